#!/bin/bash
# Variant builds of libhpxhip.so for the sort probes (round 5): sort.hip
# compiled with -D flags, linked with the shipped objects of the other sources
# (make lib first).  Output: scripts/ubench/seglib/<name>/libhpxhip.so
# usage: bash scripts/ubench/seglib.sh <name> [-DHPXHIP_...=...]...
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
out=scripts/ubench/seglib/$name
mkdir -p $out
HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off --offload-compress -Wall -Wno-unused-result -Wno-unused-function -Iinclude"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c hpx_amd/csrc/sort.hip -o $out/sort.o
objs=""
for k in runtime elementwise reduce scan copy_if merge stencil; do objs="$objs build/csrc/$k.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libhpxhip.so $objs $out/sort.o
rm -f $out/sort.o
echo "built $out/libhpxhip.so ($*)"
