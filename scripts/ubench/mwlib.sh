#!/bin/bash
# Variant builds of libhpxhip.so for the multiway merge probes (round 5):
# merge.hip compiled with -D flags, linked with the shipped objects of the
# other sources (make lib first).  Output: scripts/ubench/mwlib/<name>/libhpxhip.so
# usage: bash scripts/ubench/mwlib.sh <name> [-DHPXHIP_MW_...=...]...
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
out=scripts/ubench/mwlib/$name
mkdir -p $out
HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off --offload-compress -Wall -Wno-unused-result -Wno-unused-function -Iinclude"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c hpx_amd/csrc/merge.hip -o $out/merge.o
objs=""
for k in runtime elementwise reduce scan copy_if sort stencil; do objs="$objs build/csrc/$k.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libhpxhip.so $objs $out/merge.o
rm -f $out/merge.o
echo "built $out/libhpxhip.so ($*)"
