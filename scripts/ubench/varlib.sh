#!/bin/bash
# Variant builds of libhpxhip.so (round 6): one source of hpx_amd/csrc
# compiled with -D flags, linked with the shipped objects of the others (make
# lib first).  Output: scripts/ubench/seglib/<name>/libhpxhip.so
# usage: bash scripts/ubench/varlib.sh <name> <source, e.g. stencil> [-DHPXHIP_...=...]...
set -e
cd "$(dirname "$0")/../.."
name=$1; src=$2; shift 2
out=scripts/ubench/seglib/$name
mkdir -p $out
HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off --offload-compress -Wall -Wno-unused-result -Wno-unused-function -Iinclude"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c hpx_amd/csrc/$src.hip -o $out/$src.o
objs=""
for k in runtime elementwise reduce scan copy_if sort merge stencil; do
  if [ $k = $src ]; then objs="$objs $out/$src.o"; else objs="$objs build/csrc/$k.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libhpxhip.so $objs
rm -f $out/$src.o
echo "built $out/libhpxhip.so ($src $*)"
