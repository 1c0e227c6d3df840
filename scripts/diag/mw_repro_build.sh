#!/bin/bash
# Reproducer of the r05 k_mw_merge miscompile (round 6):
# the merge.hip of commit 8a18d38 (rounds compare xf(a) < xf(b) on raw keys)
# built twice with today's toolchain -- as it shipped (default occupancy
# bound, no SGPR spills) and with __launch_bounds__(256, 8) (20-26 SGPR
# spills), the build that wrote float64 keys in their ordered-bit form --
# each linked with the shipped objects of the other sources, plus the ISA
# of both (--save-temps style -S) for the analysis in
# profiles/r06_mw_merge_miscompile.txt.  Run in the container (needs git);
# the libraries travel to the GPU box, scripts/diag/mw_repro.py runs them.
set -e
cd "$(dirname "$0")/../.."
out=scripts/diag/mw_old
mkdir -p $out/default $out/minw8
git show 8a18d38:hpx_amd/csrc/merge.hip > $out/merge_old.hip
sed 's/__launch_bounds__(kMwThreads) void k_mw_merge/__launch_bounds__(kMwThreads, 8) void k_mw_merge/' \
    $out/merge_old.hip > $out/merge_old8.hip
grep -q "__launch_bounds__(kMwThreads, 8) void k_mw_merge" $out/merge_old8.hip
HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off --offload-compress -Wno-unused-result -Iinclude -Ihpx_amd/csrc"
objs=""
for k in runtime elementwise reduce scan copy_if sort stencil; do objs="$objs build/csrc/$k.o"; done
for v in default minw8; do
    src=$out/merge_old.hip
    [ $v = minw8 ] && src=$out/merge_old8.hip
    /opt/rocm/bin/hipcc $HIPFLAGS -Rpass-analysis=kernel-resource-usage -c $src -o $out/$v/merge.o 2> $out/$v/usage.txt
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/$v/libhpxhip.so $objs $out/$v/merge.o
    rm -f $out/$v/merge.o
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iinclude -Ihpx_amd/csrc \
        --cuda-device-only -S $src -o $out/$v/merge.s 2>/dev/null
done
echo "built $out/{default,minw8}/libhpxhip.so"
