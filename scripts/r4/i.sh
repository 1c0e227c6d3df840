# round 4, lease i: onesweep fixed-group look-back (LBFIX 32 / 16) vs the walk, sort at 2^30 u64 / u32;
# hybrid-sort parity tests on the LBFIX=32 build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in hpx_amd/libhpxhip.so scripts/r4/lib_fix32.so scripts/r4/lib_fix16.so; do
    for k in u64 u32; do
      echo "lib=$lib" >> gpurun_out/r4i_ab.log
      HPXHIP_LIB=$lib SORT_ONLY=$k timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4i_ab.log 2>&1 || exit $?
    done
  done
done
HPXHIP_LIB=scripts/r4/lib_fix32.so timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -q -x -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r4i_tests_fix32.log 2>&1
echo "fix32 tests rc=$?" >> gpurun_out/r4i_status.log
