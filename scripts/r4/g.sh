# round 4, lease g: fixed look-back group of 64 (shipped) vs 32 vs 16 tiles at 2^30, + parity of the 16 build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in hpx_amd/libhpxhip.so scripts/r4/lib_g32.so scripts/r4/lib_g16.so; do
    HPXHIP_LIB=$lib timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4g_ab.log 2>&1 || exit $?
  done
done
HPXHIP_LIB=scripts/r4/lib_g16.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x -k "scan or copy_if" --timeout 300 --timeout-method thread > gpurun_out/r4g_tests_g16.log 2>&1
echo "g16 tests rc=$?" >> gpurun_out/r4g_status.log
