# round 4, lease f: fixed look-back with 64 x K tiles per group (chain of E hand-offs K times shorter): A/B K=1 vs K=4
# on scan / copy_if / sort at 2^30, and the scan / copy_if parity tests on the K=4 build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in hpx_amd/libhpxhip.so scripts/r4/lib_k4.so; do
    HPXHIP_LIB=$lib timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4f_ab.log 2>&1 || exit $?
  done
done
HPXHIP_LIB=scripts/r4/lib_k4.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x -k "scan or copy_if" --timeout 300 --timeout-method thread > gpurun_out/r4f_tests_k4.log 2>&1
echo "k4 tests rc=$?" >> gpurun_out/r4f_status.log
