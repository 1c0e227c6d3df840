# round 4, lease b: the atomic segment sort -- hybrid sort tests (both segment kernels), sort probe A/B
# under rocprofv3 kernel trace, then the full GPU suite
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4b_sort_tests.log 2>&1 || exit $?
for seg in atomic stable; do
  HPXHIP_SORT_SEG=$seg SORT_ONLY=u64 timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4b_probe.log 2>&1 || exit $?
  HPXHIP_SORT_SEG=$seg SORT_ONLY=u32 timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4b_probe.log 2>&1 || exit $?
done
mkdir -p gpurun_out/r4b_prof
HPXHIP_SORT_SEG=atomic SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4b_prof.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1
echo "suite rc=$?" >> gpurun_out/r4b_status.log
timeout -k 10 300 tests/cxx/bin/closure_timing 30 > gpurun_out/r4b_closure_timing.log 2>&1
echo "closure timing rc=$?" >> gpurun_out/r4b_status.log
