# round 4, lease af: 18-bit form as the default -- sort-using GPU tests, cliff probes, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_multirank.py tests/test_gpu_parity.py tests/test_gpu_segmented_layouts.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4af_tests.log 2>&1 || exit $?
SORT_ONLY=u64corr timeout -k 10 200 python -u scripts/sort_probe.py 28 > gpurun_out/r4af_probe.log 2>&1 || exit $?
SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4af_probe.log 2>&1 || exit $?
SORT_ONLY=u64r16 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4af_probe.log 2>&1 || exit $?
SORT_ONLY=u64r24 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4af_probe.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4af_bench.log 2>&1 || exit $?
