# round 4, lease o: compact first histogram (1024 x 16 copies, D = 2), sort tests + probe + kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4o_probe.log 2>&1 || exit $?
SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4o_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4o_prof.log 2>&1 || exit $?
