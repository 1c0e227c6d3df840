# round 4, lease ax: sort look-back back-off 8 (HPXHIP_SORT_LB_SLEEP): sort tests, then the bench (sort rows)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_merge_sort.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ax_tests.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4ax_bench.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4ax_bench2.log 2>&1 || exit $?
