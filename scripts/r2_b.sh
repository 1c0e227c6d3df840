set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py tests/test_gpu_bench_ranks.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b_tests.log 2>&1
