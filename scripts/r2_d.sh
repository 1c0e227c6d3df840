set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bench_ranks.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2d_new.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r2d_bench.log 2>&1
