set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_merge_sort.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2h_cxx.log 2>&1
