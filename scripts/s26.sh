set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_for_loop.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s26_tests.log 2>&1
