set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s27_tests.log 2>&1
