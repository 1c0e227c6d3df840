set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2c_cxx.log 2>&1
