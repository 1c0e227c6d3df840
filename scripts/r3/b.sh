# round 3, lease b: full GPU suite (refactored kernels + device closures) and the bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/r3b_cxx.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r3b_bench.log 2>&1
