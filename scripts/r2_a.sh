set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2a_cxx.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/r2a_probe.log 2>&1
