set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s14_tests.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s14_probe.log 2>&1
