set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/perf_probe.py > gpurun_out/probe2.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_tests.log 2>&1
