set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5_tests.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s5_probe.log 2>&1
timeout -k 10 200 scripts/ubench/scan > gpurun_out/s5_scan.log 2>&1
