set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s11_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s11_smoke.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s11_probe.log 2>&1
