set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "stencil" > gpurun_out/s15_tests.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s15_probe.log 2>&1
