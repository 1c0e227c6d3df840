set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1_tests.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/s1_bench.log 2>&1
