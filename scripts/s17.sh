set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "copy_if" --timeout 120 --timeout-method thread > gpurun_out/s17_tests.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s17_probe.log 2>&1
