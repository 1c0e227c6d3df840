# per-kernel tile-id order: full GPU suite + bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2c_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2s2c_bench.log 2>&1
