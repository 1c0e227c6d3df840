# session-2 re-entry check: full GPU suite + bench on the rebuilt tree
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2a_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2s2a_bench.log 2>&1
