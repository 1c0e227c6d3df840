# full GPU suite after the session-2 changes
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2j_tests.log 2>&1
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2s2j_smoke.log 2>&1
