# copy_if occupancy bound: copy_if parity tests, 32-bit probe, copy_if rows
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "copy_if or copyif" --timeout 120 --timeout-method thread > gpurun_out/r2s2i_tests.log 2>&1
timeout -k 10 200 python -u scripts/probe32.py > gpurun_out/r2s2i_probe32.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/r2s2i_probe.log 2>&1
