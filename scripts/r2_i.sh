set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2i_gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2i_smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2i_bench.log 2>&1
