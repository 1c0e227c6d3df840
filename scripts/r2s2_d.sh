# HBM segment arena: full GPU suite, then bench step lines with and without the arena (fresh processes)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2d_tests.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras >> gpurun_out/r2s2d_bench_arena.log 2>&1
  HPXHIP_ARENA_GIB=0 timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras >> gpurun_out/r2s2d_bench_noarena.log 2>&1
done
