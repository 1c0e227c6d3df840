# round 3, lease a: 2^32-point stencil windowed parity + the bench with the windowed stencil check
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stencil_fullsize.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a_stencil_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r3a_bench.log 2>&1
