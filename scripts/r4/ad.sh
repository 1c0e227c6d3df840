# round 4, lease ad: DPP neighbour shift in the elementwise shifted kernels (and the scan's), parity + probe
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "shifted or misaligned or unaligned" --timeout 300 --timeout-method thread > gpurun_out/r4ad_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/unaligned_probe.py > gpurun_out/r4ad_probe.log 2>&1 || exit $?
