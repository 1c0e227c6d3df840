# round 4, lease w: shifted-input vector scan (mutually misaligned ranges), parity + probe, two tile shapes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "misaligned or shifted" --timeout 300 --timeout-method thread > gpurun_out/r4w_tests.log 2>&1 || exit $?
HPXHIP_SCAN_SHIFT_SHAPE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "misaligned or shifted" --timeout 300 --timeout-method thread > gpurun_out/r4w_tests_shape1.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/unaligned_probe.py > gpurun_out/r4w_probe.log 2>&1 || exit $?
HPXHIP_SCAN_SHIFT_SHAPE=1 timeout -k 10 300 python -u scripts/unaligned_probe.py > gpurun_out/r4w_probe_shape1.log 2>&1 || exit $?
