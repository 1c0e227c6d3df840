# misaligned ranges: head split (scan, copy_if) and 1-KiB store alignment (elementwise)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segmented_layouts.py tests/test_gpu_for_loop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2k_tests.log 2>&1
timeout -k 10 300 python3 scripts/unaligned_probe.py > gpurun_out/r2s2k_unaligned.log 2>&1
