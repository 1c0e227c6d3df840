# scan nt stores: scan/fullsize parity tests + bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py -m gpu -x -q -k "scan or fullsize or layout or multirank" --timeout 120 --timeout-method thread > gpurun_out/r2s2e_tests.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras > gpurun_out/r2s2e_bench.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras >> gpurun_out/r2s2e_bench.log 2>&1
