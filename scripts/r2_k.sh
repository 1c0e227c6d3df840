set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q -k "sort or hybrid" --timeout 120 --timeout-method thread > gpurun_out/r2k_tests.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2k_trace -o run -- python3 scripts/sort_probe.py > gpurun_out/r2k_trace.log 2>&1
