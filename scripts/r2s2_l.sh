# direct per-bucket segment sort: fullsize + hybrid sort tests, sort probe timing and trace
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_sort_hybrid.py -m gpu -x -q -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r2s2l_tests.log 2>&1
timeout -k 10 200 python -u scripts/ab_probe.py > gpurun_out/r2s2l_probe.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2s2l_trace -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s2l_trace.log 2>&1
