# 32-bit keys through the hybrid sort: hybrid + fullsize sort tests, probe timing, traces (17- and 16-bit forms)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -x -q -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r2s3a_tests.log 2>&1
timeout -k 10 200 python -u scripts/ab_probe.py > gpurun_out/r2s3a_probe.log 2>&1
export KEY=u32
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3a_trace17 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3a_trace17.log 2>&1
export HPXHIP_SORT_HYBRID=16
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3a_trace16 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3a_trace16.log 2>&1
export HPXHIP_SORT_HYBRID=0
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3a_trace0 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3a_trace0.log 2>&1
