# blockIdx tile order: scan / copy_if / sort parity tests, kernel probes, bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sort_hybrid.py -m gpu -x -q -k "scan or copy_if or sort or hybrid" --timeout 120 --timeout-method thread > gpurun_out/r2s2b_tests.log 2>&1
timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/r2s2b_probe.log 2>&1
timeout -k 10 200 python -u scripts/sort_probe.py > gpurun_out/r2s2b_sort.log 2>&1
timeout -k 10 400 python -u bench.py --no-pmc --no-cpu > gpurun_out/r2s2b_bench.log 2>&1
