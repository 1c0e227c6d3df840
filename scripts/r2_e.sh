set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2e_hybrid.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k sort -m gpu -x -v --timeout 120 --timeout-method thread >> gpurun_out/r2e_hybrid.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r2e_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e_prof -o run -- python3 bench.py --no-cpu --no-pmc > gpurun_out/r2e_prof.log 2>&1
