set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sort or hybrid" > gpurun_out/r2f_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc > gpurun_out/r2f_bench.log 2>&1
cd scripts/ubench && timeout -k 10 120 ./sortpass2 > ../../gpurun_out/r2f_sortpass2.log 2>&1
