# round 3, lease c: device closures (C++), device-planned sort, full GPU suite, sort sweep, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_cxx_api.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3c_cxx.log 2>&1
echo "cxx rc=$?" >> gpurun_out/r3c_status.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r3c_sort_tests.log 2>&1
rc=$?; echo "sort tests rc=$rc" >> gpurun_out/r3c_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r3c_sort_probe.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1
echo "suite rc=$?" >> gpurun_out/r3c_status.log
timeout -k 10 500 python -u bench.py > gpurun_out/r3c_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r3c_status.log
