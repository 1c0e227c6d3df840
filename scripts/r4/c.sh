# round 4, lease c: identity-free closure scans (noid_op), sort path back to r03 -- correctness first,
# then closure timing (reductions/scans), then the comparator sort timing last (the r4b run faulted in it)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_errors.py tests/test_gpu_sort_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > gpurun_out/r4c_closure_timing.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4c_closure_sort.log 2>&1 || exit $?
echo ok > gpurun_out/r4c_status.log
