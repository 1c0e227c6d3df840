# round 4, lease as: merge tiles of 4096 (256 threads x 16 items): merge API tests, C++ closures, comparator sort timing, merge probe
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_merge_sort.py tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4as_tests.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4as_closure_sort.log 2>&1 || exit $?
