# round 4, lease ar: comparator merge sort with 16-B staging/stores in the merge passes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ar_cxx.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4ar_closure_sort.log 2>&1 || exit $?
