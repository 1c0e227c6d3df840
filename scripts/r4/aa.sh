# round 4, lease aa: when_all completes by waiting on its inputs (no callbacks unless a continuation arms it)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4aa_cxx.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4aa_call_overhead.log 2>&1 || exit $?
