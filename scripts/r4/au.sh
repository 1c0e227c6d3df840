# round 4, lease au: stream_after falls back to a host wait; C++ programs, call overhead, smoke
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_errors.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4au_tests.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4au_call_overhead.log 2>&1 || exit $?
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4au_smoke.log 2>&1 || exit $?
