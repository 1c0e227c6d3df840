# round 4, lease t: copy_if 16-B stores + one-hop look-back (8-byte), parity + C++ programs + timing + bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_errors.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4t_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4t_cxx.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > gpurun_out/r4t_closure_timing.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4t_bench.log 2>&1 || exit $?
