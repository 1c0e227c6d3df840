# round 3, lease e: call_overhead diagnosis (task sort + reduce), f64 scan tile shapes (scan7), scan parity with the deferred round carry
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 tests/cxx/bin/compute_api 12345 > gpurun_out/r3e_compute_api.log 2>&1
echo "compute_api rc=$?" >> gpurun_out/r3e_status.log
timeout -k 10 120 tests/cxx/bin/call_overhead > gpurun_out/r3e_call_overhead.log 2>&1
echo "call_overhead rc=$?" >> gpurun_out/r3e_status.log
timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3e_scan7.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -k "scan" --timeout 120 --timeout-method thread > gpurun_out/r3e_scan_tests.log 2>&1
echo "scan tests rc=$?" >> gpurun_out/r3e_status.log
timeout -k 10 300 tests/cxx/bin/closure_algorithms 777 > gpurun_out/r3e_closure.log 2>&1
echo "closure rc=$?" >> gpurun_out/r3e_status.log
