# round 3, lease f: fixed-association FP look-back -- timing (scan7), scan parity incl. reproducibility, segmented/closure scans
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3f_scan7.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py -m gpu -q -k "scan" --timeout 200 --timeout-method thread > gpurun_out/r3f_scan_tests.log 2>&1
echo "scan tests rc=$?" >> gpurun_out/r3f_status.log
timeout -k 10 300 tests/cxx/bin/closure_algorithms 777 > gpurun_out/r3f_closure.log 2>&1
echo "closure rc=$?" >> gpurun_out/r3f_status.log
timeout -k 10 300 tests/cxx/bin/partitioned_vector > gpurun_out/r3f_pv.log 2>&1
echo "pv rc=$?" >> gpurun_out/r3f_status.log
