# round 3, lease m: 512-thread two-per-CU scan tiles -- scan/segmented/closure tests, then the bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py tests/test_gpu_bench_ranks.py -m gpu -q -k "scan or bench" --timeout 200 --timeout-method thread > gpurun_out/r3m_scan_tests.log 2>&1
rc=$?; echo "scan tests rc=$rc" >> gpurun_out/r3m_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 tests/cxx/bin/closure_algorithms 779 > gpurun_out/r3m_closure.log 2>&1
echo "closure rc=$?" >> gpurun_out/r3m_status.log
timeout -k 10 500 python -u bench.py --no-pmc > gpurun_out/r3m_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r3m_status.log
