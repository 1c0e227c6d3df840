# round 3, lease l: several reductions per for_loop (Python + C++), segmented transform_exclusive_scan, scan shapes (scan7)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_for_loop.py tests/test_gpu_segmented_layouts.py tests/test_cxx_api.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r3l_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3l_scan7.log 2>&1
echo "scan7 rc=$?" >> gpurun_out/r3l_status.log
