# round 3, lease d (re-entry): whole tree after the last commit -- C++ tests, full GPU suite, smoke, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_cxx_api.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3d_cxx.log 2>&1
rc=$?; echo "cxx rc=$rc" >> gpurun_out/r3d_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r3d_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3d_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r3d_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r3d_status.log
