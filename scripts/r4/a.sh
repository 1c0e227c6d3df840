# round 4, lease a: exception_list contract, launcher, iterator views -- full GPU suite, smoke, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r4a_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4a_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4a_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/r4a_status.log
