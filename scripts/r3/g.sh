# round 3, lease g: fixed-association look-back for every scan -- copy_if variants (copyif7), full GPU suite, smoke, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 scripts/ubench/copyif7 > gpurun_out/r3g_copyif7.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r3g_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3g_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r3g_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r3g_status.log
