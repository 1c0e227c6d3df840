# round 3, lease v: measurement set on the last tree (persistent-pass id fix, segment-sort run insertion) --
# full GPU suite, smoke, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r3v_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3v_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r3v_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/r3v_status.log
