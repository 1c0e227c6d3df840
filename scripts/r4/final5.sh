# round 4, final lease (5), the tree as it ends the round: full GPU suite, smoke, bench, rocprofv3 kernel trace + stats of the bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4final5_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r4final5_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4final5_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4final5_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/r4final5_status.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final5_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4final5_bench_under_rocprof.log 2>&1 || exit $?
echo "rocprof ok" >> gpurun_out/r4final5_status.log
