# round 4, lease j: lazy completion callbacks (C++ futures), scans on 32-tile look-back groups --
# C++ programs + call overhead, full GPU suite, smoke, bench, rocprofv3 kernel stats of the bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4j_cxx.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4j_call_overhead.log 2>&1 || exit $?
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r4j_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4j_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4j_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/r4j_status.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4j_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4j_bench_under_rocprof.log 2>&1 || exit $?
echo "rocprof ok" >> gpurun_out/r4j_status.log
