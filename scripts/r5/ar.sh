# round 5, lease ar: full validation of the tree -- GPU suite, smoke, bench, rocprofv3 kernel trace
# + stats of the bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5ar
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > ${L}_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> ${L}_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > ${L}_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
echo "bench ok" >> ${L}_status.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 bench.py --no-pmc --no-cpu > ${L}_bench_under_rocprof.log 2>&1 || exit $?
echo "rocprof ok" >> ${L}_status.log
