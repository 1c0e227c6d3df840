# round 3, lease p: measurement set on the tree -- full GPU suite, smoke, bench, rocprofv3 kernel stats of the bench, PMC passes over the 2^30 u64 sort
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r3p_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3p_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r3p_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/r3p_status.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r3p_bench_under_rocprof.log 2>&1 || exit $?
echo "rocprof ok" >> gpurun_out/r3p_status.log
export SORT_ONLY=u64
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r3p_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3p_pmc_sort$i.log 2>&1 || { echo "pmc pass $i failed rc=$?" >> gpurun_out/r3p_status.log; exit 1; }
done
echo "pmc ok" >> gpurun_out/r3p_status.log
