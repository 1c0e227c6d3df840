# round 4, lease aq: PMC passes over the 2^30 u64 sort in its r04 form (18-bit, first pass from tile offsets)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export SORT_ONLY=u64
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r4aq_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4aq_pmc_sort$i.log 2>&1 || { echo "pmc pass $i failed rc=$?" >> gpurun_out/r4aq_status.log; exit 1; }
done
echo "pmc ok" >> gpurun_out/r4aq_status.log
