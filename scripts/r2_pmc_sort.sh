# round 2: kernel trace + PMC passes over the (hybrid) sort of 2^30 u64 keys, each counter group in its own run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2_sort_trace -o run -- python3 scripts/sort_probe.py > gpurun_out/r2_sort_trace.log 2>&1 || exit 1
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r2_pmc_sort$i -o run -- python3 scripts/sort_probe.py > gpurun_out/r2_pmc_sort$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo done
