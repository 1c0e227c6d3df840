# PMC passes over the sort (each counter group in its own run)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_sort$i -o run -- python3 scripts/sort_probe.py > gpurun_out/pmc_sort$i.log 2>&1 || echo "pass $i failed rc=$?"
done
echo done
