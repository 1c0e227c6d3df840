# round 4, lease e: instruction mix of the sort kernels (PMC), 2^30 u64 and u32
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r4e_counters.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" gpurun_out/r4e_counters.txt | sort -u > gpurun_out/r4e_sq.txt
i=0
for k in u64 u32; do
for pmc in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  SORT_ONLY=$k timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r4e_pmc$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4e_pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?" >> gpurun_out/r4e_status.log; }
done
done
python3 scripts/pmc_summary.py gpurun_out/r4e_pmc1 gpurun_out/r4e_pmc2 > gpurun_out/r4e_u64.txt 2>&1
python3 scripts/pmc_summary.py gpurun_out/r4e_pmc3 gpurun_out/r4e_pmc4 > gpurun_out/r4e_u32.txt 2>&1
echo done >> gpurun_out/r4e_status.log
