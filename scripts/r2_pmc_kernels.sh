# round 2: PMC passes over scripts/kernel_probe.py (triad, reduce, scan, copy_if, stencil step at 2^30), one counter group per run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r2_pmc_k$i -o run -- python3 scripts/kernel_probe.py > gpurun_out/r2_pmc_k$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/r2_pmc_k1 gpurun_out/r2_pmc_k2 gpurun_out/r2_pmc_k3 gpurun_out/r2_pmc_k4 > gpurun_out/r2_pmc_kernels.txt
echo done
