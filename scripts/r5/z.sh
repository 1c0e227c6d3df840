# round 5, lease z: PMC passes (one counter group per run) over the 2^30 u64 sort as it ends
# round 5 and over the pipelined copy_if (FETCH_SIZE / WRITE_SIZE)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  SORT_ONLY=u64 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r5z_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r5z_pmc_sort$i.log 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5z_pmc_cif_fetch -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5z_pmc_cif_fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5z_pmc_cif_write -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5z_pmc_cif_write.log 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/r5z_pmc_sort1 gpurun_out/r5z_pmc_sort2 gpurun_out/r5z_pmc_sort3 > gpurun_out/r5z_pmc_sort.txt 2>&1
python3 scripts/pmc_summary.py gpurun_out/r5z_pmc_cif_fetch gpurun_out/r5z_pmc_cif_write > gpurun_out/r5z_pmc_copy_if.txt 2>&1
echo ok
