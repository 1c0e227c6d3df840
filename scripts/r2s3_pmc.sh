# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter per run) over the hybrid sort of 2^30 keys, u64 (direct per-bucket path) and u32
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for key in u64 u32; do
  export KEY=$key
  i=0
  for pmc in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r2s3_pmc_${key}_$i -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3_pmc_${key}_$i.log 2>&1 || { echo "pass $key $i failed rc=$?"; exit 1; }
  done
done
echo done
