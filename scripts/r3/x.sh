# round 3, lease x: prefix passes on persistent grids (HPXHIP_SORT_PERSIST_ALL=1) vs one workgroup per tile, same box, interleaved
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for p in 0 1; do
    for c in u64 u32; do
      echo "PERSIST_ALL=$p" >> gpurun_out/r3x_persist_all.log
      HPXHIP_SORT_PERSIST_ALL=$p SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r3x_persist_all.log 2>&1 || exit $?
    done
  done
done
