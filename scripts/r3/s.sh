# round 3, lease s: small-range keys (the LSD path on persistent grids) vs uniform keys
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in u64r16 u64r24 u64; do
  SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r3s_sort_ranges.log 2>&1 || exit $?
done
mkdir -p gpurun_out/r3s_prof
SORT_ONLY=u64r16 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3s_prof.log 2>&1
