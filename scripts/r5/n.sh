# round 5, lease n: segment sort PRE16 in the shipped kernel (seg8 A/B); 2^30 traces of the
# uniform and hot sorts with the strided histogram
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5n
timeout -k 10 300 ./scripts/ubench/seg8 > ${L}_seg8.log 2>&1 || exit $?
for c in u64 u64hot; do
  SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof30_$c -o s -- \
    python3 scripts/sort_probe.py 30 > ${L}_prof30_$c.log 2>&1 || exit $?
done
