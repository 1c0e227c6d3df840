# round 4, lease ag: small key ranges (r16, r24) under the 17- and 18-bit forms on one box
cd $GRAFT_REPO_ROOT
for m in 17 18 17 18; do
  echo "HPXHIP_SORT_HYBRID=$m" >> gpurun_out/r4ag_probe.log
  HPXHIP_SORT_HYBRID=$m SORT_ONLY=u64r16 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ag_probe.log 2>&1 || exit $?
  HPXHIP_SORT_HYBRID=$m SORT_ONLY=u64r24 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ag_probe.log 2>&1 || exit $?
done
