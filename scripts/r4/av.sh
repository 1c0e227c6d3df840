# round 4, lease av: look-back poll sleep (HPXHIP_LB_SLEEP 0/1/3/8) in the sort's prefix passes (sortpass3 ubench)
cd $GRAFT_REPO_ROOT
for s in 1 0 3 8 1; do
  echo "== sleep $s" >> gpurun_out/r4av_lbsleep_sort.log
  timeout -k 10 120 scripts/ubench/tmpbin/sp3_s$s >> gpurun_out/r4av_lbsleep_sort.log 2>&1 || exit $?
done
