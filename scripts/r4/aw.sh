# round 4, lease aw: look-back poll sleep 1/8/16/32 in the sort's prefix passes, alternated over fresh processes (placements)
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
for s in 1 8 16 32; do
  echo "== sleep $s rep $rep" >> gpurun_out/r4aw_lbsleep_sort.log
  timeout -k 10 120 scripts/ubench/tmpbin/sp3_s$s >> gpurun_out/r4aw_lbsleep_sort.log 2>&1 || exit $?
done
done
