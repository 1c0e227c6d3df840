# round 4, lease r: one-hop fixed look-back A/B (scan + copy_if, 2^30 int64)
cd $GRAFT_REPO_ROOT
for b in lb_onehop0 lb_onehop1 lb_onehop0 lb_onehop1; do
  timeout -k 10 150 scripts/r4/lb/$b >> gpurun_out/r4r_onehop.log 2>&1 || exit $?
done
