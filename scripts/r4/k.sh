# round 4, lease k: look-back poll interval x group size (scan, copy_if at 2^30 int64)
cd $GRAFT_REPO_ROOT
for b in lb_s1_g64 lb_s4_g64 lb_s16_g64 lb_s1_g32 lb_s4_g32 lb_s16_g32; do
  timeout -k 10 150 scripts/r4/lb/$b >> gpurun_out/r4k_lb.log 2>&1 || exit $?
done
