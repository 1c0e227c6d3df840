# round 4, lease ay: same-box A/B of the sort's look-back back-off, 1 vs 8 (two library builds, alternated processes)
cd $GRAFT_REPO_ROOT
for rep in 1 2 3 4; do
for s in 1 8; do
  HPXHIP_LIB=scripts/ubench/tmpbin/libhpxhip_s$s.so timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4ay_ab_sort_lbsleep.log 2>&1 || exit $?
done
done
