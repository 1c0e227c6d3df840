# round 5, lease ag: seg10 -- the segment sort's one-pass atomic ranking (ONE = 12/13/14) against the
# shipped two-pass form at 2^30 u64 in 4096-key segments
cd $GRAFT_REPO_ROOT
L=gpurun_out/r5ag
timeout -k 10 300 scripts/ubench/seg10 > ${L}_seg10.log 2>&1 || exit $?
