# round 4, lease bb: fill into a fresh allocation (first writes) vs again
cd $GRAFT_REPO_ROOT
timeout -k 10 120 scripts/ubench/fill > gpurun_out/r4bb_fill.log 2>&1 || exit $?
