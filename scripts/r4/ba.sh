# round 4, lease ba: fill (write-only stream) shapes at 2^30 doubles
cd $GRAFT_REPO_ROOT
timeout -k 10 120 scripts/ubench/fill > gpurun_out/r4ba_fill.log 2>&1 || exit $?
timeout -k 10 120 scripts/ubench/fill >> gpurun_out/r4ba_fill.log 2>&1 || exit $?
