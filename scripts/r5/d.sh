# round 5, lease d: first prefix pass (offset-fed) tile order: counter vs blockIdx vs XCD regions
cd $GRAFT_REPO_ROOT
timeout -k 10 300 ./scripts/ubench/sortpass5 > gpurun_out/r5d_sortpass5.log 2>&1 || exit $?
