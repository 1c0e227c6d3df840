# round 5, lease y: pipelined persistent scan (scan8) against the shipped k_scan shapes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 ./scripts/ubench/scan8 > gpurun_out/r5y_scan8.log 2>&1 || exit $?
