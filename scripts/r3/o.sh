# round 3, lease o: look-back width of the hybrid sort's prefix passes (sortpass3)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 scripts/ubench/sortpass3 > gpurun_out/r3o_sortpass3.log 2>&1
