# round 3, lease i: copy_if write-out variants on the fixed look-back (copyif7)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 scripts/ubench/copyif7 > gpurun_out/r3i_copyif7.log 2>&1
