# round 3, lease n: copy_if tile shapes with more workgroups per CU (copyif7)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 scripts/ubench/copyif7 > gpurun_out/r3n_copyif7.log 2>&1
