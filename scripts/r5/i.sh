# round 5, lease i: pipelined persistent copy_if against the shipped kernel (copyif9);
# segment sort phase split and register-side run detection (seg5)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5i
timeout -k 10 240 ./scripts/ubench/copyif9 > ${L}_copyif9.log 2>&1 || exit $?
timeout -k 10 240 ./scripts/ubench/seg5 > ${L}_seg5.log 2>&1 || exit $?
