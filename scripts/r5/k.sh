# round 5, lease k: segment sort -- run detection from a 16-bit prefix array (PRE16) and a
# persistent form that loads the next segment before sorting the current one (seg6)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5k
timeout -k 10 300 ./scripts/ubench/seg6 > ${L}_seg6.log 2>&1 || exit $?
