# round 5, lease aa: segment sort thread / item shapes for ~4096-key segments (seg9)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 ./scripts/ubench/seg9 > gpurun_out/r5aa_seg9.log 2>&1 || exit $?
