# round 5, lease f: kernel trace of the skewed sorts (u64hot at 2^28 and 2^30)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lg in 28 30; do
  SORT_ONLY=u64hot timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5f_prof$lg -o hot -- \
    python3 scripts/sort_probe.py $lg > gpurun_out/r5f_hot$lg.log 2>&1 || exit $?
done
