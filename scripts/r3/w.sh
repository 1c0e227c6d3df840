# round 3, lease w: kernel stats of the 2^30 u64 sort on the last tree
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3w_prof
SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3w_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3w_prof.log 2>&1
