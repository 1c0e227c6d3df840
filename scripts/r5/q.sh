# round 5, lease q: where the one-pass run merge's time goes (kernel trace of the probe at 2^30);
# multirank segmented sorts with empty sample runs fixed
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5q
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
  python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
  > ${L}_multirank.log 2>&1 || exit $?
