# round 5, lease v: one-pass run merge with a padded LDS layout (one pad key every 8) -- tests, timing

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5v
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
  > ${L}_tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
  python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
  > ${L}_multirank.log 2>&1 || exit $?
