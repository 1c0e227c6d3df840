# round 5, lease p: one-pass merge of up to 8 sorted runs (hpxhip_merge_runs) -- parity tests,
# 2^30 x 8 runs element for element, single-rank and 4-rank segmented sorts, timing vs pairwise
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5p
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
  > ${L}_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
  > ${L}_multirank.log 2>&1 || exit $?
