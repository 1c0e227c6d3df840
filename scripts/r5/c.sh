# round 5, lease c: oversized-bucket finish (segmented LSD), range errors from clamped scatters,
# deterministic device_closures pending check, 4-rank host-staged multirank; sort probes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5c
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
  tests/test_gpu_errors.py tests/test_gpu_merge_sort.py "tests/test_cxx_api.py" tests/test_gpu_multirank.py \
  > ${L}_tests.log 2>&1 || exit $?
for c in u64hot u64corr u64; do
  SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
done
for c in u64 u32 u64hot; do
  SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k sort \
  > ${L}_fullsize.log 2>&1 || exit $?
