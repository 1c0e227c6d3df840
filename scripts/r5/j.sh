# round 5, lease j: histogram peels only shared cells (uniform keys: one ballot per key);
# pipelined copy_if shipped: copy_if parity tests, sort tests, probes uniform/hot/corr, traces
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "copy_if" > ${L}_tests_copyif.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
  tests/test_gpu_merge_sort.py > ${L}_tests.log 2>&1 || exit $?
for c in u64 u32 u64hot; do
  SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
done
for c in u64hot u64corr u64; do
  SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
done
for c in u64 u64hot; do
  SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof_$c -o s -- \
    python3 scripts/sort_probe.py 30 > ${L}_prof_$c.log 2>&1 || exit $?
done
