# round 5, lease m: seg7 (seg6 variants without the opaque ids in the one-shot kernels); histogram tiles
# strided over the grid, chunk totals from k_chunk_sums -- sort tests, probes, traces

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5m
timeout -k 10 300 ./scripts/ubench/seg7 > ${L}_seg7.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -k "sort or copy_if" \
  > ${L}_tests.log 2>&1 || exit $?
for c in u64 u64hot; do
  SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
done
for c in u64hot u64; do
  SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
done
for c in u64 u64hot; do
  SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof28_$c -o s -- \
    python3 scripts/sort_probe.py 28 > ${L}_prof28_$c.log 2>&1 || exit $?
done
