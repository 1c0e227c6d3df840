# round 5, lease e: XCD-region prefix passes (XREG; the top-9 pass in 8 field regions with joint-histogram
# bin starts), bounded oversized-bucket finish v2 (LDS seg table, optimistic plan): sort tests + probes + kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
  tests/test_gpu_merge_sort.py > ${L}_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k sort \
  >> ${L}_tests.log 2>&1 || exit $?
for c in u64 u32; do
  SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
done
for c in u64hot u64corr u64; do
  SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
done
SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o sort -- \
  python3 scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
