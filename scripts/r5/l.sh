# round 5, lease l: segment sort variants again (LDS arrays declared in the shared body: the
# first seg6 build passed them down as flat pointers); histogram with a per-wave cache of hot
# cells -- sort tests, probes, traces at 2^28 and 2^30
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5l
timeout -k 10 300 ./scripts/ubench/seg6 > ${L}_seg6.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
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
