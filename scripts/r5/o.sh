# round 5, lease o: histogram prefetches the next tile (double-buffered counts); 2^30 sorts
# element for element against a closed form; C++ programs (closure copy_if on the pipelined
# kernel); sort tests, probes and a 2^30 trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py \
  -k "element_exact or permutation_and_order or oversized" > ${L}_fullsize.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cxx_api.py \
  tests/test_gpu_sort_hybrid.py > ${L}_tests.log 2>&1 || exit $?
for c in u64 u32 u64hot; do
  SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
done
for c in u64hot u64corr u64; do
  SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
done
SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof30_u64 -o s -- \
  python3 scripts/sort_probe.py 30 > ${L}_prof30_u64.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > ${L}_closure_timing.log 2>&1 || exit $?
