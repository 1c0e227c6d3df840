# round 5, lease ak: (1) lease aj's content -- the branch-free merge step in merge_in_lds too
# (k_merge: hpx::merge and the pairwise rounds): merge / multirank / C++ API GPU tests and
# scripts/merge_runs_probe.py 30; (2) the segment sort's first LDS pass ranked by LDS atomics
# (scripts/ubench/seglib/atom1, HPXHIP_SEG_ATOM1=1): the sort tests on that build, then
# scripts/sort_probe.py 30 for u64 and u32 on the shipped build and on atom1, twice each
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5ak
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
  tests/test_gpu_multirank.py tests/test_cxx_api.py -m gpu > ${L}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> ${L}_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
tail -4 ${L}_probe.log >> ${L}_status.log
A=$PWD/scripts/ubench/seglib/atom1/libhpxhip.so
HPXHIP_LIB=$A timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -k "sort" > ${L}_tests_atom1.log 2>&1
rc=$?; echo "atom1 sort tests rc=$rc" >> ${L}_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
  for v in default atom1; do
    for c in u64 u32; do
      if [ $v = default ]; then unset HPXHIP_LIB; else export HPXHIP_LIB=$A; fi
      SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 > ${L}_sort_${v}_${c}_$i.log 2>&1 || exit $?
      echo "$v $c $i: $(grep -v '^#' ${L}_sort_${v}_${c}_$i.log | tail -1)" >> ${L}_status.log
    done
  done
done
