# round 5, lease aj: the branch-free merge step in merge_in_lds too (k_merge: hpx::merge and the
# pairwise rounds) -- merge / multirank / C++ API GPU tests, scripts/merge_runs_probe.py 30
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5aj
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
  tests/test_gpu_multirank.py tests/test_cxx_api.py -m gpu > ${L}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> ${L}_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
tail -4 ${L}_probe.log >> ${L}_status.log
