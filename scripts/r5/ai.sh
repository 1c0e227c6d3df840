# round 5, lease ai: multiway merge with the branch-free step (lease ah: bl) and the staging loads
# flattened over the runs (one global round trip per task instead of one per run) -- the merge
# and multirank GPU tests, scripts/merge_runs_probe.py 30 on the shipped build and on the
# no-rounds ablation (timing only)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5ai
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
  tests/test_gpu_multirank.py > ${L}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> ${L}_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
tail -4 ${L}_probe.log >> ${L}_status.log
HPXHIP_LIB=$PWD/scripts/ubench/mwlib/ablate/libhpxhip.so HPXHIP_PROBE_NOCHECK=1 \
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe_ablate.log 2>&1 || exit $?
tail -4 ${L}_probe_ablate.log >> ${L}_status.log
