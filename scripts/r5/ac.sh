# round 5, lease ac: line-aligned write-outs (copy_if pipe, multiway merge) -- parity tests and the
# merge probe
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5ac
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
  tests/test_gpu_parity.py -k "merge or copy_if" > ${L}_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
