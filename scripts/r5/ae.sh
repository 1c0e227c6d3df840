# round 5, lease ae: multiway merge with ordered bits staged in LDS -- the merge_runs tests and the
# merge probe for the shipped build (256 threads) and the variant builds that miscompiled before
# (512 threads, 256 x 8 waves) plus 512 x 2 waves
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5ae
for v in default t512 t256w8 t512w2; do
  if [ $v = default ]; then unset HPXHIP_LIB; else export HPXHIP_LIB=$PWD/scripts/ubench/mwlib/$v/libhpxhip.so; fi
  echo "== $v" >> ${L}_status.log
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    -k "merge_runs" > ${L}_tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe_$v.log 2>&1 || exit $?
done
