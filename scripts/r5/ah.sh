# round 5, lease ah: multiway merge round variants (scripts/ubench/mwlib.sh) -- bl = branch-free
# merge step (one LDS read per output), blw4 = bl at 4 waves per SIMD, bl16 = bl with 128 threads x 16
# keys, t128i16 = shipped step with 128 x 16, ablate = no LDS rounds (timing only, wrong output);
# the merge_runs tests per variant, then scripts/merge_runs_probe.py 30
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r5ah
for v in default bl blw4 bl16 t128i16 ablate; do
  if [ $v = default ]; then unset HPXHIP_LIB; else export HPXHIP_LIB=$PWD/scripts/ubench/mwlib/$v/libhpxhip.so; fi
  echo "== $v" >> ${L}_status.log
  if [ $v != ablate ]; then
    timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_merge_sort.py \
      -k "merge_runs" > ${L}_tests_$v.log 2>&1
    rc=$?; echo "$v tests rc=$rc" >> ${L}_status.log
    if [ $rc -gt 1 ]; then exit $rc; fi
  fi
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe_$v.log 2>&1 || exit $?
  tail -4 ${L}_probe_$v.log >> ${L}_status.log
done
