# round 4, lease ao: same-box A/B, first prefix pass from precomputed tile offsets vs look-back (HPXHIP_SORT_NOPRE)
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1 0 1; do
  echo "NOPRE=$v" >> gpurun_out/r4ao_probe.log
  if [ $v = 1 ]; then export HPXHIP_SORT_NOPRE=1; else unset HPXHIP_SORT_NOPRE; fi
  SORT_ONLY=u64 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ao_probe.log 2>&1 || exit $?
  SORT_ONLY=u32 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ao_probe.log 2>&1 || exit $?
done
