# round 4, lease ai: 18-bit form, the top-byte pass (16-bit fallback only): persistent vs one workgroup per tile (HPXHIP_B_PLAIN)
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  echo "B_PLAIN=$v" >> gpurun_out/r4ai_probe.log
  if [ $v = 1 ]; then export HPXHIP_B_PLAIN=1; else unset HPXHIP_B_PLAIN; fi
  SORT_ONLY=u64 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ai_probe.log 2>&1 || exit $?
  SORT_ONLY=u64r16 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ai_probe.log 2>&1 || exit $?
  SORT_ONLY=u64r24 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ai_probe.log 2>&1 || exit $?
done
