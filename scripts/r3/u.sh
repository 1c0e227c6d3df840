# round 3, lease u: same-box A/B of three library builds (scripts/ab3/, built from the commits named):
#   lib_pre = 7fbb622 (before the persistent-pass id fix), lib_oe = a704c64 (id fix, odd-even rounds),
#   lib_ins = the run-insertion step of the segment sort; interleaved twice
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in pre oe ins; do
    HPXHIP_LIB=scripts/ab3/lib_$v.so timeout -k 10 120 python -u scripts/ab_probe.py >> gpurun_out/r3u_ab.log 2>&1 || exit $?
  done
done
