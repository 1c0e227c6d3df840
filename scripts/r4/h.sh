# round 4, lease h: fixed look-back group 64 / 48 / 40 / 32 / 24 tiles, scan and copy_if at 2^30
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in hpx_amd/libhpxhip.so scripts/r4/lib_g48.so scripts/r4/lib_g40.so scripts/r4/lib_g32.so scripts/r4/lib_g24.so; do
    HPXHIP_LIB=$lib NOSORT=1 timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4h_ab.log 2>&1 || exit $?
  done
done
