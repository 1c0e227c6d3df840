# round 4, lease aj: kernel traces of the u64r16 sort (keys below 2^16) under the 17- and 18-bit forms, second count skipping constant digits
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in 17 18; do
  HPXHIP_SORT_HYBRID=$m SORT_ONLY=u64r16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4aj_prof$m -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4aj_prof$m.log 2>&1 || exit $?
done
