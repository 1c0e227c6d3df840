# same-box A/B of the line-aligned k_bucket_sort write-back (old / new / old / new)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
  for v in old new; do
    HPXHIP_LIB=$PWD/scripts/ablib/libhpxhip_$v.so timeout -k 10 200 python -u scripts/ab_probe.py 2>&1 | grep sort >> gpurun_out/r2s3f_ab.log
    HPXHIP_LIB=$PWD/scripts/ablib/libhpxhip_$v.so timeout -k 10 200 python -u scripts/kv_probe.py 2>&1 | grep "u64/u64\|u32/u64" | sed "s/^/$v /" >> gpurun_out/r2s3f_ab.log
  done
done
