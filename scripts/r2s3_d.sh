# sort_by_key at 2^29 pairs: direct per-bucket segments (default) vs host-packed (HPXHIP_SORT_DIRECT=0)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LOGN=29 timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s3d_probe.log 2>&1
LOGN=29 HPXHIP_SORT_DIRECT=0 timeout -k 10 200 python -u scripts/kv_probe.py 2>&1 | sed 's/^hybrid /packed /' >> gpurun_out/r2s3d_probe.log
