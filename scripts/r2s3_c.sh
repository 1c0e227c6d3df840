# direct per-bucket segment sort for sort_by_key and smaller keys-only sorts: threshold ablation + forced-direct tests
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s3c_probe.log 2>&1
HPXHIP_SORT_DIRECT=4 timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s3c_probe.log 2>&1
for lg in 28 29; do
  LOGN=$lg timeout -k 10 200 python -u scripts/ab_probe.py 2>&1 | grep sort >> gpurun_out/r2s3c_probe.log
  LOGN=$lg HPXHIP_SORT_DIRECT=4 timeout -k 10 200 python -u scripts/ab_probe.py 2>&1 | grep sort | sed 's/^shipped /direct4 /' >> gpurun_out/r2s3c_probe.log
done
HPXHIP_SORT_DIRECT=100000 timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s3c_tests.log 2>&1
