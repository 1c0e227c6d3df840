# sort_by_key with 32-bit keys through the hybrid: hybrid sort tests, KV probe hybrid vs LSD
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -x -q -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r2s3b_tests.log 2>&1
timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s3b_kv.log 2>&1
HPXHIP_SORT_HYBRID=0 timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s3b_kv.log 2>&1
