# hybrid sort_by_key: hybrid + parity sort tests, kv probe (hybrid vs LSD)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -x -q -k "sort" --timeout 120 --timeout-method thread > gpurun_out/r2s2h_tests.log 2>&1
timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s2h_kv.log 2>&1
HPXHIP_SORT_HYBRID=0 timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s2h_kv.log 2>&1
