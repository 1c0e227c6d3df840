# line-aligned write-back in k_bucket_sort: hybrid sort tests (incl. forced direct path), sort probes, WRITE_SIZE pass
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s3e_tests.log 2>&1
timeout -k 10 200 python -u scripts/ab_probe.py > gpurun_out/r2s3e_probe.log 2>&1
timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s3e_probe.log 2>&1
export KEY=u64
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2s3e_pmc_u64 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3e_pmc_u64.log 2>&1
