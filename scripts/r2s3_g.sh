# keys-only plain write-back restored, sort_by_key aligned: hybrid sort tests + smoke
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -k "sort" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s3g_tests.log 2>&1
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2s3g_smoke.log 2>&1
