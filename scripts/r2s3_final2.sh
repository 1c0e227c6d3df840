# round-2 final measurement set: full GPU suite, smoke, bench (PMC + host baseline), rocprofv3 stats of the same bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s3fin2_tests.log 2>&1
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2s3fin2_smoke.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r2s3fin2_bench.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3fin2_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2s3fin2_bench_under_rocprof.log 2>&1
