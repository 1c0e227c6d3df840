# round 2 measurement set: bench (with its own PMC passes), rocprofv3 kernel stats of the same command
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/r2f_bench_final.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2f_bench_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2f_bench_under_rocprof.log 2>&1
