# round-2 measurement set (session 2): bench with PMC + host baseline, rocprofv3 kernel stats of the same command
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > gpurun_out/r2s2f_bench.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s2f_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2s2f_bench_under_rocprof.log 2>&1
