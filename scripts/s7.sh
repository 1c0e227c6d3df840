set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/s7_bench.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s7_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/s7_prof.log 2>&1
