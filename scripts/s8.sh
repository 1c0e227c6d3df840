set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 scripts/ubench/sortpass2 > gpurun_out/s8_sort.log 2>&1
