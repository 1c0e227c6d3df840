set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 scripts/ubench/scan > gpurun_out/s6_scan.log 2>&1
