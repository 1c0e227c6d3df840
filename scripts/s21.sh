set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./scripts/ubench/scan > gpurun_out/s21_scan.log 2>&1
