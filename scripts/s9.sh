set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 scripts/ubench/copyif > gpurun_out/s9_copyif.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "copy_if or copyif" > gpurun_out/s9_tests.log 2>&1
