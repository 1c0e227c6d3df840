set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 scripts/ubench/stencil > gpurun_out/s10_stencil.log 2>&1
