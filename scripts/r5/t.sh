# round 5, lease t: debug the float64 one-pass run merge mismatch
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/mw_debug.py > gpurun_out/r5t_debug.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/mw_debug2.py > gpurun_out/r5t_debug2.log 2>&1 || exit $?
