# round 4, lease u: closure copy_if back to its r03 form; bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > gpurun_out/r4u_closure_timing.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4u_bench.log 2>&1 || exit $?
