# round 4, lease an: precomputed-offset first pass with counter-ordered tiles; PMC write traffic of that pass
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SORT_ONLY=u64 timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4an_probe.log 2>&1 || exit $?
SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4an_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4an_prof.log 2>&1 || exit $?
SORT_ONLY=u64 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_onesweep --output-format csv -d gpurun_out/r4an_pmc -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4an_pmc.log 2>&1 || exit $?
