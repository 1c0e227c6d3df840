# round 4, lease am: the 18-bit form's first prefix pass from precomputed tile offsets (no look-back)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -q -x -k "18" --timeout 300 --timeout-method thread > gpurun_out/r4am_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4am_probe.log 2>&1 || exit $?
SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4am_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4am_prof.log 2>&1 || exit $?
