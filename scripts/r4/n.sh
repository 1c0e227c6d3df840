# round 4, lease n: the 17-bit first histogram counts one byte digit (k_hist), copy_if nt stores
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4n_probe.log 2>&1 || exit $?
SORT_ONLY=u64corr timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4n_probe.log 2>&1 || exit $?
SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4n_probe.log 2>&1 || exit $?
SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4n_prof.log 2>&1 || exit $?
