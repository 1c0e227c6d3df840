# round 4, lease ae: the 18-bit sort form (HPXHIP_SORT_HYBRID=18): sort tests in all forms, probe 17 vs 18, kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ae_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4ae_probe17.log 2>&1 || exit $?
HPXHIP_SORT_HYBRID=18 timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4ae_probe18.log 2>&1 || exit $?
HPXHIP_SORT_HYBRID=18 SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ae_prof18 -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4ae_prof18.log 2>&1 || exit $?
