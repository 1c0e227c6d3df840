# round 4, lease ak: second histogram skips constant digits; sort tests (all forms), probes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ak_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4ak_probe.log 2>&1 || exit $?
for c in u64r16 u64r24; do SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ak_probe.log 2>&1 || exit $?; done
for c in u64corr u64hot; do SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4ak_probe.log 2>&1 || exit $?; done
