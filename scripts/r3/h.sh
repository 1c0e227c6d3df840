# round 3, lease h: persistent onesweep / segment-sort grids in the device-planned sort -- sort tests, probe, kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_parity.py -m gpu -q -k "sort" --timeout 200 --timeout-method thread > gpurun_out/r3h_sort_tests.log 2>&1
rc=$?; echo "sort tests rc=$rc" >> gpurun_out/r3h_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r3h_sort_probe.log 2>&1 || exit $?
mkdir -p gpurun_out/r3h_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3h_prof -o run --output-format csv -- python3 scripts/sort_probe.py 30 > gpurun_out/r3h_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/r3h_status.log
