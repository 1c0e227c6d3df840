# round 3, lease t: persistent passes with per-tile id re-derivation (102-105 VGPRs, was 156) and the segment sort's run-insertion step --
# sort tests, then small-range keys (LSD path, persistent grids) vs uniform keys, then kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_parity.py -m gpu -q -k "sort" --timeout 200 --timeout-method thread > gpurun_out/r3t_sort_tests.log 2>&1
rc=$?; echo "sort tests rc=$rc" >> gpurun_out/r3t_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
for c in u64r16 u64r24 u64 u32 pairs; do
  SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r3t_sort_ranges.log 2>&1 || exit $?
done
mkdir -p gpurun_out/r3t_prof
SORT_ONLY=u64r24 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3t_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/r3t_status.log
