# round 4, lease d: comparator-sort timing (race fixed), C++ call overhead (event get), match_digit A/B
# (builtin ballot vs round-3 asm), full suite, smoke, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4d_closure_sort.log 2>&1 || exit $?
timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4d_call_overhead.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in hpx_amd/libhpxhip.so scripts/r4/lib_asm.so; do
    for k in u64 u32; do
      echo "lib=$lib" >> gpurun_out/r4d_ab.log
      HPXHIP_LIB=$lib SORT_ONLY=$k timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4d_ab.log 2>&1 || exit $?
    done
  done
done
mkdir -p gpurun_out/r4d_prof
SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4d_prof.log 2>&1 || exit $?
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r4d_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4d_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r4d_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/r4d_status.log
for c in u64corr u64hot; do SORT_ONLY=$c timeout -k 10 300 python -u scripts/sort_probe.py 28 >> gpurun_out/r4d_cliff.log 2>&1 || exit $?; done
