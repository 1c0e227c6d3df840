# round 5, lease b: C++ futures layer (shared_future / dataflow / unwrapping / when_all / wait_all,
# completion engine), device-side stream ordering in heat_solver; C++ test programs
cd $GRAFT_REPO_ROOT
L=gpurun_out/r5b_cxx.log
for t in "futures" "compute_api 12345" "dataflow_stencil" "stencil_partitioned" "stencil_partitioned_r04" \
         "partitioned_vector" "call_overhead" "exception_list" "for_loop_merge" "device_closures 4242" "algorithms_known_answer 20260101"; do
  echo "== $t" >> $L
  timeout -k 10 300 ./tests/cxx/bin/$t >> $L 2>&1
  rc=$?
  echo "== rc=$rc" >> $L
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
