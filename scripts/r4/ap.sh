# round 4, lease ap: compressed code objects (--offload-compress) load and run; same-box A/B of the precomputed first-pass offsets
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4ap_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ap_tests.log 2>&1 || exit $?
for v in 0 1 0 1 0 1; do
  echo "NOPRE=$v" >> gpurun_out/r4ap_probe.log
  if [ $v = 1 ]; then export HPXHIP_SORT_NOPRE=1; else unset HPXHIP_SORT_NOPRE; fi
  SORT_ONLY=u64 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ap_probe.log 2>&1 || exit $?
  SORT_ONLY=u32 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ap_probe.log 2>&1 || exit $?
done
