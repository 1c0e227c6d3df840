# round 4, lease x: one-rank RCCL run of the segmented orchestration; full GPU suite; smoke
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v -x --timeout 240 --timeout-method thread > gpurun_out/r4x_multirank.log 2>&1 || exit $?
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4x_tests.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r4x_status.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4x_smoke.log 2>&1 || exit $?
