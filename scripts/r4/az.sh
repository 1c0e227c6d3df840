# round 4, lease az: the rebuilt library after the reverted experiment: smoke, sort / scan / copy_if parity
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4az_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4az_tests.log 2>&1 || exit $?
