# round 3, lease r: 2^30 FP scan reproducibility test
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -k "reproducible" --timeout 250 --timeout-method thread > gpurun_out/r3r_tests.log 2>&1
