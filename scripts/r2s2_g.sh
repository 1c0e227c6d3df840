# roctx ranges: GPU parity subset incl. the annotation test, then a marker trace of the perf probe
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2g_tests.log 2>&1
export HPXHIP_ROCTX=1 LOGN=26
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/r2s2g_marker -o run -- python3 scripts/perf_probe.py > gpurun_out/r2s2g_marker.log 2>&1
