# Lease scripts of round 2, session 2 (scripts/r2s2_*.sh): what each gpurun call of that round ran,
# kept as one shell function per former file (provenance of the profiles/
# logs that cite them).  `bash scripts/leases/r2s2.sh NAME` runs lease NAME.

# ---- scripts/r2s2_a.sh
lease_r2s2_a() {
  # session-2 re-entry check: full GPU suite + bench on the rebuilt tree
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2a_tests.log 2>&1
  timeout -k 10 400 python -u bench.py > gpurun_out/r2s2a_bench.log 2>&1
}

# ---- scripts/r2s2_b.sh
lease_r2s2_b() {
  # blockIdx tile order: scan / copy_if / sort parity tests, kernel probes, bench
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sort_hybrid.py -m gpu -x -q -k "scan or copy_if or sort or hybrid" --timeout 120 --timeout-method thread > gpurun_out/r2s2b_tests.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/r2s2b_probe.log 2>&1
  timeout -k 10 200 python -u scripts/sort_probe.py > gpurun_out/r2s2b_sort.log 2>&1
  timeout -k 10 400 python -u bench.py --no-pmc --no-cpu > gpurun_out/r2s2b_bench.log 2>&1
}

# ---- scripts/r2s2_c.sh
lease_r2s2_c() {
  # per-kernel tile-id order: full GPU suite + bench
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2c_tests.log 2>&1
  timeout -k 10 400 python -u bench.py > gpurun_out/r2s2c_bench.log 2>&1
}

# ---- scripts/r2s2_d.sh
lease_r2s2_d() {
  # HBM segment arena: full GPU suite, then bench step lines with and without the arena (fresh processes)
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2d_tests.log 2>&1
  for i in 1 2 3; do
    timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras >> gpurun_out/r2s2d_bench_arena.log 2>&1
    HPXHIP_ARENA_GIB=0 timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras >> gpurun_out/r2s2d_bench_noarena.log 2>&1
  done
}

# ---- scripts/r2s2_e.sh
lease_r2s2_e() {
  # scan nt stores: scan/fullsize parity tests + bench
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py -m gpu -x -q -k "scan or fullsize or layout or multirank" --timeout 120 --timeout-method thread > gpurun_out/r2s2e_tests.log 2>&1
  timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras > gpurun_out/r2s2e_bench.log 2>&1
  timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-extras >> gpurun_out/r2s2e_bench.log 2>&1
}

# ---- scripts/r2s2_f.sh
lease_r2s2_f() {
  # round-2 measurement set (session 2): bench with PMC + host baseline, rocprofv3 kernel stats of the same command
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 500 python -u bench.py > gpurun_out/r2s2f_bench.log 2>&1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s2f_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2s2f_bench_under_rocprof.log 2>&1
}

# ---- scripts/r2s2_final.sh
lease_r2s2_final() {
  # round-2 final measurement set: full GPU suite, smoke, bench (PMC + host baseline), rocprofv3 stats of the same bench
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2fin_tests.log 2>&1
  timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2fin_smoke.log 2>&1
  timeout -k 10 500 python -u bench.py > gpurun_out/r2fin_bench.log 2>&1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2fin_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2fin_bench_under_rocprof.log 2>&1
}

# ---- scripts/r2s2_g.sh
lease_r2s2_g() {
  # roctx ranges: GPU parity subset incl. the annotation test, then a marker trace of the perf probe
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2g_tests.log 2>&1
  export HPXHIP_ROCTX=1 LOGN=26
  timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/r2s2g_marker -o run -- python3 scripts/perf_probe.py > gpurun_out/r2s2g_marker.log 2>&1
}

# ---- scripts/r2s2_h.sh
lease_r2s2_h() {
  # hybrid sort_by_key: hybrid + parity sort tests, kv probe (hybrid vs LSD)
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -x -q -k "sort" --timeout 120 --timeout-method thread > gpurun_out/r2s2h_tests.log 2>&1
  timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s2h_kv.log 2>&1
  HPXHIP_SORT_HYBRID=0 timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s2h_kv.log 2>&1
}

# ---- scripts/r2s2_i.sh
lease_r2s2_i() {
  # copy_if occupancy bound: copy_if parity tests, 32-bit probe, copy_if rows
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "copy_if or copyif" --timeout 120 --timeout-method thread > gpurun_out/r2s2i_tests.log 2>&1
  timeout -k 10 200 python -u scripts/probe32.py > gpurun_out/r2s2i_probe32.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/r2s2i_probe.log 2>&1
}

# ---- scripts/r2s2_j.sh
lease_r2s2_j() {
  # full GPU suite after the session-2 changes
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2j_tests.log 2>&1
  timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2s2j_smoke.log 2>&1
}

# ---- scripts/r2s2_k.sh
lease_r2s2_k() {
  # misaligned ranges: head split (scan, copy_if) and 1-KiB store alignment (elementwise)
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segmented_layouts.py tests/test_gpu_for_loop.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2k_tests.log 2>&1
  timeout -k 10 300 python3 scripts/unaligned_probe.py > gpurun_out/r2s2k_unaligned.log 2>&1
}

# ---- scripts/r2s2_l.sh
lease_r2s2_l() {
  # direct per-bucket segment sort: fullsize + hybrid sort tests, sort probe timing and trace
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_sort_hybrid.py -m gpu -x -q -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r2s2l_tests.log 2>&1
  timeout -k 10 200 python -u scripts/ab_probe.py > gpurun_out/r2s2l_probe.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2s2l_trace -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s2l_trace.log 2>&1
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: r2s2_a r2s2_b r2s2_c r2s2_d r2s2_e r2s2_f r2s2_final r2s2_g r2s2_h r2s2_i r2s2_j r2s2_k r2s2_l"; fi
