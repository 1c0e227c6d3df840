# Lease scripts of round 2, session 1 (scripts/r2_*.sh): what each gpurun call of that round ran,
# kept as one shell function per former file (provenance of the profiles/
# logs that cite them).  `bash scripts/leases/r2.sh NAME` runs lease NAME.

# ---- scripts/r2_a.sh
lease_r2_a() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2a_cxx.log 2>&1
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/r2a_probe.log 2>&1
}

# ---- scripts/r2_b.sh
lease_r2_b() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py tests/test_gpu_bench_ranks.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b_tests.log 2>&1
}

# ---- scripts/r2_c.sh
lease_r2_c() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2c_cxx.log 2>&1
}

# ---- scripts/r2_d.sh
lease_r2_d() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bench_ranks.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2d_new.log 2>&1
  timeout -k 10 300 python -u bench.py > gpurun_out/r2d_bench.log 2>&1
}

# ---- scripts/r2_e.sh
lease_r2_e() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2e_hybrid.log 2>&1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k sort -m gpu -x -v --timeout 120 --timeout-method thread >> gpurun_out/r2e_hybrid.log 2>&1
  timeout -k 10 300 python -u bench.py > gpurun_out/r2e_bench.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e_prof -o run -- python3 bench.py --no-cpu --no-pmc > gpurun_out/r2e_prof.log 2>&1
}

# ---- scripts/r2_f.sh
lease_r2_f() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sort or hybrid" > gpurun_out/r2f_tests.log 2>&1
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc > gpurun_out/r2f_bench.log 2>&1
  cd scripts/ubench && timeout -k 10 120 ./sortpass2 > ../../gpurun_out/r2f_sortpass2.log 2>&1
}

# ---- scripts/r2_final.sh
lease_r2_final() {
  # round 2 measurement set: bench (with its own PMC passes), rocprofv3 kernel stats of the same command
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u bench.py > gpurun_out/r2f_bench_final.log 2>&1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2f_bench_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2f_bench_under_rocprof.log 2>&1
}

# ---- scripts/r2_g.sh
lease_r2_g() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2g_gpu_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2g_smoke.log 2>&1
}

# ---- scripts/r2_h.sh
lease_r2_h() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_merge_sort.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2h_cxx.log 2>&1
}

# ---- scripts/r2_i.sh
lease_r2_i() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2i_gpu_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2i_smoke.log 2>&1
  timeout -k 10 400 python -u bench.py > gpurun_out/r2i_bench.log 2>&1
}

# ---- scripts/r2_j.sh
lease_r2_j() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_parity.py -m gpu -x -q -k "sort or hybrid" --timeout 120 --timeout-method thread > gpurun_out/r2j_tests.log 2>&1
  timeout -k 10 120 python -u scripts/sort_probe.py > gpurun_out/r2j_probe.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2j_trace -o run -- python3 scripts/sort_probe.py > gpurun_out/r2j_trace.log 2>&1
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc > gpurun_out/r2j_bench.log 2>&1
}

# ---- scripts/r2_k.sh
lease_r2_k() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q -k "sort or hybrid" --timeout 120 --timeout-method thread > gpurun_out/r2k_tests.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2k_trace -o run -- python3 scripts/sort_probe.py > gpurun_out/r2k_trace.log 2>&1
}

# ---- scripts/r2_pmc_kernels.sh
lease_r2_pmc_kernels() {
  # round 2: PMC passes over scripts/kernel_probe.py (triad, reduce, scan, copy_if, stencil step at 2^30), one counter group per run
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r2_pmc_k$i -o run -- python3 scripts/kernel_probe.py > gpurun_out/r2_pmc_k$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  done
  python3 scripts/pmc_summary.py gpurun_out/r2_pmc_k1 gpurun_out/r2_pmc_k2 gpurun_out/r2_pmc_k3 gpurun_out/r2_pmc_k4 > gpurun_out/r2_pmc_kernels.txt
  echo done
}

# ---- scripts/r2_pmc_sort.sh
lease_r2_pmc_sort() {
  # round 2: kernel trace + PMC passes over the (hybrid) sort of 2^30 u64 keys, each counter group in its own run
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2_sort_trace -o run -- python3 scripts/sort_probe.py > gpurun_out/r2_sort_trace.log 2>&1 || exit 1
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r2_pmc_sort$i -o run -- python3 scripts/sort_probe.py > gpurun_out/r2_pmc_sort$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  done
  echo done
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: r2_a r2_b r2_c r2_d r2_e r2_f r2_final r2_g r2_h r2_i r2_j r2_k r2_pmc_kernels r2_pmc_sort"; fi
