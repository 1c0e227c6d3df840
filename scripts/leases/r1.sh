# Lease scripts of round 1 (scripts/sN.sh, scripts/gpu.sh): what each gpurun call of that round ran,
# kept as one shell function per former file (provenance of the profiles/
# logs that cite them).  `bash scripts/leases/r1.sh NAME` runs lease NAME.

# ---- scripts/s1.sh
lease_s1() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1_tests.log 2>&1
  timeout -k 10 300 python -u bench.py > gpurun_out/s1_bench.log 2>&1
}

# ---- scripts/s2.sh
lease_s2() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 120 python -u scripts/perf_probe.py > gpurun_out/probe2.log 2>&1
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_tests.log 2>&1
}

# ---- scripts/s3.sh
lease_s3() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u bench.py > gpurun_out/r01_bench_full.log 2>&1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/prof_full.log 2>&1
}

# ---- scripts/s4.sh
lease_s4() {
  # PMC passes over the sort (each counter group in its own run)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_sort$i -o run -- python3 scripts/sort_probe.py > gpurun_out/pmc_sort$i.log 2>&1 || echo "pass $i failed rc=$?"
  done
  echo done
}

# ---- scripts/s5.sh
lease_s5() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5_tests.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s5_probe.log 2>&1
  timeout -k 10 200 scripts/ubench/scan > gpurun_out/s5_scan.log 2>&1
}

# ---- scripts/s6.sh
lease_s6() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 200 scripts/ubench/scan > gpurun_out/s6_scan.log 2>&1
}

# ---- scripts/s7.sh
lease_s7() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u bench.py > gpurun_out/s7_bench.log 2>&1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s7_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/s7_prof.log 2>&1
}

# ---- scripts/s8.sh
lease_s8() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 200 scripts/ubench/sortpass2 > gpurun_out/s8_sort.log 2>&1
}

# ---- scripts/s9.sh
lease_s9() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 200 scripts/ubench/copyif > gpurun_out/s9_copyif.log 2>&1
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "copy_if or copyif" > gpurun_out/s9_tests.log 2>&1
}

# ---- scripts/s10.sh
lease_s10() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 200 scripts/ubench/stencil > gpurun_out/s10_stencil.log 2>&1
}

# ---- scripts/s11.sh
lease_s11() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s11_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s11_smoke.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s11_probe.log 2>&1
}

# ---- scripts/s12.sh
lease_s12() {
  # PMC passes over scripts/kernel_probe.py, one counter group per run
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_k$i -o run -- python3 scripts/kernel_probe.py > gpurun_out/pmc_k$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  done
  python3 scripts/pmc_summary.py gpurun_out/pmc_k1 gpurun_out/pmc_k2 gpurun_out/pmc_k3 gpurun_out/pmc_k4 > gpurun_out/pmc_kernels.txt
  echo done
}

# ---- scripts/s13.sh
lease_s13() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "stencil" > gpurun_out/s13_tests.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s13_probe.log 2>&1
}

# ---- scripts/s14.sh
lease_s14() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s14_tests.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s14_probe.log 2>&1
}

# ---- scripts/s15.sh
lease_s15() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "stencil" > gpurun_out/s15_tests.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s15_probe.log 2>&1
}

# ---- scripts/s16.sh
lease_s16() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s16_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s16_smoke.log 2>&1
  timeout -k 10 600 python -u bench.py > gpurun_out/s16_bench.log 2>&1
}

# ---- scripts/s17.sh
lease_s17() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "copy_if" --timeout 120 --timeout-method thread > gpurun_out/s17_tests.log 2>&1
  timeout -k 10 200 python -u scripts/perf_probe.py > gpurun_out/s17_probe.log 2>&1
}

# ---- scripts/s18.sh
lease_s18() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s18_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s18_smoke.log 2>&1
  timeout -k 10 300 python -u bench.py > gpurun_out/s18_bench.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s18_prof -o run -- python3 -u bench.py --no-pmc --no-cpu > gpurun_out/s18_bench_under_rocprof.log 2>&1
}

# ---- scripts/s19.sh
lease_s19() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_for_loop.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s19_tests.log 2>&1
}

# ---- scripts/s20.sh
lease_s20() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_for_loop.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s20_tests.log 2>&1
}

# ---- scripts/s21.sh
lease_s21() {
  set -e
  cd $GRAFT_REPO_ROOT
  timeout -k 10 120 ./scripts/ubench/scan > gpurun_out/s21_scan.log 2>&1
}

# ---- scripts/s22.sh
lease_s22() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s22_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s22_smoke.log 2>&1
  timeout -k 10 300 python -u bench.py > gpurun_out/s22_bench.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s22_prof -o run -- python3 -u bench.py --no-pmc --no-cpu > gpurun_out/s22_bench_under_rocprof.log 2>&1
}

# ---- scripts/s23.sh
lease_s23() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_for_loop.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s23_tests.log 2>&1
}

# ---- scripts/s24.sh
lease_s24() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_for_loop.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s24_tests.log 2>&1
}

# ---- scripts/s25.sh
lease_s25() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s25_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s25_smoke.log 2>&1
  timeout -k 10 300 python -u bench.py > gpurun_out/s25_bench.log 2>&1
}

# ---- scripts/s26.sh
lease_s26() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_for_loop.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s26_tests.log 2>&1
}

# ---- scripts/s27.sh
lease_s27() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s27_tests.log 2>&1
}

# ---- scripts/s28.sh
lease_s28() {
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s28_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s28_smoke.log 2>&1
}

# ---- scripts/gpu.sh
lease_gpu() {
  #!/bin/bash
  # Run a command on the GPU box via gpurun; re-submit ONLY when the box failed
  # to come up (status=transient: nothing ran, nothing charged).  Never retries
  # a command that ran and failed.
  # usage: scripts/gpu.sh <timeout-seconds> '<command>'
  T=$1; shift
  for attempt in 1 2 3 4 5; do
    out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
    echo "$out" | tail -4
    if echo "$out" | grep -q "status=transient\|backing off\|no box\|slot"; then
      if echo "$out" | grep -q "status=ok\|rc=[0-9]"; then break; fi
      sleep 45; continue
    fi
    break
  done
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: s1 s2 s3 s4 s5 s6 s7 s8 s9 s10 s11 s12 s13 s14 s15 s16 s17 s18 s19 s20 s21 s22 s23 s24 s25 s26 s27 s28 gpu"; fi
