# Lease scripts of round 3 (scripts/r3/X.sh): what each gpurun call of that round ran,
# kept as one shell function per former file (provenance of the profiles/
# logs that cite them).  `bash scripts/leases/r3.sh NAME` runs lease NAME.

# ---- scripts/r3/a.sh
lease_a() {
  # round 3, lease a: 2^32-point stencil windowed parity + the bench with the windowed stencil check
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_stencil_fullsize.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a_stencil_tests.log 2>&1
  timeout -k 10 500 python -u bench.py > gpurun_out/r3a_bench.log 2>&1
}

# ---- scripts/r3/b.sh
lease_b() {
  # round 3, lease b: full GPU suite (refactored kernels + device closures) and the bench
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/r3b_cxx.log 2>&1
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
  timeout -k 10 500 python -u bench.py > gpurun_out/r3b_bench.log 2>&1
}

# ---- scripts/r3/c.sh
lease_c() {
  # round 3, lease c: device closures (C++), device-planned sort, full GPU suite, sort sweep, bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest tests/test_cxx_api.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3c_cxx.log 2>&1
  echo "cxx rc=$?" >> gpurun_out/r3c_status.log
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r3c_sort_tests.log 2>&1
  rc=$?; echo "sort tests rc=$rc" >> gpurun_out/r3c_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r3c_sort_probe.log 2>&1 || exit $?
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1
  echo "suite rc=$?" >> gpurun_out/r3c_status.log
  timeout -k 10 500 python -u bench.py > gpurun_out/r3c_bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/r3c_status.log
}

# ---- scripts/r3/d.sh
lease_d() {
  # round 3, lease d (re-entry): whole tree after the last commit -- C++ tests, full GPU suite, smoke, bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest tests/test_cxx_api.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3d_cxx.log 2>&1
  rc=$?; echo "cxx rc=$rc" >> gpurun_out/r3d_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r3d_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3d_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r3d_bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/r3d_status.log
}

# ---- scripts/r3/e.sh
lease_e() {
  # round 3, lease e: call_overhead diagnosis (task sort + reduce), f64 scan tile shapes (scan7), scan parity with the deferred round carry
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 120 tests/cxx/bin/compute_api 12345 > gpurun_out/r3e_compute_api.log 2>&1
  echo "compute_api rc=$?" >> gpurun_out/r3e_status.log
  timeout -k 10 120 tests/cxx/bin/call_overhead > gpurun_out/r3e_call_overhead.log 2>&1
  echo "call_overhead rc=$?" >> gpurun_out/r3e_status.log
  timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3e_scan7.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -k "scan" --timeout 120 --timeout-method thread > gpurun_out/r3e_scan_tests.log 2>&1
  echo "scan tests rc=$?" >> gpurun_out/r3e_status.log
  timeout -k 10 300 tests/cxx/bin/closure_algorithms 777 > gpurun_out/r3e_closure.log 2>&1
  echo "closure rc=$?" >> gpurun_out/r3e_status.log
}

# ---- scripts/r3/f.sh
lease_f() {
  # round 3, lease f: fixed-association FP look-back -- timing (scan7), scan parity incl. reproducibility, segmented/closure scans
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3f_scan7.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py -m gpu -q -k "scan" --timeout 200 --timeout-method thread > gpurun_out/r3f_scan_tests.log 2>&1
  echo "scan tests rc=$?" >> gpurun_out/r3f_status.log
  timeout -k 10 300 tests/cxx/bin/closure_algorithms 777 > gpurun_out/r3f_closure.log 2>&1
  echo "closure rc=$?" >> gpurun_out/r3f_status.log
  timeout -k 10 300 tests/cxx/bin/partitioned_vector > gpurun_out/r3f_pv.log 2>&1
  echo "pv rc=$?" >> gpurun_out/r3f_status.log
}

# ---- scripts/r3/g.sh
lease_g() {
  # round 3, lease g: fixed-association look-back for every scan -- copy_if variants (copyif7), full GPU suite, smoke, bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 scripts/ubench/copyif7 > gpurun_out/r3g_copyif7.log 2>&1 || exit $?
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r3g_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3g_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r3g_bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/r3g_status.log
}

# ---- scripts/r3/h.sh
lease_h() {
  # round 3, lease h: persistent onesweep / segment-sort grids in the device-planned sort -- sort tests, probe, kernel stats
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_parity.py -m gpu -q -k "sort" --timeout 200 --timeout-method thread > gpurun_out/r3h_sort_tests.log 2>&1
  rc=$?; echo "sort tests rc=$rc" >> gpurun_out/r3h_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r3h_sort_probe.log 2>&1 || exit $?
  mkdir -p gpurun_out/r3h_prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3h_prof -o run --output-format csv -- python3 scripts/sort_probe.py 30 > gpurun_out/r3h_prof.log 2>&1
  echo "prof rc=$?" >> gpurun_out/r3h_status.log
}

# ---- scripts/r3/i.sh
lease_i() {
  # round 3, lease i: copy_if write-out variants on the fixed look-back (copyif7)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 scripts/ubench/copyif7 > gpurun_out/r3i_copyif7.log 2>&1
}

# ---- scripts/r3/j.sh
lease_j() {
  # round 3, lease j: measurement set on the tree -- full GPU suite, smoke, bench, rocprofv3 kernel stats of the bench, PMC passes over the 2^30 u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3j_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r3j_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3j_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r3j_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r3j_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3j_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r3j_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r3j_status.log
  export SORT_ONLY=u64
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r3j_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3j_pmc_sort$i.log 2>&1 || { echo "pmc pass $i failed rc=$?" >> gpurun_out/r3j_status.log; exit 1; }
  done
  echo "pmc ok" >> gpurun_out/r3j_status.log
}

# ---- scripts/r3/k.sh
lease_k() {
  # round 3, lease k: scan tile shapes with several workgroups per CU on the fixed look-back (scan7)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3k_scan7.log 2>&1
}

# ---- scripts/r3/l.sh
lease_l() {
  # round 3, lease l: several reductions per for_loop (Python + C++), segmented transform_exclusive_scan, scan shapes (scan7)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_for_loop.py tests/test_gpu_segmented_layouts.py tests/test_cxx_api.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> gpurun_out/r3l_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3l_scan7.log 2>&1
  echo "scan7 rc=$?" >> gpurun_out/r3l_status.log
}

# ---- scripts/r3/m.sh
lease_m() {
  # round 3, lease m: 512-thread two-per-CU scan tiles -- scan/segmented/closure tests, then the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_segmented_layouts.py tests/test_gpu_multirank.py tests/test_gpu_bench_ranks.py -m gpu -q -k "scan or bench" --timeout 200 --timeout-method thread > gpurun_out/r3m_scan_tests.log 2>&1
  rc=$?; echo "scan tests rc=$rc" >> gpurun_out/r3m_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 tests/cxx/bin/closure_algorithms 779 > gpurun_out/r3m_closure.log 2>&1
  echo "closure rc=$?" >> gpurun_out/r3m_status.log
  timeout -k 10 500 python -u bench.py --no-pmc > gpurun_out/r3m_bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/r3m_status.log
}

# ---- scripts/r3/n.sh
lease_n() {
  # round 3, lease n: copy_if tile shapes with more workgroups per CU (copyif7)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 scripts/ubench/copyif7 > gpurun_out/r3n_copyif7.log 2>&1
}

# ---- scripts/r3/o.sh
lease_o() {
  # round 3, lease o: look-back width of the hybrid sort's prefix passes (sortpass3)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 scripts/ubench/sortpass3 > gpurun_out/r3o_sortpass3.log 2>&1
}

# ---- scripts/r3/p.sh
lease_p() {
  # round 3, lease p: measurement set on the tree -- full GPU suite, smoke, bench, rocprofv3 kernel stats of the bench, PMC passes over the 2^30 u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r3p_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3p_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r3p_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r3p_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r3p_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r3p_status.log
  export SORT_ONLY=u64
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r3p_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3p_pmc_sort$i.log 2>&1 || { echo "pmc pass $i failed rc=$?" >> gpurun_out/r3p_status.log; exit 1; }
  done
  echo "pmc ok" >> gpurun_out/r3p_status.log
}

# ---- scripts/r3/q.sh
lease_q() {
  # round 3, lease q: more scan tile shapes on the fixed look-back (scan7: 384/768-thread tiles)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3q_scan7.log 2>&1
}

# ---- scripts/r3/r.sh
lease_r() {
  # round 3, lease r: 2^30 FP scan reproducibility test
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -k "reproducible" --timeout 250 --timeout-method thread > gpurun_out/r3r_tests.log 2>&1
}

# ---- scripts/r3/s.sh
lease_s() {
  # round 3, lease s: small-range keys (the LSD path on persistent grids) vs uniform keys
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for c in u64r16 u64r24 u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r3s_sort_ranges.log 2>&1 || exit $?
  done
  mkdir -p gpurun_out/r3s_prof
  SORT_ONLY=u64r16 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3s_prof.log 2>&1
}

# ---- scripts/r3/t.sh
lease_t() {
  # round 3, lease t: persistent passes with per-tile id re-derivation (102-105 VGPRs, was 156) and the segment sort's run-insertion step --
  # sort tests, then small-range keys (LSD path, persistent grids) vs uniform keys, then kernel stats
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_parity.py -m gpu -q -k "sort" --timeout 200 --timeout-method thread > gpurun_out/r3t_sort_tests.log 2>&1
  rc=$?; echo "sort tests rc=$rc" >> gpurun_out/r3t_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  for c in u64r16 u64r24 u64 u32 pairs; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r3t_sort_ranges.log 2>&1 || exit $?
  done
  mkdir -p gpurun_out/r3t_prof
  SORT_ONLY=u64r24 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3t_prof.log 2>&1
  echo "prof rc=$?" >> gpurun_out/r3t_status.log
}

# ---- scripts/r3/u.sh
lease_u() {
  # round 3, lease u: same-box A/B of three library builds (scripts/ab3/, built from the commits named):
  #   lib_pre = 7fbb622 (before the persistent-pass id fix), lib_oe = a704c64 (id fix, odd-even rounds),
  #   lib_ins = the run-insertion step of the segment sort; interleaved twice
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for rep in 1 2; do
    for v in pre oe ins; do
      HPXHIP_LIB=scripts/ab3/lib_$v.so timeout -k 10 120 python -u scripts/ab_probe.py >> gpurun_out/r3u_ab.log 2>&1 || exit $?
    done
  done
}

# ---- scripts/r3/v.sh
lease_v() {
  # round 3, lease v: measurement set on the last tree (persistent-pass id fix, segment-sort run insertion) --
  # full GPU suite, smoke, bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r3v_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r3v_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r3v_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r3v_status.log
}

# ---- scripts/r3/w.sh
lease_w() {
  # round 3, lease w: kernel stats of the 2^30 u64 sort on the last tree
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  mkdir -p gpurun_out/r3w_prof
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3w_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r3w_prof.log 2>&1
}

# ---- scripts/r3/x.sh
lease_x() {
  # round 3, lease x: prefix passes on persistent grids (HPXHIP_SORT_PERSIST_ALL=1) vs one workgroup per tile, same box, interleaved
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for rep in 1 2; do
    for p in 0 1; do
      for c in u64 u32; do
        echo "PERSIST_ALL=$p" >> gpurun_out/r3x_persist_all.log
        HPXHIP_SORT_PERSIST_ALL=$p SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r3x_persist_all.log 2>&1 || exit $?
      done
    done
  done
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: a b c d e f g h i j k l m n o p q r s t u v w x"; fi
