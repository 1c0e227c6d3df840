# Lease scripts of round 5 (scripts/r5/X.sh): what each gpurun call of that round ran,
# kept as one shell function per former file (provenance of the profiles/
# logs that cite them).  `bash scripts/leases/r5.sh NAME` runs lease NAME.

# ---- scripts/r5/a.sh
lease_a() {
  # round 5, lease a: triad placement vs physical mapping (scripts/ubench/vmm.hip), 6 fresh processes
  cd $GRAFT_REPO_ROOT
  for i in 1 2 3 4 5 6; do
    echo "== process $i" >> gpurun_out/r5a_vmm.log
    timeout -k 10 120 ./scripts/ubench/vmm 2 >> gpurun_out/r5a_vmm.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/b.sh
lease_b() {
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
}

# ---- scripts/r5/c.sh
lease_c() {
  # round 5, lease c: oversized-bucket finish (segmented LSD), range errors from clamped scatters,
  # deterministic device_closures pending check, 4-rank host-staged multirank; sort probes
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5c
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_errors.py tests/test_gpu_merge_sort.py "tests/test_cxx_api.py" tests/test_gpu_multirank.py \
    > ${L}_tests.log 2>&1 || exit $?
  for c in u64hot u64corr u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64 u32 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k sort \
    > ${L}_fullsize.log 2>&1 || exit $?
}

# ---- scripts/r5/d.sh
lease_d() {
  # round 5, lease d: first prefix pass (offset-fed) tile order: counter vs blockIdx vs XCD regions
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 ./scripts/ubench/sortpass5 > gpurun_out/r5d_sortpass5.log 2>&1 || exit $?
}

# ---- scripts/r5/e.sh
lease_e() {
  # round 5, lease e: XCD-region prefix passes (XREG; the top-9 pass in 8 field regions with joint-histogram
  # bin starts), bounded oversized-bucket finish v2 (LDS seg table, optimistic plan): sort tests + probes + kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5e
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_merge_sort.py > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k sort \
    >> ${L}_tests.log 2>&1 || exit $?
  for c in u64 u32; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64hot u64corr u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o sort -- \
    python3 scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
}

# ---- scripts/r5/f.sh
lease_f() {
  # round 5, lease f: kernel trace of the skewed sorts (u64hot at 2^28 and 2^30)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for lg in 28 30; do
    SORT_ONLY=u64hot timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5f_prof$lg -o hot -- \
      python3 scripts/sort_probe.py $lg > gpurun_out/r5f_hot$lg.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/g.sh
lease_g() {
  # round 5, lease g: pass-2 look-back widths over XCD regions (sortpass6), pass-1 orders again (sortpass5),
  # skewed-sort fixes (wave-uniform histogram adds, b2 for concentrated skew): tests + probes + trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5g
  timeout -k 10 300 ./scripts/ubench/sortpass6 > ${L}_sortpass6.log 2>&1 || exit $?
  timeout -k 10 300 ./scripts/ubench/sortpass5 > ${L}_sortpass5.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    > ${L}_tests.log 2>&1 || exit $?
  for c in u64 u32 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64hot u64corr u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  SORT_ONLY=u64hot timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof28 -o hot -- \
    python3 scripts/sort_probe.py 28 > ${L}_prof.log 2>&1 || exit $?
}

# ---- scripts/r5/h.sh
lease_h() {
  # round 5, lease h: two-peel histogram adds and wave-parallel plan statistics; first-pass ubench
  # (its k_hist_tiles feeds the offsets), sort tests, probes uniform/hot/corr
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5h
  timeout -k 10 300 ./scripts/ubench/sortpass5 > ${L}_sortpass5.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_merge_sort.py > ${L}_tests.log 2>&1 || exit $?
  for c in u64 u32 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64hot u64corr u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof_$c -o s -- \
      python3 scripts/sort_probe.py 28 > ${L}_prof_$c.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/i.sh
lease_i() {
  # round 5, lease i: pipelined persistent copy_if against the shipped kernel (copyif9);
  # segment sort phase split and register-side run detection (seg5)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5i
  timeout -k 10 240 ./scripts/ubench/copyif9 > ${L}_copyif9.log 2>&1 || exit $?
  timeout -k 10 240 ./scripts/ubench/seg5 > ${L}_seg5.log 2>&1 || exit $?
}

# ---- scripts/r5/j.sh
lease_j() {
  # round 5, lease j: histogram peels only shared cells (uniform keys: one ballot per key);
  # pipelined copy_if shipped: copy_if parity tests, sort tests, probes uniform/hot/corr, traces
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5j
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "copy_if" > ${L}_tests_copyif.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_merge_sort.py > ${L}_tests.log 2>&1 || exit $?
  for c in u64 u32 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64hot u64corr u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof_$c -o s -- \
      python3 scripts/sort_probe.py 30 > ${L}_prof_$c.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/k.sh
lease_k() {
  # round 5, lease k: segment sort -- run detection from a 16-bit prefix array (PRE16) and a
  # persistent form that loads the next segment before sorting the current one (seg6)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5k
  timeout -k 10 300 ./scripts/ubench/seg6 > ${L}_seg6.log 2>&1 || exit $?
}

# ---- scripts/r5/l.sh
lease_l() {
  # round 5, lease l: segment sort variants again (LDS arrays declared in the shared body: the
  # first seg6 build passed them down as flat pointers); histogram with a per-wave cache of hot
  # cells -- sort tests, probes, traces at 2^28 and 2^30
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5l
  timeout -k 10 300 ./scripts/ubench/seg6 > ${L}_seg6.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    > ${L}_tests.log 2>&1 || exit $?
  for c in u64 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64hot u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof28_$c -o s -- \
      python3 scripts/sort_probe.py 28 > ${L}_prof28_$c.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/m.sh
lease_m() {
  # round 5, lease m: seg7 (seg6 variants without the opaque ids in the one-shot kernels); histogram tiles
  # strided over the grid, chunk totals from k_chunk_sums -- sort tests, probes, traces

  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5m
  timeout -k 10 300 ./scripts/ubench/seg7 > ${L}_seg7.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -k "sort or copy_if" \
    > ${L}_tests.log 2>&1 || exit $?
  for c in u64 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64hot u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof28_$c -o s -- \
      python3 scripts/sort_probe.py 28 > ${L}_prof28_$c.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/n.sh
lease_n() {
  # round 5, lease n: segment sort PRE16 in the shipped kernel (seg8 A/B); 2^30 traces of the
  # uniform and hot sorts with the strided histogram
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5n
  timeout -k 10 300 ./scripts/ubench/seg8 > ${L}_seg8.log 2>&1 || exit $?
  for c in u64 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof30_$c -o s -- \
      python3 scripts/sort_probe.py 30 > ${L}_prof30_$c.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/o.sh
lease_o() {
  # round 5, lease o: histogram prefetches the next tile (double-buffered counts); 2^30 sorts
  # element for element against a closed form; C++ programs (closure copy_if on the pipelined
  # kernel); sort tests, probes and a 2^30 trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5o
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py \
    -k "element_exact or permutation_and_order or oversized" > ${L}_fullsize.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cxx_api.py \
    tests/test_gpu_sort_hybrid.py > ${L}_tests.log 2>&1 || exit $?
  for c in u64 u32 u64hot; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
  done
  for c in u64hot u64corr u64; do
    SORT_ONLY=$c timeout -k 10 120 python -u scripts/sort_probe.py 28 >> ${L}_probe.log 2>&1 || exit $?
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof30_u64 -o s -- \
    python3 scripts/sort_probe.py 30 > ${L}_prof30_u64.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > ${L}_closure_timing.log 2>&1 || exit $?
}

# ---- scripts/r5/p.sh
lease_p() {
  # round 5, lease p: one-pass merge of up to 8 sorted runs (hpxhip_merge_runs) -- parity tests,
  # 2^30 x 8 runs element for element, single-rank and 4-rank segmented sorts, timing vs pairwise
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5p
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
    > ${L}_multirank.log 2>&1 || exit $?
}

# ---- scripts/r5/q.sh
lease_q() {
  # round 5, lease q: where the one-pass run merge's time goes (kernel trace of the probe at 2^30);
  # multirank segmented sorts with empty sample runs fixed
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5q
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
    python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
    > ${L}_multirank.log 2>&1 || exit $?
}

# ---- scripts/r5/r.sh
lease_r() {
  # round 5, lease r: one-pass run merge with 256-thread tasks on one 16-KiB LDS buffer (several
  # per CU), splitters every 3p samples, bounds through the runs' own samples -- tests, timing
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5r
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
    python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
    > ${L}_multirank.log 2>&1 || exit $?
}

# ---- scripts/r5/s.sh
lease_s() {
  # round 5, lease s: one-pass run merge -- static output slots in the LDS rounds, 16-B staging loads and
  # stores, upper bounds from the lower bound -- tests, timing
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5s
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
    python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
    > ${L}_multirank.log 2>&1 || exit $?
}

# ---- scripts/r5/t.sh
lease_t() {
  # round 5, lease t: debug the float64 one-pass run merge mismatch
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u scripts/mw_debug.py > gpurun_out/r5t_debug.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/mw_debug2.py > gpurun_out/r5t_debug2.log 2>&1 || exit $?
}

# ---- scripts/r5/u.sh
lease_u() {
  # round 5, lease u: one-pass run merge with 16-B LDS write-back in the rounds -- tests, timing

  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5u
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
    python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
    > ${L}_multirank.log 2>&1 || exit $?
}

# ---- scripts/r5/v.sh
lease_v() {
  # round 5, lease v: one-pass run merge with a padded LDS layout (one pad key every 8) -- tests, timing

  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5v
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
    python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
    > ${L}_multirank.log 2>&1 || exit $?
}

# ---- scripts/r5/w.sh
lease_w() {
  # round 5, lease w: one-pass run merge, padded LDS + 16-B staging loads -- tests, timing

  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5w
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o s -- \
    python3 scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
    > ${L}_multirank.log 2>&1 || exit $?
}

# ---- scripts/r5/x.sh
lease_x() {
  # round 5, lease x: full validation of the tree -- GPU suite, smoke, bench, rocprofv3 kernel trace
  # + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5x
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > ${L}_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > ${L}_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
  echo "bench ok" >> ${L}_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 bench.py --no-pmc --no-cpu > ${L}_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> ${L}_status.log
}

# ---- scripts/r5/y.sh
lease_y() {
  # round 5, lease y: pipelined persistent scan (scan8) against the shipped k_scan shapes
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 ./scripts/ubench/scan8 > gpurun_out/r5y_scan8.log 2>&1 || exit $?
}

# ---- scripts/r5/z.sh
lease_z() {
  # round 5, lease z: PMC passes (one counter group per run) over the 2^30 u64 sort as it ends
  # round 5 and over the pipelined copy_if (FETCH_SIZE / WRITE_SIZE)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    SORT_ONLY=u64 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r5z_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r5z_pmc_sort$i.log 2>&1 || exit 1
  done
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5z_pmc_cif_fetch -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5z_pmc_cif_fetch.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5z_pmc_cif_write -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5z_pmc_cif_write.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/r5z_pmc_sort1 gpurun_out/r5z_pmc_sort2 gpurun_out/r5z_pmc_sort3 > gpurun_out/r5z_pmc_sort.txt 2>&1
  python3 scripts/pmc_summary.py gpurun_out/r5z_pmc_cif_fetch gpurun_out/r5z_pmc_cif_write > gpurun_out/r5z_pmc_copy_if.txt 2>&1
  echo ok
}

# ---- scripts/r5/aa.sh
lease_aa() {
  # round 5, lease aa: segment sort thread / item shapes for ~4096-key segments (seg9)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 ./scripts/ubench/seg9 > gpurun_out/r5aa_seg9.log 2>&1 || exit $?
}

# ---- scripts/r5/ab.sh
lease_ab() {
  # round 5, lease ab: pipelined copy_if write-out with 128-B aligned vectors -- timing, and the
  # WRITE_SIZE of both forms (the 16-B form wrote 1.02x its bytes)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 240 ./scripts/ubench/copyif9 > gpurun_out/r5ab_copyif9.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5ab_pmc_write -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5ab_pmc_write.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5ab_pmc_fetch -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5ab_pmc_fetch.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/r5ab_pmc_fetch gpurun_out/r5ab_pmc_write > gpurun_out/r5ab_pmc.txt 2>&1
}

# ---- scripts/r5/ac.sh
lease_ac() {
  # round 5, lease ac: line-aligned write-outs (copy_if pipe, multiway merge) -- parity tests and the
  # merge probe
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ac
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    tests/test_gpu_parity.py -k "merge or copy_if" > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
}

# ---- scripts/r5/ad.sh
lease_ad() {
  # round 5, lease ad: full validation of the tree (copy_if and multiway write-outs line-aligned) -- GPU suite, smoke, bench, rocprofv3 kernel trace
  # + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ad
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > ${L}_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > ${L}_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
  echo "bench ok" >> ${L}_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 bench.py --no-pmc --no-cpu > ${L}_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> ${L}_status.log
}

# ---- scripts/r5/ae.sh
lease_ae() {
  # round 5, lease ae: multiway merge with ordered bits staged in LDS -- the merge_runs tests and the
  # merge probe for the shipped build (256 threads) and the variant builds that miscompiled before
  # (512 threads, 256 x 8 waves) plus 512 x 2 waves
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ae
  for v in default t512 t256w8 t512w2; do
    if [ $v = default ]; then unset HPXHIP_LIB; else export HPXHIP_LIB=$PWD/scripts/ubench/mwlib/$v/libhpxhip.so; fi
    echo "== $v" >> ${L}_status.log
    timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
      -k "merge_runs" > ${L}_tests_$v.log 2>&1
    rc=$?; echo "$v tests rc=$rc" >> ${L}_status.log
    if [ $rc -gt 1 ]; then exit $rc; fi
    timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe_$v.log 2>&1 || exit $?
  done
}

# ---- scripts/r5/ag.sh
lease_ag() {
  # round 5, lease ag: seg10 -- the segment sort's one-pass atomic ranking (ONE = 12/13/14) against the
  # shipped two-pass form at 2^30 u64 in 4096-key segments
  cd $GRAFT_REPO_ROOT
  L=gpurun_out/r5ag
  timeout -k 10 300 scripts/ubench/seg10 > ${L}_seg10.log 2>&1 || exit $?
}

# ---- scripts/r5/ah.sh
lease_ah() {
  # round 5, lease ah: multiway merge round variants (scripts/ubench/mwlib.sh) -- bl = branch-free
  # merge step (one LDS read per output), blw4 = bl at 4 waves per SIMD, bl16 = bl with 128 threads x 16
  # keys, t128i16 = shipped step with 128 x 16, ablate = no LDS rounds (timing only, wrong output);
  # the merge_runs tests per variant, then scripts/merge_runs_probe.py 30
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ah
  for v in default bl blw4 bl16 t128i16 ablate; do
    if [ $v = default ]; then unset HPXHIP_LIB; else export HPXHIP_LIB=$PWD/scripts/ubench/mwlib/$v/libhpxhip.so; fi
    echo "== $v" >> ${L}_status.log
    if [ $v != ablate ]; then
      timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_merge_sort.py \
        -k "merge_runs" > ${L}_tests_$v.log 2>&1
      rc=$?; echo "$v tests rc=$rc" >> ${L}_status.log
      if [ $rc -gt 1 ]; then exit $rc; fi
    fi
    timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe_$v.log 2>&1 || exit $?
    tail -4 ${L}_probe_$v.log >> ${L}_status.log
  done
}

# ---- scripts/r5/ai.sh
lease_ai() {
  # round 5, lease ai: multiway merge with the branch-free step (lease ah: bl) and the staging loads
  # flattened over the runs (one global round trip per task instead of one per run) -- the merge
  # and multirank GPU tests, scripts/merge_runs_probe.py 30 on the shipped build and on the
  # no-rounds ablation (timing only)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ai
  timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    tests/test_gpu_multirank.py > ${L}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  tail -4 ${L}_probe.log >> ${L}_status.log
  HPXHIP_LIB=$PWD/scripts/ubench/mwlib/ablate/libhpxhip.so HPXHIP_PROBE_NOCHECK=1 \
    timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe_ablate.log 2>&1 || exit $?
  tail -4 ${L}_probe_ablate.log >> ${L}_status.log
}

# ---- scripts/r5/aj.sh
lease_aj() {
  # round 5, lease aj: the branch-free merge step in merge_in_lds too (k_merge: hpx::merge and the
  # pairwise rounds) -- merge / multirank / C++ API GPU tests, scripts/merge_runs_probe.py 30
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5aj
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    tests/test_gpu_multirank.py tests/test_cxx_api.py -m gpu > ${L}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  tail -4 ${L}_probe.log >> ${L}_status.log
}

# ---- scripts/r5/ak.sh
lease_ak() {
  # round 5, lease ak: (1) lease aj's content -- the branch-free merge step in merge_in_lds too
  # (k_merge: hpx::merge and the pairwise rounds): merge / multirank / C++ API GPU tests and
  # scripts/merge_runs_probe.py 30; (2) the segment sort's first LDS pass ranked by LDS atomics
  # (scripts/ubench/seglib/atom1, HPXHIP_SEG_ATOM1=1): the sort tests on that build, then
  # scripts/sort_probe.py 30 for u64 and u32 on the shipped build and on atom1, twice each
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ak
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    tests/test_gpu_multirank.py tests/test_cxx_api.py -m gpu > ${L}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u scripts/merge_runs_probe.py 30 > ${L}_probe.log 2>&1 || exit $?
  tail -4 ${L}_probe.log >> ${L}_status.log
  A=$PWD/scripts/ubench/seglib/atom1/libhpxhip.so
  HPXHIP_LIB=$A timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -k "sort" > ${L}_tests_atom1.log 2>&1
  rc=$?; echo "atom1 sort tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  for i in 1 2; do
    for v in default atom1; do
      for c in u64 u32; do
        if [ $v = default ]; then unset HPXHIP_LIB; else export HPXHIP_LIB=$A; fi
        SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 > ${L}_sort_${v}_${c}_$i.log 2>&1 || exit $?
        echo "$v $c $i: $(grep -v '^#' ${L}_sort_${v}_${c}_$i.log | tail -1)" >> ${L}_status.log
      done
    done
  done
}

# ---- scripts/r5/al.sh
lease_al() {
  # round 5, lease al: the offset-fed first prefix pass ranked by LDS atomics (scripts/ubench/seglib/os1,
  # HPXHIP_OS_ATOM1=1): the sort tests on that build, then scripts/sort_probe.py 30 for u64 and u32 on
  # the shipped build and on os1, alternating, three times each
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5al
  A=$PWD/scripts/ubench/seglib/os1/libhpxhip.so
  HPXHIP_LIB=$A timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -k "sort" > ${L}_tests_os1.log 2>&1
  rc=$?; echo "os1 sort tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  for i in 1 2 3; do
    for v in default os1; do
      for c in u64 u32; do
        if [ $v = default ]; then unset HPXHIP_LIB; else export HPXHIP_LIB=$A; fi
        SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 > ${L}_sort_${v}_${c}_$i.log 2>&1 || exit $?
        echo "$v $c $i: $(grep -v '^#' ${L}_sort_${v}_${c}_$i.log | tail -1)" >> ${L}_status.log
      done
    done
  done
}

# ---- scripts/r5/am.sh
lease_am() {
  # round 5, lease am: full validation of the tree -- GPU suite, smoke, bench, rocprofv3 kernel trace
  # + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5am
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > ${L}_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > ${L}_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
  echo "bench ok" >> ${L}_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 bench.py --no-pmc --no-cpu > ${L}_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> ${L}_status.log
}

# ---- scripts/r5/an.sh
lease_an() {
  # round 5, lease an: the pipelined persistent offset-fed first prefix pass (k_prefix_pipe, build
  # scripts/ubench/seglib.sh pipe -DHPXHIP_PREFIX_PIPE=1): the sort tests on that build, then
  # scripts/sort_probe.py 30 for u64 and u32 on the shipped build and on pipe (u32 also with 2
  # workgroups per CU), alternating, three times each; a kernel trace of the pipe u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5an
  A=$PWD/scripts/ubench/seglib/pipe/libhpxhip.so
  HPXHIP_LIB=$A timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -k "sort" > ${L}_tests_pipe.log 2>&1
  rc=$?; echo "pipe sort tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  for i in 1 2 3; do
    for v in default pipe pipe2; do
      for c in u64 u32; do
        if [ $v = pipe2 ] && [ $c = u64 ]; then continue; fi
        unset HPXHIP_LIB HPXHIP_PIPE_WG
        if [ $v != default ]; then export HPXHIP_LIB=$A; fi
        if [ $v = pipe2 ]; then export HPXHIP_PIPE_WG=2; fi
        SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 > ${L}_sort_${v}_${c}_$i.log 2>&1 || exit $?
        echo "$v $c $i: $(grep -v '^#' ${L}_sort_${v}_${c}_$i.log | tail -1)" >> ${L}_status.log
      done
    done
  done
  unset HPXHIP_PIPE_WG
  HPXHIP_LIB=$A SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
  echo "prof ok" >> ${L}_status.log
}

# ---- scripts/r5/ao.sh
lease_ao() {
  # round 5, lease ao: the pipelined persistent offset-fed first prefix pass (k_prefix_pipe, build
  # (ao: unconditional loads and stores, the next tile's offsets loaded with its keys -- the compiler had waited
  # for every outstanding load and store, vmcnt(0), at the top of each tile)
  # scripts/ubench/seglib.sh pipe -DHPXHIP_PREFIX_PIPE=1): the sort tests on that build, then
  # scripts/sort_probe.py 30 for u64 and u32 on the shipped build and on pipe (u32 also with 2
  # workgroups per CU), alternating, three times each; a kernel trace of the pipe u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ao
  A=$PWD/scripts/ubench/seglib/pipe/libhpxhip.so
  HPXHIP_LIB=$A timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -k "sort" > ${L}_tests_pipe.log 2>&1
  rc=$?; echo "pipe sort tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  for i in 1 2 3; do
    for v in default pipe; do
      for c in u64 u32; do
        if [ $v = pipe2 ] && [ $c = u64 ]; then continue; fi
        unset HPXHIP_LIB HPXHIP_PIPE_WG
        if [ $v != default ]; then export HPXHIP_LIB=$A; fi
        if [ $v = pipe2 ]; then export HPXHIP_PIPE_WG=2; fi
        SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 > ${L}_sort_${v}_${c}_$i.log 2>&1 || exit $?
        echo "$v $c $i: $(grep -v '^#' ${L}_sort_${v}_${c}_$i.log | tail -1)" >> ${L}_status.log
      done
    done
  done
  unset HPXHIP_PIPE_WG
  HPXHIP_LIB=$A SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
  echo "prof ok" >> ${L}_status.log
}

# ---- scripts/r5/ap.sh
lease_ap() {
  # round 5, lease ap: k_onesweep's tile loads without per-key branches (build scripts/ubench/seglib.sh uncond
  # -DHPXHIP_OS_UNCOND_LOAD=1; every prefix pass): the sort tests on that build, then scripts/sort_probe.py 30 for
  # u64 and u32 on the shipped build and on uncond, alternating, three times each; a kernel trace of the uncond u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ap
  A=$PWD/scripts/ubench/seglib/uncond/libhpxhip.so
  HPXHIP_LIB=$A timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -k "sort" > ${L}_tests_uncond.log 2>&1
  rc=$?; echo "uncond sort tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  for i in 1 2 3; do
    for v in default uncond; do
      for c in u64 u32; do
        if [ $v = pipe2 ] && [ $c = u64 ]; then continue; fi
        unset HPXHIP_LIB HPXHIP_PIPE_WG
        if [ $v != default ]; then export HPXHIP_LIB=$A; fi
        if [ $v = pipe2 ]; then export HPXHIP_PIPE_WG=2; fi
        SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 > ${L}_sort_${v}_${c}_$i.log 2>&1 || exit $?
        echo "$v $c $i: $(grep -v '^#' ${L}_sort_${v}_${c}_$i.log | tail -1)" >> ${L}_status.log
      done
    done
  done
  unset HPXHIP_PIPE_WG
  HPXHIP_LIB=$A SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
  echo "prof ok" >> ${L}_status.log
}

# ---- scripts/r5/aq.sh
lease_aq() {
  # round 5, lease aq: k_onesweep and k_bucket_sort loads without per-key branches (build scripts/ubench/seglib.sh
  # uncond2 -DHPXHIP_OS_UNCOND_LOAD=1 -DHPXHIP_SEG_UNCOND_LOAD=1): the sort tests on that build, then
  # scripts/sort_probe.py 30 for u64 and u32 on the shipped build, uncond (lease ap) and uncond2, alternating,
  # three times each; a kernel trace of the uncond2 u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5aq
  B=$PWD/scripts/ubench/seglib
  HPXHIP_LIB=$B/uncond2/libhpxhip.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -k "sort" > ${L}_tests_uncond2.log 2>&1
  rc=$?; echo "uncond2 sort tests rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  for i in 1 2 3; do
    for v in default uncond uncond2; do
      for c in u64 u32; do
        unset HPXHIP_LIB
        if [ $v != default ]; then export HPXHIP_LIB=$B/$v/libhpxhip.so; fi
        SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 > ${L}_sort_${v}_${c}_$i.log 2>&1 || exit $?
        echo "$v $c $i: $(grep -v '^#' ${L}_sort_${v}_${c}_$i.log | tail -1)" >> ${L}_status.log
      done
    done
  done
  HPXHIP_LIB=$B/uncond2/libhpxhip.so SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
  echo "prof ok" >> ${L}_status.log
}

# ---- scripts/r5/ar.sh
lease_ar() {
  # round 5, lease ar: full validation of the tree -- GPU suite, smoke, bench, rocprofv3 kernel trace
  # + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5ar
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > ${L}_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > ${L}_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
  echo "bench ok" >> ${L}_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 bench.py --no-pmc --no-cpu > ${L}_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> ${L}_status.log
}

# ---- lease as (added after the fold)
lease_as() {
  # round 5, lease as: PMC passes (one counter group per run) over the 2^30 u64 sort with the onesweep tile
  # loads without per-key branches (the round's last sort) -- FETCH_SIZE, WRITE_SIZE, LDS / wave counters
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    SORT_ONLY=u64 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r5as_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r5as_pmc_sort$i.log 2>&1 || exit 1
  done
  python3 scripts/pmc_summary.py gpurun_out/r5as_pmc_sort1 gpurun_out/r5as_pmc_sort2 gpurun_out/r5as_pmc_sort3 > gpurun_out/r5as_pmc_sort.txt 2>&1
  echo ok
}

# ---- lease at (added after the fold)
lease_at() {
  # round 5, lease at: the round's last sort over the size sweep (2^20..2^30, u64 / u32 / pairs) and the
  # skewed cases at 2^28 (u64hot, u64corr, u64r16, u64r24) -- regression check of the branch-free tile loads
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r5at
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > ${L}_sweep.log 2>&1 || exit $?
  for c in u64hot u64corr u64r16 u64r24; do
    SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 28 > ${L}_$c.log 2>&1 || exit $?
    echo "$c: $(grep -v '^#' ${L}_$c.log | tail -1)" >> ${L}_status.log
  done
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: a aa ab ac ad ae ag ah ai aj ak al am an ao ap aq ar b c d e f g h i j k l m n o p q r s t u v w x y z as at"; fi
