# Lease scripts of round 4 (scripts/r4/X.sh): what each gpurun call of that round ran,
# kept as one shell function per former file (provenance of the profiles/
# logs that cite them).  `bash scripts/leases/r4.sh NAME` runs lease NAME.

# ---- scripts/r4/a.sh
lease_a() {
  # round 4, lease a: exception_list contract, launcher, iterator views -- full GPU suite, smoke, bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4a_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4a_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4a_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4a_status.log
}

# ---- scripts/r4/aa.sh
lease_aa() {
  # round 4, lease aa: when_all completes by waiting on its inputs (no callbacks unless a continuation arms it)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4aa_cxx.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4aa_call_overhead.log 2>&1 || exit $?
}

# ---- scripts/r4/ab.sh
lease_ab() {
  # round 4, lease ab: copy_if one-hop look-back, group 64/32 x poll sleep 1/3 (scan and int32 rows ride along)
  cd $GRAFT_REPO_ROOT
  for b in oh_g64_s1 oh_g32_s1 oh_g64_s3 oh_g32_s3 oh_g64_s1 oh_g32_s1; do
    timeout -k 10 150 scripts/r4/lb/$b >> gpurun_out/r4ab_onehop_group.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/ad.sh
lease_ad() {
  # round 4, lease ad: DPP neighbour shift in the elementwise shifted kernels (and the scan's), parity + probe
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "shifted or misaligned or unaligned" --timeout 300 --timeout-method thread > gpurun_out/r4ad_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/unaligned_probe.py > gpurun_out/r4ad_probe.log 2>&1 || exit $?
}

# ---- scripts/r4/ae.sh
lease_ae() {
  # round 4, lease ae: the 18-bit sort form (HPXHIP_SORT_HYBRID=18): sort tests in all forms, probe 17 vs 18, kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ae_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4ae_probe17.log 2>&1 || exit $?
  HPXHIP_SORT_HYBRID=18 timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4ae_probe18.log 2>&1 || exit $?
  HPXHIP_SORT_HYBRID=18 SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ae_prof18 -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4ae_prof18.log 2>&1 || exit $?
}

# ---- scripts/r4/af.sh
lease_af() {
  # round 4, lease af: 18-bit form as the default -- sort-using GPU tests, cliff probes, bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py tests/test_gpu_multirank.py tests/test_gpu_parity.py tests/test_gpu_segmented_layouts.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4af_tests.log 2>&1 || exit $?
  SORT_ONLY=u64corr timeout -k 10 200 python -u scripts/sort_probe.py 28 > gpurun_out/r4af_probe.log 2>&1 || exit $?
  SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4af_probe.log 2>&1 || exit $?
  SORT_ONLY=u64r16 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4af_probe.log 2>&1 || exit $?
  SORT_ONLY=u64r24 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4af_probe.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4af_bench.log 2>&1 || exit $?
}

# ---- scripts/r4/ag.sh
lease_ag() {
  # round 4, lease ag: small key ranges (r16, r24) under the 17- and 18-bit forms on one box
  cd $GRAFT_REPO_ROOT
  for m in 17 18 17 18; do
    echo "HPXHIP_SORT_HYBRID=$m" >> gpurun_out/r4ag_probe.log
    HPXHIP_SORT_HYBRID=$m SORT_ONLY=u64r16 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ag_probe.log 2>&1 || exit $?
    HPXHIP_SORT_HYBRID=$m SORT_ONLY=u64r24 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ag_probe.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/ai.sh
lease_ai() {
  # round 4, lease ai: 18-bit form, the top-byte pass (16-bit fallback only): persistent vs one workgroup per tile (HPXHIP_B_PLAIN)
  cd $GRAFT_REPO_ROOT
  for v in 0 1 0 1; do
    echo "B_PLAIN=$v" >> gpurun_out/r4ai_probe.log
    if [ $v = 1 ]; then export HPXHIP_B_PLAIN=1; else unset HPXHIP_B_PLAIN; fi
    SORT_ONLY=u64 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ai_probe.log 2>&1 || exit $?
    SORT_ONLY=u64r16 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ai_probe.log 2>&1 || exit $?
    SORT_ONLY=u64r24 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ai_probe.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/aj.sh
lease_aj() {
  # round 4, lease aj: kernel traces of the u64r16 sort (keys below 2^16) under the 17- and 18-bit forms, second count skipping constant digits
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for m in 17 18; do
    HPXHIP_SORT_HYBRID=$m SORT_ONLY=u64r16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4aj_prof$m -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4aj_prof$m.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/ak.sh
lease_ak() {
  # round 4, lease ak: second histogram skips constant digits; sort tests (all forms), probes
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_merge_sort.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ak_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4ak_probe.log 2>&1 || exit $?
  for c in u64r16 u64r24; do SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ak_probe.log 2>&1 || exit $?; done
  for c in u64corr u64hot; do SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4ak_probe.log 2>&1 || exit $?; done
}

# ---- scripts/r4/am.sh
lease_am() {
  # round 4, lease am: the 18-bit form's first prefix pass from precomputed tile offsets (no look-back)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -q -x -k "18" --timeout 300 --timeout-method thread > gpurun_out/r4am_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4am_probe.log 2>&1 || exit $?
  SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4am_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4am_prof.log 2>&1 || exit $?
}

# ---- scripts/r4/an.sh
lease_an() {
  # round 4, lease an: precomputed-offset first pass with counter-ordered tiles; PMC write traffic of that pass
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  SORT_ONLY=u64 timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4an_probe.log 2>&1 || exit $?
  SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4an_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4an_prof.log 2>&1 || exit $?
  SORT_ONLY=u64 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_onesweep --output-format csv -d gpurun_out/r4an_pmc -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4an_pmc.log 2>&1 || exit $?
}

# ---- scripts/r4/ao.sh
lease_ao() {
  # round 4, lease ao: same-box A/B, first prefix pass from precomputed tile offsets vs look-back (HPXHIP_SORT_NOPRE)
  cd $GRAFT_REPO_ROOT
  for v in 0 1 0 1 0 1; do
    echo "NOPRE=$v" >> gpurun_out/r4ao_probe.log
    if [ $v = 1 ]; then export HPXHIP_SORT_NOPRE=1; else unset HPXHIP_SORT_NOPRE; fi
    SORT_ONLY=u64 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ao_probe.log 2>&1 || exit $?
    SORT_ONLY=u32 timeout -k 10 200 python -u scripts/sort_probe.py 30 >> gpurun_out/r4ao_probe.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/ap.sh
lease_ap() {
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
}

# ---- scripts/r4/aq.sh
lease_aq() {
  # round 4, lease aq: PMC passes over the 2^30 u64 sort in its r04 form (18-bit, first pass from tile offsets)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  export SORT_ONLY=u64
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r4aq_pmc_sort$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4aq_pmc_sort$i.log 2>&1 || { echo "pmc pass $i failed rc=$?" >> gpurun_out/r4aq_status.log; exit 1; }
  done
  echo "pmc ok" >> gpurun_out/r4aq_status.log
}

# ---- scripts/r4/ar.sh
lease_ar() {
  # round 4, lease ar: comparator merge sort with 16-B staging/stores in the merge passes
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ar_cxx.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4ar_closure_sort.log 2>&1 || exit $?
}

# ---- scripts/r4/as.sh
lease_as() {
  # round 4, lease as: merge tiles of 4096 (256 threads x 16 items): merge API tests, C++ closures, comparator sort timing, merge probe
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_merge_sort.py tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4as_tests.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4as_closure_sort.log 2>&1 || exit $?
}

# ---- scripts/r4/at.sh
lease_at() {
  # round 4, lease at: pooled events created on their pool's device; C++ programs, call overhead, smoke
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_errors.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4at_tests.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4at_call_overhead.log 2>&1 || exit $?
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4at_smoke.log 2>&1 || exit $?
}

# ---- scripts/r4/au.sh
lease_au() {
  # round 4, lease au: stream_after falls back to a host wait; C++ programs, call overhead, smoke
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_errors.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4au_tests.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4au_call_overhead.log 2>&1 || exit $?
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4au_smoke.log 2>&1 || exit $?
}

# ---- scripts/r4/av.sh
lease_av() {
  # round 4, lease av: look-back poll sleep (HPXHIP_LB_SLEEP 0/1/3/8) in the sort's prefix passes (sortpass3 ubench)
  cd $GRAFT_REPO_ROOT
  for s in 1 0 3 8 1; do
    echo "== sleep $s" >> gpurun_out/r4av_lbsleep_sort.log
    timeout -k 10 120 scripts/ubench/tmpbin/sp3_s$s >> gpurun_out/r4av_lbsleep_sort.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/aw.sh
lease_aw() {
  # round 4, lease aw: look-back poll sleep 1/8/16/32 in the sort's prefix passes, alternated over fresh processes (placements)
  cd $GRAFT_REPO_ROOT
  for rep in 1 2 3; do
  for s in 1 8 16 32; do
    echo "== sleep $s rep $rep" >> gpurun_out/r4aw_lbsleep_sort.log
    timeout -k 10 120 scripts/ubench/tmpbin/sp3_s$s >> gpurun_out/r4aw_lbsleep_sort.log 2>&1 || exit $?
  done
  done
}

# ---- scripts/r4/ax.sh
lease_ax() {
  # round 4, lease ax: sort look-back back-off 8 (HPXHIP_SORT_LB_SLEEP): sort tests, then the bench (sort rows)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_merge_sort.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ax_tests.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4ax_bench.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4ax_bench2.log 2>&1 || exit $?
}

# ---- scripts/r4/ay.sh
lease_ay() {
  # round 4, lease ay: same-box A/B of the sort's look-back back-off, 1 vs 8 (two library builds, alternated processes)
  cd $GRAFT_REPO_ROOT
  for rep in 1 2 3 4; do
  for s in 1 8; do
    HPXHIP_LIB=scripts/ubench/tmpbin/libhpxhip_s$s.so timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4ay_ab_sort_lbsleep.log 2>&1 || exit $?
  done
  done
}

# ---- scripts/r4/az.sh
lease_az() {
  # round 4, lease az: the rebuilt library after the reverted experiment: smoke, sort / scan / copy_if parity
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4az_smoke.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4az_tests.log 2>&1 || exit $?
}

# ---- scripts/r4/b.sh
lease_b() {
  # round 4, lease b: the atomic segment sort -- hybrid sort tests (both segment kernels), sort probe A/B
  # under rocprofv3 kernel trace, then the full GPU suite
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4b_sort_tests.log 2>&1 || exit $?
  for seg in atomic stable; do
    HPXHIP_SORT_SEG=$seg SORT_ONLY=u64 timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4b_probe.log 2>&1 || exit $?
    HPXHIP_SORT_SEG=$seg SORT_ONLY=u32 timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4b_probe.log 2>&1 || exit $?
  done
  mkdir -p gpurun_out/r4b_prof
  HPXHIP_SORT_SEG=atomic SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4b_prof.log 2>&1 || exit $?
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1
  echo "suite rc=$?" >> gpurun_out/r4b_status.log
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 > gpurun_out/r4b_closure_timing.log 2>&1
  echo "closure timing rc=$?" >> gpurun_out/r4b_status.log
}

# ---- scripts/r4/ba.sh
lease_ba() {
  # round 4, lease ba: fill (write-only stream) shapes at 2^30 doubles
  cd $GRAFT_REPO_ROOT
  timeout -k 10 120 scripts/ubench/fill > gpurun_out/r4ba_fill.log 2>&1 || exit $?
  timeout -k 10 120 scripts/ubench/fill >> gpurun_out/r4ba_fill.log 2>&1 || exit $?
}

# ---- scripts/r4/bb.sh
lease_bb() {
  # round 4, lease bb: fill into a fresh allocation (first writes) vs again
  cd $GRAFT_REPO_ROOT
  timeout -k 10 120 scripts/ubench/fill > gpurun_out/r4bb_fill.log 2>&1 || exit $?
}

# ---- scripts/r4/c.sh
lease_c() {
  # round 4, lease c: identity-free closure scans (noid_op), sort path back to r03 -- correctness first,
  # then closure timing (reductions/scans), then the comparator sort timing last (the r4b run faulted in it)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py tests/test_gpu_errors.py tests/test_gpu_sort_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > gpurun_out/r4c_closure_timing.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4c_closure_sort.log 2>&1 || exit $?
  echo ok > gpurun_out/r4c_status.log
}

# ---- scripts/r4/d.sh
lease_d() {
  # round 4, lease d: comparator-sort timing (race fixed), C++ call overhead (event get), match_digit A/B
  # (builtin ballot vs round-3 asm), full suite, smoke, bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 sort > gpurun_out/r4d_closure_sort.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4d_call_overhead.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/r4/lib_asm.so; do
      for k in u64 u32; do
        echo "lib=$lib" >> gpurun_out/r4d_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$k timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4d_ab.log 2>&1 || exit $?
      done
    done
  done
  mkdir -p gpurun_out/r4d_prof
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4d_prof.log 2>&1 || exit $?
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4d_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4d_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4d_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4d_status.log
  for c in u64corr u64hot; do SORT_ONLY=$c timeout -k 10 300 python -u scripts/sort_probe.py 28 >> gpurun_out/r4d_cliff.log 2>&1 || exit $?; done
}

# ---- scripts/r4/e.sh
lease_e() {
  # round 4, lease e: instruction mix of the sort kernels (PMC), 2^30 u64 and u32
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r4e_counters.txt 2>&1
  grep -o "SQ_[A-Z0-9_]*" gpurun_out/r4e_counters.txt | sort -u > gpurun_out/r4e_sq.txt
  i=0
  for k in u64 u32; do
  for pmc in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"; do
    i=$((i+1))
    SORT_ONLY=$k timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r4e_pmc$i -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4e_pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?" >> gpurun_out/r4e_status.log; }
  done
  done
  python3 scripts/pmc_summary.py gpurun_out/r4e_pmc1 gpurun_out/r4e_pmc2 > gpurun_out/r4e_u64.txt 2>&1
  python3 scripts/pmc_summary.py gpurun_out/r4e_pmc3 gpurun_out/r4e_pmc4 > gpurun_out/r4e_u32.txt 2>&1
  echo done >> gpurun_out/r4e_status.log
}

# ---- scripts/r4/f.sh
lease_f() {
  # round 4, lease f: fixed look-back with 64 x K tiles per group (chain of E hand-offs K times shorter): A/B K=1 vs K=4
  # on scan / copy_if / sort at 2^30, and the scan / copy_if parity tests on the K=4 build
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/r4/lib_k4.so; do
      HPXHIP_LIB=$lib timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4f_ab.log 2>&1 || exit $?
    done
  done
  HPXHIP_LIB=scripts/r4/lib_k4.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x -k "scan or copy_if" --timeout 300 --timeout-method thread > gpurun_out/r4f_tests_k4.log 2>&1
  echo "k4 tests rc=$?" >> gpurun_out/r4f_status.log
}

# ---- scripts/r4/final.sh
lease_final() {
  # round 4, final lease: full GPU suite, smoke, bench, rocprofv3 kernel trace + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4final_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4final_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4final_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4final_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4final_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4final_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r4final_status.log
}

# ---- scripts/r4/final2.sh
lease_final2() {
  # round 4, final lease (2): full GPU suite, smoke, bench, rocprofv3 kernel trace + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4final2_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4final2_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4final2_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4final2_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4final2_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final2_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4final2_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r4final2_status.log
}

# ---- scripts/r4/final3.sh
lease_final3() {
  # round 4, final lease (3): full GPU suite, smoke, bench, rocprofv3 kernel trace + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4final3_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4final3_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4final3_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4final3_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4final3_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final3_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4final3_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r4final3_status.log
}

# ---- scripts/r4/final4.sh
lease_final4() {
  # round 4, final lease (4), after the event-pool and stream-ordering fixes: full GPU suite, smoke, bench, rocprofv3 kernel trace + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4final4_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4final4_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4final4_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4final4_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4final4_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final4_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4final4_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r4final4_status.log
}

# ---- scripts/r4/final5.sh
lease_final5() {
  # round 4, final lease (5), the tree as it ends the round: full GPU suite, smoke, bench, rocprofv3 kernel trace + stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4final5_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4final5_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4final5_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4final5_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4final5_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4final5_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4final5_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r4final5_status.log
}

# ---- scripts/r4/g.sh
lease_g() {
  # round 4, lease g: fixed look-back group of 64 (shipped) vs 32 vs 16 tiles at 2^30, + parity of the 16 build
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/r4/lib_g32.so scripts/r4/lib_g16.so; do
      HPXHIP_LIB=$lib timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4g_ab.log 2>&1 || exit $?
    done
  done
  HPXHIP_LIB=scripts/r4/lib_g16.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x -k "scan or copy_if" --timeout 300 --timeout-method thread > gpurun_out/r4g_tests_g16.log 2>&1
  echo "g16 tests rc=$?" >> gpurun_out/r4g_status.log
}

# ---- scripts/r4/h.sh
lease_h() {
  # round 4, lease h: fixed look-back group 64 / 48 / 40 / 32 / 24 tiles, scan and copy_if at 2^30
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/r4/lib_g48.so scripts/r4/lib_g40.so scripts/r4/lib_g32.so scripts/r4/lib_g24.so; do
      HPXHIP_LIB=$lib NOSORT=1 timeout -k 10 200 python -u scripts/ab_probe.py >> gpurun_out/r4h_ab.log 2>&1 || exit $?
    done
  done
}

# ---- scripts/r4/i.sh
lease_i() {
  # round 4, lease i: onesweep fixed-group look-back (LBFIX 32 / 16) vs the walk, sort at 2^30 u64 / u32;
  # hybrid-sort parity tests on the LBFIX=32 build
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/r4/lib_fix32.so scripts/r4/lib_fix16.so; do
      for k in u64 u32; do
        echo "lib=$lib" >> gpurun_out/r4i_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$k timeout -k 10 120 python -u scripts/sort_probe.py 30 >> gpurun_out/r4i_ab.log 2>&1 || exit $?
      done
    done
  done
  HPXHIP_LIB=scripts/r4/lib_fix32.so timeout -k 10 900 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -q -x -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r4i_tests_fix32.log 2>&1
  echo "fix32 tests rc=$?" >> gpurun_out/r4i_status.log
}

# ---- scripts/r4/j.sh
lease_j() {
  # round 4, lease j: lazy completion callbacks (C++ futures), scans on 32-tile look-back groups --
  # C++ programs + call overhead, full GPU suite, smoke, bench, rocprofv3 kernel stats of the bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4j_cxx.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/call_overhead > gpurun_out/r4j_call_overhead.log 2>&1 || exit $?
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4j_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4j_smoke.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4j_bench.log 2>&1 || exit $?
  echo "bench ok" >> gpurun_out/r4j_status.log
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4j_prof -o run -- python3 bench.py --no-pmc --no-cpu > gpurun_out/r4j_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> gpurun_out/r4j_status.log
}

# ---- scripts/r4/k.sh
lease_k() {
  # round 4, lease k: look-back poll interval x group size (scan, copy_if at 2^30 int64)
  cd $GRAFT_REPO_ROOT
  for b in lb_s1_g64 lb_s4_g64 lb_s16_g64 lb_s1_g32 lb_s4_g32 lb_s16_g32; do
    timeout -k 10 150 scripts/r4/lb/$b >> gpurun_out/r4k_lb.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/l.sh
lease_l() {
  # round 4, lease l: copy_if phase split + PMC traffic of the shipped kernel
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 200 scripts/r4/lb/copyif8 > gpurun_out/r4l_copyif8.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_copy_if --output-format csv -d gpurun_out/r4l_pmc_fetch -o run -- scripts/r4/lb/copyif8 only > gpurun_out/r4l_pmc_fetch.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_copy_if --output-format csv -d gpurun_out/r4l_pmc_write -o run -- scripts/r4/lb/copyif8 only > gpurun_out/r4l_pmc_write.log 2>&1 || exit $?
}

# ---- scripts/r4/n.sh
lease_n() {
  # round 4, lease n: the 17-bit first histogram counts one byte digit (k_hist), copy_if nt stores
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4n_probe.log 2>&1 || exit $?
  SORT_ONLY=u64corr timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4n_probe.log 2>&1 || exit $?
  SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 28 >> gpurun_out/r4n_probe.log 2>&1 || exit $?
  SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4n_prof.log 2>&1 || exit $?
}

# ---- scripts/r4/o.sh
lease_o() {
  # round 4, lease o: compact first histogram (1024 x 16 copies, D = 2), sort tests + probe + kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/sort_probe.py 30 > gpurun_out/r4o_probe.log 2>&1 || exit $?
  SORT_ONLY=u64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4o_prof -o run -- python3 scripts/sort_probe.py 30 > gpurun_out/r4o_prof.log 2>&1 || exit $?
}

# ---- scripts/r4/r.sh
lease_r() {
  # round 4, lease r: one-hop fixed look-back A/B (scan + copy_if, 2^30 int64)
  cd $GRAFT_REPO_ROOT
  for b in lb_onehop0 lb_onehop1 lb_onehop0 lb_onehop1; do
    timeout -k 10 150 scripts/r4/lb/$b >> gpurun_out/r4r_onehop.log 2>&1 || exit $?
  done
}

# ---- scripts/r4/t.sh
lease_t() {
  # round 4, lease t: copy_if 16-B stores + one-hop look-back (8-byte), parity + C++ programs + timing + bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_errors.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4t_tests.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests/test_cxx_api.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4t_cxx.log 2>&1 || exit $?
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > gpurun_out/r4t_closure_timing.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4t_bench.log 2>&1 || exit $?
}

# ---- scripts/r4/u.sh
lease_u() {
  # round 4, lease u: closure copy_if back to its r03 form; bench
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 tests/cxx/bin/closure_timing 30 reduce > gpurun_out/r4u_closure_timing.log 2>&1 || exit $?
  timeout -k 10 500 python -u bench.py > gpurun_out/r4u_bench.log 2>&1 || exit $?
}

# ---- scripts/r4/w.sh
lease_w() {
  # round 4, lease w: shifted-input vector scan (mutually misaligned ranges), parity + probe, two tile shapes
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "misaligned or shifted" --timeout 300 --timeout-method thread > gpurun_out/r4w_tests.log 2>&1 || exit $?
  HPXHIP_SCAN_SHIFT_SHAPE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "misaligned or shifted" --timeout 300 --timeout-method thread > gpurun_out/r4w_tests_shape1.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/unaligned_probe.py > gpurun_out/r4w_probe.log 2>&1 || exit $?
  HPXHIP_SCAN_SHIFT_SHAPE=1 timeout -k 10 300 python -u scripts/unaligned_probe.py > gpurun_out/r4w_probe_shape1.log 2>&1 || exit $?
}

# ---- scripts/r4/x.sh
lease_x() {
  # round 4, lease x: one-rank RCCL run of the segmented orchestration; full GPU suite; smoke
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v -x --timeout 240 --timeout-method thread > gpurun_out/r4x_multirank.log 2>&1 || exit $?
  timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4x_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> gpurun_out/r4x_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/r4x_smoke.log 2>&1 || exit $?
}

# ---- scripts/r4/y.sh
lease_y() {
  # round 4, lease y: bench's N > 1 path rehearsed on one GPU -- one rank under torchrun, RCCL group through TorchComm
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  HPXHIP_RCCL_SELF=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4y_bench_rccl_self.log 2>&1 || exit $?
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: a aa ab ad ae af ag ai aj ak am an ao ap aq ar as at au av aw ax ay az b ba bb c d e f final final2 final3 final4 final5 g h i j k l n o r t u w x y"; fi
