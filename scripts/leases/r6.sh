# Lease scripts of round 6: what each gpurun call of the round ran, one
# shell function per lease (provenance of the profiles/r06_* logs).
# `bash scripts/leases/r6.sh NAME` runs lease NAME.

lease_a() {
  # round 6, lease a: the r05 multiway-merge miscompile reproduced with today's toolchain
  # (scripts/diag/mw_repro.py over the commit-8a18d38 builds, the shipped build and its variants),
  # the merge tests (variant builds included), the bench with the new strong-scaling rows, and a
  # baseline 2^30 u64 / u32 sort per kernel (rocprofv3 --kernel-trace --stats), and the prefix passes
  # with 4096- / 6144- / 8192-key tiles (scripts/ubench/sortpass7.hip)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6a
  timeout -k 10 300 python -u scripts/diag/mw_repro.py > ${L}_mw_repro.log 2>&1; rc=$?
  echo "mw_repro rc=$rc" >> ${L}_status.log
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_merge_sort.py \
    > ${L}_merge_tests.log 2>&1 || exit $?
  timeout -k 10 900 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
  timeout -k 10 300 ./scripts/ubench/sortpass7 > ${L}_sortpass7.log 2>&1 || exit $?
  for c in u64 u32; do
    SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6a_prof_$c -o run -- \
      python3 -u scripts/sort_probe.py 30 > ${L}_sort_$c.log 2>&1 || exit $?
  done
}

lease_b() {
  # round 6, lease b: second prefix pass ranked by LDS atomics on tiles inside one field bin
  # (HPXHIP_REGION_ATOM): sort tests, then A/B against the ballot-ranked build (seglib noratom)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6b
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_parity.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k sort \
    > ${L}_fullsize.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/noratom/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
}


lease_c() {
  # round 6, lease c: the one-pass segment sort (k_bucket_sort ONEB = 13, in-bin ranking by counting,
  # long bins handed to the two-pass form): sort tests, then A/B against ONE = 0 (the r05 two-pass form)
  # and ONE = 12, u64 / u32 / u64hot at 2^30 / 2^28, and a kernel trace of the u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6c
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/one0/libhpxhip.so scripts/ubench/seglib/one12/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
      echo "== $lib u64hot rep $rep" >> ${L}_ab.log
      HPXHIP_LIB=$lib SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
}

lease_d() {
  # round 6, lease d: the padded second prefix pass (k_pad_scatter: bucket slots claimed by global atomics,
  # no look-back) + the one-pass segment sort reading the slots: sort tests (all hybrid forms, oversized /
  # overflow fallbacks, 2^30 element-exact), then A/B against pad0 (look-back pass) and one0pad0 (r05 form),
  # u64 / u32 / u64hot / u64corr, and a kernel trace of the u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6d
  timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/pad0/libhpxhip.so scripts/ubench/seglib/one0pad0/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
      for c in u64hot u64corr; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
}

lease_e() {
  # round 6, lease e: why the padded pass is 4.7 ms against 3.9 for the offset-fed first pass -- kernel
  # trace of the no-atomics ablation (padabl: fixed claims, wrong output, timing only), and PMC passes
  # (FETCH_SIZE, WRITE_SIZE, SQ group) over the shipped u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6e
  HPXHIP_LIB=scripts/ubench/seglib/padabl/libhpxhip.so SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace \
    --stats -d gpurun_out/r6e_prof_abl -o run -- python3 -u scripts/sort_probe.py 30 > ${L}_abl.log 2>&1 || exit $?
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    SORT_ONLY=u64 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r6e_pmc_sort$i -o run -- \
      python3 scripts/sort_probe.py 30 > gpurun_out/r6e_pmc_sort$i.log 2>&1 || exit 1
  done
  python3 scripts/pmc_summary.py gpurun_out/r6e_pmc_sort1 gpurun_out/r6e_pmc_sort2 gpurun_out/r6e_pmc_sort3 \
    > gpurun_out/r6e_pmc_sort.txt 2>&1
}

lease_f() {
  # round 6, lease f: padded pass with the two-launch bounds scan: sort tests, A/B against pad0, kernel
  # trace; the C++ drop-in bench program alone; then bench.py (its cxx_drop_in row included)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6f
  timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/pad0/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6f_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
  timeout -k 10 300 ./tests/cxx/bin/bench_targets --targets 4 --logn 28 --heat-logn 26 > ${L}_cxx.log 2>&1 || exit $?
  timeout -k 10 900 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
}

lease_g() {
  # round 6, lease g: counters behind two claims.
  # 1. triad placement: six fresh processes of scripts/ubench/triad_place (each its own placement), each
  #    under two PMC passes (TCC_EA0_RDREQ, TCC_EA0_WRREQ) with the rocpd output (per-instance rows kept);
  # 2. the fused stencil's VALU load: SQ VALU counters over scripts/stencil_probe.py 30.
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6g
  timeout -s KILL 60 rocprofv3 -L > ${L}_counters.txt 2>&1 || true
  for i in 1 2 3 4 5 6; do
    timeout -k 10 60 ./scripts/ubench/triad_place 30 >> ${L}_triad_plain.log 2>&1 || exit $?
  done
  for i in 1 2 3; do
    for pmc in TCC_EA0_RDREQ TCC_EA0_WRREQ; do
      echo "== run $i $pmc" >> ${L}_triad_pmc.log
      timeout -s KILL 120 rocprofv3 --pmc $pmc -d gpurun_out/r6g_triad_${i}_${pmc} -o run -- \
        ./scripts/ubench/triad_place 30 >> ${L}_triad_pmc.log 2>&1 || exit 1
    done
  done
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 --output-format csv -d gpurun_out/r6g_heat_sq \
    -o run -- python3 scripts/stencil_probe.py 30 > ${L}_heat_sq.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6g_heat_fetch -o run -- \
    python3 scripts/stencil_probe.py 30 > ${L}_heat_fetch.log 2>&1 || exit 1
}

lease_h() {
  # round 6, lease h: triad placement below the L2 (lease g: the L2 channels get exactly equal request
  # counts in fast and slow runs) -- eight fresh processes of scripts/ubench/triad_place, each under one
  # PMC pass of the fabric-side queue levels and DRAM credit stalls (per instance in the rocpd database)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6h
  for i in 1 2 3 4 5 6 7 8; do
    echo "== run $i" >> ${L}_triad_pmc.log
    timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_LEVEL TCC_EA0_RDREQ_DRAM_CREDIT_STALL \
      TCC_EA0_WRREQ_DRAM_CREDIT_STALL -d gpurun_out/r6h_triad_$i -o run -- ./scripts/ubench/triad_place 30 \
      >> ${L}_triad_pmc.log 2>&1 || exit 1
  done
}

lease_i() {
  # round 6, lease i: sort_by_key in 512 x 9 pair segments (C_SEGD, two workgroups per CU) when the buckets
  # fit, and the planner's joint-histogram check (u64corr: no futile prefix passes; kv0 predates both): the sort tests (all pairs cases in every hybrid form, parity, 2^30 element-exact), then A/B against
  # kv0 (the 1024 x 9 segments only), 2^28 pairs, and a kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6i
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/kv0/libhpxhip.so; do
      echo "== $lib pairs rep $rep" >> ${L}_ab.log
      HPXHIP_LIB=$lib SORT_ONLY=pairs timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
      for c in u64 u64corr u64hot; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
  SORT_ONLY=pairs timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6i_prof_pairs -o run -- \
    python3 -u scripts/sort_probe.py 28 > ${L}_prof.log 2>&1 || exit $?
}

lease_j() {
  # round 6, lease j: the optimistic first pass (k_slot_pass1: field slots, no histogram read; k_opt_plan;
  # padded second pass over the slots): sort tests, then A/B against opt0 (the full path), u64 / u32 at
  # 2^30 and u64 / u64hot / u64corr at 2^28, and a kernel trace of the 2^30 u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6j
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/opt0/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
      for c in u64 u64hot u64corr; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6j_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
}

lease_k() {
  # round 6, lease k: validation of the tree -- the whole GPU suite, smoke, bench, and the bench under
  # rocprofv3 --kernel-trace --stats
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=${LEASE_OUT:-gpurun_out/r6k}
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > ${L}_tests.log 2>&1
  rc=$?; echo "suite rc=$rc" >> ${L}_status.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${L}_smoke.log 2>&1 || exit $?
  timeout -k 10 600 python -u bench.py > ${L}_bench.log 2>&1 || exit $?
  echo "bench ok" >> ${L}_status.log
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d ${L}_prof -o run -- python3 bench.py --no-pmc \
    --no-cpu > ${L}_bench_under_rocprof.log 2>&1 || exit $?
  echo "rocprof ok" >> ${L}_status.log
}

lease_l() {
  # round 6, lease l: the padded pass's slot counters packed four per 64-bit word (128 claims per tile
  # instead of 512): sort tests, A/B against pad32 (one 32-bit counter per bucket), kernel trace, and a
  # WRITE_SIZE pass over the u64 sort
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6l
  timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/pad32/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
      echo "== $lib u64hot rep $rep" >> ${L}_ab.log
      HPXHIP_LIB=$lib SORT_ONLY=u64hot timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6l_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
  SORT_ONLY=u64 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6l_pmc_w -o run -- \
    python3 scripts/sort_probe.py 30 > ${L}_pmc_w.log 2>&1 || exit 1
}

lease_m() {
  # round 6, lease m: k_hist_tiles counts the joint / top-9 histograms on every 8th tile only (one LDS
  # atomic per key), the planner scales them, the look-back pass gets an exact recount (k_joint_exact);
  # the offset-fed pass zeroes only its tile counter: sort tests, A/B against base13 (lease l's build),
  # u64 / u32 2^30, u64hot / u64corr 2^28, and a kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6m
  timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/base13/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
      for c in u64hot u64corr; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6m_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
}

lease_n() {
  # round 6, lease n: final validation (as lease k) of the round's last tree, plus a 2^30 u64 / u32 sort
  # kernel trace and one sort probe sweep
  LEASE_OUT=gpurun_out/r6n lease_k || exit $?
  cd $GRAFT_REPO_ROOT
  L=gpurun_out/r6n
  for c in u64 u32; do
    SORT_ONLY=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6n_prof_$c -o run -- \
      python3 -u scripts/sort_probe.py 30 > ${L}_sort_$c.log 2>&1 || exit $?
  done
  # the N > 1 rows on one GPU over a real one-rank RCCL group (segmented reduce's per-call overhead)
  HPXHIP_RCCL_SELF=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --no-cpu --no-pmc > ${L}_rccl_self.log 2>&1 || exit $?
}

lease_o() {
  # round 6, lease o: the offset-fed first pass deals its tiles to the XCD regions statically (no claim
  # counter): sort tests, A/B against xdyn (claims from the per-region counters), kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6o
  timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/xdyn/libhpxhip.so; do
      for c in u64 u32; do
        echo "== $lib $c rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
      done
      echo "== $lib u64 2^28 rep $rep" >> ${L}_ab.log
      HPXHIP_LIB=$lib SORT_ONLY=u64 timeout -k 10 200 python -u scripts/sort_probe.py 28 >> ${L}_ab.log 2>&1 || exit $?
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6o_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
}

lease_p() {
  # round 6, lease p: the pairs segment sort in the one-pass form (HPXHIP_SEG_ONE_KV): sort tests (with the
  # new pairs mixed-bins case), the C++ drop-in program test, A/B against kv1off (two-pass pairs), kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6p
  timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cxx_api.py \
    -k "drop_in" > ${L}_cxx.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/kv1off/libhpxhip.so; do
      for lg in 28 26; do
        echo "== $lib pairs 2^$lg rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=pairs timeout -k 10 200 python -u scripts/sort_probe.py $lg >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
  SORT_ONLY=pairs timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6p_prof_pairs -o run -- \
    python3 -u scripts/sort_probe.py 28 > ${L}_prof.log 2>&1 || exit $?
}

lease_q() {
  # round 6, lease q: lease p's steps after its sort tests (green there): the C++ drop-in program test
  # (the one-target check index fixed), the pairs A/B against kv1off, kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6q
  timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cxx_api.py \
    -k "drop_in" > ${L}_cxx.log 2>&1 || exit $?
  for rep in 1 2; do
    for lib in hpx_amd/libhpxhip.so scripts/ubench/seglib/kv1off/libhpxhip.so; do
      for lg in 28 26; do
        echo "== $lib pairs 2^$lg rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=pairs timeout -k 10 200 python -u scripts/sort_probe.py $lg >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
  SORT_ONLY=pairs timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6q_prof_pairs -o run -- \
    python3 -u scripts/sort_probe.py 28 > ${L}_prof.log 2>&1 || exit $?
}

lease_r() {
  # round 6, lease r: the fused heat kernel's window shape (rows x points per lane; shipped 2 x 4): stencil
  # probe at 2^30 for each build, twice, then the stencil tests under the 4 x 4 and 2 x 8 builds
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6r
  for rep in 1 2; do
    for v in main r4p4 r2p8 r4p8 r1p8; do
      lib=scripts/ubench/seglib/$v/libhpxhip.so
      [ $v = main ] && lib=hpx_amd/libhpxhip.so
      echo "== $v rep $rep" >> ${L}_ab.log
      HPXHIP_LIB=$lib timeout -k 10 200 python -u scripts/stencil_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
    done
  done
  for v in r4p4 r2p8; do
    HPXHIP_LIB=scripts/ubench/seglib/$v/libhpxhip.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 \
      --timeout-method thread tests -m gpu -k "stencil or heat" > ${L}_tests_$v.log 2>&1 || exit $?
  done
}

lease_s() {
  # round 6, lease s: final validation (as lease k) of the tree with the 4-row heat windows, then the
  # stencil probe at 2^30 and a kernel trace of the 2^28 pairs sort
  LEASE_OUT=gpurun_out/r6s lease_k || exit $?
  cd $GRAFT_REPO_ROOT
  L=gpurun_out/r6s
  timeout -k 10 200 python -u scripts/stencil_probe.py 30 > ${L}_stencil.log 2>&1 || exit $?
  SORT_ONLY=pairs timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6s_prof_pairs -o run -- \
    python3 -u scripts/sort_probe.py 28 > ${L}_sort_pairs.log 2>&1 || exit $?
}

lease_t() {
  # round 6, lease t: the fused heat kernel with lane runs (HPXHIP_HEAT_LANERUN: each lane steps 16 / 8
  # consecutive points, the window transposed through LDS): stencil tests under it, then the stencil probe
  # at 2^30 for main (4 x 4 rows), lanerun (4 x 4) and lr2 (2 x 4), twice
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6t
  HPXHIP_LIB=scripts/ubench/seglib/lanerun/libhpxhip.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 \
    --timeout-method thread tests -m gpu -k "stencil or heat" > ${L}_tests_lanerun.log 2>&1 || exit $?
  for rep in 1 2; do
    for v in main lanerun lr2; do
      lib=scripts/ubench/seglib/$v/libhpxhip.so
      [ $v = main ] && lib=hpx_amd/libhpxhip.so
      echo "== $v rep $rep" >> ${L}_ab.log
      HPXHIP_LIB=$lib timeout -k 10 200 python -u scripts/stencil_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
    done
  done
}

lease_u() {
  # round 6, lease u: final validation (as lease k) of the tree with the lane-run heat kernel, then the
  # stencil probe at 2^30 and the C++ drop-in program at the bench's 1-GPU size
  LEASE_OUT=gpurun_out/r6u lease_k || exit $?
  cd $GRAFT_REPO_ROOT
  L=gpurun_out/r6u
  timeout -k 10 200 python -u scripts/stencil_probe.py 30 > ${L}_stencil.log 2>&1 || exit $?
}

lease_v() {
  # round 6, lease v: the planner without f64 divisions and the padded pass's look-back fallback as a
  # persistent grid: sort tests (with the new forced-overflow cases), 2^30 u64 / u32 probes, u64 kernel trace
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6v
  timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "sort" > ${L}_tests.log 2>&1 || exit $?
  for rep in 1 2; do
    for c in u64 u32; do
      SORT_ONLY=$c timeout -k 10 200 python -u scripts/sort_probe.py 30 >> ${L}_probe.log 2>&1 || exit $?
    done
  done
  SORT_ONLY=u64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6v_prof_u64 -o run -- \
    python3 -u scripts/sort_probe.py 30 > ${L}_prof.log 2>&1 || exit $?
}

lease_w() {
  # round 6, lease w: final validation (as lease k) of the round's last tree
  LEASE_OUT=gpurun_out/r6w lease_k || exit $?
}

lease_x() {
  # round 6, lease x: sort_by_key's prefix-pass tile (HPXHIP_KV_THREADS x HPXHIP_KV_ITEMS; shipped 256 x 16,
  # 2 workgroups = 8 waves per CU): sort_by_key tests under 512 x 8, then pairs 2^28 / 2^26 for main,
  # kv512x8 and kv512x6, twice
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6x
  HPXHIP_LIB=scripts/ubench/seglib/kv512x8/libhpxhip.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 \
    --timeout-method thread tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -k "by_key or pairs" \
    > ${L}_tests_kv512x8.log 2>&1 || exit $?
  for rep in 1 2; do
    for v in main kv512x8 kv512x6; do
      lib=scripts/ubench/seglib/$v/libhpxhip.so
      [ $v = main ] && lib=hpx_amd/libhpxhip.so
      for lg in 28 26; do
        echo "== $v pairs 2^$lg rep $rep" >> ${L}_ab.log
        HPXHIP_LIB=$lib SORT_ONLY=pairs timeout -k 10 200 python -u scripts/sort_probe.py $lg >> ${L}_ab.log 2>&1 || exit $?
      done
    done
  done
}

lease_y() {
  # round 6, lease y: the library rebuilt from the committed tree (the tile knob only): smoke, the sort and
  # stencil GPU tests, and the one-rank RCCL rehearsal of the N > 1 rows (segmented reduce / scan / sort,
  # the 2^32 stencil) with the lane-run heat kernel
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6y
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${L}_smoke.log 2>&1 || exit $?
  timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    -k "sort or stencil or heat" > ${L}_tests.log 2>&1 || exit $?
  HPXHIP_RCCL_SELF=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --no-cpu --no-pmc > ${L}_rccl_self.log 2>&1 || exit $?
}

lease_z() {
  # round 6, lease z: the lane-run heat kernel's LDS transpose in two halves (HPXHIP_HEAT_LDS_HALF: 16 KiB
  # per block, 6 waves per SIMD instead of 5): stencil tests under it, then the stencil probe at 2^30 for
  # main and half, twice
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6z
  HPXHIP_LIB=scripts/ubench/seglib/half/libhpxhip.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 \
    --timeout-method thread tests -m gpu -k "stencil or heat" > ${L}_tests_half.log 2>&1 || exit $?
  for rep in 1 2; do
    for v in main half; do
      lib=scripts/ubench/seglib/$v/libhpxhip.so
      [ $v = main ] && lib=hpx_amd/libhpxhip.so
      echo "== $v rep $rep" >> ${L}_ab.log
      HPXHIP_LIB=$lib timeout -k 10 200 python -u scripts/stencil_probe.py 30 >> ${L}_ab.log 2>&1 || exit $?
    done
  done
}

lease_fin() {
  # round 6, last lease: the whole GPU suite and smoke on the round's final tree (library relinked after z)
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  L=gpurun_out/r6fin
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > ${L}_tests.log 2>&1 || exit $?
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${L}_smoke.log 2>&1 || exit $?
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: a b c d e f g h i j k l m n o p q r s t u v w x y z fin"; fi
