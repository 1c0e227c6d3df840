# Lease scripts of round 2, session 3 (scripts/r2s3_*.sh): what each gpurun call of that round ran,
# kept as one shell function per former file (provenance of the profiles/
# logs that cite them).  `bash scripts/leases/r2s3.sh NAME` runs lease NAME.

# ---- scripts/r2s3_a.sh
lease_r2s3_a() {
  # 32-bit keys through the hybrid sort: hybrid + fullsize sort tests, probe timing, traces (17- and 16-bit forms)
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -m gpu -x -q -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r2s3a_tests.log 2>&1
  timeout -k 10 200 python -u scripts/ab_probe.py > gpurun_out/r2s3a_probe.log 2>&1
  export KEY=u32
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3a_trace17 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3a_trace17.log 2>&1
  export HPXHIP_SORT_HYBRID=16
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3a_trace16 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3a_trace16.log 2>&1
  export HPXHIP_SORT_HYBRID=0
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3a_trace0 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3a_trace0.log 2>&1
}

# ---- scripts/r2s3_b.sh
lease_r2s3_b() {
  # sort_by_key with 32-bit keys through the hybrid: hybrid sort tests, KV probe hybrid vs LSD
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_parity.py -m gpu -x -q -k "sort" --timeout 300 --timeout-method thread > gpurun_out/r2s3b_tests.log 2>&1
  timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s3b_kv.log 2>&1
  HPXHIP_SORT_HYBRID=0 timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s3b_kv.log 2>&1
}

# ---- scripts/r2s3_c.sh
lease_r2s3_c() {
  # direct per-bucket segment sort for sort_by_key and smaller keys-only sorts: threshold ablation + forced-direct tests
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s3c_probe.log 2>&1
  HPXHIP_SORT_DIRECT=4 timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s3c_probe.log 2>&1
  for lg in 28 29; do
    LOGN=$lg timeout -k 10 200 python -u scripts/ab_probe.py 2>&1 | grep sort >> gpurun_out/r2s3c_probe.log
    LOGN=$lg HPXHIP_SORT_DIRECT=4 timeout -k 10 200 python -u scripts/ab_probe.py 2>&1 | grep sort | sed 's/^shipped /direct4 /' >> gpurun_out/r2s3c_probe.log
  done
  HPXHIP_SORT_DIRECT=100000 timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s3c_tests.log 2>&1
}

# ---- scripts/r2s3_d.sh
lease_r2s3_d() {
  # sort_by_key at 2^29 pairs: direct per-bucket segments (default) vs host-packed (HPXHIP_SORT_DIRECT=0)
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  LOGN=29 timeout -k 10 200 python -u scripts/kv_probe.py > gpurun_out/r2s3d_probe.log 2>&1
  LOGN=29 HPXHIP_SORT_DIRECT=0 timeout -k 10 200 python -u scripts/kv_probe.py 2>&1 | sed 's/^hybrid /packed /' >> gpurun_out/r2s3d_probe.log
}

# ---- scripts/r2s3_e.sh
lease_r2s3_e() {
  # line-aligned write-back in k_bucket_sort: hybrid sort tests (incl. forced direct path), sort probes, WRITE_SIZE pass
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s3e_tests.log 2>&1
  timeout -k 10 200 python -u scripts/ab_probe.py > gpurun_out/r2s3e_probe.log 2>&1
  timeout -k 10 200 python -u scripts/kv_probe.py >> gpurun_out/r2s3e_probe.log 2>&1
  export KEY=u64
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2s3e_pmc_u64 -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3e_pmc_u64.log 2>&1
}

# ---- scripts/r2s3_f.sh
lease_r2s3_f() {
  # same-box A/B of the line-aligned k_bucket_sort write-back (old / new / old / new)
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for r in 1 2; do
    for v in old new; do
      HPXHIP_LIB=$PWD/scripts/ablib/libhpxhip_$v.so timeout -k 10 200 python -u scripts/ab_probe.py 2>&1 | grep sort >> gpurun_out/r2s3f_ab.log
      HPXHIP_LIB=$PWD/scripts/ablib/libhpxhip_$v.so timeout -k 10 200 python -u scripts/kv_probe.py 2>&1 | grep "u64/u64\|u32/u64" | sed "s/^/$v /" >> gpurun_out/r2s3f_ab.log
    done
  done
}

# ---- scripts/r2s3_final.sh
lease_r2s3_final() {
  # round-2 final measurement set: full GPU suite, smoke, bench (PMC + host baseline), rocprofv3 stats of the same bench
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s3fin_tests.log 2>&1
  timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2s3fin_smoke.log 2>&1
  timeout -k 10 500 python -u bench.py > gpurun_out/r2s3fin_bench.log 2>&1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3fin_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2s3fin_bench_under_rocprof.log 2>&1
}

# ---- scripts/r2s3_final2.sh
lease_r2s3_final2() {
  # round-2 final measurement set: full GPU suite, smoke, bench (PMC + host baseline), rocprofv3 stats of the same bench
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s3fin2_tests.log 2>&1
  timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2s3fin2_smoke.log 2>&1
  timeout -k 10 500 python -u bench.py > gpurun_out/r2s3fin2_bench.log 2>&1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2s3fin2_trace -o run -- python3 bench.py --no-pmc > gpurun_out/r2s3fin2_bench_under_rocprof.log 2>&1
}

# ---- scripts/r2s3_g.sh
lease_r2s3_g() {
  # keys-only plain write-back restored, sort_by_key aligned: hybrid sort tests + smoke
  set -e
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sort_hybrid.py tests/test_gpu_fullsize.py -k "sort" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2s3g_tests.log 2>&1
  timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r2s3g_smoke.log 2>&1
}

# ---- scripts/r2s3_pmc.sh
lease_r2s3_pmc() {
  # PMC passes (FETCH_SIZE, WRITE_SIZE; one counter per run) over the hybrid sort of 2^30 keys, u64 (direct per-bucket path) and u32
  cd $GRAFT_REPO_ROOT
  export TMPDIR=/tmp
  for key in u64 u32; do
    export KEY=$key
    i=0
    for pmc in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r2s3_pmc_${key}_$i -o run -- python3 scripts/sort_probe.py > gpurun_out/r2s3_pmc_${key}_$i.log 2>&1 || { echo "pass $key $i failed rc=$?"; exit 1; }
    done
  done
  echo done
}

if [ $# -eq 1 ]; then "lease_$1"; else echo "leases: r2s3_a r2s3_b r2s3_c r2s3_d r2s3_e r2s3_f r2s3_final r2s3_final2 r2s3_g r2s3_pmc"; fi
