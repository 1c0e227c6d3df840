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
