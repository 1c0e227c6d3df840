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
