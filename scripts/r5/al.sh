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
