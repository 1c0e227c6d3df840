# round 5, lease a: triad placement vs physical mapping (scripts/ubench/vmm.hip), 6 fresh processes
cd $GRAFT_REPO_ROOT
for i in 1 2 3 4 5 6; do
  echo "== process $i" >> gpurun_out/r5a_vmm.log
  timeout -k 10 120 ./scripts/ubench/vmm 2 >> gpurun_out/r5a_vmm.log 2>&1 || exit $?
done
