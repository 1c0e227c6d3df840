# round 4, lease l: copy_if phase split + PMC traffic of the shipped kernel
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 scripts/r4/lb/copyif8 > gpurun_out/r4l_copyif8.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_copy_if --output-format csv -d gpurun_out/r4l_pmc_fetch -o run -- scripts/r4/lb/copyif8 only > gpurun_out/r4l_pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_copy_if --output-format csv -d gpurun_out/r4l_pmc_write -o run -- scripts/r4/lb/copyif8 only > gpurun_out/r4l_pmc_write.log 2>&1 || exit $?
