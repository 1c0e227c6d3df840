# round 5, lease ab: pipelined copy_if write-out with 128-B aligned vectors -- timing, and the
# WRITE_SIZE of both forms (the 16-B form wrote 1.02x its bytes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 240 ./scripts/ubench/copyif9 > gpurun_out/r5ab_copyif9.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5ab_pmc_write -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5ab_pmc_write.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_copy_if_pipe --output-format csv -d gpurun_out/r5ab_pmc_fetch -o run -- ./scripts/ubench/copyif9 quick > gpurun_out/r5ab_pmc_fetch.log 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/r5ab_pmc_fetch gpurun_out/r5ab_pmc_write > gpurun_out/r5ab_pmc.txt 2>&1
