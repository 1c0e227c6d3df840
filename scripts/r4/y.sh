# round 4, lease y: bench's N > 1 path rehearsed on one GPU -- one rank under torchrun, RCCL group through TorchComm
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
HPXHIP_RCCL_SELF=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4y_bench_rccl_self.log 2>&1 || exit $?
