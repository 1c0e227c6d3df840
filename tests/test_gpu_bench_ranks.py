"""bench.py's N > 1 path end to end, two processes on one MI355X: the
partitioned step (segmented triad / transform_reduce / inclusive_scan with
the all-gathered carries), the max-over-ranks clock, the self-checks, and
the multi-GPU extras (segmented sort, partitioned 1d_stencil).  The
collectives run over the host-staged gloo double of TorchComm
(tests/staged_comm.py); the per-partition kernels are the product's."""
import contextlib
import io
import json
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _worker(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        import hpx_amd as hpx
        from staged_comm import HostStagedComm
        import bench
        tgt = hpx.target(0)
        comm = HostStagedComm(tgt)
        out = io.StringIO()
        with contextlib.redirect_stdout(out):
            bench.main(["--gpus", str(size), "--steps", "2", "--warmup", "1", "--logn", "22", "--no-cpu",
                        "--no-pmc", "--stencil-logn", "22", "--stencil-steps", "40"], comm_tgt=(comm, tgt))
        q.put((rank, out.getvalue()))
    except Exception as e:
        q.put((rank, e))
        raise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_one_json_line(gpu_target):
    import torch.multiprocessing as mp
    size = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=110) for _ in range(size))
    for p in procs:
        p.join(timeout=30)
    for r in range(size):
        assert not isinstance(res[r], Exception), res[r]
    lines = [ln for ln in res[0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and res[1].strip() == ""
    d = json.loads(lines[0])
    assert d["ranks"] == 2 and [r[0] for r in d["rank_devices"]] == [0, 1]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["global_elements"] == 2 * (1 << 22)
    x = d["extras"]
    assert x["segmented_sort_uint64"]["sorted_and_ordered"] is True
    assert x["stencil_heat_dist"]["window_check_bit_exact"] is True and x["stencil_heat_dist"]["points"] == 1 << 22
    r = x["segmented_reduce_int64"]
    assert r["ranks"] == 2 and r["gbs_per_rank"] > 0
