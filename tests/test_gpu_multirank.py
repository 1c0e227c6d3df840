"""Two and four ranks on the GPU: the product engine (HipEngine: radix sort, sorted-
range searches, merge, heat steps, reduce/scan/fold kernels) driven by the
multi-rank orchestration of hpx_amd.segmented, with both processes on
cuda:0.  RCCL refuses two ranks on one device, so the collectives here go
through a host-staged gloo test double (device -> host -> gloo -> device);
TorchComm's RCCL calls themselves run the same body on a one-rank RCCL
group (and tests/test_gpu_merge_sort.py's wrapper test).  Results are
checked against the oracle."""
import ctypes
import os
import socket

import numpy as np
import pytest

from staged_comm import HostStagedComm

pytestmark = pytest.mark.gpu


def _worker(rank, size, port, q, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    if backend == "nccl":  # one rank: the product's TorchComm over RCCL
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=size, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        import hpx_amd as hpx
        from hpx_amd import execution as ex, functional as F
        from hpx_amd import segmented as S
        tgt = hpx.target(0)
        pol = ex.par.on(hpx.default_executor(tgt))
        comm = S.TorchComm(tgt) if backend == "nccl" else HostStagedComm(tgt)
        alg = S.segmented()
        res = {}
        n = (1 << 20) + 12345
        for dt, kind in ((np.uint64, "bits"), (np.int64, "range")):
            pv = S.partitioned_vector(n, dt, comm=comm, tgt=tgt)
            alg.generate(pol, pv.begin(), pv.end(), kind, 99, -50, 50)
            for desc in (False, True):
                alg.sort(pol, pv.begin(), pv.end(), F.greater if desc else F.less)
                tgt.synchronize()
                res[("sort", np.dtype(dt).name, desc)] = (pv.lo, pv.local.to_host())
        x = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt)
        alg.generate(pol, x.begin(), x.end(), "range", 0x5EED, -1000, 1000)
        res["reduce"] = alg.reduce(pol, x.begin(), x.end(), 3, F.plus)
        y = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt)
        alg.inclusive_scan(pol, x.begin(), x.end(), y.begin(), F.plus, 3)
        tgt.synchronize()
        res["scan"] = (y.lo, y.local.to_host())
        # container_layout(5) over the two ranks, scan into a container_layout output
        CL = S.container_layout
        x5 = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt, layout=CL(5))
        alg.generate(pol, x5.begin(), x5.end(), "range", 0x5EED, -1000, 1000)
        res["reduce5"] = alg.reduce(pol, x5.begin(), x5.end(), 3, F.plus)
        y2 = S.partitioned_vector(n, np.int64, comm=comm, tgt=tgt, layout=CL)
        alg.inclusive_scan(pol, x5.begin(), x5.end(), y2.begin(), F.plus, 3)
        tgt.synchronize()
        res["scan5"] = (y2.lo, y2.local.to_host())
        for nx, nt in ((1 << 20, 6), (1001, 9)):
            init = np.random.default_rng(nx).standard_normal(nx)
            hs = S.heat_solver(nx, comm, tgt, init=init)
            out = hs.do_work(nt)
            hs.synchronize()
            res[("heat", nx)] = (hs.lo, out.to_host())
        q.put((rank, res))
    except Exception as e:  # report to the parent
        q.put((rank, e))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("size,backend", [(2, "gloo"), (4, "gloo"), (1, "nccl")])
def test_ranks_on_gpu_segmented_sort_reduce_scan_stencil(gpu_target, size, backend):
    """size 2 and 4: processes sharing cuda:0, collectives host-staged over
    gloo (4 ranks: 3 sort cuts, 2 merge rounds, a 4-rank halo ring);
    size 1 over RCCL: the same orchestration through the product's
    TorchComm (RCCL all-gathers on device buffers, all_to_all_single into
    destination views, the halo ring's batch_isend_irecv to itself) -- the
    N > 1 code path of the 8-GPU run, on the one GPU this box has."""
    import torch.multiprocessing as mp
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q, backend)) for r in range(size)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(size))
    for p in procs:
        p.join(timeout=30)
    for r in range(size):
        assert not isinstance(results[r], Exception), results[r]
    n = (1 << 20) + 12345
    for dt, kind in ((np.uint64, "bits"), (np.int64, "range")):
        base = O.generate(dt, kind, n, 99, -50, 50)
        for desc in (False, True):
            got = np.concatenate([results[r][("sort", np.dtype(dt).name, desc)][1] for r in range(size)])
            np.testing.assert_array_equal(got, O.sort(base, desc))
    x = O.generate(np.int64, "range", n, 0x5EED, -1000, 1000)
    assert all(results[r]["reduce"] == 3 + int(x.sum()) for r in range(size))
    got = np.concatenate([results[r]["scan"][1] for r in range(size)])
    np.testing.assert_array_equal(got, O.segmented_scan(x, 3, size, True))
    assert all(results[r]["reduce5"] == 3 + int(x.sum()) for r in range(size))
    got = np.concatenate([results[r]["scan5"][1] for r in range(size)])
    np.testing.assert_array_equal(got, O.segmented_scan(x, 3, 5, True))
    for nx, nt in ((1 << 20, 6), (1001, 9)):
        init = np.random.default_rng(nx).standard_normal(nx)
        got = np.concatenate([results[r][("heat", nx)][1] for r in range(size)])
        np.testing.assert_array_equal(got, O.stencil_heat(init, nt))
