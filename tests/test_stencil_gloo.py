"""examples/1d_stencil over a partitioned periodic ring on CPU (gloo, 1-4 and 8
ranks): the halo ring, the double-buffered halo slots and the edge /
exchange / interior ordering of hpx_amd.segmented.heat_solver, against the
serial oracle (1d_stencil_1.cpp:41-72).  Per-partition kernels are replaced
by the oracle's one-step restatement *in this test only*; the product engine
(HipEngine + hpxhip_stencil_heat_steps) is exercised on the GPU by
tests/test_gpu_parity.py and tests/test_gpu_merge_sort.py."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from hpx_amd import segmented as S  # noqa: E402


class OneRankComm:
    """A ring of one (the product's LocalComm does this on the device)."""
    rank, size = 0, 1

    def halo_exchange(self, send_left, send_right, recv_left, recv_right, stream, count=1):
        c = int(count)
        recv_left[:c] = send_right[:c]
        recv_right[:c] = send_left[:c]


class HeatEngine:
    stream = None

    def heat_buffers(self, n, offset, init=None):
        if isinstance(init, tuple):  # device-generated state (kind, seed) of the global sequence
            u0 = O.unit_at(np.arange(offset, offset + n, dtype=np.uint64), init[1])
        else:
            u0 = np.arange(offset, offset + n, dtype=np.float64) if init is None else np.array(init, np.float64)
        return [u0, np.zeros(n)]

    def halo_buffer(self):
        return np.zeros(4 * S.HALO_MAX)

    def loc(self, buf, idx):
        return buf[int(idx):]  # a view: the comm reads / writes through it

    def heat_steps(self, cur, nxt, n, lo, hi, left, right, steps, k, dt, dx, stream):
        """`steps` oracle single steps on [left halo | cur | right halo]; its
        inner points [steps + lo, steps + hi) are exact."""
        ext = np.concatenate([left[:steps], cur[:n], right[:steps]])
        for _ in range(steps):
            ext = O.stencil_heat_step(ext, 0.0, 0.0, k, dt, dx)
        nxt[lo:hi] = ext[steps + lo:steps + hi]

    def read_values(self, buf, n):
        return buf[:n].copy()

    def write_values(self, buf, vals):
        buf[:len(vals)] = vals

    def side_stream(self):
        return None

    def record(self, stream):
        return None

    def wait(self, stream, ev):
        pass

    def synchronize(self):
        pass


# (nx, nt, initial state, halo width cap: None = HALO_MAX fused steps per pass,
# 1 = one step per exchange as in 1d_stencil_8, 4 = four)
CASES = [(1001, 25, "ramp", None), (1001, 25, "random", None), (9, 7, "random", None), (64, 40, "random", None),
         (1001, 11, "random", 1), (1001, 13, "random", 4), (37, 9, "random", None), (1001, 30, "gen", None),
         # r05, for the 8-rank ring: 25-point partitions (W = 16 halos), and 17-point partitions whose last
         # one (11 points) is shorter than HALO_MAX (passes of <= 11 steps)
         (200, 40, "random", None), (130, 33, "random", None)]
GEN = ("unit", 0xC0FFEE)  # device-generated state: splitmix64(seed ^ global i) in [0, 1)


def _u0(nx, kind):
    if kind == "ramp":
        return np.arange(nx, dtype=np.float64)
    if kind == "gen":
        return O.unit_at(np.arange(nx, dtype=np.uint64), GEN[1])
    return np.random.default_rng(nx).standard_normal(nx)


def _worker(rank, size, port, q, ckdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        # ranks >= 2: the product's TorchComm (ring_halo_ops over batch_isend_irecv)
        comm = S.TorchComm(None, memory="host") if size > 1 else OneRankComm()
        res = {}
        for nx, nt, kind, fuse in CASES:
            init = {"ramp": None, "gen": GEN}[kind] if kind in ("ramp", "gen") else _u0(nx, kind)
            try:
                hs = S.heat_solver(nx, comm, engine=HeatEngine(), init=init, fuse=fuse)
            except ValueError:
                res[(nx, nt, kind, fuse)] = None   # empty partition: rejected on every rank
                continue
            out = hs.do_work(nt)
            res[(nx, nt, kind, fuse)] = (hs.lo, out.copy())
        # checkpoint after 7 steps, restart in a fresh solver, 9 more steps
        nx = 1001
        init = np.random.default_rng(5).standard_normal(nx)
        hs = S.heat_solver(nx, comm, engine=HeatEngine(), init=init)
        hs.do_work(7)
        hs.save_checkpoint(os.path.join(ckdir, "heat_7"))
        dist.barrier()
        hs2 = S.heat_solver(nx, comm, engine=HeatEngine())
        assert hs2.restore_checkpoint(os.path.join(ckdir, "heat_7")) == 7
        res["restart"] = (hs2.lo, hs2.do_work(9).copy())
        q.put((rank, res))
    except Exception as e:  # surface worker failures in the parent
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


@pytest.mark.parametrize("size", [1, 2, 3, 4, 8])
def test_heat_solver_ring_gloo(size, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q, str(tmp_path))) for r in range(size)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(size))
    for p in procs:
        p.join(timeout=60)
    for r in range(size):
        assert not isinstance(results[r], Exception), results[r]
    for case in CASES:
        nx, nt, kind, fuse = case
        exp = O.stencil_heat(_u0(nx, kind), nt)
        if results[0][case] is None:
            assert -(-nx // size) * (size - 1) >= nx
            continue
        got = np.zeros(nx)
        for r in range(size):
            lo, loc = results[r][case]
            got[lo:lo + loc.size] = loc
        np.testing.assert_array_equal(got, exp, err_msg=f"nx={nx} nt={nt} {kind} fuse={fuse} ranks={size}")
    # restart from the step-7 checkpoint == an uninterrupted 16-step run
    exp = O.stencil_heat(np.random.default_rng(5).standard_normal(1001), 16)
    got = np.zeros(1001)
    for r in range(size):
        lo, loc = results[r]["restart"]
        got[lo:lo + loc.size] = loc
    np.testing.assert_array_equal(got, exp)


def test_heat_solver_rejects_empty_partitions():
    class C:
        rank, size = 0, 8
    with pytest.raises(ValueError):
        S.heat_solver(9, C(), engine=HeatEngine())
