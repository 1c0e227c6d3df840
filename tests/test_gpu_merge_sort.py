"""GPU parity of hpx::parallel::merge (merge.hpp:476, stable: first range
first on ties, merge.hpp:52-80) and of the sorted-range searches behind the
segmented sort, against the oracle; the single-rank segmented sort on the
device; and the RCCL all-to-all / all-gather wrappers of TorchComm on a
one-rank process group (device memory of the library wrapped without a
copy)."""
import numpy as np
import pytest

import hpx_amd as hpx
from hpx_amd import _lib as L
from hpx_amd import execution as ex, functional as F
from hpx_amd import parallel as P
from hpx_amd import segmented as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DTS = [np.int32, np.uint32, np.int64, np.uint64, np.float32, np.float64]


@pytest.fixture(scope="module")
def pol(gpu_target):
    return ex.par.on(hpx.default_executor(gpu_target))


def rnd(dt, n, seed, lo=None, hi=None):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dt)
    if dt.kind == "f":
        x = rng.standard_normal(n).astype(dt)
        if n > 40:
            x[::13] = 0.0
            x[::11] = -0.0
        return x
    info = np.iinfo(dt)
    lo = info.min if lo is None else lo
    hi = info.max if hi is None else hi
    return rng.integers(lo, hi, n, dtype=dt, endpoint=True)


def bits(x):
    return np.ascontiguousarray(x).view(np.uint8)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("n1,n2", [(0, 0), (0, 5), (7, 0), (1, 1), (2047, 1), (2048, 2048), (3000, 77),
                                   (100003, 65537), (1 << 20, (1 << 20) + 3)])
def test_merge_bit_exact(pol, gpu_target, dt, n1, n2):
    a = O.sort(rnd(dt, n1, 1))
    b = O.sort(rnd(dt, n2, 2))
    da, db = hpx.vector.from_host(a, gpu_target), hpx.vector.from_host(b, gpu_target)
    out = hpx.vector(n1 + n2, dtype=dt, tgt=gpu_target)
    r = P.merge(pol, da.begin(), da.end(), db.begin(), db.end(), out.begin())
    assert r[2] == out.begin() + (n1 + n2)
    np.testing.assert_array_equal(bits(out.to_host()), bits(O.merge(a, b)))


@pytest.mark.parametrize("dt", [np.int64, np.uint32, np.float64])
def test_merge_descending_ties_and_misaligned(pol, gpu_target, dt):
    # heavy ties: stability (first range first) is visible through -0.0/+0.0
    # for floats and is the only order for equal integers
    for desc in (False, True):
        comp = F.greater if desc else F.less
        a = O.sort(rnd(dt, 5003, 3, 0, 9) if np.dtype(dt).kind != "f" else np.tile([0.0, -0.0, 1.0], 1700), desc)
        b = O.sort(rnd(dt, 4001, 4, 0, 9) if np.dtype(dt).kind != "f" else np.tile([-0.0, 0.0, 2.0], 1300), desc)
        a, b = a.astype(dt), b.astype(dt)
        base = np.concatenate([np.zeros(3, dt), a, np.zeros(1, dt), b])
        d = hpx.vector.from_host(base, gpu_target)
        out = hpx.vector(a.size + b.size + 1, dtype=dt, tgt=gpu_target)
        a0, b0 = 3, 3 + a.size + 1
        P.merge(pol, d.begin() + a0, d.begin() + a0 + a.size, d.begin() + b0, d.begin() + b0 + b.size,
                out.begin() + 1, comp)
        np.testing.assert_array_equal(bits(out.to_host()[1:]), bits(O.merge(a, b, desc)))


@pytest.mark.parametrize("dt", [np.int64, np.float64, np.uint32])
def test_sorted_bounds(gpu_target, dt):
    x = O.sort(rnd(dt, 100003, 5, 0, 1000) if np.dtype(dt).kind != "f" else rnd(dt, 100003, 5))
    eng = S.HipEngine(gpu_target)
    v = hpx.vector.from_host(x, gpu_target)
    probes = np.concatenate([x[::997], rnd(dt, 300, 6, 0, 1000) if np.dtype(dt).kind != "f" else rnd(dt, 300, 6)])
    lo = eng.bounds(v, 0, x.size, probes, False, False)
    hi = eng.bounds(v, 0, x.size, probes, True, False)
    if np.dtype(dt).kind == "f":
        # IEEE total order: compare through the ordered bit patterns
        from test_segmented_sort_gloo import _ordered
        xs, ps = _ordered(x, False), _ordered(probes.astype(dt), False)
    else:
        xs, ps = x, probes.astype(dt)
    np.testing.assert_array_equal(lo, np.searchsorted(xs, ps, "left"))
    np.testing.assert_array_equal(hi, np.searchsorted(xs, ps, "right"))
    # sub-range
    lo2 = eng.bounds(v, 1000, 50000, probes, False, False)
    np.testing.assert_array_equal(lo2, np.searchsorted(xs[1000:50000], ps, "left"))


def test_segmented_sort_single_rank(gpu_target):
    pol = ex.par.on(hpx.default_executor(gpu_target))
    x = O.generate(np.uint64, "bits", 1 << 20, 11)
    pv = S.partitioned_vector(x.size, np.uint64, tgt=gpu_target)
    S.algorithms.generate(pol, pv.begin(), pv.end(), "bits", 11)
    S.algorithms.sort(pol, pv.begin(), pv.end())
    np.testing.assert_array_equal(pv.local.to_host(), O.sort(x))


def test_torchcomm_alltoallv_and_allgather_one_rank(gpu_target):
    """The RCCL wrappers on a one-rank group: all_to_all_single over library
    device memory (no copy) and the host all-gather."""
    import os
    import torch
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group already exists")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(gpu_target.device)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", gpu_target.device))
    try:
        comm = S.TorchComm(gpu_target)
        g = comm.allgather_host(np.array([3, -4, 5], np.int64))
        np.testing.assert_array_equal(g, [[3, -4, 5]])
        x = np.arange(1000, dtype=np.int64) * 7
        src = hpx.vector.from_host(x, gpu_target)
        dst = hpx.vector(990, dtype=np.int64, tgt=gpu_target)
        comm.alltoallv(src, 10, [990], dst, [990], 8, gpu_target.stream)
        gpu_target.synchronize()
        np.testing.assert_array_equal(dst.to_host(), x[10:])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nx,nt,kind", [(100003, 12, "random"), (1 << 20, 5, "ramp"), (5, 9, "random"),
                                        (4, 3, "random")])
def test_heat_solver_one_partition(gpu_target, nx, nt, kind):
    """segmented.heat_solver (edge / exchange / interior split, side-stream
    halo ring) on one rank == the serial 1d_stencil oracle, bit for bit."""
    init = None if kind == "ramp" else np.random.default_rng(nx).standard_normal(nx)
    hs = S.heat_solver(nx, S.LocalComm(gpu_target), gpu_target, init=init)
    out = hs.do_work(nt)
    hs.synchronize()
    u0 = np.arange(nx, dtype=np.float64) if init is None else init
    np.testing.assert_array_equal(out.to_host(), O.stencil_heat(u0, nt))


def test_heat_solver_checkpoint_restart(gpu_target, tmp_path):
    """1d_stencil_4_checkpoint: save at step 5, revive into a fresh solver,
    continue -- equals the uninterrupted run bit for bit."""
    nx = (1 << 18) + 5
    init = np.random.default_rng(3).standard_normal(nx)
    hs = S.heat_solver(nx, S.LocalComm(gpu_target), gpu_target, init=init)
    hs.do_work(5)
    hs.save_checkpoint(str(tmp_path / "heat"))
    hs2 = S.heat_solver(nx, S.LocalComm(gpu_target), gpu_target)
    assert hs2.restore_checkpoint(str(tmp_path / "heat")) == 5
    out = hs2.do_work(6)
    hs2.synchronize()
    np.testing.assert_array_equal(out.to_host(), O.stencil_heat(init, 11))
