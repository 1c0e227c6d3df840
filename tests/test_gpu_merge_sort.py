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
from hpx_amd.compute import dtype_code
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


def _merge_runs(gpu_target, runs, dt, desc, lead=0):
    """hpxhip_merge_runs over the runs laid back to back after `lead` keys."""
    src = np.concatenate([np.zeros(lead, dt)] + [np.asarray(r, dt) for r in runs])
    offsets = [lead] + list(lead + np.cumsum([len(r) for r in runs]))
    eng = S.HipEngine(gpu_target)
    d = hpx.vector.from_host(src if src.size else np.zeros(1, dt), gpu_target)
    out = hpx.vector(max(1, offsets[-1] - lead + 1), dtype=dt, tgt=gpu_target)
    eng.merge_runs(dtype_code(dt), d, 0, offsets, out, 1, desc)
    gpu_target.synchronize()
    return out.to_host()[1:1 + offsets[-1] - lead]


@pytest.mark.parametrize("p", [2, 3, 5, 8])
@pytest.mark.parametrize("dt", [np.uint64, np.int32, np.float64])
def test_merge_runs_bit_exact(gpu_target, p, dt):
    """The segmented sort's one-pass merge of p <= 8 sorted runs
    (hpxhip_merge_runs): ragged and empty runs, keys with heavy repeats
    (the copied equal-key blocks), against the oracle sort of the union."""
    rng = np.random.default_rng(p)
    for shape in ("random", "repeats", "empty_runs"):
        lens = rng.integers(0, 300000, p)
        if shape == "empty_runs":
            lens[::2] = 0
        runs = []
        for j, n in enumerate(lens):
            if shape == "repeats":
                x = rnd(dt, int(n), 10 + j, 0, 40) if np.dtype(dt).kind != "f" else np.round(rnd(dt, int(n), 10 + j), 1)
            else:
                x = rnd(dt, int(n), 10 + j)
            runs.append(O.sort(np.asarray(x, dt)))
        for desc in (False, True):
            rs = [O.sort(r, desc) for r in runs]
            got = _merge_runs(gpu_target, rs, dt, desc, lead=3)
            np.testing.assert_array_equal(bits(got), bits(O.sort(np.concatenate(rs), desc)),
                                          err_msg=f"{shape} desc={desc}")


def merge_runs_with(lib_path, gpu_target, runs, dt, desc, lead=3):
    """hpxhip_merge_runs of another build of the library (a variant under
    hpx_amd/variants/, loaded RTLD_LOCAL beside the shipped one), on buffers
    and the stream of the shipped library."""
    import ctypes
    import os
    lib = ctypes.CDLL(lib_path, mode=os.RTLD_LOCAL)
    fn = lib.hpxhip_merge_runs
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    src = np.concatenate([np.zeros(lead, dt)] + [np.asarray(r, dt) for r in runs])
    offsets = [lead] + list(lead + np.cumsum([len(r) for r in runs]))
    d = hpx.vector.from_host(src if src.size else np.zeros(1, dt), gpu_target)
    out = hpx.vector(max(1, offsets[-1] - lead + 1), dtype=dt, tgt=gpu_target)
    offs = (ctypes.c_uint64 * len(offsets))(*[int(o) for o in offsets])
    it = np.dtype(dt).itemsize
    rc = fn(dtype_code(dt), d.data(), offs, len(offsets) - 1, out.data() + it, 1 if desc else 0,
            gpu_target.stream, None, 0)
    assert rc == 0, f"{lib_path}: hpxhip_merge_runs returned {rc}"
    gpu_target.synchronize()
    return out.to_host()[1:1 + offsets[-1] - lead]


VARIANTS = ["mw512", "mwminw4"]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("dt", [np.uint64, np.int32, np.float64])
def test_merge_runs_variant_builds(gpu_target, variant, dt):
    """the multiway merge built with 512-thread tasks and at the
    default occupancy bound (Makefile mw-variants) stays bit-exact beside
    the shipped 256-thread, 8-waves-per-SIMD build -- float64 included, the
    dtype an earlier form was miscompiled for.  The shapes of
    test_merge_runs_bit_exact, the failing one of lease r5/ad first."""
    import os
    path = os.path.join(os.path.dirname(hpx.__file__), "variants", variant, "libhpxhip.so")
    assert os.path.exists(path), f"{path} missing: build() builds it (make mw-variants)"
    for p in (2, 3, 8):
        rng = np.random.default_rng(p)
        lens = rng.integers(0, 300000, p)
        runs = [O.sort(np.asarray(rnd(dt, int(n), 10 + j), dt)) for j, n in enumerate(lens)]
        for desc in (False, True):
            rs = [O.sort(r, desc) for r in runs]
            got = merge_runs_with(path, gpu_target, rs, dt, desc)
            np.testing.assert_array_equal(bits(got), bits(O.sort(np.concatenate(rs), desc)),
                                          err_msg=f"{variant} p={p} desc={desc}")


@pytest.mark.parametrize("case", ["all_equal", "two_values", "one_long_run", "tiny"])
def test_merge_runs_edge_cases(gpu_target, case):
    """All keys equal (one task copies them), two values, one run holding
    nearly everything, and runs shorter than a sample stride."""
    dt = np.int64
    rng = np.random.default_rng(7)
    if case == "all_equal":
        # (repeated splitters: only the last task with the value copies them)
        runs = [np.full(n, 5, dt) for n in (70000, 3, 50000, 1, 120000, 0, 9, 40000)]
    elif case == "two_values":
        runs = [O.sort(rng.integers(0, 2, n).astype(dt)) for n in (80000, 60000, 1, 99999, 5)]
    elif case == "one_long_run":
        runs = [O.sort(rnd(dt, 1 << 21, 8))] + [O.sort(rnd(dt, 3, 9 + j)) for j in range(6)]
    else:
        runs = [O.sort(rnd(dt, n, 20 + n)) for n in (1, 2, 0, 7, 1, 0, 3, 1)]
    for desc in (False, True):
        rs = [O.sort(r, desc) for r in runs]
        got = _merge_runs(gpu_target, rs, dt, desc)
        np.testing.assert_array_equal(got, O.sort(np.concatenate(rs), desc), err_msg=f"{case} desc={desc}")


def test_merge_runs_2p30_eight_runs(gpu_target):
    """The 8-GPU sort's merge at full size: 2^30 u64 keys in 8 runs (the
    all-to-all's slices), generated and checked on the device (torch: the
    runs are the sorted columns of a permutation-closed form; the merged
    array must be 0, 1, ..., n-1, element for element)."""
    import torch
    dev = torch.device("cuda", gpu_target.device)
    n, p = 1 << 30, 8
    # run j = sorted keys (i << 3 | j) for i < n/p: merged = 0 .. n-1 in order
    m = n // p
    src = hpx.vector(n, dtype=np.uint64, tgt=gpu_target)
    out = hpx.vector(n, dtype=np.uint64, tgt=gpu_target)
    import ctypes
    for j in range(p):
        t = (torch.arange(m, dtype=torch.int64, device=dev) << 3) | j
        torch.cuda.synchronize(dev)
        L.call("hpxhip_memcpy_async", ctypes.c_void_p(src.data() + j * m * 8), ctypes.c_void_p(t.data_ptr()), m * 8,
               L.D2D, gpu_target.stream)
        gpu_target.synchronize()
        del t
    eng = S.HipEngine(gpu_target)
    eng.merge_runs(L.U64, src, 0, [j * m for j in range(p + 1)], out, 0, False)
    gpu_target.synchronize()
    chunk = 1 << 26
    got = torch.empty(chunk, dtype=torch.int64, device=dev)
    for lo in range(0, n, chunk):
        L.call("hpxhip_memcpy_async", ctypes.c_void_p(got.data_ptr()), ctypes.c_void_p(out.data() + lo * 8), chunk * 8,
               L.D2D, gpu_target.stream)
        gpu_target.synchronize()
        exp = torch.arange(lo, lo + chunk, dtype=torch.int64, device=dev)
        assert int((got != exp).sum()) == 0, lo
    src.free()
    out.free()


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
