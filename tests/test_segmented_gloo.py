"""Multi-rank orchestration of the segmented algorithms on CPU (gloo,
world sizes 2 and 3): partition bounds, segment-order folds of the RCCL
all-gathered totals, scan carries, copy_if offsets and the stencil halo ring.

The per-partition kernels are replaced by a numpy test engine *in this test
only* (the product engine is HipEngine, exercised by tests/test_gpu_*.py);
the code under test is hpx_amd.segmented's orchestration and the product's
TorchComm collective sequence (all_gather_into_tensor, uneven
all_to_all_single into views) run over host buffers on gloo."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from hpx_amd import functional as F  # noqa: E402
from hpx_amd import segmented as S  # noqa: E402

OPS = {0: np.add, 1: np.multiply, 2: np.minimum, 3: np.maximum, 4: np.bitwise_and, 5: np.bitwise_or, 6: np.bitwise_xor}


class NumpyEngine:
    """Test double of HipEngine: same calls, numpy arithmetic, values held
    as 8-byte words like the device slots."""
    stream = None

    def _w2v(self, words, dt):
        return np.asarray(words, np.int64).view(dt)

    def reduce_into(self, vec, lo, hi, op, conv, acc_dt, out):
        dt = np.dtype(vec.dtype)
        x = [dt.type(conv(v)) for v in vec[lo:hi].astype(dt)]
        ident = S._identity(op.kind, {np.dtype(np.int64): 2, np.dtype(np.float64): 5}[dt])
        r = np.array([ident], dt)[0]
        for v in x:
            r = OPS[op.kind](r, v)
        out[0] = np.array([r], dt).view(np.int64)[0]

    def fold(self, dt_code, op, init, values, count, out):
        dt = {2: np.int64, 5: np.float64}[dt_code]
        acc = np.array([init], dt)[0]
        for v in self._w2v(values[:count], dt):
            acc = OPS[op.kind](acc, v)
        out[0] = np.array([acc], dt).view(np.int64)[0]

    def scratch(self):
        return np.zeros(1, np.int64)

    def read(self, h, dt_code):
        return self._w2v(h[:1], {2: np.int64, 5: np.float64}[dt_code])[0]

    def scan(self, src, lo, hi, dst, dlo, op, conv, inclusive, carry):
        dt = src.dtype
        acc = self._w2v(carry[:1], dt)[0]
        for i in range(lo, hi):
            nxt = OPS[op.kind](acc, dt.type(conv(src[i])))
            dst[dlo + i - lo] = nxt if inclusive else acc
            acc = nxt

    def copy_if(self, src, lo, hi, dst, dlo, pred, count):
        sel = [v for v in src[lo:hi] if pred(v)]
        dst[dlo:dlo + len(sel)] = sel
        count[0] = len(sel)

    def read_words(self, h, count, dt):
        return list(h[:count])

    def word(self, arr, i, size=8):
        return arr[i:]

    def transform(self, pol, pv, lo, hi, dst, dlo, f):
        dst[dlo:dlo + hi - lo] = [f(v) for v in pv.local[lo:hi]]

    def put(self, slot, dt_code, value):
        dt = {2: np.int64, 5: np.float64}[dt_code]
        slot[0] = np.array([value], dt).view(np.int64)[0]

    def buffer(self, like, n):
        return np.zeros(max(1, n), like.dtype)

    def release(self, buf):
        pass


class HostPV(S.partitioned_vector):
    def __init__(self, glob, comm, layout=None):
        self.comm = comm
        self.tgt = None
        self.n = glob.size
        self.dtype = {np.dtype(np.int64): 2, np.dtype(np.float64): 5}[glob.dtype]
        self._set_layout(layout)
        self.local = glob[self.lo:self.hi].copy()


def _gather(results, key, n, dtype=np.int64):
    got = np.zeros(n, dtype)
    for r in results:
        lo, loc = results[r][key]
        got[lo:lo + loc.size] = loc
    return got


def _layout_worker(rank, size, port, q):
    """partitioned_vector_inclusive_scan.cpp:321-340 and
    partitioned_vector_reduce.cpp:47-76 restated: container_layout,
    container_layout(3), (1000), (10), and scans whose output has another
    layout than the input."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        comm = S.TorchComm(None, memory="host")  # the product comm over host buffers
        alg = S.segmented(NumpyEngine())
        CL = S.container_layout
        res = {}
        n = 10007
        ones = np.ones(n, np.int64)
        x = O.generate(np.int64, "range", n, 0x5EED, -1000, 1000)
        xf = O.generate(np.float64, "unit", n, 0x5EED)
        for name, lay in (("default", CL), ("3", CL(3)), ("8", CL(8)), ("10", CL(10)), ("13", CL(13)),
                          ("1000", CL(1000)), ("1", CL(1))):
            pv = HostPV(ones, comm, lay)
            res[("reduce_ones", name)] = alg.reduce(None, pv.begin(), pv.end(), 1, F.plus)
            pf = HostPV(xf, comm, lay)
            res[("reduce_f64", name)] = alg.reduce(None, pf.begin(), pf.end(), 0.5, F.plus)
            pi = HostPV(x, comm, lay)
            out = HostPV(np.zeros(n, np.int64), comm, lay)
            alg.inclusive_scan(None, pi.begin(), pi.end(), out.begin(), F.plus, 3)
            res[("incl", name)] = (out.lo, out.local.copy())
            alg.exclusive_scan(None, pi.begin() + 17, pi.end() - 5, out.begin() + 17, 2)
            res[("excl_sub", name)] = (out.lo, out.local.copy())
            res[("parts", name)] = (pi.get_num_partitions(), pi.my_segments())
            # transform_exclusive_scan (segmented_algorithms/transform_exclusive_scan.hpp:31)
            alg.transform_exclusive_scan(None, pi.begin(), pi.end(), out.begin(), -4, F.plus, F.multiply_step(3))
            res[("texcl", name)] = (out.lo, out.local.copy())
            fo = HostPV(np.zeros(n, np.float64), comm, lay)
            alg.inclusive_scan(None, pf.begin(), pf.end(), fo.begin(), F.plus, 0.25)
            res[("incl_f64", name)] = (fo.lo, fo.local.copy())
        # segmented output layouts (inclusive_scan_tests_segmented_out_with_policy)
        for name, lin, lout in (("loc->3", CL, CL(3)), ("loc->10", CL, CL(10)), ("7->loc", CL(7), CL),
                                ("3->1", CL(3), CL(1))):
            pi = HostPV(x, comm, lin)
            out = HostPV(np.zeros(n, np.int64), comm, lout)
            alg.inclusive_scan(None, pi.begin(), pi.end(), out.begin(), F.plus, 0)
            res[("mixed", name)] = (out.lo, out.local.copy())
            out2 = HostPV(np.zeros(n, np.int64), comm, lout)
            alg.transform(None, pi.begin(), pi.end(), out2.begin(), F.add_value(5))
            res[("mixed_transform", name)] = (out2.lo, out2.local.copy())
            # shifted destination: out[100 + i] = scan(x[0 .. i]) over x[0, n-100)
            out3 = HostPV(np.zeros(n, np.int64), comm, lout)
            alg.inclusive_scan(None, pi.begin(), pi.end() - 100, out3.begin() + 100, F.plus, 0)
            res[("shifted", name)] = (out3.lo, out3.local.copy())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _worker(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        comm = S.TorchComm(None, memory="host")  # the product comm over host buffers
        alg = S.segmented(NumpyEngine())
        res = {}
        n = 10007
        x = O.generate(np.int64, "range", n, 0x5EED, -1000, 1000)
        pv = HostPV(x, comm)
        # partitioned_vector_reduce.cpp: ones + init 1 == n + 1
        ones = HostPV(np.ones(n, np.int64), comm)
        res["reduce_ones"] = alg.reduce(None, ones.begin(), ones.end(), 1, F.plus)
        res["reduce"] = alg.reduce(None, pv.begin(), pv.end(), 7, F.plus)
        res["reduce_max"] = alg.reduce(None, pv, None, -(1 << 62), F.maximum)
        out = HostPV(np.zeros(n, np.int64), comm)
        alg.inclusive_scan(None, pv.begin(), pv.end(), out.begin(), F.plus, 5)
        res["incl"] = (out.lo, out.local.copy())
        alg.exclusive_scan(None, pv.begin(), pv.end(), out.begin(), 5)
        res["excl"] = (out.lo, out.local.copy())
        # sub-range scan
        alg.inclusive_scan(None, pv.begin() + 1234, pv.end() - 77, out.begin() + 1234, F.plus, 0)
        res["sub"] = (out.lo, out.local.copy())
        dst = HostPV(np.zeros(n, np.int64), comm)
        total, off, cnt = alg.copy_if(None, pv.begin(), pv.end(), dst, F.not_less_than(0))
        res["copy_if"] = (total, off, dst.local[:cnt].copy())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("size", [2, 3, 8])
def test_segmented_algorithms_gloo(size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(size))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 10007
    x = O.generate(np.int64, "range", n, 0x5EED, -1000, 1000)
    for r in range(size):
        res = results[r]
        assert res["reduce_ones"] == n + 1
        assert res["reduce"] == O.segmented_reduce(x, 7, size) == 7 + int(x.sum())
        assert res["reduce_max"] == x.max()
    incl = O.segmented_scan(x, 5, size, True)
    excl = O.segmented_scan(x, 5, size, False)
    sub = np.zeros(n, np.int64)
    sub[1234:n - 77] = np.cumsum(x[1234:n - 77])
    for key, exp in (("incl", incl), ("excl", excl)):
        got = np.zeros(n, np.int64)
        for r in range(size):
            lo, loc = results[r][key]
            got[lo:lo + loc.size] = loc
        np.testing.assert_array_equal(got, exp)
    got = np.zeros(n, np.int64)
    for r in range(size):
        lo, loc = results[r]["sub"]
        got[lo:lo + loc.size] = loc
    np.testing.assert_array_equal(got[1234:n - 77], sub[1234:n - 77])
    sel = O.copy_if(x, "not_less_than", 0)
    parts = sorted((results[r]["copy_if"][1], results[r]["copy_if"][2]) for r in range(size))
    assert all(results[r]["copy_if"][0] == sel.size for r in range(size))
    np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), sel)


@pytest.mark.parametrize("size", [2, 3, 8])
def test_partitioned_vector_layouts_gloo(size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(size))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 10007
    x = O.generate(np.int64, "range", n, 0x5EED, -1000, 1000)
    xf = O.generate(np.float64, "unit", n, 0x5EED)
    for name, k in (("default", size), ("3", 3), ("8", 8), ("10", 10), ("13", 13), ("1000", 1000), ("1", 1)):
        for r in range(size):
            assert results[r][("reduce_ones", name)] == n + 1
            # FP: the segment-order fold of the reference (init (+) S_0 (+) ... over k segments)
            assert results[r][("reduce_f64", name)] == O.segmented_reduce(xf, 0.5, k)
            nparts, (j0, j1) = results[r][("parts", name)]
            assert nparts == k and (j0, j1) == S.rank_partitions(k, size, r)
        np.testing.assert_array_equal(_gather(results, ("incl", name), n), O.segmented_scan(x, 3, k, True))
        sub = _gather(results, ("excl_sub", name), n)
        exp = np.concatenate([[2], 2 + np.cumsum(x[17:n - 5])[:-1]])
        np.testing.assert_array_equal(sub[17:n - 5], exp)
        np.testing.assert_array_equal(_gather(results, ("incl_f64", name), n, np.float64),
                                      O.segmented_scan(xf, 0.25, k, True))
        # transform_exclusive_scan(init -4, plus, x -> 3x): exact for integers
        np.testing.assert_array_equal(_gather(results, ("texcl", name), n),
                                      np.concatenate([[-4], -4 + np.cumsum(3 * x)[:-1]]))
    for name in ("loc->3", "loc->10", "7->loc", "3->1"):
        np.testing.assert_array_equal(_gather(results, ("mixed", name), n), np.cumsum(x))
        np.testing.assert_array_equal(_gather(results, ("mixed_transform", name), n), x + 5)
        got = _gather(results, ("shifted", name), n)
        np.testing.assert_array_equal(got[100:], np.cumsum(x[:n - 100]))


def test_layout_maps():
    # partitioned_vector_impl.hpp:325 partition sizes; contiguous partition runs per rank
    for n, k, p in [(10007, 3, 2), (10007, 10, 3), (1000, 1000, 3), (10, 4, 3), (5, 8, 3), (0, 3, 2)]:
        m = S.layout_map(n, k, p)
        runs = [m.rank_segments(r) for r in range(p)]
        assert runs[0][0] == 0 and runs[-1][1] == k and all(a1 == b0 for (_, a1), (b0, _) in zip(runs, runs[1:]))
        bounds = [m.rank_bounds(r) for r in range(p)]
        assert bounds[0][0] == 0 and bounds[-1][1] == n
        assert all(a1 == b0 for (_, a1), (b0, _) in zip(bounds, bounds[1:]))
        for r in range(p):
            j0, j1 = runs[r]
            if j1 > j0:
                assert bounds[r] == (m.segment_bounds(j0)[0], m.segment_bounds(j1 - 1)[1])
    with pytest.raises(ValueError):
        S.container_layout(0)


def test_partition_bounds_match_reference_layout():
    # partitioned_vector_impl.hpp:325: ceil(n/parts) per partition, last shorter
    for n, p in [(10007, 2), (10007, 3), (10, 4), (3, 8), (0, 2), (2 ** 32, 8)]:
        b = [S.partition_bounds(n, p, k) for k in range(p)]
        assert b[0][0] == 0 and b[-1][1] == n
        for (a0, a1), (b0, b1) in zip(b, b[1:]):
            assert a1 == b0
        part = -(-n // p)
        assert all(e - s <= part for s, e in b)
