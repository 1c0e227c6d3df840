"""Segmented sort across ranks on CPU (gloo, world sizes 2-4 and 8): the exact
global cut (radix select over ordered key bits + rank-order split of equal
keys), the uneven all-to-all and the pairwise merge rounds of
hpx_amd.segmented.segmented.sort.  The per-partition kernels are replaced by
the oracle (sort.hpp:364 std::sort, merge.hpp:52-80 sequential_merge) and
numpy searchsorted *in this test only*; the product engine is HipEngine
(tests/test_gpu_parity.py covers hpxhip_merge / hpxhip_sorted_bounds and the
single-rank path on the GPU)."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from hpx_amd import _lib as L  # noqa: E402
from hpx_amd import functional as F  # noqa: E402
from hpx_amd import segmented as S  # noqa: E402

CODES = {np.dtype(np.int64): L.I64, np.dtype(np.uint64): L.U64, np.dtype(np.float64): L.F64,
         np.dtype(np.int32): L.I32, np.dtype(np.uint32): L.U32, np.dtype(np.float32): L.F32}


def _ordered(x, desc):
    """Host restatement of the key order (common.hpp ordered_bits)."""
    it = x.dtype.itemsize
    ut = np.uint64 if it == 8 else np.uint32
    raw = x.view(ut)
    sign = ut(1) << ut(8 * it - 1)
    if x.dtype.kind == "f":
        o = np.where(raw & sign, ~raw, raw | sign).astype(ut)
    elif x.dtype.kind == "i":
        o = raw ^ sign
    else:
        o = raw.copy()
    return ~o if desc else o


class SortEngine:
    stream = None

    def sort(self, vec, lo, hi, desc):
        vec[lo:hi] = O.sort(vec[lo:hi], desc)

    def bounds(self, vec, lo, hi, values, upper, desc):
        keys = _ordered(vec[lo:hi], desc)
        v = _ordered(np.asarray(values, vec.dtype), desc)
        return np.searchsorted(keys, v, side="right" if upper else "left").astype(np.int64)

    def read_ranges(self, vec, starts, counts):
        return [vec[int(a):int(a) + int(c)].copy() for a, c in zip(starts, counts)]

    def buffer(self, like, n):
        return np.zeros(max(1, n), like.dtype)

    def merge(self, dt, a, a_off, na, b, b_off, nb, out, out_off, desc):
        out[out_off:out_off + na + nb] = O.merge(a[a_off:a_off + na], b[b_off:b_off + nb], desc)

    def copy(self, dt, src, s_off, n, dst, d_off):
        dst[d_off:d_off + n] = src[s_off:s_off + n]

    def release(self, buf):
        pass


class RunsEngine(SortEngine):
    """With the one-pass merge of up to 8 runs (hpxhip_merge_runs's role):
    the oracle's merge folded over the runs."""

    def merge_runs(self, dt, src, s_off, offsets, out, out_off, desc):
        acc = src[s_off + offsets[0]:s_off + offsets[0]]
        for a, b in zip(offsets[:-1], offsets[1:]):
            acc = O.merge(acc, src[s_off + a:s_off + b], desc)
        out[out_off:out_off + acc.size] = acc


class HostPV(S.partitioned_vector):
    def __init__(self, glob, comm, layout=None):
        self.comm = comm
        self.tgt = None
        self.n = glob.size
        self.dtype = CODES[glob.dtype]
        self._set_layout(layout)
        self.local = glob[self.lo:self.hi].copy()


def cases():
    rng = np.random.default_rng(0x5EED)
    f = rng.standard_normal(3001)
    f[::17] = 0.0
    f[::19] = -0.0
    f[5] = np.inf
    f[6] = -np.inf
    return {
        "i64_random": O.generate(np.int64, "range", 10007, 0x5EED, -1000, 1000),
        "u64_bits": O.generate(np.uint64, "bits", 4099, 7),
        "i64_dups": rng.integers(0, 3, 5000).astype(np.int64),
        "i64_const": np.full(777, 42, np.int64),
        "f64_signed_zeros": f,
        "u32": rng.integers(0, 2 ** 32, 3333, dtype=np.uint64).astype(np.uint32),
        "i32_small": np.array([5, -1, 3], np.int32),
        "f32": rng.standard_normal(2048).astype(np.float32),
        "empty": np.zeros(0, np.int64),
        # r05: 8-rank cases -- fewer keys than ranks, a few keys per rank,
        # uniform 64-bit keys (the 2-round-trip select), repeated wide keys
        # straddling the cuts (gathered blocks with equal keys)
        "i64_five": np.array([9, -3, 9, 0, -3], np.int64),
        "u64_thirteen": rng.integers(0, 2 ** 63, 13, dtype=np.uint64),
        "u64_uniform": O.generate(np.uint64, "bits", 200003, 11),
        "i64_wide_dups": np.repeat(rng.integers(-2 ** 62, 2 ** 62, 9000, dtype=np.int64), 3),
    }


class CountingComm:
    """The product comm, counting the host-level exchanges of the select."""
    def __init__(self, comm):
        self.comm = comm
        self.rounds = 0

    def __getattr__(self, name):
        return getattr(self.comm, name)

    def allreduce_host(self, words):
        self.rounds += 1
        return self.comm.allreduce_host(words)

    def allgather_host(self, words):
        self.rounds += 1
        return self.comm.allgather_host(words)


def _worker(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        comm = CountingComm(S.TorchComm(None, memory="host"))  # the product comm over host buffers
        res = {}
        # the shipped block size and one forcing more rounds, with the
        # one-pass run merge (p <= 8); the shipped block size with the
        # pairwise merge rounds (p > 8)
        for eng, gather in ((RunsEngine, S.segmented.SELECT_GATHER), (RunsEngine, 16),
                            (SortEngine, S.segmented.SELECT_GATHER)):
            alg = S.segmented(eng())
            alg.SELECT_GATHER = gather
            for name, x in cases().items():
                for desc in (False, True):
                    pv = HostPV(x, comm)
                    comm.rounds = 0
                    alg.sort(None, pv.begin(), pv.end(), F.greater if desc else F.less)
                    res[(eng.__name__, gather, name, desc)] = (pv.lo, pv.local.copy(), comm.rounds)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("size", [2, 3, 4, 8])
def test_segmented_sort_gloo(size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(size))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for (eng, gather, name, desc) in results[0]:
        x = cases()[name]
        got = np.zeros_like(x)
        sizes = []
        for r in range(size):
            lo, loc, rounds = results[r][(eng, gather, name, desc)]
            got[lo:lo + loc.size] = loc
            sizes.append(loc.size)
        if name == "u64_uniform" and gather == S.segmented.SELECT_GATHER:
            # one all-reduce round of 16-bit digits, then the gathered blocks
            assert rounds == 2, rounds
        # at most 4 digit rounds + the gather for 64-bit keys
        assert rounds <= 5, (name, rounds)
        # partition sizes unchanged (partitioned_vector_impl.hpp:325) and
        # the concatenation is the oracle sort bit for bit
        assert sizes == [b - a for a, b in (S.partition_bounds(x.size, size, k) for k in range(size))]
        exp = O.sort(x, desc)
        np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8),
                                      err_msg=f"{name} desc={desc} gather={gather} {eng}")
