"""ctypes wrapper of the CPU oracle (oracle/oracle.cpp).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / host baseline.  The product
(hpx_amd/) never imports it.

Parity pinning: tests/test_oracle_golden.py checks every function used as a
checker against tests/golden/*.npz (closed forms of the reference's own
known-answer tests, see tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(HERE, "_build", "liboracle.so")

DT = {"int32": 0, "uint32": 1, "int64": 2, "uint64": 3, "float32": 4, "float64": 5}
OPS = {"plus": 0, "multiplies": 1, "min": 2, "max": 3, "bit_and": 4, "bit_or": 5, "bit_xor": 6}
UNARY = {"identity": 0, "scale": 1, "add_scalar": 2, "affine": 3, "negate": 4, "abs": 5, "square": 6}
BINARY = {"add": 0, "triad": 1, "sub": 2, "mul": 3, "axpy": 4, "min": 5, "max": 6}
PRED = {"lt": 0, "le": 1, "gt": 2, "ge": 3, "eq": 4, "ne": 5, "not_less_than": 6, "bits": 7}

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(SO):
        subprocess.run(["make", "-C", ROOT, "oracle"], check=True, capture_output=True)
    lib = ctypes.CDLL(SO)
    d = ctypes.c_double
    lib.oracle_par_triad.restype = d
    lib.oracle_par_reduce_i64.restype = d
    lib.oracle_par_scan_i64.restype = d
    lib.oracle_par_sort_u64.restype = d
    lib.oracle_par_copy_if_i64.restype = d
    lib.oracle_par_alloc.restype = ctypes.c_void_p
    lib.oracle_par_alloc.argtypes = [ctypes.c_uint64, ctypes.c_int]
    lib.oracle_par_free.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _scal(dtype, vals):
    a = np.zeros(2, dtype)
    for i, v in enumerate(vals):
        a[i] = v
    return a


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"oracle {what} failed: {rc}")


def dtname(a) -> str:
    return np.dtype(a).name


def for_each(data, kind, scalars=()):
    out = np.array(data, copy=True)
    _check(load().oracle_for_each(DT[dtname(out.dtype)], UNARY[kind], _p(_scal(out.dtype, scalars)), _p(out),
                                  ctypes.c_uint64(out.size)), "for_each")
    return out


def transform(a, kind, scalars=(), compute=None, out_dtype=None):
    cd = np.dtype(compute or a.dtype)
    out = np.empty(a.size, out_dtype or a.dtype)
    _check(load().oracle_transform(DT[dtname(a.dtype)], DT[cd.name], DT[dtname(out.dtype)], UNARY[kind],
                                   _p(_scal(cd, scalars)), _p(np.ascontiguousarray(a)), _p(out),
                                   ctypes.c_uint64(a.size)), "transform")
    return out


def transform_binary(a, b, kind, scalars=(), compute=None, out_dtype=None):
    cd = np.dtype(compute or a.dtype)
    out = np.empty(a.size, out_dtype or a.dtype)
    _check(load().oracle_transform_binary(DT[dtname(a.dtype)], DT[cd.name], DT[dtname(out.dtype)], BINARY[kind],
                                          _p(_scal(cd, scalars)), _p(np.ascontiguousarray(a)),
                                          _p(np.ascontiguousarray(b)), _p(out), ctypes.c_uint64(a.size)),
           "transform_binary")
    return out


def transform_reduce(a, init, op="plus", conv="identity", scalars=(), acc=None, cores=0):
    ad = np.dtype(acc or a.dtype)
    out = np.zeros(1, ad)
    iv = np.array([init], ad)
    _check(load().oracle_transform_reduce(DT[dtname(a.dtype)], DT[ad.name], OPS[op], UNARY[conv],
                                          _p(_scal(ad, scalars)), _p(iv), _p(np.ascontiguousarray(a)),
                                          ctypes.c_uint64(a.size), _p(out), cores), "transform_reduce")
    return out[0]


def transform_reduce_binary(a, b, init, op="plus", kind="mul", scalars=(), acc=None, cores=0):
    ad = np.dtype(acc or a.dtype)
    out = np.zeros(1, ad)
    iv = np.array([init], ad)
    _check(load().oracle_transform_reduce_binary(DT[dtname(a.dtype)], DT[ad.name], OPS[op], BINARY[kind],
                                                 _p(_scal(ad, scalars)), _p(iv), _p(np.ascontiguousarray(a)),
                                                 _p(np.ascontiguousarray(b)), ctypes.c_uint64(a.size), _p(out),
                                                 cores), "transform_reduce_binary")
    return out[0]


def scan(a, init, inclusive=True, op="plus", conv="identity", scalars=(), cores=0):
    a = np.ascontiguousarray(a)
    out = np.empty_like(a)
    iv = np.array([init], a.dtype)
    _check(load().oracle_scan(DT[dtname(a.dtype)], OPS[op], 1 if inclusive else 0, UNARY[conv],
                              _p(_scal(a.dtype, scalars)), _p(iv), _p(a), _p(out), ctypes.c_uint64(a.size),
                              cores), "scan")
    return out


def copy_if(a, pred, arg=0):
    a = np.ascontiguousarray(a)
    out = np.empty_like(a)
    cnt = ctypes.c_uint64()
    argv = np.array([arg], a.dtype)
    _check(load().oracle_copy_if(DT[dtname(a.dtype)], PRED[pred], _p(argv), _p(a), _p(out), ctypes.c_uint64(a.size),
                                 ctypes.byref(cnt)), "copy_if")
    return out[:cnt.value].copy()


def sort(a, descending=False):
    out = np.array(a, copy=True)
    _check(load().oracle_sort(DT[dtname(out.dtype)], _p(out), ctypes.c_uint64(out.size), 1 if descending else 0),
           "sort")
    return out


def merge(a, b, descending=False):
    """merge.hpp:52-80: stable merge of two sorted arrays (oracle_merge)."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b, dtype=a.dtype)
    out = np.empty(a.size + b.size, a.dtype)
    _check(load().oracle_merge(DT[dtname(a.dtype)], _p(a), ctypes.c_uint64(a.size), _p(b), ctypes.c_uint64(b.size),
                               _p(out), 1 if descending else 0), "merge")
    return out


def sort_by_key(keys, values, descending=False):
    k = np.array(keys, copy=True)
    v = np.array(values, copy=True)
    _check(load().oracle_sort_by_key(DT[dtname(k.dtype)], DT[dtname(v.dtype)], _p(k), _p(v), ctypes.c_uint64(k.size),
                                     1 if descending else 0), "sort_by_key")
    return k, v


def stencil_heat(u, nt, k=0.5, dt=1.0, dx=1.0):
    out = np.array(u, np.float64, copy=True)
    _check(load().oracle_stencil_heat(_p(out), ctypes.c_uint64(out.size), ctypes.c_uint64(nt), ctypes.c_double(k),
                                      ctypes.c_double(dt), ctypes.c_double(dx)), "stencil")
    return out


def unit_at(idx, seed):
    """generate("unit") at arbitrary global indices (hpxhip_generate_at GEN_UNIT):
    (splitmix64(seed ^ i) >> 11) * 2^-53."""
    z = splitmix64(np.uint64(seed) ^ np.asarray(idx, np.uint64))
    return (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def stencil_window(nx, nt, seed, lo, count, k=0.5, dt=1.0, dx=1.0):
    """Points [lo, lo + count) of the periodic nx-point heat ring after nt
    steps of 1d_stencil_1.cpp:41-72 from U0[i] = unit_at(i, seed).  After nt
    steps point i depends only on U0[i - nt .. i + nt], so the serial stepper
    runs on that window only (each step drops one point per side); the
    window wraps around the ring.  Needs count + 2 nt <= nx."""
    if count + 2 * nt > nx:
        u = stencil_heat(unit_at(np.arange(nx, dtype=np.uint64), seed), nt, k, dt, dx)
        return u[(lo + np.arange(count)) % nx]
    g = (np.int64(lo) - nt + np.arange(count + 2 * nt, dtype=np.int64)) % np.int64(nx)
    w = unit_at(g.astype(np.uint64), seed)
    for _ in range(nt):
        w = stencil_heat_step(w[1:-1], w[0], w[-1], k, dt, dx)
    return w


def stencil_heat_step(cur, left, right, k=0.5, dt=1.0, dx=1.0):
    cur = np.ascontiguousarray(cur, np.float64)
    out = np.empty_like(cur)
    _check(load().oracle_stencil_heat_step(_p(cur), _p(out), ctypes.c_uint64(cur.size), ctypes.c_double(left),
                                           ctypes.c_double(right), ctypes.c_double(k), ctypes.c_double(dt),
                                           ctypes.c_double(dx)), "stencil step")
    return out


def stream_expected(iterations, scalar=3.0):
    a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    _check(load().oracle_stream_expected(ctypes.c_uint64(iterations), ctypes.c_double(scalar), ctypes.byref(a),
                                         ctypes.byref(b), ctypes.byref(c)), "stream")
    return a.value, b.value, c.value


def segmented_reduce(a, init, parts, op="plus"):
    a = np.ascontiguousarray(a)
    out = np.zeros(1, a.dtype)
    iv = np.array([init], a.dtype)
    _check(load().oracle_segmented_reduce(DT[dtname(a.dtype)], OPS[op], _p(iv), _p(a), ctypes.c_uint64(a.size),
                                          parts, _p(out)), "segmented_reduce")
    return out[0]


def segmented_scan(a, init, parts, inclusive=True, op="plus"):
    a = np.ascontiguousarray(a)
    out = np.empty_like(a)
    iv = np.array([init], a.dtype)
    _check(load().oracle_segmented_scan(DT[dtname(a.dtype)], OPS[op], 1 if inclusive else 0, _p(iv), _p(a), _p(out),
                                        ctypes.c_uint64(a.size), parts), "segmented_scan")
    return out


# ---------------------------------------------------------------- generators
MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 (the device generator's functor)."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def generate(dtype, kind, n, seed=0x5EED, lo=0, hi=0, offset=0):
    """Host restatement of hpxhip_generate (include/hpxhip.h) for index range
    [offset, offset + n)."""
    dt = np.dtype(dtype)
    i = np.arange(offset, offset + n, dtype=np.uint64)
    if kind == "iota":
        return (np.int64(lo) + i.astype(np.int64)).astype(dt)
    z = splitmix64(np.uint64(seed) ^ i)
    if kind in ("bits", "splitmix"):
        if dt.itemsize == 8:
            return z.view(dt)
        return (z >> np.uint64(32)).astype(np.uint32).view(dt)
    if kind == "range":
        span = np.uint64((hi - lo + 1) & 0xFFFFFFFFFFFFFFFF)
        r = z % span if span else z
        with np.errstate(over="ignore"):
            v = (np.uint64(lo & 0xFFFFFFFFFFFFFFFF) + r).view(np.int64)
        return v.astype(dt)
    if kind == "unit":
        if dt.itemsize == 8:
            return ((z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53).astype(dt)
        return ((z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)).astype(dt)
    raise ValueError(kind)


# ------------------------------------------------------------- host baseline
def par_stream(n, threads, scalar=3.0, iterations=10):
    """HPX-par restatement of the whole STREAM benchmark (stream.cpp:294-375):
    returns ({kernel: (best s, avg s)}, (a0, b0, c0))."""
    lib = load()
    best, avg, abc = (ctypes.c_double * 4)(), (ctypes.c_double * 4)(), (ctypes.c_double * 3)()
    lib.oracle_par_stream.argtypes = [ctypes.c_uint64, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    _check(lib.oracle_par_stream(n, scalar, iterations, threads, best, avg, abc), "par_stream")
    names = ("copy", "scale", "add", "triad")
    return {k: (best[i], avg[i]) for i, k in enumerate(names)}, tuple(abc)


def par_triad(n, threads, scalar=3.0, reps=3):
    """HPX-par restatement of STREAM triad on `threads` host threads; returns
    best seconds."""
    lib = load()
    b = lib.oracle_par_alloc(n * 8, threads)
    c = lib.oracle_par_alloc(n * 8, threads)
    a = lib.oracle_par_alloc(n * 8, threads)
    try:
        lib.oracle_par_triad.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_double, ctypes.c_int]
        best = min(lib.oracle_par_triad(a, b, c, n, scalar, threads) for _ in range(reps))
    finally:
        for p in (a, b, c):
            lib.oracle_par_free(p, n * 8)
    return best


def par_reduce_i64(a: np.ndarray, threads, reps=3):
    lib = load()
    out = ctypes.c_int64()
    lib.oracle_par_reduce_i64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64,
                                          ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    best = min(lib.oracle_par_reduce_i64(_p(a), a.size, 0, ctypes.byref(out), threads) for _ in range(reps))
    return best, out.value


def par_scan_i64(a: np.ndarray, threads, reps=3):
    lib = load()
    out = np.empty_like(a)
    lib.oracle_par_scan_i64.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    best = min(lib.oracle_par_scan_i64(_p(a), _p(out), a.size, threads) for _ in range(reps))
    return best, out


def par_sort_u64(a: np.ndarray, threads):
    lib = load()
    k = np.array(a, copy=True)
    lib.oracle_par_sort_u64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    t = lib.oracle_par_sort_u64(_p(k), k.size, threads)
    return t, k


def par_stencil(u, nt, threads, k=0.5, dt=1.0, dx=1.0):
    """HPX-par restatement of the 1d_stencil heat solver (1d_stencil_4_parallel.cpp:87-156)
    on `threads` host threads; returns (seconds, final state)."""
    lib = load()
    u0 = np.array(u, np.float64, copy=True)
    u1 = np.empty_like(u0)
    lib.oracle_par_stencil.restype = ctypes.c_double
    lib.oracle_par_stencil.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int]
    t = lib.oracle_par_stencil(_p(u0), _p(u1), u0.size, int(nt), k, dt, dx, threads)
    return t, (u0 if nt % 2 == 0 else u1)


def par_copy_if_i64(a: np.ndarray, threads, reps=3):
    lib = load()
    out = np.empty_like(a)
    cnt = ctypes.c_uint64()
    lib.oracle_par_copy_if_i64.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    best = min(lib.oracle_par_copy_if_i64(_p(a), _p(out), a.size, ctypes.byref(cnt), threads) for _ in range(reps))
    return best, out[:cnt.value]
