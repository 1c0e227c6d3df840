"""Debug 2: the float64 one-pass run merge -- LB / UB rows and the sample
read back from an explicit scratch buffer (layout replicated from mw_plan)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import hpx_amd as hpx
from hpx_amd import _lib as L
from hpx_amd.compute import dtype_code
from oracle import oracle as O
from test_gpu_merge_sort import rnd


def ordered(x):
    u = np.ascontiguousarray(x).view(np.uint64)
    if x.dtype.kind == "f":
        neg = (u >> np.uint64(63)) == 1
        return np.where(neg, ~u, u | np.uint64(1 << 63))
    return u


def align(x):
    return (x + 255) // 256 * 256


tgt = hpx.target(0)
for dt in (np.float64, np.uint64):
    p = 2
    rng = np.random.default_rng(p)
    lens = rng.integers(0, 300000, p)
    runs = [O.sort(np.asarray(rnd(dt, int(n), 10 + j), dt)) for j, n in enumerate(lens)]
    src = np.concatenate(runs)
    d = hpx.vector.from_host(src, tgt)
    out = hpx.vector(src.size, dtype=dt, tgt=tgt)
    CAP, Q = 2048, 3
    S = CAP // ((Q + 1) * p)
    q = Q * p
    ns = [(int(n) + S - 1) // S for n in lens]
    M = sum(ns)
    K = max(1, (M + q - 1) // q)
    off = 0
    o_runsamp = off; off = align(off + M * 8)
    o_sa = off; off = align(off + M * 8)
    o_sb = off; off = align(off + M * 8)
    o_splits = off; off = align(off + ((M + 2047) // 2048 + 1) * 8)
    o_lb = off; off = align(off + (K + 1) * p * 8)
    o_ub = off; off = align(off + (K + 1) * p * 8)
    total = off
    scr = hpx.vector(total // 8 + 64, dtype=np.uint64, tgt=tgt)
    offs = (ctypes.c_uint64 * (p + 1))(0, int(lens[0]), int(lens[0] + lens[1]))
    L.call("hpxhip_merge_runs", dtype_code(dt), ctypes.c_void_p(d.data()), offs, p, ctypes.c_void_p(out.data()), 0,
           tgt.stream, ctypes.c_void_p(scr.data()), total)
    tgt.synchronize()
    raw = scr.to_host()
    got = out.to_host()
    exp = O.sort(src)
    print(dt.__name__, "M", M, "K", K, "mismatches", int((got.view(np.uint64) != exp.view(np.uint64)).sum()))
    samp = raw[o_runsamp // 8:o_runsamp // 8 + M]
    srt = raw[o_sa // 8:o_sa // 8 + M]
    LB = raw[o_lb // 8:o_lb // 8 + (K + 1) * p].reshape(K + 1, p)
    UB = raw[o_ub // 8:o_ub // 8 + (K + 1) * p].reshape(K + 1, p)
    oks = [ordered(r) for r in runs]
    exp_samp = np.concatenate([r[::S] for r in runs]).view(np.uint64)
    print(" runsamp ok", bool((samp == exp_samp).all()))
    es = np.sort(ordered(np.concatenate([r[::S] for r in runs])))
    print(" sorted sample ok", bool((ordered(srt.view(dt)) == es).all()))
    bad = 0
    for k in range(1, K):
        v = ordered(srt.view(dt))[k * q]
        for j in range(p):
            lb = np.searchsorted(oks[j], v, "left")
            ub = np.searchsorted(oks[j], v, "right")
            if LB[k, j] != lb or UB[k, j] != ub:
                if bad < 5:
                    print("  k", k, "j", j, "LB", LB[k, j], lb, "UB", UB[k, j], ub)
                bad += 1
    print(" bad bounds", bad)
