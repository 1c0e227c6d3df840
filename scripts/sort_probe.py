"""Sort size sweep on one GPU: hpxhip_sort / hpxhip_sort_by_key over random
keys at 2^20..2^30, device time from HIP events (best of 3, generation
subtracted), host time of the call itself, and an is_sorted + checksum
check of every result.  usage: python scripts/sort_probe.py [maxlog]
(SORT_ONLY=u64|u32|pairs|u64r16|u64r24|u64corr|u64hot: that case at 2^maxlog
only; u64corr: the 9-bit field under the top byte is a function of the top
byte -- uniform marginal histograms, 256 populated buckets of n/256 keys, so
every bucket is oversized and the plan falls back to the full LSD after the
prefix passes; u64hot: uniform keys plus one prefix holding
n/64 extra keys -- one oversized bucket sends the whole sort to the LSD)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import hpx_amd as hpx  # noqa: E402
from hpx_amd import _lib as L  # noqa: E402
from hpx_amd import execution as ex, functional as F, parallel as P  # noqa: E402
from hpx_amd.compute import dtype_code  # noqa: E402

t = hpx.target(0)
pol = ex.par.on(hpx.default_executor(t))
S = t.stream


def ev():
    h = ctypes.c_void_p()
    L.call("hpxhip_event_create", ctypes.byref(h))
    return h


e0, e1, e2 = ev(), ev(), ev()


def ms(a, b):
    f = ctypes.c_float()
    L.call("hpxhip_event_elapsed_ms", a, b, ctypes.byref(f))
    return f.value


def correlate(k, n, hot=False):
    """u64corr: bits [47, 56) := bits [56, 64) << 1 (a function of the top
    byte); u64hot: keys [0, n/64) moved onto one 17-bit prefix."""
    from hpx_amd import functional as F  # noqa: F401
    import numpy as np_
    h = k.to_host()
    if hot:
        m = n // 64
        h[:m] = (np_.uint64(0x1234B) << np_.uint64(47)) | (h[:m] & np_.uint64((1 << 47) - 1))
    else:
        top = h >> np_.uint64(56)
        h = (h & ~np_.uint64(0x1FF << 47)) | ((top << np_.uint64(48)) & np_.uint64(0x1FF << 47))
    L.call("hpxhip_memcpy_async", ctypes.c_void_p(k.data()), h.ctypes.data_as(ctypes.c_void_p), 8 * n, L.H2D, S)
    t.synchronize()


def run(dt, logn, kv=False, reps=3, key_range=None, shape=None):
    n = 1 << logn
    k = hpx.vector(n, dtype=dt, tgt=t)
    v = hpx.vector(n, dtype=np.uint64, tgt=t) if kv else None
    best, host = 1e30, 1e30
    for r in range(reps):
        if key_range:
            P.generate(pol, k.begin(), k.end(), "range", 7 + r, 0, key_range - 1)
        else:
            P.generate(pol, k.begin(), k.end(), "bits", 7 + r)
        if shape:
            correlate(k, n, hot=shape == "hot")
        if kv:
            P.generate(pol, v.begin(), v.end(), "iota", 0, 0, 0)
        t.synchronize()
        L.call("hpxhip_event_record", e0, S)
        h0 = time.perf_counter()
        if kv:
            L.call("hpxhip_sort_by_key", dtype_code(dt), L.U64, ctypes.c_void_p(k.data()), ctypes.c_void_p(v.data()),
                   n, 0, S, None, 0)
        else:
            L.call("hpxhip_sort", dtype_code(dt), ctypes.c_void_p(k.data()), n, 0, S, None, 0)
        h1 = time.perf_counter()
        L.call("hpxhip_event_record", e1, S)
        t.synchronize()
        best = min(best, ms(e0, e1))
        host = min(host, 1e3 * (h1 - h0))
    ok = bool(P.is_sorted(pol, k.begin(), k.end()))
    if kv:  # values are a permutation of iota: sum check
        ok = ok and P.reduce(pol, v.begin(), v.end(), 0, F.plus) == n * (n - 1) // 2
        v.free()
    k.free()
    return best, host, ok


maxlog = int(sys.argv[1]) if len(sys.argv) > 1 else 30
# SORT_ONLY=u64|u32|pairs: that case at 2^maxlog only (PMC target runs)
only = os.environ.get("SORT_ONLY")
print(f"{'case':28s} {'ms':>9s} {'Gkeys/s':>8s} {'host_ms':>8s} ok", flush=True)
if only:
    # u64r16 / u64r24: keys below 2^16 / 2^24 (two / three live digits)
    dt, kv, kr = {"u64": (np.uint64, False, None), "u32": (np.uint32, False, None),
                  "pairs": (np.uint64, True, None), "u64r16": (np.uint64, False, 1 << 16),
                  "u64r24": (np.uint64, False, 1 << 24), "u64corr": (np.uint64, False, None),
                  "u64hot": (np.uint64, False, None)}[only]
    shape = {"u64corr": "corr", "u64hot": "hot"}.get(only)
    d, h, ok = run(dt, maxlog, kv, reps=2, key_range=kr, shape=shape)
    print(f"{only + ' 2^' + str(maxlog):28s} {d:9.3f} {(1 << maxlog) / d / 1e6:8.2f} {h:8.3f} {ok}", flush=True)
    sys.exit(0)
for logn in range(20, maxlog + 1, 2):
    for dt, kv, name in ((np.uint64, False, "u64"), (np.uint32, False, "u32"), (np.uint64, True, "u64/u64 pairs")):
        if kv and logn > 28:
            continue
        d, h, ok = run(dt, logn, kv)
        print(f"{name + ' 2^' + str(logn):28s} {d:9.3f} {(1 << logn) / d / 1e6:8.2f} {h:8.3f} {ok}", flush=True)
