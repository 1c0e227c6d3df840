"""1d_stencil heat at 2^32 points (one GPU, the partitioned solver): time of
100 steps after 100 warm-up steps, ramp U0[i] = i vs random U0 = unit(seed),
and the fused single-GPU run on the same two states.  usage:
python scripts/stencil_probe.py [logn]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import hpx_amd as hpx  # noqa: E402
from hpx_amd import _lib as L  # noqa: E402
from hpx_amd import segmented as S  # noqa: E402

logn = int(sys.argv[1]) if len(sys.argv) > 1 else 32
nx, nt = 1 << logn, 100
t = hpx.target(0)
comm = S.LocalComm(t)
for init in (None, ("unit", 0xC0FFEE), None, ("unit", 0xC0FFEE)):
    hs = S.heat_solver(nx, comm, t, init=init)
    hs.do_work(nt)
    hs.synchronize()
    t0 = time.perf_counter()
    hs.do_work(nt)
    hs.synchronize()
    el = time.perf_counter() - t0
    print(f"heat_solver {'ramp' if init is None else 'random'}: {1e3 * el:.2f} ms for {nt} steps", flush=True)
    for v in hs.U + [hs.H]:
        v.free()
for kind in (L.GEN_IOTA, L.GEN_UNIT, L.GEN_IOTA, L.GEN_UNIT):
    a = hpx.vector(nx, dtype=np.float64, tgt=t)
    b = hpx.vector(nx, dtype=np.float64, tgt=t)
    L.call("hpxhip_generate_at", L.F64, kind, 0xC0FFEE, 0, 0, 0, ctypes.c_void_p(a.data()), nx, t.stream)
    which = ctypes.c_int()
    for rep in range(2):
        t.synchronize()
        t0 = time.perf_counter()
        L.call("hpxhip_stencil_heat_run_fused", ctypes.c_void_p(a.data()), ctypes.c_void_p(b.data()), nx, nt,
               ctypes.c_double(0.5), ctypes.c_double(1.0), ctypes.c_double(1.0), ctypes.byref(which), t.stream)
        t.synchronize()
        el = time.perf_counter() - t0
    print(f"heat_run_fused {'ramp' if kind == L.GEN_IOTA else 'random'}: {1e3 * el:.2f} ms for {nt} steps", flush=True)
    a.free()
    b.free()
