"""Fused stencil timing through the C ABI: 16 steps per pass over 2^30 points
(hpxhip_stencil_heat_steps, periodic ring: halos taken from the ring's ends)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "30"))
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
a, b = alloc(8 * N), alloc(8 * N)
L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 1, 0, 0, a, N, st))
e0, e1 = vp(), vp(); lib.hpxhip_event_create(ctypes.byref(e0)); lib.hpxhip_event_create(ctypes.byref(e1))
for S in (8, 16):
    lh = vp(a.value + 8 * (N - S))
    best = 1e9
    for _ in range(6):
        lib.hpxhip_event_record(e0, st)
        L.check(lib.hpxhip_stencil_heat_steps(a, b, ctypes.c_uint64(N), ctypes.c_uint64(0), ctypes.c_uint64(N), lh, a,
                                              S, ctypes.c_double(0.5), ctypes.c_double(1.0), ctypes.c_double(1.0), st))
        lib.hpxhip_event_record(e1, st)
        L.check(lib.hpxhip_event_synchronize(e1))
        ms = ctypes.c_float(); lib.hpxhip_event_elapsed_ms(e0, e1, ctypes.byref(ms)); best = min(best, ms.value)
    print(f"fused {S:2d} steps over 2^{N.bit_length()-1} points: {best:.3f} ms = {best / S:.3f} ms/step, "
          f"{N * S / best / 1e9:.2f} T point-steps/s", flush=True)
