"""Scan / copy_if / reduce / triad on sub-ranges that are not 16-B aligned
(2^30 - 8 int64 / f64 elements, in/out offset by whole elements), event-timed."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = (1 << 30)
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
e0, e1 = vp(), vp(); lib.hpxhip_event_create(ctypes.byref(e0)); lib.hpxhip_event_create(ctypes.byref(e1))
x, y, z, cnt = alloc(8 * N), alloc(8 * N), alloc(8 * N), alloc(64)
def off(p, k): return vp(p.value + 8 * k)
def timeit(name, fn, bytes_):
    fn(); L.check(lib.hpxhip_stream_synchronize(st)); ts = []
    for _ in range(6):
        lib.hpxhip_event_record(e0, st); L.check(fn()); lib.hpxhip_event_record(e1, st)
        L.check(lib.hpxhip_event_synchronize(e1)); ms = ctypes.c_float(); lib.hpxhip_event_elapsed_ms(e0, e1, ctypes.byref(ms)); ts.append(ms.value)
    ts.sort(); print(f"{name:44s} best {ts[0]:7.3f} ms  {bytes_/ts[0]/1e6:7.1f} GB/s", flush=True)
n = N - 8
L.check(lib.hpxhip_generate(L.I64, L.GEN_RANGE, 5, -9, 9, x, N, st))
i0 = L.scalar_buf(L.I64, 0); s3 = L.scalars_buf(L.F64, [3.0])
for a, b in ((0, 0), (1, 1), (1, 0), (0, 3)):
    timeit(f"incl scan i64 in+{a} out+{b}", lambda: lib.hpxhip_scan(L.I64, L.PLUS, 1, L.U_IDENTITY, None, i0, None, off(x, a), off(y, b), n, st, None, 0), 16 * n)
for a, b in ((0, 0), (1, 1), (1, 0)):
    timeit(f"copy_if i64 in+{a} out+{b}", lambda: lib.hpxhip_copy_if(L.I64, L.P_NOT_LT, i0, off(x, a), off(y, b), n, cnt, st, None, 0), 12 * n)
for a in (0, 1):
    timeit(f"reduce i64 in+{a}", lambda: lib.hpxhip_transform_reduce(L.I64, L.I64, L.PLUS, L.U_IDENTITY, None, i0, off(x, a), n, cnt, st, None, 0), 8 * n)
for a, b, c in ((0, 0, 0), (1, 1, 1), (1, 0, 0), (0, 1, 3)):
    timeit(f"triad f64 b+{a} c+{b} a+{c}", lambda: lib.hpxhip_transform_binary(L.F64, L.F64, L.F64, L.B_TRIAD, s3, off(x, a), off(y, b), off(z, c), n, st), 24 * n)
d = ctypes.c_uint32(); L.check(lib.hpxhip_device_error(0, ctypes.byref(d))); print("deverr", d.value)
