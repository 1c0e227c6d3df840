"""32-bit element paths at 2^31 elements (8 GiB per array, the same bytes as
the 2^30 x 8-B headline): reduce / scan / copy_if over int32, triad over f32,
event-timed through the C ABI."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "31"))
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
e0, e1 = vp(), vp(); lib.hpxhip_event_create(ctypes.byref(e0)); lib.hpxhip_event_create(ctypes.byref(e1))
def timeit(name, fn, bytes_, reps=8):
    fn(); L.check(lib.hpxhip_stream_synchronize(st))
    ts = []
    for _ in range(reps):
        lib.hpxhip_event_record(e0, st); L.check(fn()); lib.hpxhip_event_record(e1, st)
        L.check(lib.hpxhip_event_synchronize(e1)); ms = ctypes.c_float(); lib.hpxhip_event_elapsed_ms(e0, e1, ctypes.byref(ms))
        ts.append(ms.value)
    ts.sort()
    print(f"{name:26s} best {ts[0]:8.3f} ms  {bytes_/ts[0]/1e6:8.1f} GB/s ({bytes_/ts[0]/1e6/80:5.1f}% of 8 TB/s)", flush=True)
x, y, z, cnt = alloc(4 * N), alloc(4 * N), alloc(4 * N), alloc(64)
L.check(lib.hpxhip_generate(L.I32, L.GEN_RANGE, 5, -1000, 1000, x, N, st))
i0 = L.scalar_buf(L.I32, 0); i64 = L.scalar_buf(L.I64, 0)
timeit("reduce i32 -> i64", lambda: lib.hpxhip_transform_reduce(L.I32, L.I64, L.PLUS, L.U_IDENTITY, None, i64, x, N, cnt, st, None, 0), 4 * N)
timeit("reduce i32", lambda: lib.hpxhip_transform_reduce(L.I32, L.I32, L.PLUS, L.U_IDENTITY, None, i0, x, N, cnt, st, None, 0), 4 * N)
timeit("incl scan i32", lambda: lib.hpxhip_scan(L.I32, L.PLUS, 1, L.U_IDENTITY, None, i0, None, x, y, N, st, None, 0), 8 * N)
timeit("copy_if i32 x>=0", lambda: lib.hpxhip_copy_if(L.I32, L.P_NOT_LT, i0, x, y, N, cnt, st, None, 0), 6 * N)
L.check(lib.hpxhip_generate(L.F32, L.GEN_UNIT, 1, 0, 0, x, N, st)); L.check(lib.hpxhip_generate(L.F32, L.GEN_UNIT, 2, 0, 0, y, N, st))
s3 = L.scalars_buf(L.F32, [3.0])
timeit("triad f32", lambda: lib.hpxhip_transform_binary(L.F32, L.F32, L.F32, L.B_TRIAD, s3, x, y, z, N, st), 12 * N)
timeit("incl scan f32", lambda: lib.hpxhip_scan(L.F32, L.PLUS, 1, L.U_IDENTITY, None, L.scalar_buf(L.F32, 0.0), None, x, z, N, st, None, 0), 8 * N)
d = ctypes.c_uint32(); L.check(lib.hpxhip_device_error(0, ctypes.byref(d))); print("deverr", d.value)
