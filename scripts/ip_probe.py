"""transform_reduce binary (inner product, transform_reduce_binary.hpp:323)
at 2^30 doubles and int64, event-timed; HPXHIP_LIB selects the build."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "30"))
tag = os.environ.get("HPXHIP_LIB", "shipped").split("/")[-1]
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
e0, e1 = vp(), vp(); lib.hpxhip_event_create(ctypes.byref(e0)); lib.hpxhip_event_create(ctypes.byref(e1))
a, b, out = alloc(8 * N), alloc(8 * N), alloc(64)
def timeit(name, fn, bytes_):
    fn(); L.check(lib.hpxhip_stream_synchronize(st)); ts = []
    for _ in range(10):
        lib.hpxhip_event_record(e0, st); L.check(fn()); lib.hpxhip_event_record(e1, st)
        L.check(lib.hpxhip_event_synchronize(e1)); ms = ctypes.c_float(); lib.hpxhip_event_elapsed_ms(e0, e1, ctypes.byref(ms)); ts.append(ms.value)
    ts.sort(); print(f"{tag:22s} {name:24s} best {ts[0]:7.3f} ms  {bytes_/ts[0]/1e6:7.1f} GB/s", flush=True)
L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 1, 0, 0, a, N, st)); L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 2, 0, 0, b, N, st))
f0 = L.scalar_buf(L.F64, 0.0); i0 = L.scalar_buf(L.I64, 0)
timeit("inner product f64", lambda: lib.hpxhip_transform_reduce_binary(L.F64, L.F64, L.PLUS, L.B_MUL, None, f0, a, b, N, out, st, None, 0), 16 * N)
timeit("inner product i64", lambda: lib.hpxhip_transform_reduce_binary(L.I64, L.I64, L.PLUS, L.B_MUL, None, i0, a, b, N, out, st, None, 0), 16 * N)
timeit("reduce f64", lambda: lib.hpxhip_transform_reduce(L.F64, L.F64, L.PLUS, L.U_IDENTITY, None, f0, a, N, out, st, None, 0), 8 * N)
