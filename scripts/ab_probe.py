"""A/B of two library builds on one box: scan, copy_if and sort at 2^30,
event-timed through the C ABI.  HPXHIP_LIB selects the build."""
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
def timeit(name, fn, bytes_, reps=10, pre=None):
    if pre: pre()
    fn(); L.check(lib.hpxhip_stream_synchronize(st))
    ts = []
    for _ in range(reps):
        if pre: pre()
        lib.hpxhip_event_record(e0, st); fn(); lib.hpxhip_event_record(e1, st)
        L.check(lib.hpxhip_event_synchronize(e1)); ms = ctypes.c_float(); lib.hpxhip_event_elapsed_ms(e0, e1, ctypes.byref(ms))
        ts.append(ms.value)
    ts.sort()
    print(f"{tag:20s} {name:22s} best {ts[0]:8.3f} ms  med {ts[len(ts)//2]:8.3f} ms  {bytes_/ts[0]/1e6:8.1f} GB/s", flush=True)
x, y, cnt = alloc(8 * N), alloc(8 * N), alloc(64)
L.check(lib.hpxhip_generate(L.I64, L.GEN_RANGE, 0x5EED, -(1 << 20), 1 << 20, x, N, st))
i0 = L.scalar_buf(L.I64, 0)
timeit("incl scan i64", lambda: lib.hpxhip_scan(L.I64, L.PLUS, 1, L.U_IDENTITY, None, i0, None, x, y, N, st, None, 0), 16 * N)
z = L.scalar_buf(L.I64, 0)
timeit("copy_if i64 x>=0", lambda: lib.hpxhip_copy_if(L.I64, L.P_NOT_LT, z, x, y, N, cnt, st, None, 0), 12 * N)
L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 3, 0, 0, x, N, st))
timeit("incl scan f64", lambda: lib.hpxhip_scan(L.F64, L.PLUS, 1, L.U_IDENTITY, None, L.scalar_buf(L.F64, 0.0), None, x, y, N, st, None, 0), 16 * N)
if os.environ.get("NOSORT"):
    L.check(lib.hpxhip_stream_synchronize(st))
    sys.exit(0)
gen = lambda: L.check(lib.hpxhip_generate(L.U64, L.GEN_BITS, 7, 0, 0, x, N, st))
timeit("sort u64 (hybrid)", lambda: lib.hpxhip_sort(L.U64, x, N, 0, st, None, 0), 56 * N, reps=4, pre=gen)
gen32 = lambda: L.check(lib.hpxhip_generate(L.U32, L.GEN_BITS, 11, 0, 0, x, N, st))
timeit("sort u32 (hybrid)", lambda: lib.hpxhip_sort(L.U32, x, N, 0, st, None, 0), 36 * N, reps=4, pre=gen32)
L.check(lib.hpxhip_stream_synchronize(st))
d = ctypes.c_uint32()
L.check(lib.hpxhip_device_error(0, ctypes.byref(d))); print("deverr", d.value)
