"""Host-side cost of one C-ABI call (enqueue only, no synchronisation):
perf_counter around each call, 2^logn elements, after warm-up."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "26"))
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
a, b, c, out = alloc(8 * N), alloc(8 * N), alloc(8 * N), alloc(64)
L.check(lib.hpxhip_generate(L.I64, L.GEN_RANGE, 5, -9, 9, b, N, st))
i0 = L.scalar_buf(L.I64, 0); s3 = L.scalars_buf(L.F64, [3.0])
calls = {
    "transform_binary (triad)": lambda: lib.hpxhip_transform_binary(L.F64, L.F64, L.F64, L.B_TRIAD, s3, b, c, a, N, st),
    "transform_reduce": lambda: lib.hpxhip_transform_reduce(L.I64, L.I64, L.PLUS, L.U_IDENTITY, None, i0, b, N, out, st, None, 0),
    "scan": lambda: lib.hpxhip_scan(L.I64, L.PLUS, 1, L.U_IDENTITY, None, i0, None, b, a, N, st, None, 0),
    "event_record": None,
}
for name, fn in calls.items():
    if fn is None:
        continue
    for _ in range(3):
        L.check(fn())
    L.check(lib.hpxhip_stream_synchronize(st))
    ts = []
    for _ in range(20):
        t0 = time.perf_counter(); L.check(fn()); ts.append(1e6 * (time.perf_counter() - t0))
    L.check(lib.hpxhip_stream_synchronize(st))
    ts.sort()
    print(f"{name:28s} host us per call: min {ts[0]:8.1f} med {ts[10]:8.1f} max {ts[-1]:8.1f}", flush=True)
