"""Perf probe at 2^30: event-timed kernels through the C ABI."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "30"))
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
e0, e1 = vp(), vp(); lib.hpxhip_event_create(ctypes.byref(e0)); lib.hpxhip_event_create(ctypes.byref(e1))
def timeit(name, fn, bytes_, reps=10):
    fn(); L.check(lib.hpxhip_stream_synchronize(st))
    best = 1e9; tot = 0
    for _ in range(reps):
        lib.hpxhip_event_record(e0, st); fn(); lib.hpxhip_event_record(e1, st)
        L.check(lib.hpxhip_event_synchronize(e1)); ms = ctypes.c_float(); lib.hpxhip_event_elapsed_ms(e0, e1, ctypes.byref(ms))
        best = min(best, ms.value); tot += ms.value
    print(f"{name:28s} best {best:8.3f} ms  avg {tot/reps:8.3f} ms  {bytes_/best/1e6:8.1f} GB/s ({bytes_/best/1e6/8000*100:5.1f}% of 8 TB/s)", flush=True)
a, b, c = alloc(8*N), alloc(8*N), alloc(8*N)
L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 1, 0, 0, b, N, st)); L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 2, 0, 0, c, N, st))
s3 = L.scalars_buf(L.F64, [3.0])
timeit("copy f64", lambda: lib.hpxhip_copy(L.F64, b, a, N, st), 16*N)
timeit("triad f64", lambda: lib.hpxhip_transform_binary(L.F64, L.F64, L.F64, L.B_TRIAD, s3, b, c, a, N, st), 24*N)
x, y, out = b, c, alloc(64)
L.check(lib.hpxhip_generate(L.I64, L.GEN_RANGE, 0x5EED, -(1<<20), 1<<20, x, N, st))
i0 = L.scalar_buf(L.I64, 0); f0 = L.scalar_buf(L.F64, 0.0)
timeit("reduce i64", lambda: lib.hpxhip_transform_reduce(L.I64, L.I64, L.PLUS, L.U_IDENTITY, None, i0, x, N, out, st, None, 0), 8*N)
timeit("incl scan i64", lambda: lib.hpxhip_scan(L.I64, L.PLUS, 1, L.U_IDENTITY, None, i0, None, x, y, N, st, None, 0), 16*N)
timeit("excl scan i64", lambda: lib.hpxhip_scan(L.I64, L.PLUS, 0, L.U_IDENTITY, None, i0, None, x, y, N, st, None, 0), 16*N)
cnt = alloc(64)
timeit("copy_if i64 (x>=0)", lambda: lib.hpxhip_copy_if(L.I64, L.P_NOT_LT, i0, x, y, N, cnt, st, None, 0), 12*N)
L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 3, 0, 0, x, N, st))
timeit("reduce f64", lambda: lib.hpxhip_transform_reduce(L.F64, L.F64, L.PLUS, L.U_IDENTITY, None, f0, x, N, out, st, None, 0), 8*N)
timeit("incl scan f64", lambda: lib.hpxhip_scan(L.F64, L.PLUS, 1, L.U_IDENTITY, None, f0, None, x, y, N, st, None, 0), 16*N)
cur = alloc(8*N); L.check(lib.hpxhip_generate(L.F64, L.GEN_IOTA, 0, 0, 0, cur, N, st))
timeit("stencil step f64", lambda: lib.hpxhip_stencil_heat_step(cur, a, N, cur, cur, 0.5, 1.0, 1.0, st), 16*N)
# temporal blocking: 8 steps in one pass (16.5 B/point of HBM traffic); GB/s column = 16 B/point/step model
timeit("stencil 8 fused steps f64", lambda: lib.hpxhip_stencil_heat_steps(cur, a, N, 0, N, cur, cur, 8, 0.5, 1.0, 1.0, st), 8*16*N)
timeit("stencil 16 fused steps f64", lambda: lib.hpxhip_stencil_heat_steps(cur, a, N, 0, N, cur, cur, 16, 0.5, 1.0, 1.0, st), 16*16*N)
keys = a
def srt():
    L.check(lib.hpxhip_generate(L.U64, L.GEN_BITS, 7, 0, 0, keys, N, st))
    return lib.hpxhip_sort(L.U64, keys, N, 0, st, None, 0)
# time generate separately to subtract
timeit("generate u64", lambda: lib.hpxhip_generate(L.U64, L.GEN_BITS, 7, 0, 0, keys, N, st), 8*N, reps=3)
timeit("gen+sort u64", srt, 136*N, reps=3)
code = ctypes.c_uint32(); L.check(lib.hpxhip_device_error(0, ctypes.byref(code))); print("deverr", code.value)
# merge of two sorted 2^(LOGN-1) u64 runs (evens and odds: alternating path)
h = N // 2
ma, mb, mo = a, vp(c.value), vp(b.value)
L.check(lib.hpxhip_generate(L.U64, L.GEN_IOTA, 0, 0, 0, ma, h, st))
L.check(lib.hpxhip_transform(L.U64, L.U64, L.U64, L.U_AFFINE, L.scalars_buf(L.U64, [2, 0]), ma, ma, h, st))
L.check(lib.hpxhip_transform(L.U64, L.U64, L.U64, L.U_AFFINE, L.scalars_buf(L.U64, [1, 1]), ma, mb, h, st))
timeit("merge u64 (2x2^29 -> 2^30)", lambda: lib.hpxhip_merge(L.U64, ma, h, mb, h, mo, 0, st, None, 0), 16 * N)
code = ctypes.c_uint32(); L.check(lib.hpxhip_device_error(0, ctypes.byref(code))); print("deverr", code.value)
