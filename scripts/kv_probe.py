"""sort_by_key u64/u64, u64/u32, u32/u64 and u32/u32 at 2^logn pairs (random keys), event-timed
through the C ABI; HPXHIP_SORT_HYBRID=0 gives the plain LSD for comparison."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "28"))
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
e0, e1 = vp(), vp(); lib.hpxhip_event_create(ctypes.byref(e0)); lib.hpxhip_event_create(ctypes.byref(e1))
k, v = alloc(8 * N), alloc(8 * N)
tag = "hybrid" if os.environ.get("HPXHIP_SORT_HYBRID", "17") != "0" else "lsd"
for kdt, kname, vdt, vname in ((L.U64, "u64", L.U64, "u64"), (L.U64, "u64", L.U32, "u32"),
                               (L.U32, "u32", L.U64, "u64"), (L.U32, "u32", L.U32, "u32")):
    def gen():
        L.check(lib.hpxhip_generate(kdt, L.GEN_BITS, 13, 0, 0, k, N, st))
        L.check(lib.hpxhip_generate(vdt, L.GEN_IOTA, 0, 0, 0, v, N, st))
    best = 1e9
    for rep in range(4):
        gen()
        lib.hpxhip_event_record(e0, st)
        L.check(lib.hpxhip_sort_by_key(kdt, vdt, k, v, N, 0, st, None, 0))
        lib.hpxhip_event_record(e1, st)
        L.check(lib.hpxhip_event_synchronize(e1)); ms = ctypes.c_float(); lib.hpxhip_event_elapsed_ms(e0, e1, ctypes.byref(ms))
        if rep: best = min(best, ms.value)
    print(f"{tag:7s} sort_by_key {kname}/{vname} 2^{N.bit_length()-1}: {best:8.3f} ms  {N/best/1e6:7.3f} Gpairs/s", flush=True)
d = ctypes.c_uint32(); L.check(lib.hpxhip_device_error(0, ctypes.byref(d))); print("deverr", d.value)
