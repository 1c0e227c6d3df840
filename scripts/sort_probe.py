"""Sort-only run for rocprof breakdown: 2^30 keys (KEY=u64 | u32), sorted twice."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "30"))
KT, KB = (L.U32, 4) if os.environ.get("KEY") == "u32" else (L.U64, 8)
k = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(k), KB * N))
for r in range(2):
    L.check(lib.hpxhip_generate(KT, L.GEN_BITS, 7 + r, 0, 0, k, N, st))
    L.check(lib.hpxhip_sort(KT, k, N, 0, st, None, 0))
L.check(lib.hpxhip_stream_synchronize(st))
print("done")
