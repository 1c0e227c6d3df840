"""PMC target run (no timing): the bench's hot kernels at 2^30 elements,
each launched 3 times, for rocprofv3 --pmc passes (scripts/s12.sh)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L
lib = L.load(); vp = ctypes.c_void_p
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))
N = 1 << int(os.environ.get("LOGN", "30"))
def alloc(b):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), b)); return p
a, b, c, out, cnt = alloc(8 * N), alloc(8 * N), alloc(8 * N), alloc(64), alloc(64)
L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 1, 0, 0, b, N, st))
L.check(lib.hpxhip_generate(L.F64, L.GEN_UNIT, 2, 0, 0, c, N, st))
s3 = L.scalars_buf(L.F64, [3.0]); i0 = L.scalar_buf(L.I64, 0)
for _ in range(3):
    L.check(lib.hpxhip_transform_binary(L.F64, L.F64, L.F64, L.B_TRIAD, s3, b, c, a, N, st))
L.check(lib.hpxhip_generate(L.I64, L.GEN_RANGE, 0x5EED, -(1 << 20), 1 << 20, b, N, st))
for _ in range(3):
    L.check(lib.hpxhip_transform_reduce(L.I64, L.I64, L.PLUS, L.U_IDENTITY, None, i0, b, N, out, st, None, 0))
for _ in range(3):
    L.check(lib.hpxhip_scan(L.I64, L.PLUS, 1, L.U_IDENTITY, None, i0, None, b, c, N, st, None, 0))
for _ in range(3):
    L.check(lib.hpxhip_copy_if(L.I64, L.P_NOT_LT, i0, b, c, N, cnt, st, None, 0))
L.check(lib.hpxhip_generate(L.F64, L.GEN_IOTA, 0, 0, 0, a, N, st))
for _ in range(3):
    L.check(lib.hpxhip_stencil_heat_step(a, c, N, a, a, 0.5, 1.0, 1.0, st))
L.check(lib.hpxhip_stream_synchronize(st))
print("done")
