"""Early GPU probe: raw C-ABI calls on small arrays, checked with numpy."""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpx_amd import _lib as L

lib = L.load()
vp = ctypes.c_void_p
cnt = ctypes.c_int()
L.check(lib.hpxhip_get_device_count(ctypes.byref(cnt)))
print("devices", cnt.value, "torch loaded:", "torch" in sys.modules)
props = L.DeviceProps(); L.check(lib.hpxhip_device_props_get(0, ctypes.byref(props)))
print(props.name, props.arch, props.compute_units)
st = vp(); L.check(lib.hpxhip_stream_create(0, ctypes.byref(st)))

def dev(arr):
    p = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(p), max(arr.nbytes, 16)))
    L.check(lib.hpxhip_memcpy_async(p, arr.ctypes.data, arr.nbytes, L.H2D, st)); return p
def host(p, n, dt):
    a = np.empty(n, dt); L.check(lib.hpxhip_memcpy_async(a.ctypes.data, p, a.nbytes, L.D2H, st))
    L.check(lib.hpxhip_stream_synchronize(st)); return a

ok = True
def rep(name, good):
    global ok
    ok &= bool(good); print(("PASS " if good else "FAIL ") + name, flush=True)

rng = np.random.default_rng(1)
for n in [1, 5, 1000, 100003, 1 << 22]:
    b = rng.random(n); c = rng.random(n)
    pb, pc, pa = dev(b), dev(c), dev(np.zeros(n))
    s = L.scalars_buf(L.F64, [3.0])
    L.check(lib.hpxhip_transform_binary(L.F64, L.F64, L.F64, L.B_TRIAD, s, pb, pc, pa, n, st))
    a = host(pa, n, np.float64)
    rep(f"triad n={n}", np.array_equal(a, b + c * 3.0))
    x = rng.integers(-2**20, 2**20, n, dtype=np.int64); px = dev(x)
    out = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(out), 64))
    init = L.scalar_buf(L.I64, 7)
    L.check(lib.hpxhip_transform_reduce(L.I64, L.I64, L.PLUS, L.U_IDENTITY, None, init, px, n, out, st, None, 0))
    r = host(out, 1, np.int64)[0]
    rep(f"reduce i64 n={n}", r == 7 + int(x.sum()))
    py = dev(np.zeros(n, np.int64))
    L.check(lib.hpxhip_scan(L.I64, L.PLUS, 1, L.U_IDENTITY, None, init, None, px, py, n, st, None, 0))
    y = host(py, n, np.int64)
    rep(f"incl scan i64 n={n}", np.array_equal(y, 7 + np.cumsum(x)))
    L.check(lib.hpxhip_scan(L.I64, L.PLUS, 0, L.U_IDENTITY, None, init, None, px, py, n, st, None, 0))
    y = host(py, n, np.int64)
    ex = np.concatenate([[7], 7 + np.cumsum(x)[:-1]])
    rep(f"excl scan i64 n={n}", np.array_equal(y, ex))
    cntp = vp(); L.check(lib.hpxhip_malloc(0, ctypes.byref(cntp), 64))
    zero = L.scalar_buf(L.I64, 0)
    L.check(lib.hpxhip_copy_if(L.I64, L.P_NOT_LT, zero, px, py, n, cntp, st, None, 0))
    k = int(host(cntp, 1, np.uint64)[0]); sel = x[~(x < 0)]
    y = host(py, n, np.int64)
    rep(f"copy_if n={n}", k == sel.size and np.array_equal(y[:k], sel))
    keys = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True); pk = dev(keys)
    L.check(lib.hpxhip_sort(L.U64, pk, n, 0, st, None, 0))
    sk = host(pk, n, np.uint64)
    rep(f"sort u64 n={n}", np.array_equal(sk, np.sort(keys)))
    for p in (pb, pc, pa, px, out, py, cntp, pk): lib.hpxhip_free(p)
code = ctypes.c_uint32(); L.check(lib.hpxhip_device_error(0, ctypes.byref(code)))
rep("device error word clear", code.value == 0)
print("ALL OK" if ok else "SOME FAILED")
sys.exit(0 if ok else 1)
