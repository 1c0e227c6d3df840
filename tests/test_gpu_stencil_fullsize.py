"""Full-size parity of the 1d_stencil heat solver (BASELINE.json configs[3]:
2^32 points) from a NON-steady initial state.

U0[i] = (splitmix64(seed ^ i) >> 11) * 2^-53, generated on the device for the
global index i (hpxhip_generate_at).  After nt steps point i depends only on
U0[i - nt .. i + nt] (1d_stencil_1.cpp:41-72: next[i] = heat(cur[i-1], cur[i],
cur[i+1])), so the serial oracle runs on a window of +-nt points around each
checked range (oracle.stencil_window) and the comparison is bit for bit.

Unlike the ramp U0[i] = i (a fixed point of the update away from the seam,
which a no-op kernel also passes), random data makes every wrong neighbour
offset, skipped step or 32-bit index wrap visible.  Windows sit at the
periodic seam (0 and nx - 1), at 2^31 +- nt points (signed 32-bit element
index), at 2^28 and 2^29 points (2^31 and 2^32 bytes), at 2^32 - 1 and at
seeded random positions."""
import ctypes

import numpy as np
import pytest

import hpx_amd as hpx
from hpx_amd import _lib as L
from hpx_amd import segmented as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

NX = 1 << 32
SEED = 0xC0FFEE


def windows(nx, nt, seed=7):
    w = [(0, 64), (nx - 64, 64), ((1 << 31) - nt - 32, 2 * nt + 64), ((1 << 28) - 32, 64),
         ((1 << 29) - 32, 64), ((1 << 30) + 511, 130), (nx // 2 + 1000, 64), (nx - 1, 1)]
    rng = np.random.default_rng(seed)
    w += [(int(s), 96) for s in rng.integers(0, nx - 96, 4)]
    return [(lo % nx, c) for lo, c in w if lo + c <= nx]


def read(vec, lo, count, stream, tgt):
    out = np.empty(count, np.float64)
    L.call("hpxhip_memcpy_async", out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(vec.data() + 8 * lo),
           8 * count, L.D2H, stream)
    tgt.synchronize()
    return out


def check_windows(vec, nx, nt, seed, tgt):
    for lo, c in windows(nx, nt):
        got = read(vec, lo, c, tgt.stream, tgt)
        exp = O.stencil_window(nx, nt, seed, lo, c)
        np.testing.assert_array_equal(got, exp, err_msg=f"nx={nx} nt={nt} window [{lo}, {lo + c})")


@pytest.mark.parametrize("nt", [100, 37])
def test_heat_solver_2p32_random_state_windows(gpu_target, nt):
    """heat_solver (hpx_amd.segmented, the partitioned solver the bench runs):
    2^32 points on one GPU, halo ring onto itself, passes of 16 steps (and an
    odd remainder for nt = 37)."""
    tgt = gpu_target
    hs = S.heat_solver(NX, S.LocalComm(tgt), tgt, init=("unit", SEED))
    try:
        hs.do_work(nt)
        hs.synchronize()
        assert hs.t == nt
        check_windows(hs.current, NX, nt, SEED, tgt)
    finally:
        for v in hs.U:
            v.free()
        hs.H.free()


def test_heat_run_fused_2p32_random_state_windows(gpu_target):
    """hpxhip_stencil_heat_run_fused (the single-GPU periodic run, temporal
    blocking with the ring's own ends as halos) at 2^32 points, 100 steps."""
    tgt, nt = gpu_target, 100
    a = hpx.vector(NX, dtype=np.float64, tgt=tgt)
    b = hpx.vector(NX, dtype=np.float64, tgt=tgt)
    try:
        L.call("hpxhip_generate_at", L.F64, L.GEN_UNIT, SEED, 0, 0, 0, ctypes.c_void_p(a.data()), NX, tgt.stream)
        which = ctypes.c_int(-1)
        L.call("hpxhip_stencil_heat_run_fused", ctypes.c_void_p(a.data()), ctypes.c_void_p(b.data()), NX, nt,
               ctypes.c_double(0.5), ctypes.c_double(1.0), ctypes.c_double(1.0), ctypes.byref(which), tgt.stream)
        tgt.synchronize()
        assert which.value in (0, 1)
        check_windows(b if which.value else a, NX, nt, SEED, tgt)
    finally:
        a.free()
        b.free()


def test_heat_solver_random_state_small_full(gpu_target):
    """The same generated state at a size the oracle runs whole: every point
    bit for bit (ties the windowed check to the full-ring oracle)."""
    tgt, nx, nt = gpu_target, 100003, 45
    hs = S.heat_solver(nx, S.LocalComm(tgt), tgt, init=("unit", SEED))
    hs.do_work(nt)
    hs.synchronize()
    exp = O.stencil_heat(O.unit_at(np.arange(nx, dtype=np.uint64), SEED), nt)
    np.testing.assert_array_equal(hs.current.to_host(), exp)
    for lo, c in windows(nx, nt):
        np.testing.assert_array_equal(exp[lo:lo + c], O.stencil_window(nx, nt, SEED, lo, c))
