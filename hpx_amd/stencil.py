"""examples/1d_stencil heat solver on MI355X.

Reference: examples/1d_stencil/1d_stencil_1.cpp:41-72 (serial stepper),
1d_stencil_4_parallel.cpp:87-156 (partitions + dataflow), 1d_stencil_8.cpp
(distributed partitions with halo exchange).  One partition per GPU here;
the single-GPU solver runs the whole periodic ring on one device
(hpxhip_stencil_heat_run, temporal blocking: up to MAX_FUSED steps per pass
over HBM), the multi-GPU solver (hpx_amd.segmented.heat_solver) exchanges
halos of one pass's width between neighbouring ranks once per pass.
Initial condition of the benchmark: U0[i] = i (1d_stencil_4.cpp:64-66).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from .compute import target, vector

K, DT, DX = 0.5, 1.0, 1.0  # 1d_stencil_1.cpp:25-28
MAX_FUSED = L.STENCIL_MAX_FUSED   # steps per HBM pass (hpxhip_stencil_heat_steps)
FUSED_WINDOW = 1024               # points per wave window of the fused kernel (stencil.hip kFusedWin)
FUSED_MIN_POINTS = 2 * FUSED_WINDOW


def fused_passes(n: int, nt: int, match_parity: bool = False) -> list:
    """Steps per HBM pass for nt steps on an n-point ring (mirror of the
    planner in stencil.hip, run_passes): passes of up to MAX_FUSED (even)
    steps, a single step for an odd remainder.  match_parity=True is the plan
    of hpxhip_stencil_heat_run (pass count with nt's parity, so the result
    lands in u0 for even nt); False that of hpxhip_stencil_heat_run_fused."""
    out = []
    fuse = n >= FUSED_MIN_POINTS
    done = 0
    while done < nt:
        cap = 60 * MAX_FUSED if fuse else 64
        chunk = min(nt - done, cap)
        p, r = [], chunk
        while fuse and r >= 2:
            st = MAX_FUSED if r >= MAX_FUSED else r & ~1
            p.append(st)
            r -= st
        p += [1] * r
        if match_parity and len(p) % 2 != chunk % 2:
            big = [i for i, v in enumerate(p) if v >= 4]
            i = big[0] if big else p.index(2)
            d = 2 if big else 1
            p[i] -= d
            p.insert(i + 1, d)
        out += p
        done += chunk
    return out


def pass_hbm_bytes(n: int, steps: int) -> float:
    """HBM bytes of one pass over n points: every wave window of FUSED_WINDOW points
    is read once and its FUSED_WINDOW - 2*steps exact points written (a single step
    reads and writes each point once)."""
    if steps == 1:
        return 16.0 * n
    return 8.0 * n * FUSED_WINDOW / (FUSED_WINDOW - 2 * steps) + 8.0 * n


def heat_run(u0, nt: int, k: float = K, dt: float = DT, dx: float = DX, tgt: target | None = None):
    """nt periodic steps of the heat equation from host array u0; returns the
    host result (1d_stencil_1.cpp do_work)."""
    tgt = tgt or target(0)
    u0 = np.ascontiguousarray(u0, np.float64)
    n = u0.size
    if n == 0 or nt == 0:
        return u0.copy()
    a = vector.from_host(u0, tgt)
    b = vector(n, dtype=np.float64, tgt=tgt)
    which = ctypes.c_int(0)
    L.call("hpxhip_stencil_heat_run_fused", ctypes.c_void_p(a.data()), ctypes.c_void_p(b.data()), n, nt,
           ctypes.c_double(k), ctypes.c_double(dt), ctypes.c_double(dx), ctypes.byref(which), tgt.stream)
    res = b if which.value else a
    out = res.to_host()
    tgt.synchronize()
    return out


class stepper:
    """Device-resident stepper (1d_stencil_4 `stepper` with U[2] buffers)."""

    def __init__(self, nx: int, tgt: target | None = None, k: float = K, dt: float = DT, dx: float = DX,
                 offset: int = 0):
        self.tgt = tgt or target(0)
        self.nx = int(nx)
        self.k, self.dt, self.dx = k, dt, dx
        self.U = [vector(self.nx, dtype=np.float64, tgt=self.tgt), vector(self.nx, dtype=np.float64, tgt=self.tgt)]
        self.t = 0
        self._cur = 0  # index of the buffer holding step t
        # U0[i] = global index (1d_stencil_4.cpp:64-66)
        L.call("hpxhip_generate", L.F64, L.GEN_IOTA, 0, int(offset), 0, ctypes.c_void_p(self.U[0].data()),
               self.nx, self.tgt.stream)

    @property
    def current(self) -> vector:
        return self.U[self._cur]

    @property
    def next(self) -> vector:
        return self.U[1 - self._cur]

    def step_with_halos(self, left_dev: int, right_dev: int, stream=None):
        """One step; left/right halo values are read from device addresses."""
        cur, nxt = self.current, self.next
        L.call("hpxhip_stencil_heat_step", ctypes.c_void_p(cur.data()), ctypes.c_void_p(nxt.data()), self.nx,
               ctypes.c_void_p(left_dev), ctypes.c_void_p(right_dev), ctypes.c_double(self.k),
               ctypes.c_double(self.dt), ctypes.c_double(self.dx), stream or self.tgt.stream)
        self.t += 1
        self._cur = 1 - self._cur

    def do_work(self, nt: int):
        """nt periodic steps of a single partition (temporal blocking: up to
        MAX_FUSED steps per pass over HBM)."""
        a, b = self.current, self.next
        which = ctypes.c_int(0)
        L.call("hpxhip_stencil_heat_run_fused", ctypes.c_void_p(a.data()), ctypes.c_void_p(b.data()), self.nx, nt,
               ctypes.c_double(self.k), ctypes.c_double(self.dt), ctypes.c_double(self.dx), ctypes.byref(which),
               self.tgt.stream)
        self.t += nt
        if which.value:
            self._cur = 1 - self._cur
        return self.current
