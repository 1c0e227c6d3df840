"""examples/1d_stencil heat solver on MI355X.

Reference: examples/1d_stencil/1d_stencil_1.cpp:41-72 (serial stepper),
1d_stencil_4_parallel.cpp:87-156 (partitions + dataflow), 1d_stencil_8.cpp
(distributed partitions with halo exchange).  One partition per GPU here;
the single-GPU solver runs the whole periodic ring on one device
(hpxhip_stencil_heat_run), the multi-GPU solver (hpx_amd.segmented.
heat_solver) exchanges one-point halos between neighbouring ranks each step.
Initial condition of the benchmark: U0[i] = i (1d_stencil_4.cpp:64-66).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from .compute import target, vector

K, DT, DX = 0.5, 1.0, 1.0  # 1d_stencil_1.cpp:25-28


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
    L.call("hpxhip_stencil_heat_run", ctypes.c_void_p(a.data()), ctypes.c_void_p(b.data()), n, nt,
           ctypes.c_double(k), ctypes.c_double(dt), ctypes.c_double(dx), tgt.stream)
    res = a if nt % 2 == 0 else b
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
        # U0[i] = global index (1d_stencil_4.cpp:64-66)
        L.call("hpxhip_generate", L.F64, L.GEN_IOTA, 0, int(offset), 0, ctypes.c_void_p(self.U[0].data()),
               self.nx, self.tgt.stream)

    @property
    def current(self) -> vector:
        return self.U[self.t % 2]

    @property
    def next(self) -> vector:
        return self.U[(self.t + 1) % 2]

    def step_with_halos(self, left_dev: int, right_dev: int, stream=None):
        """One step; left/right halo values are read from device addresses."""
        cur, nxt = self.current, self.next
        L.call("hpxhip_stencil_heat_step", ctypes.c_void_p(cur.data()), ctypes.c_void_p(nxt.data()), self.nx,
               ctypes.c_void_p(left_dev), ctypes.c_void_p(right_dev), ctypes.c_double(self.k),
               ctypes.c_double(self.dt), ctypes.c_double(self.dx), stream or self.tgt.stream)
        self.t += 1

    def do_work(self, nt: int):
        """nt periodic steps of a single partition."""
        a, b = self.current, self.next
        L.call("hpxhip_stencil_heat_run", ctypes.c_void_p(a.data()), ctypes.c_void_p(b.data()), self.nx, nt,
               ctypes.c_double(self.k), ctypes.c_double(self.dt), ctypes.c_double(self.dx), self.tgt.stream)
        self.t += nt
        return self.current
