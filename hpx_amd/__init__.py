"""hpx_amd -- MI355X (gfx950) backend for HPX's data-parallel algorithm layer.

Python mirror of the reference interface for the hot path (the C++ mirror
lives in include/hpx/).  Layout:

  hpx_amd.compute      hip::target, hip::allocator, hip executors,
                       compute::vector / iterator
  hpx_amd.execution    seq, par, par_unseq, task, .on(), .with_()
  hpx_amd.parallel     the algorithms (for_each ... sort), hpx::parallel::*
  hpx_amd.functional   named functors the C ABI can carry
  hpx_amd.future       hpx::future, when_all, dataflow
  hpx_amd.segmented    partitioned_vector + segmented algorithms over N GPUs
  hpx_amd.stencil      examples/1d_stencil heat solver

The kernels live in libhpxhip.so (hpx_amd/csrc, C ABI include/hpxhip.h).
"""
from . import _lib
from . import algorithms as parallel
from . import compute, execution, functional, future as _future_mod
from .compute import (allocator, concurrent_executor, default_executor, get_local_targets, iterator, target,
                      vector)
from .future import dataflow, future, make_ready_future, wait_all, when_all

__all__ = [
    "allocator", "compute", "concurrent_executor", "dataflow", "default_executor", "execution",
    "functional", "future", "get_local_targets", "iterator", "make_ready_future", "parallel", "target",
    "vector", "wait_all", "when_all",
]


def library():
    """The loaded ctypes library (raises ImportError if it is not built)."""
    return _lib.load()
