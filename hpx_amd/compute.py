"""hpx::compute for MI355X: hip::target, hip::allocator, hip executors,
compute::vector and its iterator.

Mirrors (HPX 1.4.0):
  * hpx/compute/cuda/target.hpp:36-200 and src/compute/cuda/cuda_target.cpp
    -> :class:`target` (device id, lazily created non-blocking stream,
    ``synchronize()``, ``get_future()``), get_local_targets
    (src/compute/cuda/get_cuda_targets.cpp:30-65);
  * hpx/compute/cuda/allocator.hpp:36-259 -> :class:`allocator`
    (``allocate``/``deallocate``/``max_size``/``target``; out-of-memory maps to
    :class:`hpx_amd._lib.OutOfMemory` like allocator.hpp:118-124);
  * hpx/compute/vector.hpp:28-372 + detail/iterator.hpp:23-85 ->
    :class:`vector`, :class:`iterator`; host element access goes through a
    1-element copy like value_proxy.hpp:25-124 / access_target.hpp:21-52;
  * hpx/compute/cuda/default_executor.hpp:42-260 -> :class:`default_executor`;
    concurrent_executor.hpp:29-234 -> :class:`concurrent_executor`
    (several streams on one device, round robin).

Documented deviation: ``vector(n)`` value-initialises its elements with the
fill kernel; the reference's ``bulk_construct`` is a no-op on the host path
(allocator.hpp:173-195), leaving device memory uninitialised.
"""
from __future__ import annotations

import ctypes
import itertools
import threading

import numpy as np

from . import _lib as L
from .future import future, make_ready_future

_NP = {L.I32: np.int32, L.U32: np.uint32, L.I64: np.int64, L.U64: np.uint64,
       L.F32: np.float32, L.F64: np.float64}


def dtype_code(dt) -> int:
    """numpy dtype / name / code -> hpxhip dtype code."""
    if isinstance(dt, int):
        if dt in _NP:
            return dt
        raise TypeError(f"unknown dtype code {dt}")
    name = np.dtype(dt).name
    if name not in L.NAME_DTYPE:
        raise TypeError(f"dtype {name} is not supported (int32/uint32/int64/uint64/float32/float64)")
    return L.NAME_DTYPE[name]


def np_dtype(code: int):
    return np.dtype(_NP[code])


# ------------------------------------------------------------------ targets
def get_device_count() -> int:
    c = ctypes.c_int()
    L.call("hpxhip_get_device_count", ctypes.byref(c))
    return c.value


class target:
    """hpx::compute::hip::target -- one GPU plus its (lazily created) stream.

    Like cuda::target, a *copy* gets its own stream (cuda_target.cpp:203-211);
    ``target(t)`` shares nothing but the device id.
    """

    def __init__(self, device: int = 0):
        if isinstance(device, target):
            device = device.device
        self.device = int(device)
        self._stream = None
        self._lock = threading.Lock()

    # native_handle().get_stream(), lazily created (cuda_target.cpp:255-280)
    @property
    def stream(self):
        if self._stream is None:
            with self._lock:
                if self._stream is None:
                    s = ctypes.c_void_p()
                    L.call("hpxhip_stream_create", self.device, ctypes.byref(s))
                    self._stream = s
        return self._stream

    def native_handle(self):
        return self

    def get_device(self) -> int:
        return self.device

    def get_stream(self):
        return self.stream

    def synchronize(self):
        """cuda_target.cpp:290-300: wait for all work on the stream."""
        if self._stream is not None:
            L.call("hpxhip_stream_synchronize", self._stream)
        device_error_check(self.device)

    def get_future(self) -> future:
        """cuda_target.cpp:307-317: a future ready when queued work is done."""
        return future.on_stream(self.stream)

    def properties(self) -> dict:
        p = L.DeviceProps()
        L.call("hpxhip_device_props_get", self.device, ctypes.byref(p))
        return {"name": p.name.decode(), "arch": p.arch.decode(), "compute_units": p.compute_units,
                "wave_size": p.wave_size, "total_global_mem": p.total_global_mem,
                "clock_khz": p.clock_khz, "memory_clock_khz": p.memory_clock_khz,
                "memory_bus_width": p.memory_bus_width, "pci_bus_id": p.pci_bus_id,
                "pci_device_id": p.pci_device_id}

    def processing_units_count(self) -> int:
        return self.properties()["compute_units"]

    def __eq__(self, other):
        return isinstance(other, target) and other.device == self.device

    def __hash__(self):
        return hash(("hip-target", self.device))

    def __repr__(self):
        return f"hip::target(device={self.device})"

    def __del__(self):
        try:
            if self._stream is not None:
                L.load().hpxhip_stream_destroy(self._stream)
        except Exception:
            pass


def get_local_targets():
    """get_cuda_targets.cpp:30-65: one target per visible device."""
    return [target(d) for d in range(get_device_count())]


def device_error_check(device: int):
    code = ctypes.c_uint32()
    L.call("hpxhip_device_error", device, ctypes.byref(code))
    if code.value:
        raise L.HpxHipError(L.ERROR_DEVICE_TIMEOUT, f"device {device} kernel error word {code.value}")


# ---------------------------------------------------------------- allocator
class allocator:
    """hpx::compute::hip::allocator<T> (cuda/allocator.hpp:36-259)."""

    def __init__(self, dtype, tgt: target | None = None):
        self.dtype = dtype_code(dtype)
        self._target = tgt if tgt is not None else target(0)

    @property
    def value_size(self) -> int:
        return L.DTYPE_SIZE[self.dtype]

    def target(self) -> target:
        return self._target

    def allocate(self, n: int) -> int:
        p = ctypes.c_void_p()
        L.call("hpxhip_malloc", self._target.device, ctypes.byref(p), int(n) * self.value_size)
        return p.value or 0

    def deallocate(self, ptr: int, n: int = 0):
        if ptr:
            L.call("hpxhip_free", ctypes.c_void_p(ptr))

    def max_size(self) -> int:
        free = ctypes.c_size_t()
        total = ctypes.c_size_t()
        L.call("hpxhip_mem_info", self._target.device, ctypes.byref(free), ctypes.byref(total))
        return total.value // self.value_size

    def __eq__(self, other):
        return isinstance(other, allocator) and other.dtype == self.dtype and other._target == self._target


# ---------------------------------------------------------------- executors
class default_executor:
    """hpx::compute::hip::default_executor (cuda/default_executor.hpp:139-260).

    Traits: parallel_execution_tag, one-/two-way, bulk one-/two-way.  The
    algorithms recognise a policy rebound to this executor and run whole-
    algorithm kernels on its target's stream.
    """
    execution_category = "parallel_execution_tag"
    is_one_way_executor = True
    is_two_way_executor = True
    is_bulk_one_way_executor = True
    is_bulk_two_way_executor = True

    def __init__(self, tgt: target | int = 0):
        self._target = tgt if isinstance(tgt, target) else target(tgt)

    def target(self) -> target:
        return self._target

    def context(self) -> target:
        return self._target

    def stream_for_call(self):
        return self._target.stream

    def processing_units_count(self) -> int:
        return self._target.processing_units_count()

    # executor customisation points for hpx_amd operations (callables taking a stream)
    def post(self, fn, *args):
        fn(self.stream_for_call(), *args)

    def sync_execute(self, fn, *args):
        s = self.stream_for_call()
        r = fn(s, *args)
        L.call("hpxhip_stream_synchronize", s)  # the stream the call ran on (concurrent_executor rotates)
        return r

    def async_execute(self, fn, *args) -> future:
        s = self.stream_for_call()
        r = fn(s, *args)
        return future.on_stream(s, thunk=lambda: r)

    def bulk_async_execute(self, fn, shape, *args):
        s = self.stream_for_call()
        for idx in shape:
            fn(s, idx, *args)
        return [future.on_stream(s)]

    def bulk_sync_execute(self, fn, shape, *args):
        for f in self.bulk_async_execute(fn, shape, *args):
            f.get()

    def synchronize(self):
        self._target.synchronize()

    def __eq__(self, other):
        return isinstance(other, default_executor) and other._target == self._target

    def __hash__(self):
        return hash(self._target)


class concurrent_executor(default_executor):
    """cuda/concurrent_executor.hpp:29-234: several streams on one device;
    successive calls rotate over the streams (independent calls overlap)."""

    def __init__(self, tgt: target | int = 0, num_streams: int = 4):
        super().__init__(tgt)
        self._targets = [target(self._target.device) for _ in range(max(1, num_streams))]
        self._rr = itertools.cycle(range(len(self._targets)))

    def stream_for_call(self):
        return self._targets[next(self._rr)].stream

    def synchronize(self):
        for t in self._targets:
            t.synchronize()


# ------------------------------------------------------------------- vector
class iterator:
    """compute::detail::iterator (detail/iterator.hpp:23-85): random access
    over a device vector; dereference on the host is a value proxy."""
    __slots__ = ("vec", "pos")

    def __init__(self, vec: "vector", pos: int):
        self.vec = vec
        self.pos = int(pos)

    @property
    def address(self) -> int:
        return self.vec.data() + self.pos * self.vec.value_size

    @property
    def dtype(self) -> int:
        return self.vec.dtype

    def target(self) -> target:
        return self.vec.target()

    def __add__(self, k):
        return iterator(self.vec, self.pos + int(k))

    __radd__ = __add__

    def __sub__(self, other):
        if isinstance(other, iterator):
            if other.vec is not self.vec:
                raise ValueError("iterators of different vectors")
            return self.pos - other.pos
        return iterator(self.vec, self.pos - int(other))

    def __eq__(self, other):
        return isinstance(other, iterator) and other.vec is self.vec and other.pos == self.pos

    def __hash__(self):
        return hash((id(self.vec), self.pos))

    def __lt__(self, other):
        return self.pos < other.pos

    def get(self):
        return self.vec[self.pos]

    def set(self, value):
        self.vec[self.pos] = value

    def __repr__(self):
        return f"iterator(pos={self.pos}, n={len(self.vec)})"


class vector:
    """hpx::compute::vector<T, hip::allocator<T>> (vector.hpp:28-372)."""

    def __init__(self, n: int = 0, alloc=None, value=None, dtype=None, tgt: target | None = None):
        if alloc is None:
            alloc = allocator(dtype if dtype is not None else np.float64, tgt)
        elif not isinstance(alloc, allocator):
            alloc = allocator(alloc, tgt)
        self._alloc = alloc
        self._size = int(n)
        self._data = alloc.allocate(self._size) if self._size else 0
        if self._size:
            # value-initialise (documented deviation from bulk_construct)
            from . import algorithms
            algorithms._fill_raw(self._alloc.target().stream, self.dtype, self._data, self._size,
                                 0 if value is None else value)

    # -- construction from / to host ---------------------------------------
    @classmethod
    def from_host(cls, arr, tgt: target | None = None, alloc: allocator | None = None):
        arr = np.ascontiguousarray(arr)
        a = alloc or allocator(arr.dtype, tgt)
        v = cls.__new__(cls)
        v._alloc = a
        v._size = arr.size
        v._data = a.allocate(arr.size) if arr.size else 0
        if arr.size:
            s = a.target().stream
            L.call("hpxhip_memcpy_async", ctypes.c_void_p(v._data), arr.ctypes.data_as(ctypes.c_void_p),
                   arr.nbytes, L.H2D, s)
            L.call("hpxhip_stream_synchronize", s)
        return v

    def to_host(self, out=None):
        arr = out if out is not None else np.empty(self._size, np_dtype(self.dtype))
        if self._size:
            s = self._alloc.target().stream
            L.call("hpxhip_memcpy_async", arr.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(self._data),
                   self._size * self.value_size, L.D2H, s)
            L.call("hpxhip_stream_synchronize", s)
        return arr

    # -- std::vector-like interface -------------------------------------------
    def __len__(self):
        return self._size

    def size(self) -> int:
        return self._size

    def capacity(self) -> int:
        return self._size

    def empty(self) -> bool:
        return self._size == 0

    def data(self) -> int:
        """device_data() (vector.hpp:253-260)."""
        return self._data

    device_data = data

    @property
    def dtype(self) -> int:
        return self._alloc.dtype

    @property
    def value_size(self) -> int:
        return self._alloc.value_size

    def get_allocator(self) -> allocator:
        return self._alloc

    def target(self) -> target:
        return self._alloc.target()

    def begin(self) -> iterator:
        return iterator(self, 0)

    def end(self) -> iterator:
        return iterator(self, self._size)

    cbegin, cend = begin, end

    def __getitem__(self, i):
        """value_proxy read: one element D2H (access_target.hpp:28-37)."""
        i = int(i)
        if i < 0:
            i += self._size
        if not 0 <= i < self._size:
            raise IndexError(i)
        out = np.empty(1, np_dtype(self.dtype))
        s = self.target().stream
        L.call("hpxhip_memcpy_async", out.ctypes.data_as(ctypes.c_void_p),
               ctypes.c_void_p(self._data + i * self.value_size), self.value_size, L.D2H, s)
        L.call("hpxhip_stream_synchronize", s)
        return out[0].item()

    def __setitem__(self, i, value):
        """value_proxy write (access_target.hpp:40-50)."""
        i = int(i)
        if i < 0:
            i += self._size
        if not 0 <= i < self._size:
            raise IndexError(i)
        src = np.array([value], np_dtype(self.dtype))
        s = self.target().stream
        L.call("hpxhip_memcpy_async", ctypes.c_void_p(self._data + i * self.value_size),
               src.ctypes.data_as(ctypes.c_void_p), self.value_size, L.H2D, s)
        L.call("hpxhip_stream_synchronize", s)

    def resize(self, n: int):
        raise NotImplementedError("compute::vector::resize is not provided for device vectors")

    def free(self):
        if self._data:
            self._alloc.target().synchronize()
            self._alloc.deallocate(self._data, self._size)
            self._data = 0
            self._size = 0

    def __del__(self):
        try:
            if getattr(self, "_data", 0):
                self._alloc.deallocate(self._data, self._size)
                self._data = 0
        except Exception:
            pass

    def __repr__(self):
        return f"compute::vector<{L.DTYPE_NAME[self.dtype]}, hip::allocator>(n={self._size}, device={self.target().device})"


def ready_future(value=None):
    return make_ready_future(value)
