"""ctypes binding of the C ABI declared in include/hpxhip.h.

The library is the product path: there is no CPU fallback.  If
``libhpxhip.so`` is missing or a call fails, an exception is raised.

Process-wide HIP runtime: PyTorch-ROCm ships its own ``libamdhip64.so``
(same SONAME ``libamdhip64.so.7`` as /opt/rocm's).  To keep exactly one HIP
runtime per process, ``torch`` is imported (when available) before the
library is loaded, so the library binds to the runtime torch already mapped.
Set ``HPXHIP_NO_TORCH=1`` to skip that (single-GPU use without torch).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhpxhip.so")

# --- enums (mirror include/hpxhip.h) ------------------------------------
I32, U32, I64, U64, F32, F64 = range(6)
PLUS, MULTIPLIES, MIN, MAX, BIT_AND, BIT_OR, BIT_XOR = range(7)
U_IDENTITY, U_SCALE, U_ADD_SCALAR, U_AFFINE, U_NEGATE, U_ABS, U_SQUARE = range(7)
B_ADD, B_TRIAD, B_SUB, B_MUL, B_AXPY, B_MIN, B_MAX = range(7)
P_LT, P_LE, P_GT, P_GE, P_EQ, P_NE, P_NOT_LT, P_BITS = range(8)
H2H, H2D, D2H, D2D, DEFAULT = range(5)
GEN_IOTA, GEN_BITS, GEN_RANGE, GEN_UNIT = range(4)
ALGO_REDUCE, ALGO_SCAN, ALGO_COPY_IF, ALGO_SORT, ALGO_SORT_BY_KEY, ALGO_MERGE, ALGO_MERGE_RUNS = range(7)
STENCIL_MAX_FUSED = 16  # HPXHIP_STENCIL_MAX_FUSED

SUCCESS = 0
ERROR_INVALID_ARGUMENT = 10001
ERROR_UNSUPPORTED = 10002
ERROR_DEVICE_TIMEOUT = 10003
ERROR_OUT_OF_MEMORY = 10004
ERROR_NOT_READY = 10005

DTYPE_SIZE = {I32: 4, U32: 4, I64: 8, U64: 8, F32: 4, F64: 8}
DTYPE_NAME = {I32: "int32", U32: "uint32", I64: "int64", U64: "uint64", F32: "float32", F64: "float64"}
NAME_DTYPE = {v: k for k, v in DTYPE_NAME.items()}
CTYPE = {I32: ctypes.c_int32, U32: ctypes.c_uint32, I64: ctypes.c_int64,
         U64: ctypes.c_uint64, F32: ctypes.c_float, F64: ctypes.c_double}


class HpxHipError(RuntimeError):
    """A failing C-ABI call (hipError_t or HPXHIP_ERROR_* status)."""

    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: [{status}] {error_string(status)}")


class OutOfMemory(HpxHipError, MemoryError):
    """hpx::out_of_memory analogue (hpx/compute/cuda/allocator.hpp:118-124)."""


class exception_list(HpxHipError):
    """hpx::exception_list (hpx/exception_list.hpp:28-97): the error a
    parallel algorithm reports.  Every failure other than an allocation
    failure (OutOfMemory, a MemoryError) is wrapped in one
    (parallel/exception_list.hpp:20-111); iterating yields the original
    exceptions."""

    def __init__(self, exceptions=()):
        self.exceptions = list(exceptions)
        first = self.exceptions[0] if self.exceptions else None
        self.status = getattr(first, "status", ERROR_INVALID_ARGUMENT)
        RuntimeError.__init__(self, "; ".join(str(e) for e in self.exceptions) or "hpx::exception_list")

    def __len__(self):
        return len(self.exceptions)

    def size(self):
        return len(self.exceptions)

    def __iter__(self):
        return iter(self.exceptions)


class DeviceProps(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 256),
        ("arch", ctypes.c_char * 64),
        ("compute_units", ctypes.c_int),
        ("wave_size", ctypes.c_int),
        ("max_threads_per_block", ctypes.c_int),
        ("clock_khz", ctypes.c_int),
        ("memory_clock_khz", ctypes.c_int),
        ("memory_bus_width", ctypes.c_int),
        ("total_global_mem", ctypes.c_size_t),
        ("lds_per_block", ctypes.c_size_t),
        ("pci_bus_id", ctypes.c_int),
        ("pci_device_id", ctypes.c_int),
    ]


CALLBACK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_u64 = ctypes.c_uint64
_i = ctypes.c_int
_f = ctypes.c_float
_d = ctypes.c_double

# name -> argtypes (restype int unless noted)
SIGNATURES = {
    "hpxhip_abi_version": [],
    "hpxhip_debug_inject_error": [_i, _i],
    "hpxhip_debug_raise_device_error": [ctypes.c_void_p, ctypes.c_uint32],
    "hpxhip_debug_inject_event_error": [_i, _i],
    "hpxhip_device_error": [_i, ctypes.POINTER(ctypes.c_uint32)],
    "hpxhip_get_device_count": [ctypes.POINTER(_i)],
    "hpxhip_set_device": [_i],
    "hpxhip_get_device": [ctypes.POINTER(_i)],
    "hpxhip_device_props_get": [_i, ctypes.POINTER(DeviceProps)],
    "hpxhip_device_synchronize": [_i],
    "hpxhip_enable_peer_access": [_i, _i],
    "hpxhip_can_access_peer": [_i, _i, ctypes.POINTER(_i)],
    "hpxhip_stream_create": [_i, ctypes.POINTER(_vp)],
    "hpxhip_stream_destroy": [_vp],
    "hpxhip_stream_synchronize": [_vp],
    "hpxhip_stream_query": [_vp],
    "hpxhip_stream_add_callback": [_vp, CALLBACK, _vp],
    "hpxhip_event_create": [ctypes.POINTER(_vp)],
    "hpxhip_event_create_on": [_i, _i, ctypes.POINTER(_vp)],
    "hpxhip_stream_device": [_vp, ctypes.POINTER(_i)],
    "hpxhip_event_destroy": [_vp],
    "hpxhip_event_record": [_vp, _vp],
    "hpxhip_event_synchronize": [_vp],
    "hpxhip_event_query": [_vp],
    "hpxhip_event_elapsed_ms": [_vp, _vp, ctypes.POINTER(_f)],
    "hpxhip_stream_wait_event": [_vp, _vp],
    "hpxhip_malloc": [_i, ctypes.POINTER(_vp), _sz],
    "hpxhip_free": [_vp],
    "hpxhip_malloc_host": [ctypes.POINTER(_vp), _sz],
    "hpxhip_free_host": [_vp],
    "hpxhip_mem_info": [_i, ctypes.POINTER(_sz), ctypes.POINTER(_sz)],
    "hpxhip_memcpy_async": [_vp, _vp, _sz, _i, _vp],
    "hpxhip_memcpy_peer_async": [_vp, _i, _vp, _i, _sz, _vp],
    "hpxhip_memset_async": [_vp, _i, _sz, _vp],
    "hpxhip_scratch_bytes": [_i, _i, _i, _u64, ctypes.POINTER(_sz)],
    "hpxhip_stream_scratch": [_vp, _sz, ctypes.POINTER(_vp)],
    "hpxhip_device_error_word": [_vp, ctypes.POINTER(_vp)],
    "hpxhip_generate": [_i, _i, _u64, ctypes.c_int64, ctypes.c_int64, _vp, _u64, _vp],
    "hpxhip_generate_at": [_i, _i, _u64, _u64, ctypes.c_int64, ctypes.c_int64, _vp, _u64, _vp],
    "hpxhip_fill": [_i, _vp, _vp, _u64, _vp],
    "hpxhip_copy": [_i, _vp, _vp, _u64, _vp],
    "hpxhip_for_each": [_i, _i, _vp, _vp, _u64, _vp],
    "hpxhip_transform": [_i, _i, _i, _i, _vp, _vp, _vp, _u64, _vp],
    "hpxhip_transform_binary": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _u64, _vp],
    "hpxhip_transform_strided": [_i, _i, _i, _i, _vp, _vp, ctypes.c_int64, _vp, ctypes.c_int64, _u64, _vp],
    "hpxhip_transform_binary_strided": [_i, _i, _i, _i, _vp, _vp, ctypes.c_int64, _vp, ctypes.c_int64, _vp,
                                        ctypes.c_int64, _u64, _vp],
    "hpxhip_transform_reduce": [_i, _i, _i, _i, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _sz],
    "hpxhip_transform_reduce_binary": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _sz],
    "hpxhip_fold": [_i, _i, _vp, _vp, _u64, _vp, _vp],
    "hpxhip_fold_exclusive": [_i, _i, _vp, _vp, _u64, _vp, _vp],
    "hpxhip_scan": [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _sz],
    "hpxhip_copy_if": [_i, _i, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _sz],
    "hpxhip_sort": [_i, _vp, _u64, _i, _vp, _vp, _sz],
    "hpxhip_sort_by_key": [_i, _i, _vp, _vp, _u64, _i, _vp, _vp, _sz],
    "hpxhip_merge": [_i, _vp, _u64, _vp, _u64, _vp, _i, _vp, _vp, _sz],
    "hpxhip_merge_runs": [_i, _vp, _vp, _i, _vp, _i, _vp, _vp, _sz],
    "hpxhip_unsorted_pairs": [_i, _vp, _u64, _i, _vp, _vp],
    "hpxhip_sorted_bounds": [_i, _vp, _u64, _vp, _u64, _i, _i, _vp, _vp],
    "hpxhip_stencil_heat_step": [_vp, _vp, _u64, _vp, _vp, _d, _d, _d, _vp],
    "hpxhip_stencil_heat_run": [_vp, _vp, _u64, _u64, _d, _d, _d, _vp],
    "hpxhip_stencil_heat_steps": [_vp, _vp, _u64, _u64, _u64, _vp, _vp, _i, _d, _d, _d, _vp],
    "hpxhip_stencil_heat_run_fused": [_vp, _vp, _u64, _u64, _d, _d, _d, ctypes.POINTER(_i), _vp],
}

_lib = None
_lock = threading.Lock()


def _preload_torch():
    if os.environ.get("HPXHIP_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401  (binds the process to torch's HIP runtime)
    except Exception:
        pass


ABI_VERSION = 1  # HPXHIP_ABI_VERSION, include/hpxhip.h


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("HPXHIP_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise ImportError(
                f"hpx_amd: HIP library not built ({p}); run `make lib` or "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        _preload_torch()
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        lib.hpxhip_error_string.argtypes = [ctypes.c_int]
        lib.hpxhip_error_string.restype = ctypes.c_char_p
        # the binding and the library must agree on the C ABI (include/hpxhip.h)
        got = lib.hpxhip_abi_version()
        if got != ABI_VERSION:
            raise ImportError(f"hpx_amd: {p} implements C ABI version {got}, this binding expects {ABI_VERSION}")
        _lib = lib
        return lib


def error_string(status: int) -> str:
    try:
        return load().hpxhip_error_string(status).decode()
    except Exception:  # pragma: no cover - library unavailable
        return "unknown"


def check(status: int, what: str = "hpxhip call") -> None:
    if status == SUCCESS:
        return
    if status == ERROR_OUT_OF_MEMORY:
        raise OutOfMemory(status, what)
    raise HpxHipError(status, what)


def call(name: str, *args) -> None:
    """Call C-ABI function `name` and raise on a non-zero status."""
    check(getattr(load(), name)(*args), name)


def scalar_buf(dtype: int, value):
    """A ctypes object holding one element of `dtype` (host pointer arg)."""
    arr = (CTYPE[dtype] * 1)()
    arr[0] = value
    return arr


def scalars_buf(dtype: int, values):
    arr = (CTYPE[dtype] * max(2, len(values)))()
    for i, v in enumerate(values):
        arr[i] = v
    return arr
