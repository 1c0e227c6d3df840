"""hpx::parallel algorithms over hip device iterators.

Each function keeps the reference's name, argument order and return
convention (value for ``seq``/``par``, ``future`` for ``par(task)``) and
calls one whole-algorithm entry point of the C ABI (include/hpxhip.h):

  for_each / for_each_n      hpx/parallel/algorithms/for_each.hpp:369-552
  fill / fill_n              fill.hpp:86,159
  copy / copy_n              copy.hpp:88-114,209 (+ util/transfer.hpp for
                             host<->device ranges, cuda/transfer.hpp:188-348)
  copy_if                    copy.hpp:401-494,585
  transform (1, 2, 2')       transform.hpp:138-182,411-461,643-694,304/625/862
  reduce                     reduce.hpp:200/271/344
  transform_reduce           transform_reduce.hpp:254; binary: transform_reduce_binary.hpp:323/432
  inclusive_scan             inclusive_scan.hpp:288/320/409/511/591
  exclusive_scan             exclusive_scan.hpp:292/374
  transform_inclusive_scan   transform_inclusive_scan.hpp:320/445
  transform_exclusive_scan   transform_exclusive_scan.hpp:317
  sort / sort_by_key         sort.hpp:364, sort_by_key.hpp:42-78
  generate (splitmix/iota)   generate.hpp (device generator functors)
  for_loop / for_loop_n      for_loop.hpp:808; for_loop_strided 604,
  for_loop_n_strided         1014 (inductions: for_loop_induction.hpp;
                             reductions: for_loop_reduction.hpp:35-231)

A policy must be rebound to a hip executor (``par.on(hip_exec)``) or all
iterators must be device iterators of one target (then that target's
stream is used).  There is no host fallback: host ranges are only accepted
as the source/destination of ``copy`` (a transfer).
"""
from __future__ import annotations

import ctypes
import functools
import threading

import numpy as np

from . import _lib as L
from . import functional as F
from .compute import (default_executor, dtype_code, iterator, np_dtype, target)
from .execution import policy as _policy
from .future import future, make_ready_future


# ------------------------------------------------------------------ helpers
class _slots:
    """Per-target ring of small device result slots + pinned host mirrors."""
    N = 256

    def __init__(self, tgt: target):
        self.dev = ctypes.c_void_p()
        L.call("hpxhip_malloc", tgt.device, ctypes.byref(self.dev), 16 * self.N)
        self.host = ctypes.c_void_p()
        L.call("hpxhip_malloc_host", ctypes.byref(self.host), 16 * self.N)
        self.i = 0
        self.lock = threading.Lock()

    def next(self):
        with self.lock:
            self.i = (self.i + 1) % self.N
            return self.dev.value + 16 * self.i, self.host.value + 16 * self.i


_slot_lock = threading.Lock()


def _slots_for(tgt: target) -> _slots:
    s = getattr(tgt, "_hpx_slots", None)
    if s is None:
        with _slot_lock:
            s = getattr(tgt, "_hpx_slots", None)
            if s is None:
                s = _slots(tgt)
                tgt._hpx_slots = s
    return s


def _read_host(addr: int, dtype: int):
    return np.frombuffer((ctypes.c_char * 8).from_address(addr), dtype=np_dtype(dtype), count=1)[0].item()


def _exec_of(pol) -> tuple:
    if not isinstance(pol, _policy):
        raise TypeError(f"first argument must be an execution policy, got {pol!r}")
    return pol.executor


def _context(pol, *iters):
    """-> (stream, target, is_task) for a policy and its device iterators."""
    ex = _exec_of(pol)
    devs = [it for it in iters if isinstance(it, iterator)]
    if ex is not None:
        if not isinstance(ex, default_executor):
            raise TypeError(f"hpx_amd algorithms run on hip executors, got {type(ex).__name__}")
        tgt = ex.target()
        stream = ex.stream_for_call()
    else:
        if not devs:
            raise TypeError("policy has no hip executor and no device iterators: host algorithms "
                            "are HPX's own, hpx_amd provides the hip executor path")
        tgt = devs[0].target()
        stream = tgt.stream
    for it in devs:
        if it.target().device != tgt.device:
            raise ValueError(f"iterator on device {it.target().device} used with target on device {tgt.device}")
    return stream, tgt, pol.is_task


def _check_range(first, last):
    if not isinstance(first, iterator) or not isinstance(last, iterator):
        raise TypeError("expected device iterators (hpx_amd.compute.iterator)")
    n = last - first
    if n < 0:
        raise ValueError("last precedes first")
    return n


def _finish(is_task, stream, tgt, value_thunk):
    """Return the algorithm result: a value (sync) or a future (task)."""
    if is_task:
        return future.on_stream(stream, thunk=value_thunk)
    L.call("hpxhip_stream_synchronize", stream)
    from .compute import device_error_check
    device_error_check(tgt.device)
    return value_thunk()


def _vp(addr):
    return ctypes.c_void_p(addr)


def _fill_raw(stream, dtype, addr, n, value):
    buf = L.scalar_buf(dtype, value)
    L.call("hpxhip_fill", dtype, buf, _vp(addr), n, stream)


def _acc_dtype(elem: int, init) -> int:
    """HPX's T is the init's type: float init over integers -> double."""
    if isinstance(init, np.generic):
        return dtype_code(init.dtype)
    if isinstance(init, float) and elem not in (L.F32, L.F64):
        return L.F64
    return elem


def _compute_dtype(elem: int, fn) -> int:
    c = getattr(fn, "compute", None)
    return dtype_code(c) if c else elem


# ------------------------------------------------------------- for_each etc
def generate(pol, first, last, kind: str = "splitmix", seed: int = 0x5EED, lo: int = 0, hi: int = 0):
    """hpx::parallel::generate with a counter-based generator functor:
    kind = 'iota' (lo + i), 'bits', 'range' ([lo, hi]) or 'unit' ([0,1))."""
    kinds = {"iota": L.GEN_IOTA, "bits": L.GEN_BITS, "splitmix": L.GEN_BITS, "range": L.GEN_RANGE,
             "unit": L.GEN_UNIT}
    n = _check_range(first, last)
    stream, tgt, is_task = _context(pol, first)
    L.call("hpxhip_generate", first.dtype, kinds[kind], seed, lo, hi, _vp(first.address), n, stream)
    return _finish(is_task, stream, tgt, lambda: last)


def fill(pol, first, last, value):
    n = _check_range(first, last)
    stream, tgt, is_task = _context(pol, first)
    _fill_raw(stream, first.dtype, first.address, n, value)
    return _finish(is_task, stream, tgt, lambda: None)


def fill_n(pol, first, count, value):
    return fill(pol, first, first + count, value) if count > 0 else _finish(
        pol.is_task, *_context(pol, first)[:2], lambda: first)


def for_each(pol, first, last, f):
    """for_each.hpp:540: applies f in place; returns last (future for task)."""
    f = F.require(f, F.Unary, "for_each")
    n = _check_range(first, last)
    stream, tgt, is_task = _context(pol, first)
    sc = L.scalars_buf(first.dtype, f.scalars)
    L.call("hpxhip_for_each", first.dtype, f.kind, sc, _vp(first.address), n, stream)
    return _finish(is_task, stream, tgt, lambda: last)


def for_each_n(pol, first, count, f):
    return for_each(pol, first, first + max(0, count), f)


# ---------------------------------------------------------------- copy etc
def copy(pol, first, last, dest):
    """copy.hpp:209.  Device->device runs the copy kernel; device<->host
    ranges (numpy arrays) are transfers (util/transfer.hpp -> memcpy)."""
    if isinstance(first, np.ndarray) and isinstance(dest, iterator):
        arr = np.ascontiguousarray(first if last is None else first[:last])
        stream, tgt, is_task = _context(pol, dest)
        if np_dtype(dest.dtype) != arr.dtype:
            raise TypeError("host/device dtype mismatch")
        L.call("hpxhip_memcpy_async", _vp(dest.address), arr.ctypes.data_as(ctypes.c_void_p), arr.nbytes,
               L.H2D, stream)
        keep = arr  # noqa: F841 (alive until synchronised)
        end = dest + arr.size
        return _finish(is_task, stream, tgt, lambda: (keep, end)[1])
    n = _check_range(first, last)
    if isinstance(dest, np.ndarray):
        stream, tgt, is_task = _context(pol, first)
        if dest.size < n or not dest.flags.c_contiguous or np_dtype(first.dtype) != dest.dtype:
            raise TypeError("destination array too small, non-contiguous or of another dtype")
        L.call("hpxhip_memcpy_async", dest.ctypes.data_as(ctypes.c_void_p), _vp(first.address),
               n * first.vec.value_size, L.D2H, stream)
        return _finish(is_task, stream, tgt, lambda: dest)
    stream, tgt, is_task = _context(pol, first, dest)
    if first.dtype != dest.dtype:
        return transform(pol, first, last, dest, F.identity())
    L.call("hpxhip_copy", first.dtype, _vp(first.address), _vp(dest.address), n, stream)
    return _finish(is_task, stream, tgt, lambda: (last, dest + n))


def copy_n(pol, first, count, dest):
    return copy(pol, first, first + count, dest)


def copy_if(pol, first, last, dest, pred):
    """copy.hpp:585: stable compaction; returns (last, dest_end)."""
    pred = F.require(pred, F.Predicate, "copy_if")
    n = _check_range(first, last)
    stream, tgt, is_task = _context(pol, first, dest)
    if first.dtype != dest.dtype:
        raise TypeError("copy_if: source and destination dtypes differ")
    dev, host = _slots_for(tgt).next()
    arg = L.scalar_buf(first.dtype, pred.arg)
    L.call("hpxhip_copy_if", first.dtype, pred.kind, arg, _vp(first.address), _vp(dest.address), n,
           _vp(dev), stream, None, 0)
    L.call("hpxhip_memcpy_async", _vp(host), _vp(dev), 8, L.D2H, stream)
    return _finish(is_task, stream, tgt, lambda: (last, dest + _read_host(host, L.U64)))


# --------------------------------------------------------------- transform
def transform(pol, *args):
    """transform.hpp overloads:
         (first, last, dest, f)                    unary      (304)
         (first1, last1, first2, dest, f)          binary     (625)
         (first1, last1, first2, last2, dest, f)   binary2    (862; min length)
    Returns (in_last, out_last) like the reference's tagged pair."""
    if len(args) == 4:
        first, last, dest, f = args
        f = F.require(f, F.Unary, "transform")
        n = _check_range(first, last)
        stream, tgt, is_task = _context(pol, first, dest)
        cdt = _compute_dtype(first.dtype, f)
        sc = L.scalars_buf(cdt, f.scalars)
        L.call("hpxhip_transform", first.dtype, cdt, dest.dtype, f.kind, sc, _vp(first.address),
               _vp(dest.address), n, stream)
        return _finish(is_task, stream, tgt, lambda: (last, dest + n))
    if len(args) == 5:
        first1, last1, first2, dest, f = args
        n = _check_range(first1, last1)
    elif len(args) == 6:
        first1, last1, first2, last2, dest, f = args
        n = min(_check_range(first1, last1), _check_range(first2, last2))  # transform.hpp:683-685
    else:
        raise TypeError("transform: unsupported overload")
    f = F.require(f, F.Binary, "transform")
    stream, tgt, is_task = _context(pol, first1, first2, dest)
    if first1.dtype != first2.dtype:
        raise TypeError("transform: both input ranges must have the same dtype")
    cdt = _compute_dtype(first1.dtype, f)
    sc = L.scalars_buf(cdt, f.scalars)
    L.call("hpxhip_transform_binary", first1.dtype, cdt, dest.dtype, f.kind, sc, _vp(first1.address),
           _vp(first2.address), _vp(dest.address), n, stream)
    return _finish(is_task, stream, tgt, lambda: (first1 + n, first2 + n, dest + n))


# -------------------------------------------------------------- reductions
def reduce(pol, first, last, init=None, op=F.plus):
    """reduce.hpp:200/271/344: init defaults to T(), op to std::plus."""
    return transform_reduce(pol, first, last, 0 if init is None else init, op, F.identity())


def transform_reduce(pol, *args):
    """transform_reduce.hpp:254 (first, last, init, red_op, conv_op) and
    transform_reduce_binary.hpp:323/432 (first1, last1, first2, init[, red_op, conv_op])."""
    if len(args) >= 4 and isinstance(args[2], iterator):
        first1, last1, first2, init = args[:4]
        red = args[4] if len(args) > 4 else F.plus
        conv = args[5] if len(args) > 5 else F.multiply()
        red = F.require(red, F.BinaryOp, "transform_reduce")
        conv = F.require(conv, F.Binary, "transform_reduce")
        n = _check_range(first1, last1)
        stream, tgt, is_task = _context(pol, first1, first2)
        adt = _acc_dtype(first1.dtype, init)
        dev, host = _slots_for(tgt).next()
        L.call("hpxhip_transform_reduce_binary", first1.dtype, adt, red.kind, conv.kind,
               L.scalars_buf(adt, conv.scalars), L.scalar_buf(adt, init), _vp(first1.address),
               _vp(first2.address), n, _vp(dev), stream, None, 0)
    else:
        first, last, init, red, conv = args
        red = F.require(red, F.BinaryOp, "transform_reduce")
        conv = F.require(conv, F.Unary, "transform_reduce")
        n = _check_range(first, last)
        stream, tgt, is_task = _context(pol, first)
        adt = _acc_dtype(first.dtype, init)
        dev, host = _slots_for(tgt).next()
        L.call("hpxhip_transform_reduce", first.dtype, adt, red.kind, conv.kind,
               L.scalars_buf(adt, conv.scalars), L.scalar_buf(adt, init), _vp(first.address), n,
               _vp(dev), stream, None, 0)
    L.call("hpxhip_memcpy_async", _vp(host), _vp(dev), 8, L.D2H, stream)
    return _finish(is_task, stream, tgt, lambda: _read_host(host, adt))


# -------------------------------------------------------------------- scans
def _scan(pol, first, last, dest, op, init, inclusive, conv, prefix_dev=None):
    op = F.require(op, F.BinaryOp, "scan")
    conv = F.require(conv, F.Unary, "scan")
    n = _check_range(first, last)
    stream, tgt, is_task = _context(pol, first, dest)
    if first.dtype != dest.dtype:
        raise TypeError("scan: source and destination dtypes differ")
    dt = first.dtype
    L.call("hpxhip_scan", dt, op.kind, 1 if inclusive else 0, conv.kind, L.scalars_buf(dt, conv.scalars),
           L.scalar_buf(dt, init), None if prefix_dev is None else _vp(prefix_dev), _vp(first.address),
           _vp(dest.address), n, stream, None, 0)
    return _finish(is_task, stream, tgt, lambda: dest + n)


def inclusive_scan(pol, first, last, dest, *args):
    """Overloads (op, init) 288, (init, op) 320, (init) 409, (op) 511, () 591.
    Without init the reference uses value_type() (inclusive_scan.hpp:526,606)."""
    op, init = F.plus, 0
    if len(args) == 2:
        if isinstance(args[0], F.BinaryOp):
            op, init = args
        else:
            init, op = args
    elif len(args) == 1:
        if isinstance(args[0], F.BinaryOp):
            op = args[0]
        else:
            init = args[0]
    elif args:
        raise TypeError("inclusive_scan: unsupported overload")
    return _scan(pol, first, last, dest, op, init, True, F.identity())


def exclusive_scan(pol, first, last, dest, init, op=F.plus):
    """exclusive_scan.hpp:292 (init, op) / 374 (init)."""
    return _scan(pol, first, last, dest, op, init, False, F.identity())


def transform_inclusive_scan(pol, first, last, dest, op, conv, init=0):
    """transform_inclusive_scan.hpp:320 (op, conv, init) / 445 (op, conv)."""
    return _scan(pol, first, last, dest, op, init, True, conv)


def transform_exclusive_scan(pol, first, last, dest, init, op, conv):
    """transform_exclusive_scan.hpp:317 (init, op, conv)."""
    return _scan(pol, first, last, dest, op, init, False, conv)


# --------------------------------------------------------------------- sort
def sort(pol, first, last=None, comp=F.less):
    """sort.hpp:364; comp = std::less (default) or std::greater.  With a
    container instead of an iterator pair -- sort(pol, rng[, comp]) -- the
    range overload of container_algorithms/sort.hpp:102 (hpx::parallel::sort
    over begin(rng), end(rng)); returns the range's end iterator."""
    from .compute import vector as _vector
    if isinstance(first, _vector):
        rng = first
        if last is not None:
            comp = last
        return sort(pol, rng.begin(), rng.end(), comp)
    comp = F.require(comp, F.Compare, "sort")
    n = _check_range(first, last)
    stream, tgt, is_task = _context(pol, first)
    L.call("hpxhip_sort", first.dtype, _vp(first.address), n, 1 if comp.descending else 0, stream, None, 0)
    return _finish(is_task, stream, tgt, lambda: last)


def is_sorted(pol, first, last, comp=F.less):
    """is_sorted.hpp:40-120: True iff no adjacent pair is ordered after one
    another under comp (std::less / std::greater, the sort's key order),
    counted on the device (hpxhip_unsorted_pairs); a future under par(task)."""
    comp = F.require(comp, F.Compare, "is_sorted")
    n = _check_range(first, last)
    stream, tgt, is_task = _context(pol, first)
    dev, host = _slots_for(tgt).next()
    L.call("hpxhip_unsorted_pairs", first.dtype, _vp(first.address), n, 1 if comp.descending else 0, _vp(dev),
           stream)
    L.call("hpxhip_memcpy_async", _vp(host), _vp(dev), 8, L.D2H, stream)
    return _finish(is_task, stream, tgt, lambda: _read_host(host, L.U64) == 0)


def sort_by_key(pol, key_first, key_last, value_first, comp=F.less):
    """sort_by_key.hpp:42-78 (stable here); returns (key_last, value_last)."""
    comp = F.require(comp, F.Compare, "sort_by_key")
    n = _check_range(key_first, key_last)
    stream, tgt, is_task = _context(pol, key_first, value_first)
    L.call("hpxhip_sort_by_key", key_first.dtype, value_first.dtype, _vp(key_first.address),
           _vp(value_first.address), n, 1 if comp.descending else 0, stream, None, 0)
    return _finish(is_task, stream, tgt, lambda: (key_last, value_first + n))


def merge(pol, first1, last1, first2, last2, dest, comp=F.less):
    """merge.hpp:476: stable merge of two sorted ranges into dest (equal keys:
    the first range's first, merge.hpp:52-80); returns the tagged tuple
    (last1, last2, dest_end), or its future under par(task)."""
    comp = F.require(comp, F.Compare, "merge")
    n1 = _check_range(first1, last1)
    n2 = _check_range(first2, last2)
    if not isinstance(dest, iterator):
        raise TypeError("merge: dest must be a device iterator")
    if not (first1.dtype == first2.dtype == dest.dtype):
        raise TypeError("merge: the ranges and dest must have one dtype")
    stream, tgt, is_task = _context(pol, first1, first2, dest)
    L.call("hpxhip_merge", first1.dtype, _vp(first1.address), n1, _vp(first2.address), n2, _vp(dest.address),
           1 if comp.descending else 0, stream, None, 0)
    return _finish(is_task, stream, tgt, lambda: (last1, last2, dest + (n1 + n2)))


# ------------------------------------------------------------------ for_loop
class induction:
    """for_loop_induction.hpp:210-219: an induction variable whose value at
    iteration i is value + stride * i (pointer / iterator inductions here)."""
    __slots__ = ("value", "stride")

    def __init__(self, value, stride: int = 1):
        self.value, self.stride = value, int(stride)   # stride may be negative (a difference type)


class reduction:
    """for_loop_reduction.hpp:35-132 reduction(var, identity, combiner).

    ``var`` is the live-out object: a one-element (or 0-d) numpy array, the
    Python stand-in for the reference's ``T&``.  The reference gives every OS
    thread a view initialised with ``identity`` and, at loop exit, folds
    ``var = op(var, view_k)`` over the views (62-66).  Here one launch forms a
    single view, ``identity (op) f(x_0) (op) ... (op) f(x_{n-1})`` (the
    transform_reduce kernel with init = identity), and the exit folds it into
    ``var``.  With a neutral identity -- every reduction_* helper without an
    explicit identity -- this equals the reference's result for any thread
    count; with a non-neutral explicit identity the reference's result
    depends on its OS thread count, and ours is the one-view result."""
    __slots__ = ("var", "identity", "op")

    def __init__(self, var, identity, op):
        if not (isinstance(var, np.ndarray) and var.size == 1):
            raise TypeError("reduction: the live-out variable must be a one-element numpy array (T&)")
        self.var, self.identity, self.op = var, identity, F.require(op, F.BinaryOp, "reduction")


def _ident(var, value):
    if not isinstance(var, np.ndarray):
        raise TypeError("reduction: the live-out variable must be a one-element numpy array (T&)")
    return var.dtype.type(value)


def reduction_plus(var, identity=None):
    """for_loop_reduction.hpp:135-147 (identity T())."""
    return reduction(var, _ident(var, 0) if identity is None else identity, F.plus)


def reduction_multiplies(var, identity=None):
    """for_loop_reduction.hpp:149-161 (identity T(1))."""
    return reduction(var, _ident(var, 1) if identity is None else identity, F.multiplies)


def reduction_bit_and(var, identity=None):
    """for_loop_reduction.hpp:163-175 (identity ~T())."""
    return reduction(var, ~_ident(var, 0) if identity is None else identity, F.bit_and)


def reduction_bit_or(var, identity=None):
    """for_loop_reduction.hpp:177-189 (identity T())."""
    return reduction(var, _ident(var, 0) if identity is None else identity, F.bit_or)


def reduction_bit_xor(var, identity=None):
    """for_loop_reduction.hpp:191-203 (identity T())."""
    return reduction(var, _ident(var, 0) if identity is None else identity, F.bit_xor)


def reduction_min(var, identity=None):
    """for_loop_reduction.hpp:205-217 (identity = var's current value)."""
    return reduction(var, _ident(var, var.reshape(-1)[0]) if identity is None else identity, F.minimum)


def reduction_max(var, identity=None):
    """for_loop_reduction.hpp:219-231 (identity = var's current value)."""
    return reduction(var, _ident(var, var.reshape(-1)[0]) if identity is None else identity, F.maximum)


def _for_loop_reduce(pol, n, vars_, reds, parts):
    """The for_loop with reductions: each reduction's body (an accumulate
    naming its position) feeds the transform_reduce kernels (unary or binary
    map) -- one launch per reduction, all on the loop's stream -- and the
    loop exit folds every view into its live-out variable
    (for_loop_reduction.hpp:60-66), once all of them are back."""
    launches = []
    for red, body in zip(reds, parts):
        try:
            ins = [vars_[i] for i in body.ins]
        except IndexError:
            raise IndexError("for_loop_n: loop body refers to a variable that is not passed") from None
        if not all(isinstance(v, iterator) for v in ins):
            raise TypeError("for_loop_n: the reduction body must read device iterators")
        if n > 0 and any(it.pos < 0 or it.pos + n - 1 >= it.vec.size() for it in ins):
            raise ValueError("for_loop_n: an induction walks outside its vector")
        if isinstance(body.fn, F.Binary) and ins[0].dtype != ins[1].dtype:
            raise TypeError("for_loop_n: both inputs of a binary body must have one dtype")
        launches.append((red, body, ins))
    stream, tgt, is_task = _context(pol, *[it for _, _, ins in launches for it in ins])
    views = []
    for red, body, ins in launches:
        adt = dtype_code(red.var.dtype)
        dev, host = _slots_for(tgt).next()
        fn = body.fn
        if isinstance(fn, F.Unary):
            L.call("hpxhip_transform_reduce", ins[0].dtype, adt, red.op.kind, fn.kind, L.scalars_buf(adt, fn.scalars),
                   L.scalar_buf(adt, red.identity), _vp(ins[0].address), n, _vp(dev), stream, None, 0)
        else:
            L.call("hpxhip_transform_reduce_binary", ins[0].dtype, adt, red.op.kind, fn.kind,
                   L.scalars_buf(adt, fn.scalars), L.scalar_buf(adt, red.identity), _vp(ins[0].address),
                   _vp(ins[1].address), n, _vp(dev), stream, None, 0)
        L.call("hpxhip_memcpy_async", _vp(host), _vp(dev), 8, L.D2H, stream)
        views.append((red, host, adt))

    def exit_iteration():
        for red, host, adt in views:
            flat = red.var.reshape(-1)
            with np.errstate(over="ignore"):  # integer combiners wrap like the kernels (and T in C++)
                flat[0] = red.op(flat[0], red.var.dtype.type(_read_host(host, adt)))

    return _finish(is_task, stream, tgt, exit_iteration)


def for_loop_n(pol, first, count, *args):
    return _for_loop(pol, first, 1, count, *args)


def for_loop_strided(pol, first, last, stride, *args):
    """for_loop.hpp:604 for_loop_strided(policy, first, last, stride, args..., f):
    the loop variable visits first, first + stride, ... while it precedes
    last (follows it for a negative stride); inductions take their ordinal
    value (base + induction stride * k at the k-th application)."""
    stride = int(stride)
    if stride == 0:
        raise ValueError("for_loop_strided: stride must not be 0")
    n = _check_range(first, last) if stride > 0 else _check_range(last, first)
    count = (n + abs(stride) - 1) // abs(stride)
    return _for_loop(pol, first, stride, count, *args)


def for_loop_n_strided(pol, first, count, stride, *args):
    """for_loop.hpp:1014 for_loop_n_strided(policy, first, size, stride, args..., f)."""
    stride = int(stride)
    if stride == 0:
        raise ValueError("for_loop_n_strided: stride must not be 0")
    return _for_loop(pol, first, stride, count, *args)


def _for_loop(pol, first, first_stride, count, *args):
    """for_loop.hpp:808 for_loop_n(policy, first, size, inductions..., f) as
    for_loop_compute.cu uses it: the loop iterator and pointer inductions
    walk device ranges in lock step (induction i's value at iteration k is
    base + stride*k, for_loop_induction.hpp:210-219) and the body writes one
    of them from one or two others (functional.assign).  All-stride-1 loops
    run on the vectorised elementwise transform kernels, others on the
    strided ones; returns None (future<void> under par(task)).  With
    ``reduction`` arguments (for_loop_reduction.hpp; any number of them) the
    body is a functional.accumulate, or functional.accumulate_all of one
    accumulate per reduction, and the loop runs on the transform_reduce
    kernels."""
    if not args:
        raise TypeError("for_loop_n: missing loop body")
    *inds, body = args
    reds = [a for a in inds if isinstance(a, reduction)]
    if reds and first_stride != 1:
        raise ValueError("for_loop_n: a reduction loop walks its loop variable with stride 1")
    if reds:
        # any number of reductions (for_loop.hpp:802-812): a body that
        # accumulates into each of them -- accumulate() for one,
        # accumulate_all(accumulate(...), ...) for several
        if isinstance(body, F.Accumulate):
            parts = (body,)
        else:
            parts = F.require(body, F.Accumulates, "for_loop_n").parts
        if not isinstance(first, iterator):
            raise TypeError("for_loop_n: the loop variable must be a device iterator")
        for ind in inds:
            if isinstance(ind, induction) and ind.stride != 1:
                raise ValueError("for_loop_n: a reduction loop reads its inductions with stride 1 "
                                 "(the transform_reduce kernels are contiguous)")
        n = int(count)
        if n < 0:
            raise ValueError("for_loop_n: negative count")
        vars_ = [first] + [a.value if isinstance(a, induction) else a for a in inds]
        named = []
        for a in parts:
            if not (0 <= a.red < len(vars_)) or not isinstance(vars_[a.red], reduction):
                raise IndexError("for_loop_n: accumulate() must name a reduction's position")
            named.append(vars_[a.red])
        if len(named) != len(reds) or any(all(r is not x for x in named) for r in reds):
            raise ValueError("for_loop_n: every reduction needs exactly one accumulate() in the body")
        return _for_loop_reduce(pol, n, vars_, named, parts)
    body = F.require(body, F.LoopBody, "for_loop_n")
    for ind in inds:
        if not isinstance(ind, induction):
            raise TypeError("for_loop_n: extra arguments must be hpx::parallel::induction or "
                            "hpx::parallel::reduction objects")
        if not isinstance(ind.value, iterator):
            raise TypeError("for_loop_n: inductions over device iterators only")
    if not isinstance(first, iterator):
        raise TypeError("for_loop_n: the loop variable must be a device iterator")
    n = int(count)
    if n < 0:
        raise ValueError("for_loop_n: negative count")
    vars_ = [first] + [ind.value for ind in inds]
    strides = [first_stride] + [ind.stride for ind in inds]
    try:
        out, so = vars_[body.out], strides[body.out]
        ins = [vars_[i] for i in body.ins]
        sis = [strides[i] for i in body.ins]
    except IndexError:
        raise IndexError("for_loop_n: loop body refers to a variable that is not passed") from None
    if n > 0:
        # every iteration's element must lie inside its vector (value_proxy
        # semantics: the reference would run off the end of the allocation)
        for it, st in zip([out] + ins, [so] + sis):
            lo, hi = it.pos, it.pos + st * (n - 1)
            if min(lo, hi) < 0 or max(lo, hi) >= it.vec.size():
                raise ValueError("for_loop_n: an induction walks outside its vector")
        if so == 0 and n > 1:
            raise ValueError("for_loop_n: the written induction has stride 0")
    stream, tgt, is_task = _context(pol, out, *ins)
    fn = body.fn
    strided = any(st != 1 for st in [so] + sis)
    if isinstance(fn, F.Unary):
        cdt = _compute_dtype(ins[0].dtype, fn)
        if strided:
            L.call("hpxhip_transform_strided", ins[0].dtype, cdt, out.dtype, fn.kind, L.scalars_buf(cdt, fn.scalars),
                   _vp(ins[0].address), sis[0], _vp(out.address), so, n, stream)
        else:
            L.call("hpxhip_transform", ins[0].dtype, cdt, out.dtype, fn.kind, L.scalars_buf(cdt, fn.scalars),
                   _vp(ins[0].address), _vp(out.address), n, stream)
    else:
        if ins[0].dtype != ins[1].dtype:
            raise TypeError("for_loop_n: both inputs of a binary body must have one dtype")
        cdt = _compute_dtype(ins[0].dtype, fn)
        if strided:
            L.call("hpxhip_transform_binary_strided", ins[0].dtype, cdt, out.dtype, fn.kind,
                   L.scalars_buf(cdt, fn.scalars), _vp(ins[0].address), sis[0], _vp(ins[1].address), sis[1],
                   _vp(out.address), so, n, stream)
        else:
            L.call("hpxhip_transform_binary", ins[0].dtype, cdt, out.dtype, fn.kind, L.scalars_buf(cdt, fn.scalars),
                   _vp(ins[0].address), _vp(ins[1].address), _vp(out.address), n, stream)
    return _finish(is_task, stream, tgt, lambda: None)


def for_loop(pol, first, last, *args):
    """for_loop.hpp for_loop(policy, first, last, inductions..., f)."""
    return for_loop_n(pol, first, _check_range(first, last), *args)


# ------------------------------------------------------------ error contract
# dispatch.hpp:122-124,164-168 and parallel/exception_list.hpp:20-111: an
# algorithm's failure reaches the caller as hpx::exception_list (raised under
# a synchronous policy, held by the returned future under a task policy),
# except an allocation failure, which stays std::bad_alloc (OutOfMemory, a
# MemoryError).  Python's argument errors (TypeError for a functor with no
# device mapping, ValueError / IndexError for malformed ranges) stand for the
# reference's compile-time rejections and precondition checks and pass
# unchanged.
_ARGUMENT_ERRORS = (TypeError, ValueError, IndexError, ZeroDivisionError)


def _algorithm_error(e):
    if isinstance(e, (MemoryError, L.exception_list) + _ARGUMENT_ERRORS):
        return e
    return L.exception_list([e])


def _guarded(fn):
    @functools.wraps(fn)
    def run(pol, *args, **kw):
        try:
            r = fn(pol, *args, **kw)
        except _ARGUMENT_ERRORS:
            raise
        except Exception as e:  # noqa: BLE001 -- rethrown under the contract
            err = _algorithm_error(e)
            if getattr(pol, "is_task", False):
                from .future import make_exceptional_future
                return make_exceptional_future(err)
            if err is e:
                raise
            raise err from e
        if isinstance(r, future):
            r._error_map = _algorithm_error
        return r
    return run


for _name in ("generate", "fill", "fill_n", "for_each", "for_each_n", "copy", "copy_n", "copy_if", "transform",
              "reduce", "transform_reduce", "inclusive_scan", "exclusive_scan", "transform_inclusive_scan",
              "transform_exclusive_scan", "sort", "is_sorted", "sort_by_key", "merge", "for_loop_n", "for_loop",
              "for_loop_n_strided", "for_loop_strided"):
    if _name in globals():
        globals()[_name] = _guarded(globals()[_name])
del _name
