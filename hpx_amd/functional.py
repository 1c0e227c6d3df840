"""Function objects accepted by the hip-executor algorithms.

HPX passes arbitrary ``HPX_HOST_DEVICE`` callables to the algorithms; a
precompiled C ABI can only carry an operator *kind* plus scalars, so the
functors used by the reference's STREAM benchmark, tests and examples are
named here ("Arbitrary user functors vs a C ABI").
Anything else raises ``TypeError`` (no silent host fallback).

References:
  * multiply_step / add_step / triad_step: tests/performance/local/stream.cpp:224-272
  * `i += 5`: tests/unit/computeapi/cuda/for_each_compute.cu:40-46
  * `a + 3.0 * b` (int result): tests/unit/computeapi/cuda/transform_compute.cu:36-39
  * `!(i < 0)`: tests/unit/parallel/algorithms/copyif_random.cpp:45
"""
from __future__ import annotations

from dataclasses import dataclass, field

from . import _lib as L


# --------------------------------------------------------------- reductions
@dataclass(frozen=True)
class BinaryOp:
    """std::plus<> and friends: an associative operator with an identity."""
    kind: int
    name: str

    def __call__(self, a, b):  # host-side meaning, used by tests/docs only
        return _BINOP_PY[self.kind](a, b)


def _wrap(fn):
    return fn


_BINOP_PY = {
    L.PLUS: lambda a, b: a + b,
    L.MULTIPLIES: lambda a, b: a * b,
    L.MIN: lambda a, b: b if b < a else a,
    L.MAX: lambda a, b: b if a < b else a,
    L.BIT_AND: lambda a, b: a & b,
    L.BIT_OR: lambda a, b: a | b,
    L.BIT_XOR: lambda a, b: a ^ b,
}

plus = BinaryOp(L.PLUS, "std::plus")
multiplies = BinaryOp(L.MULTIPLIES, "std::multiplies")
minimum = BinaryOp(L.MIN, "hpx::parallel::v1::detail::min")
maximum = BinaryOp(L.MAX, "hpx::parallel::v1::detail::max")
bit_and = BinaryOp(L.BIT_AND, "std::bit_and")
bit_or = BinaryOp(L.BIT_OR, "std::bit_or")
bit_xor = BinaryOp(L.BIT_XOR, "std::bit_xor")


# ------------------------------------------------------------ unary functors
@dataclass(frozen=True)
class Unary:
    kind: int
    scalars: tuple = field(default=())
    compute: str | None = None  # compute dtype name; None = element dtype

    def __call__(self, x):
        s = self.scalars + (0, 0)
        k = self.kind
        if k == L.U_IDENTITY:
            return x
        if k == L.U_SCALE:
            return x * s[0]
        if k == L.U_ADD_SCALAR:
            return x + s[0]
        if k == L.U_AFFINE:
            return x * s[0] + s[1]
        if k == L.U_NEGATE:
            return -x
        if k == L.U_ABS:
            return abs(x)
        return x * x


def identity() -> Unary:
    """util::projection_identity."""
    return Unary(L.U_IDENTITY)


def multiply_step(factor) -> Unary:
    """stream.cpp:224-239: val * factor_."""
    return Unary(L.U_SCALE, (factor,))


def add_value(k) -> Unary:
    """for_each_compute.cu: ``i += 5``."""
    return Unary(L.U_ADD_SCALAR, (k,))


def affine(a, b) -> Unary:
    return Unary(L.U_AFFINE, (a, b))


def negate() -> Unary:
    return Unary(L.U_NEGATE)


def absolute() -> Unary:
    return Unary(L.U_ABS)


def square() -> Unary:
    return Unary(L.U_SQUARE)


# ----------------------------------------------------------- binary functors
@dataclass(frozen=True)
class Binary:
    kind: int
    scalars: tuple = field(default=())
    compute: str | None = None

    def __call__(self, x, y):
        s = self.scalars + (0,)
        k = self.kind
        if k == L.B_ADD:
            return x + y
        if k == L.B_TRIAD:
            return x + y * s[0]
        if k == L.B_SUB:
            return x - y
        if k == L.B_MUL:
            return x * y
        if k == L.B_AXPY:
            return x * s[0] + y
        if k == L.B_MIN:
            return y if y < x else x
        return y if x < y else x


def add_step() -> Binary:
    """stream.cpp:241-253: val1 + val2."""
    return Binary(L.B_ADD)


def triad_step(factor, compute: str | None = None) -> Binary:
    """stream.cpp:255-272: val1 + val2 * factor_.

    ``compute="float64"`` with int inputs reproduces transform_compute.cu's
    ``int(a + 3.0*b)``."""
    return Binary(L.B_TRIAD, (factor,), compute)


def subtract() -> Binary:
    return Binary(L.B_SUB)


def multiply() -> Binary:
    """The conv of an inner product (transform_reduce_binary.hpp:323)."""
    return Binary(L.B_MUL)


def axpy(a) -> Binary:
    return Binary(L.B_AXPY, (a,))


# ---------------------------------------------------------------- predicates
@dataclass(frozen=True)
class Predicate:
    kind: int
    arg: object = 0

    def __call__(self, x):
        a = self.arg
        k = self.kind
        return {
            L.P_LT: lambda: x < a, L.P_LE: lambda: x <= a, L.P_GT: lambda: x > a,
            L.P_GE: lambda: x >= a, L.P_EQ: lambda: x == a, L.P_NE: lambda: x != a,
            L.P_NOT_LT: lambda: not (x < a), L.P_BITS: lambda: (x & a) != 0,
        }[k]()


def less_than(a) -> Predicate:
    return Predicate(L.P_LT, a)


def less_equal(a) -> Predicate:
    return Predicate(L.P_LE, a)


def greater_than(a) -> Predicate:
    return Predicate(L.P_GT, a)


def greater_equal(a) -> Predicate:
    return Predicate(L.P_GE, a)


def equal_to(a) -> Predicate:
    return Predicate(L.P_EQ, a)


def not_equal_to(a) -> Predicate:
    return Predicate(L.P_NE, a)


def not_less_than(a) -> Predicate:
    """copyif_random.cpp: ``!(i < 0)``."""
    return Predicate(L.P_NOT_LT, a)


def any_bits(mask) -> Predicate:
    return Predicate(L.P_BITS, mask)


# ------------------------------------------------------------- loop bodies
@dataclass(frozen=True)
class LoopBody:
    """Body of for_loop / for_loop_n over pointer inductions: writes
    ``*vars[out] = fn(*vars[ins[0]] [, *vars[ins[1]]])`` where vars are the
    loop iterator (position 0) followed by the inductions in call order.
    for_loop_compute.cu:40-48's ``[](int* A, int* B, int* C) { *C = *A +
    3.0 * *B; }`` is ``assign(2, triad_step(3.0, "float64"), 0, 1)``."""
    out: int
    fn: object
    ins: tuple


def assign(out: int, fn, *ins) -> LoopBody:
    if isinstance(fn, Unary) and len(ins) == 1 or isinstance(fn, Binary) and len(ins) == 2:
        return LoopBody(int(out), fn, tuple(int(i) for i in ins))
    raise TypeError("assign: a Unary functor takes one loop variable, a Binary functor two")


@dataclass(frozen=True)
class Accumulate:
    """Body of for_loop / for_loop_n with a reduction: folds
    ``fn(*vars[ins[0]] [, *vars[ins[1]]])`` into the reduction variable at
    position ``red`` with the reduction's combiner.
    for_loop_reduction.cpp:37-44's ``[](iterator it, std::size_t& sum) { sum
    += *it; }`` is ``accumulate(1, identity(), 0)``."""
    red: int
    fn: object
    ins: tuple


def accumulate(red: int, fn, *ins) -> Accumulate:
    if isinstance(fn, Unary) and len(ins) == 1 or isinstance(fn, Binary) and len(ins) == 2:
        return Accumulate(int(red), fn, tuple(int(i) for i in ins))
    raise TypeError("accumulate: a Unary functor takes one loop variable, a Binary functor two")


@dataclass(frozen=True)
class Accumulates:
    """Body of a for_loop with several reductions (for_loop.hpp:802-812
    takes any number of reduction arguments): one Accumulate per reduction,
    e.g. ``[](it, T& sum, T& sq) { sum += *it; sq += *it * *it; }`` is
    ``accumulate_all(accumulate(1, identity(), 0), accumulate(2, square(), 0))``."""
    parts: tuple


def accumulate_all(*parts) -> Accumulates:
    if not parts or not all(isinstance(a, Accumulate) for a in parts):
        raise TypeError("accumulate_all: one or more accumulate(...) bodies")
    if len({a.red for a in parts}) != len(parts):
        raise ValueError("accumulate_all: each reduction is accumulated by one body")
    return Accumulates(tuple(parts))


# ------------------------------------------------------------------ compare
@dataclass(frozen=True)
class Compare:
    descending: bool
    name: str


less = Compare(False, "std::less")
greater = Compare(True, "std::greater")


def require(obj, cls, what: str):
    if not isinstance(obj, cls):
        raise TypeError(
            f"{what}: {obj!r} is not an hpx_amd functor ({cls.__name__}); arbitrary "
            "callables need the header-only C++ layer compiled with hipcc "
            "(include/hpx/...), the C ABI carries operator kinds only")
    return obj
