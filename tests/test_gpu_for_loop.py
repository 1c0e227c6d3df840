"""for_loop_n / for_loop with pointer inductions on the hip executor
(tests/unit/computeapi/cuda/for_loop_compute.cu:28-118 restated: N = 100 int
iotas from a random start, body *C = *A + 3.0 * *B), bit-exact against the
host expression, plus larger sizes, a unary in-place body and the argument
checks."""
import numpy as np
import pytest

import hpx_amd as hpx
from hpx_amd import execution as ex, functional as F
from hpx_amd import parallel as P

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [100, 1, 0, 4097, (1 << 20) + 3])
def test_for_loop_compute(gpu_target, n):
    rng = np.random.default_rng(n)
    a0, b0 = rng.integers(2, 102, 2)
    h_a = np.arange(a0, a0 + n, dtype=np.int32)
    h_b = np.arange(b0, b0 + n, dtype=np.int32)
    ref = (h_a.astype(np.float64) + 3.0 * h_b.astype(np.float64)).astype(np.int32)  # transform(.., a + 3.0*b)
    tA, tB = hpx.target(gpu_target.device), hpx.target(gpu_target.device)   # targetA, targetB
    d_a = hpx.vector.from_host(h_a, tA)
    d_b = hpx.vector.from_host(h_b, tB)
    d_c = hpx.vector(n, dtype=np.int32, tgt=tA)
    tA.synchronize()
    tB.synchronize()
    execu = hpx.default_executor(tB)
    body = F.assign(2, F.triad_step(3.0, "float64"), 0, 1)   # *C = *A + 3.0 * *B
    P.for_loop_n(ex.par.on(execu), d_a.begin(), n, P.induction(d_b.begin()), P.induction(d_c.begin()), body)
    np.testing.assert_array_equal(d_c.to_host(), ref)
    # for_loop over [first, last) and the task form
    d_c2 = hpx.vector(n, dtype=np.int32, tgt=tA)
    f = P.for_loop(ex.par(ex.task).on(execu), d_a.begin(), d_a.end(), P.induction(d_b.begin()),
                   P.induction(d_c2.begin()), body)
    f.get()
    np.testing.assert_array_equal(d_c2.to_host(), ref)


def test_for_loop_unary_in_place(gpu_target):
    x = np.arange(10007, dtype=np.int64)
    d = hpx.vector.from_host(x, gpu_target)
    P.for_loop_n(ex.par.on(hpx.default_executor(gpu_target)), d.begin(), d.size(), F.assign(0, F.add_value(5), 0))
    np.testing.assert_array_equal(d.to_host(), x + 5)


def test_for_loop_argument_checks(gpu_target):
    d = hpx.vector(16, dtype=np.int32, tgt=gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    with pytest.raises(TypeError):
        P.for_loop_n(pol, d.begin(), 16, lambda a: a)
    with pytest.raises(ValueError):
        P.for_loop_n(pol, d.begin(), 16, P.induction(d.begin(), 2), F.assign(1, F.add_value(1), 0))
    with pytest.raises(IndexError):
        P.for_loop_n(pol, d.begin(), 16, F.assign(3, F.add_value(1), 0))
    with pytest.raises(TypeError):
        F.assign(0, F.add_value(1), 0, 1)


# ------------------------------------------------------- for_loop reductions
# tests/unit/parallel/algorithms/for_loop_reduction.cpp:20-140 restated:
# 10007 size_t iotas from a random start, body ``r op= *it``, checked against
# std::accumulate (integer results, bit-exact; products wrap modulo 2^64).
_N = 10007


def _iota(seed, dtype=np.uint64):
    start = int(np.random.default_rng(seed).integers(0, 1 << 31))
    return np.arange(start, start + _N, dtype=dtype)


def _fold(op, init, xs, mask=(1 << 64) - 1):
    acc = int(init)
    for x in xs.tolist():
        acc = op(acc, int(x)) & mask
    return acc


@pytest.mark.parametrize("task", [False, True])
def test_for_loop_reduction_plus(gpu_target, task):
    c = _iota(1)
    d = hpx.vector.from_host(c, gpu_target)
    pol = (ex.par(ex.task) if task else ex.par).on(hpx.default_executor(gpu_target))
    s = np.zeros(1, np.uint64)
    r = P.for_loop(pol, d.begin(), d.end(), P.reduction_plus(s), F.accumulate(1, F.identity(), 0))
    if task:
        r.get()
    assert int(s[0]) == _fold(lambda a, b: a + b, 0, c)


def test_for_loop_reduction_multiplies(gpu_target):
    c = _iota(2)
    d = hpx.vector.from_host(c, gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    # for_loop_reduction.cpp:60: prod starts at 0, so the live-out stays 0
    prod = np.zeros(1, np.uint64)
    P.for_loop(pol, d.begin(), d.end(), P.reduction_multiplies(prod), F.accumulate(1, F.identity(), 0))
    assert int(prod[0]) == 0
    prod = np.ones(1, np.uint64)
    P.for_loop(pol, d.begin(), d.end(), P.reduction_multiplies(prod), F.accumulate(1, F.identity(), 0))
    assert int(prod[0]) == _fold(lambda a, b: a * b, 1, c)


@pytest.mark.parametrize("which", ["min", "max"])
def test_for_loop_reduction_minmax(gpu_target, which):
    c = _iota(3)
    np.random.default_rng(3).shuffle(c)
    d = hpx.vector.from_host(c, gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    v = np.array([c[0]], np.uint64)   # for_loop_reduction.cpp:96: minval = c[0]
    red = P.reduction_min(v) if which == "min" else P.reduction_max(v)
    P.for_loop(pol, d.begin(), d.end(), red, F.accumulate(1, F.identity(), 0))
    assert int(v[0]) == int(c.min() if which == "min" else c.max())


@pytest.mark.parametrize("which", ["and", "or", "xor"])
def test_for_loop_reduction_bits(gpu_target, which):
    c = np.random.default_rng(4).integers(0, 2**63, _N, dtype=np.int64) | np.int64(1 << 40)
    d = hpx.vector.from_host(c, gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    v = np.zeros(1, np.int64)
    if which == "and":
        v[0] = -1
        red, op, ident = P.reduction_bit_and(v), np.bitwise_and, -1
    elif which == "or":
        red, op, ident = P.reduction_bit_or(v), np.bitwise_or, 0
    else:
        red, op, ident = P.reduction_bit_xor(v), np.bitwise_xor, 0
    P.for_loop_n(pol, d.begin(), _N, red, F.accumulate(1, F.identity(), 0))
    assert int(v[0]) == int(op.reduce(c, initial=ident))


@pytest.mark.parametrize("task", [False, True])
def test_for_loop_several_reductions(gpu_target, task):
    """for_loop_n(policy, first, size, reduction..., reduction..., f) takes
    any number of reductions (for_loop.hpp:802-812): sum, min and max of one
    range plus the inner product with an induction, in one loop; every
    live-out variable is folded with its own combiner."""
    rng = np.random.default_rng(6)
    a = rng.integers(-1000, 1000, 100003, dtype=np.int64)
    b = rng.integers(-1000, 1000, 100003, dtype=np.int64)
    da, db = hpx.vector.from_host(a, gpu_target), hpx.vector.from_host(b, gpu_target)
    pol = (ex.par(ex.task) if task else ex.par).on(hpx.default_executor(gpu_target))
    s, lo, hi, dot = (np.array([v], np.int64) for v in (5, a[0], a[0], 7))
    r = P.for_loop_n(pol, da.begin(), len(a), P.reduction_plus(s), P.reduction_min(lo), P.reduction_max(hi),
                     P.induction(db.begin()), P.reduction_plus(dot),
                     F.accumulate_all(F.accumulate(1, F.identity(), 0), F.accumulate(2, F.identity(), 0),
                                      F.accumulate(3, F.identity(), 0), F.accumulate(5, F.multiply(), 0, 4)))
    if task:
        r.get()
    assert int(s[0]) == 5 + int(a.sum())
    assert int(lo[0]) == int(a.min()) and int(hi[0]) == int(a.max())
    assert int(dot[0]) == 7 + int(np.dot(a, b))


def test_for_loop_reduction_inner_product_and_empty(gpu_target):
    """A reduction body reading the loop iterator and an induction
    (transform_reduce_binary kernels); an empty loop leaves var op identity."""
    rng = np.random.default_rng(5)
    a = rng.integers(-1000, 1000, 1 << 16, dtype=np.int64)
    b = rng.integers(-1000, 1000, 1 << 16, dtype=np.int64)
    da, db = hpx.vector.from_host(a, gpu_target), hpx.vector.from_host(b, gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    s = np.array([7], np.int64)
    P.for_loop_n(pol, da.begin(), a.size, P.induction(db.begin()), P.reduction_plus(s),
                 F.accumulate(2, F.multiply(), 0, 1))
    assert int(s[0]) == 7 + int(np.dot(a, b))
    e = np.array([11], np.int64)
    P.for_loop_n(pol, da.begin(), 0, P.reduction_plus(e), F.accumulate(1, F.identity(), 0))
    assert int(e[0]) == 11


def test_for_loop_reduction_argument_checks(gpu_target):
    d = hpx.vector(16, dtype=np.int64, tgt=gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    s = np.zeros(1, np.int64)
    with pytest.raises(TypeError):   # a reduction needs an accumulate body
        P.for_loop_n(pol, d.begin(), 16, P.reduction_plus(s), F.assign(0, F.add_value(1), 0))
    with pytest.raises(IndexError):  # accumulate must name the reduction's position
        P.for_loop_n(pol, d.begin(), 16, P.reduction_plus(s), F.accumulate(0, F.identity(), 0))
    with pytest.raises(ValueError):  # two reductions, only one accumulated
        P.for_loop_n(pol, d.begin(), 16, P.reduction_plus(s), P.reduction_plus(s),
                     F.accumulate(1, F.identity(), 0))
    with pytest.raises(ValueError):  # the induction read by the body runs past its vector
        P.for_loop_n(pol, d.begin(), 16, P.induction(d.begin() + 1), P.reduction_plus(s),
                     F.accumulate(2, F.multiply(), 0, 1))
    assert int(s[0]) == 0


# ---------------------------------------------- strided pointer inductions
# for_loop_induction.hpp:210-219: induction(it, stride) has the value
# it + stride * i at iteration i (for_loop_induction.cpp's stride-2 cases).
@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.float64])
def test_for_loop_strided_inductions(gpu_target, dtype):
    n = 10007
    rng = np.random.default_rng(7)
    a = rng.integers(-1000, 1000, 3 * n).astype(dtype)
    b = rng.integers(-1000, 1000, 2 * n).astype(dtype)
    da, db = hpx.vector.from_host(a, gpu_target), hpx.vector.from_host(b, gpu_target)
    dc = hpx.vector.from_host(np.zeros(2 * n, dtype), gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    # unary: c[2i] = a[3i] + 5 (loop variable over the first n of b, unused)
    P.for_loop_n(pol, db.begin(), n, P.induction(da.begin(), 3), P.induction(dc.begin(), 2),
                 F.assign(2, F.add_value(5), 1))
    ref = np.zeros(2 * n, dtype)
    ref[0::2] = a[0::3] + dtype(5)
    np.testing.assert_array_equal(dc.to_host(), ref)
    # binary, negative stride on one input: c[i] = b[i] + 3*a[3n-1-i] ... via triad(b, a_rev)
    dd = hpx.vector.from_host(np.zeros(n, dtype), gpu_target)
    P.for_loop_n(pol, dd.begin(), n, P.induction(db.begin()), P.induction(da.begin() + (3 * n - 1), -1),
                 F.assign(0, F.add_step(), 1, 2))
    np.testing.assert_array_equal(dd.to_host(), b[:n] + a[::-1][:n])
    # task form, stride 0 on an input (broadcast of a[0])
    de = hpx.vector.from_host(np.zeros(n, dtype), gpu_target)
    f = P.for_loop_n(ex.par(ex.task).on(hpx.default_executor(gpu_target)), de.begin(), n,
                     P.induction(da.begin(), 0), F.assign(0, F.add_value(1), 1))
    f.get()
    np.testing.assert_array_equal(de.to_host(), np.full(n, a[0] + dtype(1), dtype))


def test_for_loop_strided_bounds(gpu_target):
    d = hpx.vector(100, dtype=np.int64, tgt=gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    with pytest.raises(ValueError):   # 10 + 10*9 = 100 is one past the end
        P.for_loop_n(pol, d.begin(), 10, P.induction(d.begin() + 10, 10), F.assign(0, F.add_value(1), 1))
    with pytest.raises(ValueError):   # walks below the start
        P.for_loop_n(pol, d.begin(), 10, P.induction(d.begin() + 5, -1), F.assign(0, F.add_value(1), 1))
    with pytest.raises(ValueError):   # every iteration writes one element
        P.for_loop_n(pol, d.begin(), 10, P.induction(d.begin(), 0), F.assign(1, F.add_value(1), 0))
    P.for_loop_n(pol, d.begin(), 10, P.induction(d.begin() + 9, 10), F.assign(0, F.add_value(1), 1))


# tests/unit/parallel/algorithms/for_loop_strided.cpp:29-74 restated: 10007
# size_t iotas (42 replaced by 43), every stride-th element set to 42.
@pytest.mark.parametrize("stride", [1, 2, 7, 100, 10007, 20000])
def test_for_loop_strided(gpu_target, stride):
    c = np.arange(1000, 1000 + 10007, dtype=np.uint64)
    d = hpx.vector.from_host(c, gpu_target)
    pol = ex.par.on(hpx.default_executor(gpu_target))
    P.for_loop_strided(pol, d.begin(), d.end(), stride, F.assign(0, F.affine(0, 42), 0))
    got = d.to_host()
    idx = np.arange(c.size)
    assert np.all(got[idx % stride == 0] == 42) and np.all(got[idx % stride != 0] != 42)


def test_for_loop_strided_negative_and_inductions(gpu_target):
    n = 1000
    a = np.arange(n, dtype=np.int64)
    da = hpx.vector.from_host(a, gpu_target)
    dout = hpx.vector.from_host(np.zeros(n, np.int64), gpu_target)
    pol = ex.par(ex.task).on(hpx.default_executor(gpu_target))
    # loop variable walks a backwards by 3 from the end; induction of out walks forward (ordinal)
    f = P.for_loop_strided(pol, da.begin() + (n - 1), da.begin() - 0, -3, P.induction(dout.begin()),
                           F.assign(1, F.add_value(1), 0))
    f.get()
    k = (n - 1 + 2) // 3
    ref = np.zeros(n, np.int64)
    ref[:k] = a[n - 1::-3][:k] + 1
    np.testing.assert_array_equal(dout.to_host(), ref)
    P.for_loop_n_strided(ex.par.on(hpx.default_executor(gpu_target)), dout.begin(), 5, 2,
                         F.assign(0, F.affine(0, 7), 0))
    assert list(dout.to_host()[:10:2]) == [7] * 5
    with pytest.raises(ValueError):
        P.for_loop_strided(pol, da.begin(), da.end(), 0, F.assign(0, F.add_value(1), 0))
