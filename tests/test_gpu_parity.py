"""GPU parity: every hip-executor algorithm against the CPU oracle (bit-exact
for integer work, stated tolerance for floating-point reductions/scans),
against the golden fixtures from the reference's known-answer tests, and
size-independent properties at large n.  Calls go through the Python mirror
of the HPX API into the C ABI (include/hpxhip.h)."""
import math
import os

import numpy as np
import pytest

import hpx_amd as hpx
from hpx_amd import execution as ex, functional as F
from hpx_amd import parallel as P
from conftest import golden_cases, load_golden
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 2, 3, 7, 63, 64, 65, 255, 1000, 4095, 4096, 4097, 16383, 100003, 1 << 20, (1 << 20) + 17]
INT_DT = [np.int32, np.uint32, np.int64, np.uint64]
ALL_DT = INT_DT + [np.float32, np.float64]


@pytest.fixture(scope="module")
def pol(gpu_target):
    return ex.par.on(hpx.default_executor(gpu_target))


def dev(a, t):
    return hpx.vector.from_host(np.ascontiguousarray(a), t)


def rnd(dt, n, seed=0, lo=None, hi=None):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dt)
    if dt.kind == "f":
        return rng.standard_normal(n).astype(dt)
    info = np.iinfo(dt)
    lo = info.min if lo is None else lo
    hi = info.max if hi is None else hi
    return rng.integers(lo, hi, n, dtype=dt, endpoint=True)


def fp_tol(x, dt):
    """|gpu - oracle| bound for a reordered FP sum of x (relative to sum|x|):
    gamma_k * sum|x_i| with k = 2*ceil(log2 n) + 32 (tree depth + serial run),
    u = 2^-24 (f32) / 2^-53 (f64)."""
    u = 2.0 ** -24 if np.dtype(dt) == np.float32 else 2.0 ** -53
    k = 2 * max(1, math.ceil(math.log2(max(2, x.size)))) + 32
    return k * u * float(np.sum(np.abs(x.astype(np.float64)))) + 1e-30


# ------------------------------------------------------------ elementwise
@pytest.mark.parametrize("n", SIZES)
def test_stream_triad_bit_exact(pol, gpu_target, n):
    b, c = rnd(np.float64, n, 1), rnd(np.float64, n, 2)
    db, dc, da = dev(b, gpu_target), dev(c, gpu_target), hpx.vector(n, dtype=np.float64, tgt=gpu_target)
    P.transform(pol, db.begin(), db.end(), dc.begin(), dc.end(), da.begin(), F.triad_step(3.0))
    np.testing.assert_array_equal(da.to_host(), O.transform_binary(b, c, "triad", (3.0,)))


@pytest.mark.parametrize("offset", [0, 1, 2, 3])
def test_transform_unaligned_offsets(pol, gpu_target, offset):
    n = 10000
    b, c = rnd(np.float32, n, 1), rnd(np.float32, n, 2)
    db, dc, da = dev(b, gpu_target), dev(c, gpu_target), hpx.vector(n, dtype=np.float32, tgt=gpu_target)
    # misaligned and mutually misaligned ranges (scalar fallback) and equally shifted ones
    P.transform(pol, db.begin() + offset, db.end(), dc.begin() + offset, da.begin() + offset, F.add_step())
    out = da.to_host()
    np.testing.assert_array_equal(out[offset:], O.transform_binary(b[offset:], c[offset:], "add"))
    P.transform(pol, db.begin() + offset, db.end() - 1, dc.begin(), da.begin(), F.add_step())
    np.testing.assert_array_equal(da.to_host()[: n - 1 - offset], O.transform_binary(b[offset:n - 1], c[: n - 1 - offset], "add"))


@pytest.mark.parametrize("dt", ALL_DT)
@pytest.mark.parametrize("kind,sc", [("scale", (3,)), ("add_scalar", (5,)), ("affine", (2, 7)), ("negate", ()),
                                     ("abs", ()), ("square", ()), ("identity", ())])
def test_transform_unary_kinds(pol, gpu_target, dt, kind, sc):
    n = 4099
    a = rnd(dt, n, 3, *((-1000, 1000) if np.dtype(dt).kind == "i" else (None, None)) if np.dtype(dt).kind != "f" else ())
    da, dd = dev(a, gpu_target), hpx.vector(n, dtype=dt, tgt=gpu_target)
    f = F.Unary({"scale": 1, "add_scalar": 2, "affine": 3, "negate": 4, "abs": 5, "square": 6, "identity": 0}[kind], sc)
    P.transform(pol, da.begin(), da.end(), dd.begin(), f)
    np.testing.assert_array_equal(dd.to_host(), O.transform(a, kind, sc))


@pytest.mark.parametrize("dt", ALL_DT)
def test_for_each_fill_copy(pol, gpu_target, dt):
    n = 12347
    a = rnd(dt, n, 4)
    da = dev(a, gpu_target)
    P.for_each(pol, da.begin(), da.end(), F.add_value(5))
    np.testing.assert_array_equal(da.to_host(), O.for_each(a, "add_scalar", (5,)))
    P.fill(pol, da.begin() + 3, da.end() - 2, 7)
    exp = O.for_each(a, "add_scalar", (5,))
    exp[3:n - 2] = 7
    np.testing.assert_array_equal(da.to_host(), exp)
    db = hpx.vector(n, dtype=dt, tgt=gpu_target)
    P.copy(pol, da.begin(), da.end(), db.begin())
    np.testing.assert_array_equal(db.to_host(), exp)


def test_golden_for_each_compute(pol, gpu_target):
    case = golden_cases("for_each")[0]
    g = load_golden(case)
    d = dev(g["input"], gpu_target)
    P.for_each(pol, d.begin(), d.end(), F.add_value(case["scalar"]))
    np.testing.assert_array_equal(d.to_host(), g["expected"])


def test_golden_transform_compute(pol, gpu_target):
    case = golden_cases("transform_binary")[0]
    g = load_golden(case)
    a, b = dev(g["input"], gpu_target), dev(g["input2"], gpu_target)
    c = hpx.vector(len(a), dtype=np.int32, tgt=gpu_target)
    P.transform(pol, a.begin(), a.end(), b.begin(), c.begin(), F.triad_step(3.0, compute="float64"))
    np.testing.assert_array_equal(c.to_host(), g["expected"])


@pytest.mark.parametrize("iters", [1, 2, 10])
def test_golden_stream_check_results(pol, gpu_target, iters):
    """stream.cpp:294-375 on the GPU, checked bit-exact against check_results' closed form."""
    n = 100003
    a = hpx.vector(n, dtype=np.float64, value=1.0, tgt=gpu_target)
    b = hpx.vector(n, dtype=np.float64, value=2.0, tgt=gpu_target)
    c = hpx.vector(n, dtype=np.float64, value=0.0, tgt=gpu_target)
    P.transform(pol, a.begin(), a.end(), a.begin(), F.multiply_step(2.0))
    for _ in range(iters):
        P.copy(pol, a.begin(), a.end(), c.begin())
        P.transform(pol, c.begin(), c.end(), b.begin(), F.multiply_step(3.0))
        P.transform(pol, a.begin(), a.end(), b.begin(), b.end(), c.begin(), F.add_step())
        P.transform(pol, b.begin(), b.end(), c.begin(), c.end(), a.begin(), F.triad_step(3.0))
    g = load_golden([c_ for c_ in golden_cases("stream") if c_["iterations"] == iters][0])
    aj, bj, cj = g["expected"]
    assert np.all(a.to_host() == aj) and np.all(b.to_host() == bj) and np.all(c.to_host() == cj)


def test_generate_matches_host_restatement(pol, gpu_target):
    n = 100003
    for dt, kind, lo, hi in [(np.uint64, "bits", 0, 0), (np.uint32, "bits", 0, 0), (np.int64, "range", -(1 << 20), 1 << 20),
                             (np.float64, "unit", 0, 0), (np.float32, "unit", 0, 0), (np.int64, "iota", 5, 0)]:
        v = hpx.vector(n, dtype=dt, tgt=gpu_target)
        P.generate(pol, v.begin(), v.end(), kind, 0x5EED, lo, hi)
        np.testing.assert_array_equal(v.to_host(), O.generate(dt, kind, n, 0x5EED, lo, hi))


# ------------------------------------------------------------- reductions
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dt", [np.int32, np.int64, np.uint64])
def test_reduce_int_exact(pol, gpu_target, n, dt):
    a = rnd(dt, n, 5)
    d = dev(a, gpu_target)
    for op, name in [(F.plus, "plus"), (F.minimum, "min"), (F.maximum, "max"), (F.bit_xor, "bit_xor"),
                     (F.bit_and, "bit_and"), (F.bit_or, "bit_or"), (F.multiplies, "multiplies")]:
        got = P.reduce(pol, d.begin(), d.end(), 3, op)
        assert got == O.transform_reduce(a, 3, op=name), name


@pytest.mark.parametrize("n", [1, 1000, 100003, (1 << 22) + 5])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_reduce_fp_tolerance_and_determinism(pol, gpu_target, n, dt):
    a = rnd(dt, n, 6)
    d = dev(a, gpu_target)
    got = P.reduce(pol, d.begin(), d.end(), 0.5, F.plus)
    exact = math.fsum(a.astype(np.float64).tolist()) + 0.5
    assert abs(got - exact) <= fp_tol(a, dt) + abs(exact) * (2.0 ** -24 if dt == np.float32 else 2.0 ** -53)
    assert P.reduce(pol, d.begin(), d.end(), 0.5, F.plus) == got  # run-to-run bitwise reproducible
    assert P.reduce(pol, d.begin(), d.end(), 0.0, F.maximum) == a.max()


def test_reduce_many_partials(pol, gpu_target):
    """Past 16384 block partials the fold launch (k_reduce_partials) loops:
    int64 at 2^28 + 3 (and a misaligned sub-range of it), int32 widened to
    int64 at 2^29 + 5.  Inputs are iota ranges (lo + i), so the exact
    results have closed forms and no multi-GiB host copy is needed."""
    def iota_sum(lo, n):
        return n * lo + n * (n - 1) // 2

    n, lo = (1 << 28) + 3, -(1 << 27)
    x = hpx.vector(n, dtype=np.int64, tgt=gpu_target)
    P.generate(pol, x.begin(), x.end(), "iota", 0, lo)
    assert x[0] == lo and x[n - 1] == lo + n - 1
    assert P.reduce(pol, x.begin(), x.end(), 7, F.plus) == 7 + iota_sum(lo, n)
    assert P.reduce(pol, x.begin() + 1, x.end(), 0, F.plus) == iota_sum(lo + 1, n - 1)
    assert P.reduce(pol, x.begin(), x.end(), -(1 << 40), F.maximum) == lo + n - 1
    assert P.reduce(pol, x.begin(), x.end(), 0, F.minimum) == lo
    del x
    n, lo = (1 << 29) + 5, -(1 << 28)
    y = hpx.vector(n, dtype=np.int32, tgt=gpu_target)
    P.generate(pol, y.begin(), y.end(), "iota", 0, lo)
    got = P.transform_reduce(pol, y.begin(), y.end(), np.int64(3), F.plus, F.identity())
    assert got == 3 + iota_sum(lo, n)


def test_reduce_golden(pol, gpu_target):
    for case in golden_cases("reduce"):
        g = load_golden(case)
        d = dev(g["input"], gpu_target)
        assert P.reduce(pol, d.begin(), d.end(), case["init"], F.plus) == g["expected"][0]
    case = golden_cases("transform_reduce")[0]
    g = load_golden(case)
    d = dev(g["input"], gpu_target)
    assert P.transform_reduce(pol, d.begin(), d.end(), np.uint64(1), F.multiplies, F.identity()) == g["expected"][0]


@pytest.mark.parametrize("conv,name,sc", [(F.square(), "square", ()), (F.absolute(), "abs", ()),
                                          (F.multiply_step(3), "scale", (3,))])
def test_transform_reduce_conv_widening(pol, gpu_target, conv, name, sc):
    a = rnd(np.int32, 50001, 7, -30000, 30000)
    d = dev(a, gpu_target)
    got = P.transform_reduce(pol, d.begin(), d.end(), np.int64(0), F.plus, conv)
    assert got == O.transform_reduce(a, 0, "plus", name, sc, acc=np.int64)


def test_inner_product(pol, gpu_target):
    a, b = rnd(np.int64, 70001, 8, -1000, 1000), rnd(np.int64, 70001, 9, -1000, 1000)
    da, db = dev(a, gpu_target), dev(b, gpu_target)
    assert P.transform_reduce(pol, da.begin(), da.end(), db.begin(), 0) == O.transform_reduce_binary(a, b, 0)
    assert P.transform_reduce(pol, da.begin() + 1, da.end(), db.begin(), 0) == O.transform_reduce_binary(a[1:], b[:-1], 0)


def test_reduce_task_policy_future(gpu_target):
    a = rnd(np.int64, 100000, 10, -5, 5)
    d = dev(a, gpu_target)
    pt = ex.par(ex.task).on(hpx.default_executor(gpu_target))
    futs = [P.reduce(pt, d.begin(), d.end(), i, F.plus) for i in range(5)]
    assert all(isinstance(f, hpx.future) for f in futs)
    vals = hpx.when_all(futs).get()
    assert [f.get() for f in vals] == [int(a.sum()) + i for i in range(5)]


# ------------------------------------------------------------------ scans
@pytest.mark.parametrize("n", SIZES + [(1 << 24) + 3])
@pytest.mark.parametrize("dt", [np.int32, np.uint32, np.int64, np.uint64])
def test_scan_int_exact(pol, gpu_target, n, dt):
    a = rnd(dt, n, 11)
    d, o = dev(a, gpu_target), hpx.vector(n, dtype=dt, tgt=gpu_target)
    P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), F.plus, 9)
    np.testing.assert_array_equal(o.to_host(), O.scan(a, 9, True))
    P.exclusive_scan(pol, d.begin(), d.end(), o.begin(), 9)
    np.testing.assert_array_equal(o.to_host(), O.scan(a, 9, False))


@pytest.mark.parametrize("opname", ["min", "max", "bit_xor", "bit_or", "bit_and", "multiplies"])
def test_scan_other_ops(pol, gpu_target, opname):
    op = {"min": F.minimum, "max": F.maximum, "bit_xor": F.bit_xor, "bit_or": F.bit_or, "bit_and": F.bit_and,
          "multiplies": F.multiplies}[opname]
    a = rnd(np.int64, 300001, 12, -7, 7)
    d, o = dev(a, gpu_target), hpx.vector(len(a), dtype=np.int64, tgt=gpu_target)
    for incl in (True, False):
        if incl:
            P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), op, 3)
        else:
            P.exclusive_scan(pol, d.begin(), d.end(), o.begin(), 3, op)
        np.testing.assert_array_equal(o.to_host(), O.scan(a, 3, incl, op=opname))


def test_scan_golden_and_in_place(pol, gpu_target):
    for case in golden_cases("exclusive_scan"):
        g = load_golden(case)
        d, o = dev(g["input"], gpu_target), hpx.vector(len(g["input"]), dtype=np.int32, tgt=gpu_target)
        P.exclusive_scan(pol, d.begin(), d.end(), o.begin(), case["init"], F.plus)
        np.testing.assert_array_equal(o.to_host(), g["expected"])
        P.exclusive_scan(pol, d.begin(), d.end(), d.begin(), case["init"], F.plus)  # in place
        np.testing.assert_array_equal(d.to_host(), g["expected"])
    for case in golden_cases("inclusive_scan"):
        g = load_golden(case)
        d = dev(g["input"], gpu_target)
        o = hpx.vector(len(d), dtype=g["input"].dtype, tgt=gpu_target)
        P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), F.plus, case["init"])
        np.testing.assert_array_equal(o.to_host(), g["expected"])  # bit-exact incl. the all-1.0 doubles


def test_inclusive_scan_overloads(pol, gpu_target):
    a = rnd(np.int64, 5000, 13, -100, 100)
    d, o = dev(a, gpu_target), hpx.vector(len(a), dtype=np.int64, tgt=gpu_target)
    P.inclusive_scan(pol, d.begin(), d.end(), o.begin())
    np.testing.assert_array_equal(o.to_host(), np.cumsum(a))
    P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), 4)
    np.testing.assert_array_equal(o.to_host(), 4 + np.cumsum(a))
    P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), 4, F.plus)
    np.testing.assert_array_equal(o.to_host(), 4 + np.cumsum(a))
    # no-init overload with multiplies uses value_type() == 0 (inclusive_scan.hpp:526): all zeros
    P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), F.multiplies)
    np.testing.assert_array_equal(o.to_host(), O.scan(a, 0, True, op="multiplies"))


def test_transform_scans(pol, gpu_target):
    a = rnd(np.int64, 40000, 14, -100, 100)
    d, o = dev(a, gpu_target), hpx.vector(len(a), dtype=np.int64, tgt=gpu_target)
    P.transform_inclusive_scan(pol, d.begin(), d.end(), o.begin(), F.plus, F.square(), 1)
    np.testing.assert_array_equal(o.to_host(), O.scan(a, 1, True, conv="square"))
    P.transform_exclusive_scan(pol, d.begin(), d.end(), o.begin(), 1, F.plus, F.multiply_step(3))
    np.testing.assert_array_equal(o.to_host(), O.scan(a, 1, False, conv="scale", scalars=(3,)))


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_scan_fp_tolerance(pol, gpu_target, dt):
    a = np.abs(rnd(dt, 1 << 20, 15))
    d, o = dev(a, gpu_target), hpx.vector(len(a), dtype=dt, tgt=gpu_target)
    P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), F.plus, 0)
    got = o.to_host().astype(np.longdouble)
    exact = np.cumsum(a.astype(np.longdouble))  # 64-bit-mantissa reference
    # Tolerance: non-negative inputs, so every partial sum is <=
    # out[i]; the GPU association chains the look-back across tiles
    # (ntiles adds) on top of lane (V), round (8), wave (7) and tile-wave (4)
    # levels: |err| <= (ntiles + 64) * u * out[i].
    u = 2.0 ** -24 if dt == np.float32 else 2.0 ** -53
    tile = 1024 * 8 * (16 // np.dtype(dt).itemsize)
    k = (a.size + tile - 1) // tile + 64
    assert np.all(np.abs(got - exact) <= k * u * exact + 1e-300)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("incl", [True, False])
def test_scan_fp_reproducible(pol, gpu_target, dt, incl):
    """FP scans use the fixed-association look-back (lookback.hpp
    exclusive_prefix_fixed): the result is a function of the input alone, so
    repeated runs agree bit for bit -- over many 64-tile groups (2^25 + 5
    elements: 256-1024 tiles), mixed signs, a ragged last tile -- and stay
    within the scan tolerance of a 64-bit-mantissa cumulative sum."""
    n = (1 << 25) + 5
    a = rnd(dt, n, 77) - dt(0.5)
    d = dev(a, gpu_target)
    outs = []
    for _ in range(3):
        o = hpx.vector(n, dtype=dt, tgt=gpu_target)
        if incl:
            P.inclusive_scan(pol, d.begin(), d.end(), o.begin(), F.plus, dt(0.25))
        else:
            P.exclusive_scan(pol, d.begin(), d.end(), o.begin(), dt(0.25))
        outs.append(o.to_host())
    for o in outs[1:]:
        np.testing.assert_array_equal(o.view(np.uint8), outs[0].view(np.uint8))
    exact = np.cumsum(np.concatenate([[0.25], a.astype(np.longdouble)]))
    exact = exact[1:] if incl else exact[:-1]
    u = 2.0 ** -24 if dt == np.float32 else 2.0 ** -53
    mag = np.cumsum(np.concatenate([[0.25], np.abs(a).astype(np.longdouble)]))
    mag = mag[1:] if incl else mag[:-1]
    tile = 1024 * 12 * (16 // np.dtype(dt).itemsize)
    k = (n + tile - 1) // tile + 96
    assert np.all(np.abs(outs[0].astype(np.longdouble) - exact) <= k * u * mag)


def test_scan_large_property(pol, gpu_target):
    """Size-independent property at 2^27: inclusive - exclusive == input and
    last inclusive == reduce (int64, exact)."""
    n = 1 << 27
    x = hpx.vector(n, dtype=np.int64, tgt=gpu_target)
    P.generate(pol, x.begin(), x.end(), "range", 0x5EED, -(1 << 20), 1 << 20)
    inc, exc = hpx.vector(n, dtype=np.int64, tgt=gpu_target), hpx.vector(n, dtype=np.int64, tgt=gpu_target)
    P.inclusive_scan(pol, x.begin(), x.end(), inc.begin(), F.plus, 0)
    P.exclusive_scan(pol, x.begin(), x.end(), exc.begin(), 0)
    d = hpx.vector(n, dtype=np.int64, tgt=gpu_target)
    P.transform(pol, inc.begin(), inc.end(), exc.begin(), d.begin(), F.subtract())
    P.transform(pol, d.begin(), d.end(), x.begin(), d.begin(), F.subtract())
    assert P.reduce(pol, d.begin(), d.end(), 0, F.bit_or) == 0
    total = P.reduce(pol, x.begin(), x.end(), 0, F.plus)
    assert inc[n - 1] == total
    host = O.generate(np.int64, "range", n, 0x5EED, -(1 << 20), 1 << 20)
    assert total == int(host.sum())


# ---------------------------------------------------------------- copy_if
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dt", [np.int32, np.int64, np.float64])
def test_copy_if_exact(pol, gpu_target, n, dt):
    a = rnd(dt, n, 16, *((-1000, 1000) if np.dtype(dt).kind == "i" else ()))
    d, o = dev(a, gpu_target), hpx.vector(max(n, 1), dtype=dt, tgt=gpu_target)
    _, end = P.copy_if(pol, d.begin(), d.end(), o.begin(), F.not_less_than(0))
    exp = O.copy_if(a, "not_less_than", 0)
    assert end - o.begin() == exp.size
    np.testing.assert_array_equal(o.to_host()[: exp.size], exp)


@pytest.mark.parametrize("pred,name,arg", [(F.less_than(10), "lt", 10), (F.equal_to(3), "eq", 3),
                                           (F.any_bits(4), "bits", 4), (F.greater_than(1 << 30), "gt", 1 << 30)])
def test_copy_if_predicates(pol, gpu_target, pred, name, arg):
    a = rnd(np.int64, 200003, 17, -20, 20)
    d, o = dev(a, gpu_target), hpx.vector(len(a), dtype=np.int64, tgt=gpu_target)
    _, end = P.copy_if(pol, d.begin(), d.end(), o.begin(), pred)
    exp = O.copy_if(a, name, arg)
    assert end - o.begin() == exp.size
    np.testing.assert_array_equal(o.to_host()[: exp.size], exp)


@pytest.mark.parametrize("dt,n,sel", [(np.int64, (64 * 3 + 5) * 16384 + 777, 0.5), (np.float64, (64 * 2 + 40) * 16384, 0.5),
                                      (np.int64, (64 * 2 + 1) * 16384 + 1, 0.97), (np.int64, 64 * 16384 * 2 + 3, 0.02),
                                      (np.int32, (64 * 3 + 5) * 32768 + 9, 0.5),
                                      (np.int64, 1000 * 16384 + 4321, 0.5), (np.int64, 777 * 16384, 1.0),
                                      (np.int64, 600 * 16384 + 3, 0.0), (np.int32, 700 * 32768 + 5, 0.5),
                                      (np.int32, 530 * 32768 + 2, 1.0)])
def test_copy_if_lookback_groups(pol, gpu_target, dt, n, sel):
    """Several 64-tile look-back groups and a partial last one (16384-element
    8-byte tiles, 32768-element 4-byte tiles), empty, near-empty, near-full
    and full selections, and an output that starts 8 B past a 16-B boundary.
    From 600 tiles on, each persistent workgroup of the pipelined form (one
    per CU) walks several tiles: a full tile's hits fill its LDS stage."""
    rng = np.random.default_rng(n)
    a = (rng.random(n) < sel).astype(np.int64) * 2 - 1  # +1 selected, -1 not
    a = (a * rng.integers(1, 1000, n)).astype(dt)
    d, o = dev(a, gpu_target), hpx.vector(n + 1, dtype=dt, tgt=gpu_target)
    exp = O.copy_if(a, "not_less_than", 0)
    for off in (0, 1):
        _, end = P.copy_if(pol, d.begin(), d.end(), o.begin() + off, F.not_less_than(0))
        assert end - o.begin() == exp.size + off
        np.testing.assert_array_equal(o.to_host()[off:off + exp.size], exp)


def test_copy_if_golden(pol, gpu_target):
    case = golden_cases("copy_if")[0]
    g = load_golden(case)
    d, o = dev(g["input"], gpu_target), hpx.vector(len(g["input"]), dtype=np.int32, tgt=gpu_target)
    _, end = P.copy_if(pol, d.begin(), d.end(), o.begin(), F.not_less_than(0))
    k = end - o.begin()
    assert k == g["expected"].size
    np.testing.assert_array_equal(o.to_host()[:k], g["expected"])


# ------------------------------------------------------------------- sort
@pytest.mark.parametrize("n", SIZES + [(1 << 23) + 11])
@pytest.mark.parametrize("dt", INT_DT)
def test_sort_int_exact(pol, gpu_target, n, dt):
    a = rnd(dt, n, 18)
    d = dev(a, gpu_target)
    P.sort(pol, d.begin(), d.end())
    np.testing.assert_array_equal(d.to_host(), O.sort(a))


@pytest.mark.parametrize("dt", ALL_DT)
def test_sort_descending_and_narrow_ranges(pol, gpu_target, dt):
    a = rnd(dt, 300007, 19, *((0, 3) if np.dtype(dt).kind in "iu" else ()))  # few digits -> skipped passes
    d = dev(a, gpu_target)
    P.sort(pol, d.begin(), d.end(), F.greater)
    np.testing.assert_array_equal(d.to_host(), O.sort(a, descending=True))
    P.sort(pol, d.begin(), d.end())
    np.testing.assert_array_equal(d.to_host(), O.sort(a))


def test_sort_floats_special_values(pol, gpu_target):
    a = np.array([3.0, -0.0, 0.0, -np.inf, np.inf, -1.5, 2.25, -0.0, 1e-300, -1e300] * 1000, np.float64)
    d = dev(a, gpu_target)
    P.sort(pol, d.begin(), d.end())
    np.testing.assert_array_equal(d.to_host().view(np.uint64), O.sort(a).view(np.uint64))


def test_sort_sub_range_and_sorted_input(pol, gpu_target):
    a = rnd(np.int64, 100000, 20)
    d = dev(a, gpu_target)
    P.sort(pol, d.begin() + 17, d.end() - 5)
    exp = a.copy()
    exp[17:-5] = np.sort(a[17:-5])
    np.testing.assert_array_equal(d.to_host(), exp)
    P.sort(pol, d.begin(), d.end())
    P.sort(pol, d.begin(), d.end())  # already sorted
    np.testing.assert_array_equal(d.to_host(), np.sort(a))


@pytest.mark.parametrize("vdt", [np.int32, np.uint64, np.float64])
def test_sort_by_key_stable(pol, gpu_target, vdt):
    n = 200003
    k = rnd(np.uint32, n, 21, 0, 1000)  # many duplicates: checks stability
    v = np.arange(n).astype(vdt)
    dk, dv = dev(k, gpu_target), dev(v, gpu_target)
    P.sort_by_key(pol, dk.begin(), dk.end(), dv.begin())
    ek, ev = O.sort_by_key(k, v)
    np.testing.assert_array_equal(dk.to_host(), ek)
    np.testing.assert_array_equal(dv.to_host(), ev)


# ---------------------------------------------------------------- stencil
def test_stencil_golden_and_random(gpu_target):
    from hpx_amd import stencil
    case = golden_cases("stencil")[0]
    g = load_golden(case)
    out = stencil.heat_run(g["input"], 1, tgt=gpu_target)
    np.testing.assert_array_equal(out, g["expected"])
    for nx, nt in [(1, 3), (2, 5), (3, 5), (1001, 17), (1 << 16, 50)]:
        u = rnd(np.float64, nx, 22 + nx)
        np.testing.assert_array_equal(stencil.heat_run(u, nt, tgt=gpu_target), O.stencil_heat(u, nt))


@pytest.mark.parametrize("nx", [1024, 4097, 100003])
def test_stencil_fused_run_bit_exact(gpu_target, nx):
    """hpxhip_stencil_heat_run with temporal blocking (passes of up to 16
    steps, the pass count matched to nt's parity so the result lands in the
    documented buffer) against the serial oracle, bit for bit."""
    from hpx_amd import stencil
    u = rnd(np.float64, nx, 31 + nx)
    for nt in [1, 2, 3, 4, 5, 7, 8, 9, 10, 16, 17, 26, 33, 48]:
        np.testing.assert_array_equal(stencil.heat_run(u, nt, tgt=gpu_target), O.stencil_heat(u, nt), err_msg=f"nt={nt}")
    # hpxhip_stencil_heat_run keeps its buffer contract (u0 for even nt, u1 for odd)
    import ctypes
    from hpx_amd import _lib as L
    for nt in [8, 9, 10]:
        a, b = dev(u, gpu_target), hpx.vector(nx, dtype=np.float64, tgt=gpu_target)
        L.call("hpxhip_stencil_heat_run", ctypes.c_void_p(a.data()), ctypes.c_void_p(b.data()), nx, nt,
               ctypes.c_double(0.5), ctypes.c_double(1.0), ctypes.c_double(1.0), gpu_target.stream)
        res = a if nt % 2 == 0 else b
        np.testing.assert_array_equal(res.to_host(), O.stencil_heat(u, nt), err_msg=f"heat_run nt={nt}")


@pytest.mark.parametrize("steps", [1, 2, 4, 6, 8, 10, 16])
def test_stencil_heat_steps_halos_subranges(gpu_target, steps):
    """hpxhip_stencil_heat_steps: explicit `steps`-point halos, output
    sub-ranges (even and odd starts), misaligned buffers; expected = `steps`
    single steps of the oracle on [halo | cur | halo], whose inner n points
    are exact."""
    import ctypes
    from hpx_amd import _lib as L
    rng = np.random.default_rng(40 + steps)
    for n, off in [(5000, 0), (4099, 1), (700, 0)]:
        cur = rng.standard_normal(n)
        lh, rh = rng.standard_normal(steps), rng.standard_normal(steps)
        ext = np.concatenate([lh, cur, rh])
        for _ in range(steps):
            ext = O.stencil_heat_step(ext, 0.0, 0.0)
        exp = ext[steps:steps + n]
        dcur = hpx.vector.from_host(np.concatenate([np.zeros(off), cur]), gpu_target)
        dlh, drh = hpx.vector.from_host(lh, gpu_target), hpx.vector.from_host(rh, gpu_target)
        for lo, hi in [(0, n), (1, n - 3), (n // 3, n // 3 + 1), (n - 1, n)]:
            dnext = hpx.vector(n + off, dtype=np.float64, value=-7.0, tgt=gpu_target)
            L.call("hpxhip_stencil_heat_steps", ctypes.c_void_p(dcur.data() + 8 * off),
                   ctypes.c_void_p(dnext.data() + 8 * off), n, lo, hi, ctypes.c_void_p(dlh.data()),
                   ctypes.c_void_p(drh.data()), steps, ctypes.c_double(0.5), ctypes.c_double(1.0),
                   ctypes.c_double(1.0), gpu_target.stream)
            got = dnext.to_host()[off:]
            np.testing.assert_array_equal(got[lo:hi], exp[lo:hi], err_msg=f"n={n} off={off} [{lo},{hi})")
            assert np.all(got[:lo] == -7.0) and np.all(got[hi:] == -7.0)


def test_device_error_word_clear(gpu_target):
    hpx.compute.device_error_check(gpu_target.device)


@pytest.mark.parametrize("n", [0, 1, 65, 4097, 100003, (1 << 20) + 17, 1 << 23])
def test_copy_if_state64(pol, gpu_target, n, monkeypatch):
    """The 64-bit look-back form (used from 2^32 elements on) at small n."""
    monkeypatch.setenv("HPXHIP_COPY_IF_STATE64", "1")
    a = rnd(np.int64, n, 23, -1000, 1000)
    d, o = dev(a, gpu_target), hpx.vector(max(n, 1), dtype=np.int64, tgt=gpu_target)
    _, end = P.copy_if(pol, d.begin(), d.end(), o.begin(), F.not_less_than(0))
    exp = O.copy_if(a, "not_less_than", 0)
    assert end - o.begin() == exp.size
    np.testing.assert_array_equal(o.to_host()[: exp.size], exp)


@pytest.mark.gpu
def test_roctx_annotation_path():
    """HPXHIP_ROCTX=1 (roctx range per C-ABI algorithm call, the
    annotate_function analogue) leaves results unchanged: a scan and a sort
    in a child process with the ranges on."""
    import subprocess
    import sys
    code = (
        "import numpy as np, hpx_amd as hpx\n"
        "from hpx_amd import execution as ex, parallel as P\n"
        "t = hpx.target(0); pol = ex.par.on(hpx.default_executor(t))\n"
        "v = hpx.vector(100003, dtype=np.int64, tgt=t); P.generate(pol, v.begin(), v.end(), 'range', 5, -9, 9)\n"
        "h = np.array([v[i] for i in range(0, 100003, 997)])\n"
        "w = hpx.vector(100003, dtype=np.int64, tgt=t)\n"
        "P.inclusive_scan(pol, v.begin(), v.end(), w.begin())\n"
        "s = P.reduce(pol, v.begin(), v.end(), 0)\n"
        "assert w[100002] == s, (w[100002], s)\n"
        "P.sort(pol, v.begin(), v.end()); assert P.is_sorted(pol, v.begin(), v.end())\n"
        "print('roctx ok')\n")
    env = dict(os.environ, HPXHIP_ROCTX="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "roctx ok" in r.stdout, r.stdout + r.stderr


# ---- misaligned sub-ranges through the head split (scan: input and output
# with the same offset inside 16 B -> one-thread head scan to a 1-KiB output
# boundary, vector kernel seeded with its carry; copy_if: misaligned input ->
# head compacted first, vector kernel seeded with its count) and through the
# element-wise kernels, against the oracle.  r04: mutually misaligned
# ranges (offsets that differ inside 16 B) take the vector kernel with the
# input shifted across lanes (k_scan SHIFTED) after the same head split.
@pytest.mark.parametrize("dt", [np.int64, np.int32, np.uint32, np.float64])
@pytest.mark.parametrize("oin,oout", [(1, 1), (2, 2), (3, 3), (1, 0), (0, 3), (5, 5), (0, 1), (2, 1), (3, 0),
                                      (1, 2), (6, 1)])
@pytest.mark.parametrize("incl", [True, False])
def test_scan_misaligned_subranges(pol, gpu_target, dt, oin, oout, incl):
    n = 300007
    if np.dtype(dt).kind == "f":  # small integers in doubles: exact sums in any association
        a = rnd(np.int64, n, 31, -1000, 1000).astype(dt)
    else:
        a = rnd(dt, n, 31, *((-1000, 1000) if np.dtype(dt).kind == "i" else (0, 1000)))
    d = dev(a, gpu_target)
    o = hpx.vector(n, dtype=dt, tgt=gpu_target)
    m = n - max(oin, oout) - 11
    if incl:
        P.inclusive_scan(pol, d.begin() + oin, d.begin() + oin + m, o.begin() + oout, F.plus, 7)
    else:
        P.exclusive_scan(pol, d.begin() + oin, d.begin() + oin + m, o.begin() + oout, 7)
    np.testing.assert_array_equal(o.to_host()[oout:oout + m], O.scan(a[oin:oin + m], 7, incl))


@pytest.mark.parametrize("dt,oin,oout", [(np.int64, 1, 0), (np.int64, 0, 1), (np.int32, 3, 1), (np.float64, 1, 0)])
def test_scan_shifted_input_large(pol, gpu_target, dt, oin, oout):
    # 2^24 + 5 elements: many tiles of the shifted vector kernel, the last
    # one partial; int64/int32 exact, doubles hold small integers
    n = (1 << 24) + 5
    a = rnd(np.int64, n, 41, -50, 50).astype(dt)
    d = dev(a, gpu_target)
    o = hpx.vector(n, dtype=dt, tgt=gpu_target)
    m = n - max(oin, oout) - 3
    P.inclusive_scan(pol, d.begin() + oin, d.begin() + oin + m, o.begin() + oout, F.plus, 3)
    np.testing.assert_array_equal(o.to_host()[oout:oout + m], O.scan(a[oin:oin + m], 3, True))


@pytest.mark.parametrize("off", [1, 3])
def test_scan_misaligned_in_place_f64(pol, gpu_target, off):
    # all-1.0 doubles (exact sums): in place, both ends trimmed
    n = 1 << 20
    a = np.ones(n, np.float64)
    d = dev(a, gpu_target)
    m = n - off - 5
    P.inclusive_scan(pol, d.begin() + off, d.begin() + off + m, d.begin() + off, F.plus, 0.0)
    got = d.to_host()
    np.testing.assert_array_equal(got[off:off + m], np.arange(1, m + 1, dtype=np.float64))
    assert got[0] == 1.0 and got[-1] == 1.0


@pytest.mark.parametrize("dt,off", [(np.int64, 1), (np.int32, 1), (np.int32, 2), (np.int32, 3), (np.float64, 1)])
@pytest.mark.parametrize("oout", [0, 1])
def test_copy_if_misaligned_input(pol, gpu_target, dt, off, oout):
    n = 500009
    a = rnd(dt, n, 37, *((-1000, 1000) if np.dtype(dt).kind == "i" else ()))
    a[off] = 5  # a hit inside the head
    d, o = dev(a, gpu_target), hpx.vector(n, dtype=dt, tgt=gpu_target)
    _, end = P.copy_if(pol, d.begin() + off, d.end(), o.begin() + oout, F.not_less_than(0))
    exp = O.copy_if(a[off:], "not_less_than", 0)
    assert end - (o.begin() + oout) == exp.size
    np.testing.assert_array_equal(o.to_host()[oout:oout + exp.size], exp)


# ---- mutually misaligned elementwise ranges (inputs offset from the output
# inside 16 B): the shifted-vector kernels (aligned vectors i and i+1 of each
# misaligned input, elements shifted in registers), bit-exact against the
# oracle for every relative offset of 8-B and 4-B elements, with partial
# last waves.
@pytest.mark.parametrize("dt", [np.float64, np.int64, np.int32, np.float32])
@pytest.mark.parametrize("oa,ob,oo", [(1, 0, 0), (0, 1, 3), (1, 2, 0), (3, 1, 2), (2, 2, 1), (0, 0, 1)])
@pytest.mark.parametrize("n", [100003, 3001])
def test_transform_binary_shifted(pol, gpu_target, dt, oa, ob, oo, n):
    a, b = rnd(dt, n, 41, *((-1000, 1000) if np.dtype(dt).kind == "i" else ())), rnd(dt, n, 42, *((-1000, 1000) if np.dtype(dt).kind == "i" else ()))
    da, db = dev(a, gpu_target), dev(b, gpu_target)
    do = hpx.vector(n, dtype=dt, tgt=gpu_target)
    m = n - 7
    P.transform(pol, da.begin() + oa, da.begin() + oa + m, db.begin() + ob, db.begin() + ob + m, do.begin() + oo,
                F.add_step())
    np.testing.assert_array_equal(do.to_host()[oo:oo + m], O.transform_binary(a[oa:oa + m], b[ob:ob + m], "add"))


@pytest.mark.parametrize("dt", [np.float64, np.int32])
@pytest.mark.parametrize("oi,oo", [(1, 0), (0, 1), (3, 0), (2, 5)])
def test_transform_unary_shifted(pol, gpu_target, dt, oi, oo):
    n = 100003
    x = rnd(dt, n, 43, *((-1000, 1000) if np.dtype(dt).kind == "i" else ()))
    dx = dev(x, gpu_target)
    do = hpx.vector(n, dtype=dt, tgt=gpu_target)
    m = n - 9
    P.copy(pol, dx.begin() + oi, dx.begin() + oi + m, do.begin() + oo)
    np.testing.assert_array_equal(do.to_host()[oo:oo + m], x[oi:oi + m])


# ---- concurrent_executor (cuda/concurrent_executor.hpp:29-234): several
# streams on one device, successive calls rotate over them.  Synchronous
# policies order each call; task policies give independent futures that
# when_all joins.
def test_concurrent_executor_python(gpu_target):
    cexec = hpx.concurrent_executor(gpu_target, 3)
    pol = ex.par.on(cexec)
    n = 1 << 20
    xs = [dev(np.arange(n, dtype=np.int64) * (k + 1), gpu_target) for k in range(6)]
    ys = [hpx.vector(n, dtype=np.int64, tgt=gpu_target) for _ in range(6)]
    for x, y in zip(xs, ys):  # sync calls on rotating streams
        P.inclusive_scan(pol, x.begin(), x.end(), y.begin(), F.plus, 0)
    for k, y in enumerate(ys):
        assert y[n - 1] == (k + 1) * n * (n - 1) // 2
    tpol = ex.par(ex.task).on(cexec)
    fs = [P.reduce(tpol, x.begin(), x.end(), 0, F.plus) for x in xs]
    vals = [f.get() for f in hpx.when_all(*fs).get()]
    assert vals == [(k + 1) * n * (n - 1) // 2 for k in range(6)]
    # executor customisation points on the rotating streams
    seen = []
    key = lambda s: getattr(s, "value", s)  # noqa: E731 -- stream handles are ctypes pointers
    cexec.sync_execute(lambda s: seen.append(key(s)))
    cexec.post(lambda s: seen.append(key(s)))
    cexec.async_execute(lambda s: seen.append(key(s))).get()
    assert len(set(seen)) == 3  # three calls, three different streams
    cexec.synchronize()
