"""Pin the CPU oracle against the reference's own known-answer tests
(tests/golden/*.npz, closed forms from the reference test sources) and check
its par-chunk semantics against its seq semantics where the reference's
tests require equality (seq == par for integer work)."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden
from oracle import oracle as O


@pytest.mark.parametrize("case", golden_cases("exclusive_scan"), ids=lambda c: c["name"])
@pytest.mark.parametrize("cores", [0, 1, 3, 8])
def test_exclusive_scan_validate(case, cores):
    g = load_golden(case)
    out = O.scan(g["input"], case["init"], inclusive=False, cores=cores)
    np.testing.assert_array_equal(out, g["expected"])


@pytest.mark.parametrize("case", golden_cases("inclusive_scan"), ids=lambda c: c["name"])
@pytest.mark.parametrize("cores", [0, 2, 16])
def test_inclusive_scan_golden(case, cores):
    g = load_golden(case)
    out = O.scan(g["input"], case["init"], inclusive=True, cores=cores)
    np.testing.assert_array_equal(out, g["expected"])  # bit-exact, incl. the all-ones doubles


def test_copyif_random():
    case = golden_cases("copy_if")[0]
    g = load_golden(case)
    np.testing.assert_array_equal(O.copy_if(g["input"], case["pred"], case["arg"]), g["expected"])


@pytest.mark.parametrize("case", golden_cases("reduce"), ids=lambda c: c["name"])
@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_partitioned_vector_reduce(case, parts):
    g = load_golden(case)
    got = O.segmented_reduce(g["input"], case["init"], parts)
    assert got == g["expected"][0]
    assert O.transform_reduce(g["input"], case["init"]) == g["expected"][0]
    assert O.transform_reduce(g["input"], case["init"], cores=4) == g["expected"][0]


@pytest.mark.parametrize("cores", [0, 1, 7])
def test_transform_reduce_product(cores):
    case = golden_cases("transform_reduce")[0]
    g = load_golden(case)
    got = O.transform_reduce(g["input"], case["init"], op="multiplies", cores=cores)
    assert got == g["expected"][0]


def test_transform_compute():
    case = golden_cases("transform_binary")[0]
    g = load_golden(case)
    out = O.transform_binary(g["input"], g["input2"], "triad", (3.0,), compute="float64")
    np.testing.assert_array_equal(out, g["expected"])


def test_for_each_compute():
    case = golden_cases("for_each")[0]
    g = load_golden(case)
    np.testing.assert_array_equal(O.for_each(g["input"], "add_scalar", (5,)), g["expected"])


@pytest.mark.parametrize("case", golden_cases("stream"), ids=lambda c: c["name"])
def test_stream_closed_form(case):
    g = load_golden(case)
    assert O.stream_expected(case["iterations"], case["scalar"]) == tuple(g["expected"])


def test_stream_loop_matches_closed_form():
    # the STREAM kernel sequence (stream.cpp:294-375) restated with the oracle's
    # transforms reproduces check_results' closed form exactly
    n = 1000
    a = np.full(n, 1.0)
    b = np.full(n, 2.0)
    c = np.zeros(n)
    a = O.transform(a, "scale", (2.0,))
    iters = 5
    for _ in range(iters):
        c = a.copy()
        b = O.transform(c, "scale", (3.0,))
        c = O.transform_binary(a, b, "add")
        a = O.transform_binary(b, c, "triad", (3.0,))
    aj, bj, cj = O.stream_expected(iters)
    assert np.all(a == aj) and np.all(b == bj) and np.all(c == cj)


def test_stencil_ramp_closed_form():
    case = golden_cases("stencil")[0]
    g = load_golden(case)
    np.testing.assert_array_equal(O.stencil_heat(g["input"], 1), g["expected"])
    left = g["input"][-1]
    right = g["input"][0]
    np.testing.assert_array_equal(O.stencil_heat_step(g["input"], left, right), g["expected"])


def test_sort_sortedness_and_permutation():
    # sort_tests.hpp:122-145 checks sortedness; also a permutation of the input
    rng = np.random.default_rng(3)
    for dt in (np.int32, np.uint32, np.int64, np.uint64):
        x = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, 5000, dtype=dt, endpoint=True)
        s = O.sort(x)
        np.testing.assert_array_equal(s, np.sort(x))
        np.testing.assert_array_equal(O.sort(x, descending=True), np.sort(x)[::-1])
    f = rng.standard_normal(5000)
    np.testing.assert_array_equal(O.sort(f), np.sort(f))


def test_seq_equals_par_integer():
    rng = np.random.default_rng(5)
    x = rng.integers(-1000, 1000, 12345, dtype=np.int64)
    for op in ("plus", "min", "max", "bit_xor"):
        assert O.transform_reduce(x, 3, op=op) == O.transform_reduce(x, 3, op=op, cores=5)
        for incl in (True, False):
            np.testing.assert_array_equal(O.scan(x, 3, incl, op=op), O.scan(x, 3, incl, op=op, cores=5))


def test_segmented_scan_equals_scan():
    rng = np.random.default_rng(9)
    x = rng.integers(-50, 50, 10007, dtype=np.int64)
    for parts in (1, 3, 8):
        for incl in (True, False):
            np.testing.assert_array_equal(O.segmented_scan(x, 7, parts, incl), O.scan(x, 7, incl))


def test_generate_restatement_is_deterministic():
    a = O.generate(np.uint64, "bits", 1000, seed=1)
    b = O.generate(np.uint64, "bits", 500, seed=1, offset=500)
    np.testing.assert_array_equal(a[500:], b)
    r = O.generate(np.int64, "range", 10000, seed=2, lo=-(1 << 20), hi=1 << 20)
    assert r.min() >= -(1 << 20) and r.max() <= (1 << 20)
    u = O.generate(np.float64, "unit", 10000, seed=3)
    assert u.min() >= 0.0 and u.max() < 1.0


def test_stencil_window_equals_full_ring():
    """oracle.stencil_window (the +-nt window restatement the 2^32-point GPU
    check uses) against the full periodic-ring oracle, at the seam, inside,
    wrapping both ends, and in the small-ring fallback."""
    nx, seed = 4099, 0xC0FFEE
    for nt in (1, 2, 17, 100):
        full = O.stencil_heat(O.unit_at(np.arange(nx, dtype=np.uint64), seed), nt)
        for lo, c in [(0, 64), (nx - 64, 64), (nx - 1, 1), (1000, 333), (2048 - nt, 2 * nt + 1)]:
            np.testing.assert_array_equal(O.stencil_window(nx, nt, seed, lo, c), full[lo:lo + c])
    small = O.stencil_heat(O.unit_at(np.arange(50, dtype=np.uint64), 3), 40)
    np.testing.assert_array_equal(O.stencil_window(50, 40, 3, 10, 20), small[10:30])
    # unit_at is generate("unit") at arbitrary indices
    np.testing.assert_array_equal(O.unit_at(np.arange(7, 20, dtype=np.uint64), 9),
                                  O.generate(np.float64, "unit", 13, 9, offset=7))


@pytest.mark.parametrize("iters", [2, 10])
def test_par_stream_check_results(iters):
    """The host-par STREAM (cpu_baseline's configs[0] leg) ends on
    check_results' closed form (stream.cpp:82-133), as the golden fixture."""
    times, abc = O.par_stream(100003, 3, 3.0, iters)
    assert abc == tuple(O.stream_expected(iters, 3.0))
    assert set(times) == {"copy", "scale", "add", "triad"} and all(b > 0 and a > 0 for b, a in times.values())
