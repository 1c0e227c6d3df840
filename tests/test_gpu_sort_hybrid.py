"""The hybrid tail of the sort (64- and 32-bit keys, and sort_by_key), planned
on the device (sort.hip k_sort_plan): two onesweep passes on the prefix --
the top byte and the 9 bits under it (17-bit form) or the two top live bytes
(16-bit form) --, bucket bounds by lower_bound over buckets of the top byte
plus b2 bits, b2 chosen from the histograms, one LDS-resident sort per
bucket (512- or 1024-thread segments); up to 64 buckets over their
segment's capacity are finished by a segmented LSD over their own ranges,
more send the whole array through the LSD over the live digits.  Checked element for
element against the oracle on the distributions that steer it down each
branch, in every form (HPXHIP_SORT_HYBRID=17 / 16 / 18; 18: two 9-bit
prefix passes and ~4096-key buckets).  Sizes start at the
hybrid's 2^22-key threshold.

Parity: std::sort's order for integer keys (sort.hpp:78-229, restated by the
oracle's O.sort as std::sort on the keys' ordered bits, oracle/oracle.cpp) and
the IEEE total order for doubles (-0.0 before +0.0)."""
import numpy as np
import pytest

import hpx_amd as hpx
from hpx_amd import execution as ex, functional as F
from hpx_amd import parallel as P
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pol(gpu_target):
    return ex.par.on(hpx.default_executor(gpu_target))


@pytest.fixture(params=["17", "16", "18"], autouse=True)
def form(request, monkeypatch):
    monkeypatch.setenv("HPXHIP_SORT_HYBRID", request.param)
    return request.param


def check(pol, tgt, h, desc=False):
    v = hpx.vector.from_host(h, tgt)
    P.sort(pol, v.begin(), v.end(), F.greater if desc else F.less)
    got = v.to_host()
    v.free()
    np.testing.assert_array_equal(got, O.sort(h, desc))


@pytest.mark.parametrize("logn", [22, 24, 25])
@pytest.mark.parametrize("desc", [False, True])
def test_uniform_u64(pol, gpu_target, logn, desc):
    # 2^22: buckets of ~64 keys packed into multi-bucket segments (prefix passes
    # run in LDS); 2^24: ~256-key buckets
    h = np.random.default_rng(logn).integers(0, 2**64 - 1, 1 << logn, dtype=np.uint64, endpoint=True)
    check(pol, gpu_target, h, desc)


@pytest.mark.parametrize("dt", [np.int64, np.float64])
def test_signed_and_double(pol, gpu_target, dt):
    rng = np.random.default_rng(5)
    n = (1 << 23) + 12345
    if dt is np.float64:
        h = rng.standard_normal(n) * np.exp2(rng.integers(-60, 60, n))
        h[:5] = [0.0, -0.0, np.inf, -np.inf, 1e-310]
    else:
        h = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)


def test_constant_middle_digits(pol, gpu_target):
    # bits 40..59 zero: live digits 7, 4, 3, 2, 1, 0 -> prefix (7, 4), 1024 buckets of ~8K
    rng = np.random.default_rng(11)
    n = 1 << 23
    h = (rng.integers(0, 4, n, dtype=np.uint64) << np.uint64(60)) | rng.integers(0, 1 << 40, n, dtype=np.uint64)
    check(pol, gpu_target, h)


def test_few_oversized_buckets(pol, gpu_target):
    # one prefix (0x12, 0x34) holds 30000 extra keys: its bucket exceeds the LDS
    # segment and is finished by the segmented LSD over its own range (r05);
    # the marginal histograms alone do not reveal it
    rng = np.random.default_rng(12)
    n = 1 << 23
    h = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    h[:30000] = (np.uint64(0x1234) << np.uint64(48)) | rng.integers(0, 1 << 48, 30000, dtype=np.uint64)
    h[30000:30100] = np.uint64(0x1234) << np.uint64(48)  # duplicates inside the big bucket
    check(pol, gpu_target, h)


@pytest.mark.parametrize("desc", [False, True])
def test_several_oversized_buckets(pol, gpu_target, desc):
    """r05: up to kMaxBig (64) oversized buckets are finished by a segmented
    LSD over just their ranges (sort.hip k_sort_fallback): 11 hot prefixes of
    very different sizes (one barely over a segment, one of n/8 keys), with
    duplicates inside and keys at both ends of the key range."""
    rng = np.random.default_rng(21)
    n = 1 << 23
    h = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    o = 0
    for i, m in enumerate([19000, 25000, 40000, 70000, n // 8, 9000, 12000, 30000, 5000, 100000, 20000]):
        prefix = np.uint64((0x0000 + 0x1777 * (i + 1)) & 0xFFFF) << np.uint64(48)
        h[o:o + m] = prefix | rng.integers(0, 1 << 48, m, dtype=np.uint64)
        h[o:o + m // 50] = prefix | np.uint64(7)  # a run of duplicates in the bucket
        o += m
    h[o] = np.uint64(0)
    h[o + 1] = np.uint64(2**64 - 1)
    check(pol, gpu_target, h, desc)


def test_many_oversized_buckets(pol, gpu_target):
    # digit 6 == digit 7 for every key: 256 buckets of 32K keys, more than the
    # 64 the segmented finish keeps -> the whole-array LSD
    rng = np.random.default_rng(13)
    n = 1 << 23
    top = rng.integers(0, 256, n, dtype=np.uint64)
    h = (top << np.uint64(56)) | (top << np.uint64(48)) | rng.integers(0, 1 << 48, n, dtype=np.uint64)
    check(pol, gpu_target, h)


def test_heavy_duplicates(pol, gpu_target):
    # few distinct values: most digits constant -> fewer than three live digits (LSD)
    rng = np.random.default_rng(14)
    n = 1 << 23
    vals = rng.integers(0, 2**64 - 1, 3, dtype=np.uint64, endpoint=True)
    check(pol, gpu_target, vals[rng.integers(0, 3, n)])
    # 2^16 distinct values spread over all digits: buckets of duplicates
    vals = rng.integers(0, 2**64 - 1, 1 << 16, dtype=np.uint64, endpoint=True)
    check(pol, gpu_target, vals[rng.integers(0, 1 << 16, n)])


def test_buckets_past_the_typical_grid(pol, gpu_target):
    """The segment sort is launched with one workgroup per bucket for the
    buckets a typical plan of n keys has (2 n / 8192) and a striding launch
    for the rest (sort.hip): skewed keys whose planned buckets lie past that
    grid -- top byte 0xF0 for all keys but one (17-bit form, buckets from
    0xF0 << 9 on), a constant top byte (16-bit form on the next two bytes,
    more buckets than the grid) -- must be sorted by the second launch."""
    rng = np.random.default_rng(0xB0C)
    n = 1 << 22
    low = rng.integers(0, 1 << 56, n, dtype=np.uint64)
    h = low | np.uint64(0xF0 << 56)
    h[12345] = low[12345]
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)
    check(pol, gpu_target, low | np.uint64(0xC3 << 56))


@pytest.mark.parametrize("choices", [1, 2, 8, 64])
def test_equal_prefix_runs(pol, gpu_target, choices):
    """Runs of keys equal on every bit the segment sort's two LDS passes order
    (k_bucket_sort step 2: each run sorted by insertion by the thread that
    finds its start; a run over kRunMax = 16 keys goes on to the odd-even
    rounds, and past OE_MAX rounds to the LSD): bits [20, 47) take one of
    `choices` values, so the keys sharing a 17-bit prefix split into runs of
    about 64 / choices keys (2^23 keys) with random low 20 bits."""
    rng = np.random.default_rng(0x5EED + choices)
    n = 1 << 23
    mids = rng.integers(0, 1 << 27, choices, dtype=np.uint64)
    h = (rng.integers(0, 1 << 17, n, dtype=np.uint64) << np.uint64(47)) \
        | (mids[rng.integers(0, choices, n)] << np.uint64(20)) | rng.integers(0, 1 << 20, n, dtype=np.uint64)
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)


def test_bucket_near_the_segment_capacity(pol, gpu_target):
    """A bucket close to the 512 x 18 = 9216-key segment capacity the plan
    sizes against: 4800 extra keys on the prefix (0x12, 0b101) make the plan
    take b2 = 3 (buckets of ~4096 keys) with that one bucket at ~8900 keys."""
    rng = np.random.default_rng(0xCAB)
    n = 1 << 23
    h = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    h[:4800] = (np.uint64(0x12) << np.uint64(56)) | (np.uint64(5) << np.uint64(53)) \
        | rng.integers(0, 1 << 53, 4800, dtype=np.uint64)
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)


@pytest.mark.parametrize("bits", [24, 56])
def test_low_bit_ranges(pol, gpu_target, bits):
    # keys below 2^24 (three live bytes, many duplicates: the prefix is bytes 2
    # and 1) and below 2^56 (top byte constant: the prefix moves down a byte)
    rng = np.random.default_rng(bits)
    h = rng.integers(0, 1 << bits, (1 << 23) + 5, dtype=np.uint64)
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)


# ---- 32-bit keys (keys-only): the same prefix passes on the top byte and the
# 9 bits under it ([15, 24)) or the two top bytes; the two LDS passes then
# cover every bit under the prefix, so a segment is sorted without odd-even
# rounds.
@pytest.mark.parametrize("logn", [22, 25])
@pytest.mark.parametrize("dt", [np.uint32, np.int32, np.float32])
def test_uniform_32bit(pol, gpu_target, logn, dt):
    rng = np.random.default_rng(100 + logn)
    n = (1 << logn) + 77
    if dt is np.float32:
        h = (rng.standard_normal(n) * np.exp2(rng.integers(-30, 30, n))).astype(np.float32)
        h[:6] = [0.0, -0.0, np.inf, -np.inf, 1e-40, -1e-40]
    else:
        info = np.iinfo(dt)
        h = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)


def test_32bit_oversized_and_skewed(pol, gpu_target):
    rng = np.random.default_rng(21)
    n = 1 << 24
    h = rng.integers(0, 2**32 - 1, n, dtype=np.uint32, endpoint=True)
    # one 16/17-bit prefix holds 40000 extra keys (per-bucket LSD finish)
    h[:40000] = np.uint32(0xABCD0000) | rng.integers(0, 1 << 16, 40000, dtype=np.uint32)
    check(pol, gpu_target, h)
    # top byte == second byte for every key: 256 oversized buckets (plain LSD)
    top = rng.integers(0, 256, n, dtype=np.uint32)
    h = (top << np.uint32(24)) | (top << np.uint32(16)) | rng.integers(0, 1 << 16, n, dtype=np.uint32)
    check(pol, gpu_target, h)
    # keys below 2^24: the prefix moves down a byte, many duplicates
    check(pol, gpu_target, rng.integers(0, 1 << 24, n, dtype=np.uint32))


# ---- sort_by_key through the hybrid (16-bit form with the values staged in
# LDS beside their keys; sort_by_key.hpp:42-78).  Checked pair for pair
# against the oracle's stable sort_by_key: equal keys keep their input order
# in the prefix passes, the LDS passes and the odd-even rounds.
def check_kv(pol, tgt, k, v, desc=False):
    dk = hpx.vector.from_host(k, tgt)
    dv = hpx.vector.from_host(v, tgt)
    P.sort_by_key(pol, dk.begin(), dk.end(), dv.begin(), F.greater if desc else F.less)
    gk, gv = dk.to_host(), dv.to_host()
    dk.free()
    dv.free()
    ek, ev = O.sort_by_key(k, v, desc)
    np.testing.assert_array_equal(gk, ek)
    np.testing.assert_array_equal(gv, ev)


def test_sort_by_key_equal_prefix_runs_stable(pol, gpu_target):
    # the insertion step moves values with their keys and keeps equal keys in
    # input order: runs of ~8 keys with 4 random low bits (many equal keys)
    rng = np.random.default_rng(0xAB1E)
    n = 1 << 22
    mids = rng.integers(0, 1 << 43, 4, dtype=np.uint64)
    k = (rng.integers(0, 1 << 17, n, dtype=np.uint64) << np.uint64(47)) \
        | (mids[rng.integers(0, 4, n)] << np.uint64(4)) | rng.integers(0, 16, n, dtype=np.uint64)
    v = np.arange(n, dtype=np.uint64)
    check_kv(pol, gpu_target, k, v)
    check_kv(pol, gpu_target, k, v, True)


@pytest.mark.parametrize("vdt", [np.uint64, np.uint32])
@pytest.mark.parametrize("desc", [False, True])
def test_sort_by_key_uniform(pol, gpu_target, vdt, desc):
    rng = np.random.default_rng(21)
    n = (1 << 22) + 13
    k = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    v = np.arange(n, dtype=vdt)
    check_kv(pol, gpu_target, k, v, desc)


def test_sort_by_key_duplicates_stable(pol, gpu_target):
    # 2^23 keys over 2^24 values (3 live bytes: the prefix is bytes 2 and 1,
    # buckets of ~128 pairs, many equal keys): stability decides the values
    rng = np.random.default_rng(22)
    n = 1 << 23
    k = rng.integers(0, 1 << 24, n, dtype=np.uint64)
    v = np.arange(n, dtype=np.uint64)
    check_kv(pol, gpu_target, k, v)


def test_sort_by_key_oversized_bucket(pol, gpu_target):
    # one 16-bit prefix holds 20000 extra pairs (> the 9216-pair LDS segment):
    # finished by the per-bucket LSD with its values
    rng = np.random.default_rng(23)
    n = 1 << 22
    k = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    k[:20000] = (np.uint64(0xABCD) << np.uint64(48)) | rng.integers(0, 1 << 48, 20000, dtype=np.uint64)
    k[20000:20050] = np.uint64(0xABCD) << np.uint64(48)
    v = np.arange(n, dtype=np.uint64)
    check_kv(pol, gpu_target, k, v)


@pytest.mark.parametrize("kdt", [np.int64, np.float64])
def test_sort_by_key_signed_and_double_keys(pol, gpu_target, kdt):
    rng = np.random.default_rng(24)
    n = (1 << 22) + 5
    if kdt is np.float64:
        k = rng.standard_normal(n) * np.exp2(rng.integers(-40, 40, n))
        k[:4] = [0.0, -0.0, np.inf, -np.inf]
    else:
        k = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    v = np.arange(n, dtype=np.uint64)
    check_kv(pol, gpu_target, k, v)
    check_kv(pol, gpu_target, k, v, True)


# ---- sort_by_key with 32-bit keys: the 16-bit form on the two top bytes; a
# single-bucket segment is finished by the two LDS passes, a packed run of
# small buckets by the odd-even rounds, stable throughout.
@pytest.mark.parametrize("kdt", [np.uint32, np.int32, np.float32])
@pytest.mark.parametrize("vdt", [np.uint64, np.uint32])
def test_sort_by_key_32bit_keys(pol, gpu_target, kdt, vdt):
    rng = np.random.default_rng(31)
    n = (1 << 24) + 9
    if kdt is np.float32:
        k = (rng.standard_normal(n) * np.exp2(rng.integers(-30, 30, n))).astype(np.float32)
        k[:4] = [0.0, -0.0, np.inf, -np.inf]
    else:
        info = np.iinfo(kdt)
        k = rng.integers(info.min, info.max, n, dtype=kdt, endpoint=True)
    v = np.arange(n, dtype=vdt)
    check_kv(pol, gpu_target, k, v)
    check_kv(pol, gpu_target, k, v, True)


def test_sort_by_key_32bit_duplicates_and_oversized(pol, gpu_target):
    rng = np.random.default_rng(32)
    n = 1 << 22
    v = np.arange(n, dtype=np.uint64)
    # keys below 2^20: many equal keys, packed multi-bucket segments
    check_kv(pol, gpu_target, rng.integers(0, 1 << 20, n, dtype=np.uint32), v)
    # one 16-bit prefix holds 20000 extra pairs: per-bucket LSD with its values
    k = rng.integers(0, 2**32 - 1, n, dtype=np.uint32, endpoint=True)
    k[:20000] = np.uint32(0xABCD0000) | rng.integers(0, 1 << 16, 20000, dtype=np.uint32)
    k[20000:20050] = np.uint32(0xABCD0000)
    check_kv(pol, gpu_target, k, v)


# ---- one workgroup per bucket straight from the bounds (the device plan
# picks the bucket width from the histograms), with an oversized bucket
# flagged by the segment kernel and the whole sort finished by the LSD.
@pytest.mark.parametrize("kdt", [np.uint64, np.uint32])
def test_direct_path_and_fallback(pol, gpu_target, kdt):
    rng = np.random.default_rng(41)
    n = 1 << 22
    bits = np.dtype(kdt).itemsize * 8
    k = rng.integers(0, 2**bits - 1, n, dtype=kdt, endpoint=True)
    check(pol, gpu_target, k)
    # one oversized bucket (flagged by the kernel, finished by per-bucket LSD)
    k[:30000] = kdt(0xABCD) << kdt(bits - 16) | rng.integers(0, 1 << (bits - 16), 30000, dtype=kdt)
    k[30000:30050] = kdt(0xABCD) << kdt(bits - 16)
    check(pol, gpu_target, k, True)
    v = np.arange(n, dtype=np.uint64)
    check_kv(pol, gpu_target, k, v)
    check_kv(pol, gpu_target, k, v, True)


def test_one_pass_segment_sort_mixed_bins(pol, gpu_target):
    """r06, the one-pass segment sort (k_bucket_sort ONEB = 13): most buckets
    of random keys take it; in every 16th bucket (top 11 bits) the 13 bits
    under the bucket's top take 4 values, so its bins hold ~1000 keys, over
    kOneBinMax -- those buckets are listed and sorted by the two-pass form in
    the third launch -- with duplicates and keys differing only in the low
    bits inside them."""
    rng = np.random.default_rng(0x0E13)
    n = 1 << 23
    h = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    top = h >> np.uint64(53)
    sel = (top % np.uint64(16)) == 0
    low = rng.integers(0, 4, int(sel.sum()), dtype=np.uint64) << np.uint64(40)
    h[sel] = (h[sel] & ~(np.uint64((1 << 53) - 1))) | low | (h[sel] & np.uint64((1 << 20) - 1))
    h[: 1000] = h[1000]  # a run of equal keys
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)


@pytest.mark.parametrize("kdt", [np.uint64, np.uint32])
@pytest.mark.parametrize("extra", [1000, 3000])
def test_padded_pass_overflow_fallback(pol, gpu_target, kdt, extra):
    """r06, the padded second prefix pass's fallback: `extra` keys share one
    (top-9, 4-bit field) cell of a 2^24-key sort, which the planner's
    marginal estimate (largest top-9 bin x largest field group / n, ~2100
    keys per bucket, slots of ~2500) cannot see.  The cell's slot overflows
    (k_pad_scatter raises C_PADOVF), k_pad_check hands the sort to the
    look-back pass (the persistent XREG form) from the same input; with
    3000 extra keys the bucket (~5000) is also over the 4608-key segment and
    is finished by the oversized-bucket LSD."""
    rng = np.random.default_rng(0x0F10 + extra)
    n = 1 << 24
    bits = np.dtype(kdt).itemsize * 8
    h = rng.integers(0, 2**bits - 1, n, dtype=kdt, endpoint=True)
    low = bits - 13
    cell = kdt(int(rng.integers(0, 1 << 13)) << low)
    h[:extra] = cell | rng.integers(0, 1 << low, extra, dtype=kdt)
    rng.shuffle(h)
    check(pol, gpu_target, h)
    check(pol, gpu_target, h, True)


def test_one_pass_pairs_segment_sort_mixed_bins(pol, gpu_target):
    """sort_by_key over the keys of the test above (sort_by_key's 512 x 9
    segments; buckets whose 13 bits under the top take 4 values), plus 5000
    keys each copied to ~10 scattered places: equal keys inside one segment,
    whose values must keep their input order.  (r06: it also covered the
    rejected one-pass form with values, profiles/r06_sort_pairs_onepass_rejected.log.)"""
    rng = np.random.default_rng(0x0E14)
    n = 1 << 23
    h = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    top = h >> np.uint64(53)
    sel = (top % np.uint64(16)) == 0
    low = rng.integers(0, 4, int(sel.sum()), dtype=np.uint64) << np.uint64(40)
    h[sel] = (h[sel] & ~(np.uint64((1 << 53) - 1))) | low | (h[sel] & np.uint64((1 << 20) - 1))
    h[: 1000] = h[1000]
    src = h[rng.integers(0, n, 5000)]
    h[rng.choice(n, 50000, replace=False)] = src[rng.integers(0, 5000, 50000)]
    v = np.arange(n, dtype=np.uint64)
    check_kv(pol, gpu_target, h, v)
    check_kv(pol, gpu_target, h, v, True)
    check_kv(pol, gpu_target, h, v.astype(np.uint32))
