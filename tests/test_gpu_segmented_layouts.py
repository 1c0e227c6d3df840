"""partitioned_vector layouts on one MI355X (one rank holding several
partitions): container_layout(k) for k = 1, 3, 10, 1000 and scans into a
destination with another layout, restating
tests/unit/parallel/segmented_algorithms/partitioned_vector_reduce.cpp:47-76
(10007 ones + init 1 = 10008, int and double) and
partitioned_vector_inclusive_scan.cpp:321-340 (iota from 1, compared with
sequential_inclusive_scan) through the HIP kernels, against the oracle's
segmented restatement.  Integer results are bit-exact; double results are
checked against the oracle's segment-order restatement within the stated
FP-reduction bound."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

KS = [None, 1, 3, 10, 1000]


def _pv(S, n, dt, k, tgt, host=None):
    lay = S.container_layout if k is None else S.container_layout(k)
    pv = S.partitioned_vector(n, dt, tgt=tgt, layout=lay)
    if host is not None:
        from hpx_amd import _lib as L
        import ctypes
        h = np.ascontiguousarray(host, dt)
        L.call("hpxhip_memcpy_async", ctypes.c_void_p(pv.local.data()), h.ctypes.data_as(ctypes.c_void_p), h.nbytes,
               L.H2D, tgt.stream)
        tgt.synchronize()
    return pv


@pytest.mark.parametrize("k", KS)
@pytest.mark.parametrize("dt", [np.int32, np.float64])
def test_reduce_ones_layouts(gpu_target, k, dt):
    from hpx_amd import segmented as S, execution as ex, functional as F
    import hpx_amd as hpx
    pol = ex.par.on(hpx.default_executor(gpu_target))
    pv = _pv(S, 10007, dt, k, gpu_target, np.ones(10007, dt))
    assert pv.get_num_partitions() == (1 if k is None else k)
    assert S.algorithms.reduce(pol, pv.begin(), pv.end(), dt(1), F.plus) == 10008
    f = S.algorithms.reduce(ex.par(ex.task).on(hpx.default_executor(gpu_target)), pv.begin(), pv.end(), dt(1), F.plus)
    assert f.get() == 10008


@pytest.mark.parametrize("k", KS)
def test_inclusive_scan_iota_layouts(gpu_target, k):
    from hpx_amd import segmented as S, execution as ex, functional as F
    import hpx_amd as hpx
    pol = ex.par.on(hpx.default_executor(gpu_target))
    n = 1000000
    x = np.arange(1, n + 1, dtype=np.int64)
    pv = _pv(S, n, np.int64, k, gpu_target, x)
    out = _pv(S, n, np.int64, k, gpu_target)
    S.algorithms.inclusive_scan(pol, pv.begin(), pv.end(), out.begin(), F.plus, 0)
    gpu_target.synchronize()
    np.testing.assert_array_equal(out.local.to_host(), O.scan(x, 0, True))
    # in place (inclusive_scan_tests_inplace_with_policy)
    S.algorithms.inclusive_scan(pol, pv.begin(), pv.end(), pv.begin(), F.plus, 0)
    gpu_target.synchronize()
    np.testing.assert_array_equal(pv.local.to_host(), O.scan(x, 0, True))


@pytest.mark.parametrize("kin,kout", [(None, 3), (None, 10), (7, None), (3, 1000)])
def test_scan_and_transform_mixed_layouts(gpu_target, kin, kout):
    from hpx_amd import segmented as S, execution as ex, functional as F
    import hpx_amd as hpx
    pol = ex.par.on(hpx.default_executor(gpu_target))
    n = 100003
    x = O.generate(np.int64, "range", n, 0x5EED, -1000, 1000)
    pv = _pv(S, n, np.int64, kin, gpu_target, x)
    out = _pv(S, n, np.int64, kout, gpu_target)
    S.algorithms.exclusive_scan(pol, pv.begin(), pv.end(), out.begin(), 5)
    gpu_target.synchronize()
    np.testing.assert_array_equal(out.local.to_host(), O.segmented_scan(x, 5, kin or 1, False))
    # segmented transform_exclusive_scan (transform_exclusive_scan.hpp:317 argument order)
    S.algorithms.transform_exclusive_scan(pol, pv.begin(), pv.end(), out.begin(), -4, F.plus, F.multiply_step(3))
    gpu_target.synchronize()
    np.testing.assert_array_equal(out.local.to_host(), np.concatenate([[-4], -4 + np.cumsum(3 * x)[:-1]]))
    S.algorithms.transform(pol, pv.begin() + 10, pv.end(), out.begin(), F.add_value(7))
    gpu_target.synchronize()
    np.testing.assert_array_equal(out.local.to_host()[:n - 10], x[10:] + 7)


@pytest.mark.parametrize("k", [3, 10, 1000])
def test_fp_segment_order(gpu_target, k):
    """double reduce / scan over k segments vs the oracle's segment-order
    restatement (init (+) S_0 (+) ... ; carries from segment totals):
    |d| <= (2 ceil(log2 n) + 32) u sum|x| + u |exact| per result."""
    from hpx_amd import segmented as S, execution as ex, functional as F
    import hpx_amd as hpx
    pol = ex.par.on(hpx.default_executor(gpu_target))
    n = 200003
    x = O.generate(np.float64, "unit", n, 0x5EED) - 0.5
    pv = _pv(S, n, np.float64, k, gpu_target, x)
    u = 2.0 ** -53
    bound = (2 * np.ceil(np.log2(n)) + 32) * u * np.abs(x).sum()
    got = S.algorithms.reduce(pol, pv.begin(), pv.end(), 0.25, F.plus)
    exp = O.segmented_reduce(x, 0.25, k)
    assert abs(got - exp) <= bound + u * abs(exp)
    out = _pv(S, n, np.float64, k, gpu_target)
    S.algorithms.inclusive_scan(pol, pv.begin(), pv.end(), out.begin(), F.plus, 0.25)
    gpu_target.synchronize()
    got = out.local.to_host()
    exp = O.segmented_scan(x, 0.25, k, True)
    prefix_abs = np.cumsum(np.abs(x)) + 0.25
    ntiles = n // 4096 + 2
    assert np.all(np.abs(got - exp) <= (2 * ntiles + 64) * u * prefix_abs)
