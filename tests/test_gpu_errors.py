"""The algorithms' error contract through the Python mirror (the C++ layer
has tests/cxx/exception_list.cpp): a failure is hpx::exception_list, raised
under seq/par and held by the future under par(task); an allocation failure
stays OutOfMemory (a MemoryError).  Failures are injected at the C ABI
(hpxhip_debug_inject_error / hpxhip_debug_raise_device_error), as the
reference's tests inject them with throwing functors
(tests/unit/parallel/algorithms/foreach_tests.hpp:110-205)."""
import numpy as np
import pytest

import hpx_amd as hpx
from hpx_amd import _lib as L
from hpx_amd import execution as ex, functional as F, parallel as P

pytestmark = pytest.mark.gpu


def _inject(status):
    L.call("hpxhip_debug_inject_error", status, 1)


@pytest.fixture
def vec(gpu_target):
    return hpx.vector.from_host(np.arange(10007, dtype=np.int64), gpu_target)


@pytest.mark.parametrize("pol", ["seq", "par", "par_on"])
def test_sync_failure_is_exception_list(gpu_target, vec, pol):
    p = {"seq": ex.seq, "par": ex.par, "par_on": ex.par.on(hpx.default_executor(gpu_target))}[pol]
    _inject(L.ERROR_INVALID_ARGUMENT)
    with pytest.raises(L.exception_list) as ei:
        P.for_each(p, vec.begin(), vec.end(), F.add_value(1))
    assert len(ei.value) == 1 and ei.value.status == L.ERROR_INVALID_ARGUMENT
    (inner,) = list(ei.value)
    assert isinstance(inner, L.HpxHipError) and inner.status == L.ERROR_INVALID_ARGUMENT
    assert np.array_equal(vec.to_host(), np.arange(10007))  # nothing was enqueued


def test_task_failure_is_an_exceptional_future(gpu_target, vec):
    _inject(L.ERROR_INVALID_ARGUMENT)
    f = P.reduce(ex.par(ex.task), vec.begin(), vec.end(), 0)
    assert f.has_exception()
    with pytest.raises(L.exception_list):
        f.get()


def test_out_of_memory_is_not_wrapped(gpu_target, vec):
    _inject(L.ERROR_OUT_OF_MEMORY)
    with pytest.raises(MemoryError) as ei:
        P.sort(ex.par, vec.begin(), vec.end())
    assert not isinstance(ei.value, L.exception_list)
    _inject(L.ERROR_OUT_OF_MEMORY)
    f = P.inclusive_scan(ex.par(ex.task), vec.begin(), vec.end(), vec.begin())
    with pytest.raises(MemoryError):
        f.get()


def test_device_side_failure(gpu_target, vec):
    L.call("hpxhip_debug_raise_device_error", gpu_target.stream, 5)
    with pytest.raises(L.exception_list) as ei:
        P.reduce(ex.par, vec.begin(), vec.end(), 0)
    assert ei.value.status == L.ERROR_DEVICE_TIMEOUT
    assert P.reduce(ex.par, vec.begin(), vec.end(), 0) == 10007 * 10006 // 2  # reported once, then clear


def test_argument_errors_pass_unchanged(gpu_target, vec):
    with pytest.raises(ValueError):
        P.fill(ex.par, vec.end(), vec.begin(), 1)
    L.call("hpxhip_debug_inject_error", 0, 0)


def test_inconsistent_merge_splits_raise(gpu_target):
    """merge_kernel.hpp k_merge: merge-path splits that are out of order (an
    input that is not sorted, or one changed while the merge ran, as a
    caller racing a sort from another stream does) are clamped so no access
    leaves the inputs, and the clamp raises the device error word
    (HPXHIP_DEVERR_RANGE): the caller gets exception_list, not silently wrong
    output (the clamped scatters of k_onesweep / k_merge used to
    be silent).  Here the splits come out of order deterministically: with
    2048-element tiles, a = [0]*2048 + [100]*2048 and the unsorted
    b = [10]*2048 + [-5]*2048, the diagonal 2048 splits at 2048 and the
    diagonal 4096 at 0 (path_split's binary search)."""
    a = np.concatenate([np.zeros(2048, np.int64), np.full(2048, 100, np.int64)])
    b = np.concatenate([np.full(2048, 10, np.int64), np.full(2048, -5, np.int64)])
    va, vb = hpx.vector.from_host(a, gpu_target), hpx.vector.from_host(b, gpu_target)
    out = hpx.vector(8192, dtype=np.int64, tgt=gpu_target)
    with pytest.raises(L.exception_list) as ei:
        P.merge(ex.par, va.begin(), va.end(), vb.begin(), vb.end(), out.begin())
    (inner,) = list(ei.value)
    assert ei.value.status == L.ERROR_DEVICE_TIMEOUT and "error word 2" in str(inner)
    # reported once: a consistent merge afterwards is clean and correct
    vb2 = hpx.vector.from_host(np.sort(b), gpu_target)
    P.merge(ex.par, va.begin(), va.end(), vb2.begin(), vb2.end(), out.begin())
    assert np.array_equal(out.to_host(), np.sort(np.concatenate([a, b]), kind="stable"))
