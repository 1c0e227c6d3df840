"""Host-side logic of the for_loop reduction objects (no GPU): the identities
each reduction_* helper uses (for_loop_reduction.hpp:135-231) and the
live-out checks."""
import numpy as np
import pytest

from hpx_amd import functional as F
from hpx_amd import parallel as P


def test_reduction_identities():
    v = np.array([42], np.int64)
    assert P.reduction_plus(v).identity == 0 and P.reduction_plus(v).op is F.plus
    assert P.reduction_multiplies(v).identity == 1 and P.reduction_multiplies(v).op is F.multiplies
    assert P.reduction_bit_and(v).identity == -1 and P.reduction_bit_and(v).op is F.bit_and
    assert P.reduction_bit_or(v).identity == 0 and P.reduction_bit_or(v).op is F.bit_or
    assert P.reduction_bit_xor(v).identity == 0 and P.reduction_bit_xor(v).op is F.bit_xor
    # min/max take the live-out's current value as the identity (205-231)
    assert P.reduction_min(v).identity == 42 and P.reduction_min(v).op is F.minimum
    assert P.reduction_max(v).identity == 42 and P.reduction_max(v).op is F.maximum
    u = np.zeros((), np.uint64)
    assert int(P.reduction_bit_and(u).identity) == (1 << 64) - 1
    assert P.reduction_plus(v, 5).identity == 5


def test_reduction_live_out_checks():
    with pytest.raises(TypeError):
        P.reduction_plus(3)                       # not an lvalue stand-in
    with pytest.raises(TypeError):
        P.reduction_plus(np.zeros(2, np.int64))   # not one element
    with pytest.raises(TypeError):
        P.reduction(np.zeros(1), 0.0, lambda a, b: a + b)  # not an hpx_amd combiner
    with pytest.raises(TypeError):
        F.accumulate(1, F.identity(), 0, 1)


def test_accumulate_all_validation():
    """Several reductions per for_loop (for_loop.hpp:802-812): accumulate_all
    takes one accumulate per reduction position; the loop checks that every
    reduction argument is named exactly once (no device needed: the checks
    run before any launch)."""
    with pytest.raises(ValueError):
        F.accumulate_all(F.accumulate(1, F.identity(), 0), F.accumulate(1, F.square(), 0))
    with pytest.raises(TypeError):
        F.accumulate_all()
    body = F.accumulate_all(F.accumulate(1, F.identity(), 0), F.accumulate(2, F.square(), 0))
    assert [a.red for a in body.parts] == [1, 2]
