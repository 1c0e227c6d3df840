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
