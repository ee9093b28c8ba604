"""UnivariateEvaluations<RationalField<bn254::Fr>> through the reference's
C-ABI (bn254_univariate_rational_evaluations.h; its unit test
bn254_univariate_rational_evaluations_unittest.cc): empty / set_zero /
set_trivial / set_rational / clone / len, Evaluate, and the GPU BatchEvaluate
against the oracle's field inverse and product -- zero denominators give 0
(MultiplicativeGroup::DoBatchInverse, math/base/groups.h:124-180)."""
import pytest

from oracle import oracle as O
from oracle import pyref

pytestmark = pytest.mark.gpu
FR = pyref.Field("bn254_fr")


def test_containers():
    from tachyon_amd.ntt import Radix2EvaluationDomain, RationalEvaluations
    dom = Radix2EvaluationDomain(16)
    ev = RationalEvaluations.empty(dom)
    assert len(ev) == 16
    one, zero = FR.to_bytes(1), FR.to_bytes(0)
    assert all(ev.get(i) == (zero, one) for i in range(16))
    ev.set_rational(3, FR.to_bytes(10), FR.to_bytes(4))
    cl = ev.clone()
    ev.set_trivial(3, FR.to_bytes(7))
    assert ev.get(3) == (FR.to_bytes(7), one) and cl.get(3) == (FR.to_bytes(10), FR.to_bytes(4))
    assert FR.from_bytes(cl.evaluate(3)) == 10 * pow(4, -1, FR.p) % FR.p
    cl.set_zero(3)
    assert cl.get(3) == (zero, one)
    ev.close(), cl.close(), dom.close()


@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, 1 << 16])
def test_batch_evaluate_vs_oracle(n):
    from tachyon_amd.ntt import RationalEvaluations
    nums = O.gen_scalars("bn254_fr", 70 + n, n).tobytes()
    dens = bytearray(O.gen_scalars("bn254_fr", 90 + n, n).tobytes())
    for i in range(0, n, 7):  # zero denominators, also runs of them
        dens[32 * i:32 * i + 32] = b"\0" * 32
    dens = bytes(dens)
    ev = RationalEvaluations()
    ev.resize(n)
    for i in range(n):
        ev.set_rational(i, nums[32 * i:32 * i + 32], dens[32 * i:32 * i + 32])
    got = ev.batch_evaluate()
    inv = O.field_op("bn254_fr", "inv", dens)
    want = bytearray(O.field_op("bn254_fr", "mul", nums, inv))
    for i in range(0, n, 7):
        want[32 * i:32 * i + 32] = b"\0" * 32
    assert got == bytes(want)
    ev.close()
