"""HIP NTT and KZG on the halo2 BN254 Fr domain against the reference's own
outputs (tests/golden/halo2_circuits.json, see tests/test_halo2_golden.py) and
against the oracle at sizes where the halo2 root differs from arkworks'.

Scope: math::halo2::OverrideSubgroupGenerator (bn/bn254/halo2/bn254.cc:7-30)
through the C-ABI (tachyon_mi355x_bn254_halo2_*), the domain C-ABI
(bn254_univariate_evaluation_domain.h:38-136) and the KZG extension
(UnsafeSetup(n, tau = 2) / CommitLagrange / Commit, kzg.h:173-258).
"""
import pytest

import halo2_golden as H
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = H.circuits()
IDS = [H.case_id(c) for c in CASES]


def _trim(poly):
    k = len(poly) // 32
    while k and poly[32 * (k - 1):32 * k] == b"\0" * 32:
        k -= 1
    return poly[:32 * k]


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_domain_columns_and_indicators(c):
    from tachyon_amd.ntt import Radix2EvaluationDomain, ScopedSubgroupGeneratorOverrider
    pairs = H.transform_pairs(c)
    ind = H.indicator_polys(c)
    if not pairs and ind is None:
        pytest.skip("no columns")
    n = c["n"]
    with ScopedSubgroupGeneratorOverrider():
        dom = Radix2EvaluationDomain(n)
    if "omega" in c:
        assert H.FR.from_bytes(dom.group_gen) == int(c["omega"], 16)
    for ev, poly in pairs:
        assert dom.ifft(ev) == _trim(poly)
        assert dom.fft(poly) == ev
    if ind is not None:
        for key in ("l_first", "l_last", "l_active_row"):
            poly, evals = ind[key]
            assert dom.fft(poly) == evals, key
            assert dom.ifft(evals) == _trim(poly), key
    dom.close()


@pytest.mark.parametrize("n", [16, 32])
def test_kzg_commitments(n):
    from tachyon_amd.kzg import KZG
    from tachyon_amd.ntt import ScopedSubgroupGeneratorOverrider
    cases = [c for c in CASES if c["n"] == n and H.commitment_pairs(c)]
    kzg = KZG("bn254_g1")
    with ScopedSubgroupGeneratorOverrider():
        kzg.unsafe_setup(n, H.FR.to_bytes(H.TAU))
    checked = 0
    for c in cases:
        for col, com in H.commitment_pairs(c):
            assert kzg.commit_lagrange(col) == com, H.case_id(c)
            assert kzg.commit(O.ifft(col, n).ljust(32 * n, b"\0")) == com
            checked += 1
    assert checked >= 2
    kzg.close()


@pytest.mark.parametrize("log_n", [6, 10, 16, 20])
def test_halo2_domain_vs_oracle(log_n):
    """Above n = 32 the halo2 and arkworks roots differ: the HIP transforms on
    the halo2 domain equal the oracle's halo2 transforms and differ from the
    arkworks ones; domains created after the scope use arkworks again."""
    from tachyon_amd.ntt import Radix2EvaluationDomain, ScopedSubgroupGeneratorOverrider, \
        halo2_subgroup_generator_active
    n = 1 << log_n
    coeffs = O.gen_scalars("bn254_fr", 4242 + log_n, n).tobytes()
    with ScopedSubgroupGeneratorOverrider():
        assert halo2_subgroup_generator_active()
        dom = Radix2EvaluationDomain(n)
    assert not halo2_subgroup_generator_active()
    ark = Radix2EvaluationDomain(n)
    assert H.FR.from_bytes(dom.group_gen) == pow(7, (H.FR.p - 1) // n, H.FR.p)
    with O.halo2_domain():
        want_f = O.fft(coeffs, n)
        want_i = O.ifft(coeffs, n)
    assert dom.fft(coeffs) == want_f
    assert dom.ifft(coeffs) == want_i
    assert ark.fft(coeffs) == O.fft(coeffs, n) != want_f
    dom.close()
    ark.close()


def test_halo2_kzg_lagrange_srs_vs_oracle():
    """KZG's Lagrange SRS follows the generator set active at UnsafeSetup."""
    from tachyon_amd.kzg import KZG
    from tachyon_amd.ntt import ScopedSubgroupGeneratorOverrider
    n, tau = 64, 0xC0FFEE
    R = H.FR.p
    w = pow(7, (R - 1) // n, R)
    kzg = KZG("bn254_g1")
    with ScopedSubgroupGeneratorOverrider():
        kzg.unsafe_setup(n, H.FR.to_bytes(tau))
    z = (pow(tau, n, R) - 1) % R
    g = H.G1.to_bytes(H.G1.G)
    lag = b"".join(O.ec_op("bn254_g1", "mul", g, (z * pow(n, -1, R) * pow(w, i, R) *
                                                  pow((tau - pow(w, i, R)) % R, -1, R) % R).to_bytes(32, "little"))
                   for i in range(n))
    assert kzg.g1_powers_of_tau_lagrange() == lag
    evals = O.gen_scalars("bn254_fr", 77, n).tobytes()
    with O.halo2_domain():
        coeffs = O.ifft(evals, n).ljust(32 * n, b"\0")
    assert kzg.commit_lagrange(evals) == kzg.commit(coeffs)
    kzg.close()
