"""Pin the oracle to the reference's own halo2 outputs (CPU).

tests/golden/halo2_circuits.json holds, for the reference's PLONK example
circuits, values its CPU path computed on the halo2 BN254 Fr domain: fixed /
permutation columns and their IFFTs, the l_first / l_last / l_active_row
polynomials, the domain generator, and KZG CommitLagrange commitments with
UnsafeSetup(n, tau = 2).  The oracle, switched to the halo2 generator set
(OverrideSubgroupGenerator, bn/bn254/halo2/bn254.cc:7-30), must reproduce every
one of them byte for byte.
"""
import ctypes

import pytest

import halo2_golden as H
from oracle import oracle as O

CASES = H.circuits()
IDS = [H.case_id(c) for c in CASES]
R = H.FR.p


def test_golden_file_shape():
    assert len(CASES) >= 10
    assert sum(len(H.transform_pairs(c)) for c in CASES) >= 25
    assert sum(len(H.commitment_pairs(c)) for c in CASES) >= 25


def test_halo2_constants():
    """Both constant sets satisfy GetRootOfUnity's identity large^(3^2) =
    two-adic root (prime_field_base.h:90-130), and the halo2 set is
    generator 7's (halo2curves fr.rs, cited at bn254.cc:9-23)."""
    for on, gen in ((False, 5), (True, 7)):
        with O.halo2_domain() if on else _null():
            large = H.FR.from_bytes(O.bn254_fr_large_subgroup_root())
        t = (R - 1) >> 28
        assert large == pow(gen, t // 9, R)
        assert pow(large, 9, R) == pow(gen, t, R)
    assert not O.bn254_fr_set_halo2(False)  # the scopes restored the default


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _omega(n):
    out = ctypes.create_string_buffer(96)
    assert O.lib().oracle_domain_info(O.FIELDS["bn254_fr"], n, out) == 0
    return H.FR.from_bytes(out.raw[:32])


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_domain_generator(c):
    if "omega" not in c:
        pytest.skip("no pinned verifying key")
    with O.halo2_domain():
        assert _omega(c["n"]) == int(c["omega"], 16)


def test_halo2_roots_above_32():
    """Up to n = 32 the halo2 and arkworks generators give the same w_n (so the
    example circuits, k = 4 and 5, pin the NTT and KZG but not the override);
    from n = 64 they differ.  There the halo2 root is pinned by the reference's
    literal constants (bn254.cc:18-29) through test_halo2_constants."""
    for k in range(1, 21):
        n = 1 << k
        ark = _omega(n)
        with O.halo2_domain():
            h2 = _omega(n)
        assert ark == pow(5, (R - 1) // n, R) and h2 == pow(7, (R - 1) // n, R)
        assert (ark == h2) == (k <= 5)


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_ifft_fft_columns(c):
    pairs = H.transform_pairs(c)
    if not pairs:
        pytest.skip("no columns")
    n = c["n"]
    with O.halo2_domain():
        for ev, poly in pairs:
            assert O.ifft(ev, n) == _trim(poly)
            assert O.fft(poly, n) == ev


def _trim(poly):
    """IFFT drops trailing zero coefficients (RemoveHighDegreeZeros)."""
    k = len(poly) // 32
    while k and poly[32 * (k - 1):32 * k] == b"\0" * 32:
        k -= 1
    return poly[:32 * k]


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_indicator_polys(c):
    ind = H.indicator_polys(c)
    if ind is None:
        pytest.skip("no l_first/l_last/l_active_row")
    n = c["n"]
    assert 0 < ind["u"] < n
    with O.halo2_domain():
        for key in ("l_first", "l_last", "l_active_row"):
            poly, evals = ind[key]
            assert O.fft(poly, n) == evals, key
            assert O.ifft(evals, n) == _trim(poly), key


def _srs(n, lagrange, w):
    g = H.G1.to_bytes(H.G1.G)
    if not lagrange:
        ks = [pow(H.TAU, i, R) for i in range(n)]
    else:
        z = (pow(H.TAU, n, R) - 1) % R
        ks = [z * pow(n, -1, R) * pow(w, i, R) * pow((H.TAU - pow(w, i, R)) % R, -1, R) % R for i in range(n)]
    return b"".join(O.ec_op("bn254_g1", "mul", g, k.to_bytes(32, "little")) for k in ks)


@pytest.mark.parametrize("n", [16, 32])
def test_kzg_commitments(n):
    """CommitLagrange(column) (verifying_key.h:94-100) over [L_i(2)]G on the
    halo2 domain, and Commit(poly) over [2^i]G, equal the reference's
    fixed / permutation commitments."""
    cases = [c for c in CASES if c["n"] == n and H.commitment_pairs(c)]
    assert cases
    w = pow(7, (R - 1) // n, R)
    lag, powers = _srs(n, True, w), _srs(n, False, w)
    checked = 0
    with O.halo2_domain():
        for c in cases:
            for col, com in H.commitment_pairs(c):
                assert O.msm("bn254_g1", lag, col)[0] == com, H.case_id(c)
                assert O.msm("bn254_g1", powers, O.ifft(col, n).ljust(32 * n, b"\0"))[0] == com
                checked += 1
    assert checked >= 2
    # negative control: another tau commits the same column elsewhere
    col, com = H.commitment_pairs(cases[0])[-1]
    other = _srs_tau(n, 3, w)
    assert O.msm("bn254_g1", other, col)[0] != com


def _srs_tau(n, tau, w):
    g = H.G1.to_bytes(H.G1.G)
    z = (pow(tau, n, R) - 1) % R
    ks = [z * pow(n, -1, R) * pow(w, i, R) * pow((tau - pow(w, i, R)) % R, -1, R) % R for i in range(n)]
    return b"".join(O.ec_op("bn254_g1", "mul", g, k.to_bytes(32, "little")) for k in ks)
