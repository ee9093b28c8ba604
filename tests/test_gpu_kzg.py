"""KZG commitments with a device-resident SRS (the reference's
tachyon/crypto/commitments/kzg/kzg_unittest.cc): the GPU-built SRS equals the
oracle's [tau^i]G and [L_i(tau)]G, commitments equal the oracle MSM,
Commit(poly) == CommitLagrange(FFT(poly)), batch commitments, Downsize, and the
tau-in-the-domain corner of EvaluateAllLagrangeCoefficients."""
import pytest

from oracle import oracle as O
from oracle import pyref

pytestmark = pytest.mark.gpu


def oracle_srs(curve, n, tau):
    """[tau^i] G and [L_i(tau)] G (affine bytes), L_i over the size-n radix-2 domain."""
    C = pyref.Curve(curve)
    Fr = C.Fr
    r = Fr.p
    w = Fr.root_of_unity(n)
    g = C.to_bytes(C.G)
    mul = lambda k: O.ec_op(curve, "mul", g, k.to_bytes(32, "little"))  # plain-integer scalar
    powers = b"".join(mul(pow(tau, i, r)) for i in range(n))
    z = (pow(tau, n, r) - 1) % r
    lag = []
    for i in range(n):
        wi = pow(w, i, r)
        if z == 0:
            lag.append(1 if wi == tau else 0)
        else:
            lag.append(z * pow(n, -1, r) * wi * pow((tau - wi) % r, -1, r) % r)
    return powers, b"".join(mul(k) for k in lag)


@pytest.mark.parametrize("curve,logn", [("bn254_g1", 3), ("bn254_g1", 6), ("bls12_381_g1", 4)])
def test_setup_and_commit(curve, logn):
    from tachyon_amd.kzg import KZG
    n = 1 << logn
    Fr = pyref.Curve(curve).Fr
    tau = 0x1234_5678_9ABC_DEF0 + logn
    kzg = KZG(curve)
    kzg.unsafe_setup(n, Fr.to_bytes(tau))
    assert kzg.N() == n
    powers, lag = oracle_srs(curve, n, tau)
    assert kzg.g1_powers_of_tau() == powers
    assert kzg.g1_powers_of_tau_lagrange() == lag
    coeffs = O.gen_scalars(Fr.name, 500 + logn, n).tobytes()
    c = kzg.commit(coeffs)
    assert c == O.msm(curve, powers, coeffs)[0]
    if curve == "bn254_g1":  # CommitLagrange(FFT(poly)) == Commit(poly)  (kzg_unittest.cc:39-71)
        assert kzg.commit_lagrange(O.fft(coeffs, n)) == c
    # shorter input: the first |v| SRS points (DoMSM's min(bases, scalars))
    assert kzg.commit(coeffs[:32 * (n // 2 + 1)]) == O.msm(curve, powers[:kzg.point_bytes * (n // 2 + 1)],
                                                           coeffs[:32 * (n // 2 + 1)])[0]
    kzg.close()


def test_batch_and_downsize():
    from tachyon_amd.kzg import KZG
    n = 8  # kzg_unittest.cc: K = 3
    Fr = pyref.Field("bn254_fr")
    kzg = KZG("bn254_g1")
    kzg.unsafe_setup(n)  # random tau
    polys = [O.gen_scalars("bn254_fr", 900 + i, n).tobytes() for i in range(10)]
    batch = kzg.commit_batch(polys)
    lag = kzg.commit_batch([O.fft(p, n) for p in polys], lagrange=True)
    # against the oracle's MSM over the SRS the device built (itself checked
    # against the oracle's SRS in test_setup_and_commit), not only the
    # single-polynomial path
    powers, lag_srs = kzg.g1_powers_of_tau(), kzg.g1_powers_of_tau_lagrange()
    assert batch == [O.msm("bn254_g1", powers, p)[0] for p in polys]
    assert lag == [O.msm("bn254_g1", lag_srs, O.fft(p, n))[0] for p in polys]
    assert batch == lag == [kzg.commit(p) for p in polys]
    # ragged batch incl. an empty polynomial and a zero polynomial (identity
    # commitments stay (0, 0) through the one-inversion normalisation)
    ragged = [polys[0][:32 * 3], b"", bytes(32 * n), polys[1]]
    assert kzg.commit_batch(ragged) == [O.msm("bn254_g1", powers[:len(p) * 2], p)[0] if p else bytes(64)
                                        for p in ragged]
    assert kzg.commit_batch(ragged) == [kzg.commit(p) if p else bytes(64) for p in ragged]
    assert kzg.commit_batch(ragged)[1] == bytes(64) and kzg.commit_batch(ragged)[2] == bytes(64)
    assert kzg.commit_batch([polys[0] + polys[0][:32]]) is None  # more than N: nothing written
    assert kzg.commit_batch([]) == []
    assert not kzg.downsize(n)
    assert kzg.downsize(n // 2) and kzg.N() == n // 2
    assert len(kzg.g1_powers_of_tau()) == (n // 2) * 64
    # more scalars than N: the reference's Commit / CommitLagrange return false
    assert kzg.commit(polys[0]) is None and kzg.commit_lagrange(polys[0]) is None
    assert kzg.commit(polys[0][:32 * (n // 2)]) is not None
    del Fr
    kzg.close()


def test_commit_longer_than_srs_and_before_setup():
    from tachyon_amd.kzg import KZG
    kzg = KZG("bn254_g1")
    one = pyref.Field("bn254_fr").to_bytes(1)
    assert kzg.commit(one) is None  # no setup: N = 0
    kzg.unsafe_setup(4, pyref.Field("bn254_fr").to_bytes(5))
    assert kzg.commit(one * 5) is None and kzg.commit_lagrange(one * 5) is None
    assert kzg.commit(one * 4) is not None
    kzg.close()


def test_tau_in_domain():
    """tau = w^3: L_3(tau) = 1, the other Lagrange points are the identity."""
    from tachyon_amd.kzg import KZG
    n = 16
    Fr = pyref.Field("bn254_fr")
    tau = pow(Fr.root_of_unity(n), 3, Fr.p)
    kzg = KZG("bn254_g1")
    kzg.unsafe_setup(n, Fr.to_bytes(tau))
    lag = kzg.g1_powers_of_tau_lagrange()
    G1 = pyref.Curve("bn254_g1")
    pts = [lag[i * 64:(i + 1) * 64] for i in range(n)]
    assert pts[3] == G1.to_bytes(G1.G)
    assert all(p == b"\0" * 64 for i, p in enumerate(pts) if i != 3)
    kzg.close()


def test_device_resident_scalars():
    import numpy as np
    import torch
    from tachyon_amd.kzg import KZG
    n = 64
    kzg = KZG("bn254_g1")
    kzg.unsafe_setup(n, pyref.Field("bn254_fr").to_bytes(77))
    coeffs = O.gen_scalars("bn254_fr", 7, n)
    d = torch.from_numpy(coeffs.view(np.uint8).copy()).cuda()
    assert kzg.commit(d) == kzg.commit(coeffs.tobytes())
    kzg.close()


def test_batch_grouping_ragged_and_over_limits():
    """commit_batch groups polynomials of similar length into batched MSMs and
    closes a group when zero-padding would more than double its work: one 2^12
    polynomial beside 60 short ones (the short ones are not all padded to
    2^12), and 4,500 three-term polynomials -- more than
    one batched MSM takes (4,096) -- all equal the oracle's MSM over the
    device SRS, in the caller's order."""
    import random
    from tachyon_amd.kzg import KZG
    n = 1 << 12
    kzg = KZG("bn254_g1")
    kzg.unsafe_setup(n, pyref.Field("bn254_fr").to_bytes(991))
    powers = kzg.g1_powers_of_tau()
    rng = random.Random(5)
    big = O.gen_scalars("bn254_fr", 31, n).tobytes()
    pool = O.gen_scalars("bn254_fr", 32, 4096).tobytes()
    polys = [pool[32 * rng.randrange(0, 2000):][:32 * rng.randrange(1, 41)] for _ in range(60)]
    polys.insert(17, big)
    got = kzg.commit_batch(polys)
    assert got == [O.msm("bn254_g1", powers[:len(p) * 2], p)[0] for p in polys]
    tiny = [pool[32 * (i % 4000):][:96] for i in range(4500)]
    got = kzg.commit_batch(tiny)
    assert len(got) == 4500
    for i in range(0, 4500, 7):
        assert got[i] == O.msm("bn254_g1", powers[:192], tiny[i])[0], i
    assert got[4000] == got[0] and got[4499] == got[499]
    kzg.close()
