"""Pin the C oracle (oracle/oracle.c) against the golden vectors written by the
independent Python restatement (oracle/pyref.py) and the reference's own
known-answer data.  CPU only."""
import json
import os

import pytest

from oracle import oracle as O
from oracle import pyref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


B = bytes.fromhex


@pytest.mark.parametrize("field", ["bn254_fq", "bn254_fr", "bls12_381_fq", "bls12_381_fr"])
def test_field_ops(field):
    # prime_field_unittest.cc / prime_field_correctness_gpu_test.cc semantics
    for c in load("field_ops.json")[field]:
        a, b = B(c["a"]), B(c["b"])
        assert O.field_op(field, "add", a, b).hex() == c["add"]
        assert O.field_op(field, "sub", a, b).hex() == c["sub"]
        assert O.field_op(field, "mul", a, b).hex() == c["mul"]
        assert O.field_op(field, "sqr", a).hex() == c["sqr"]
        assert O.field_op(field, "neg", a).hex() == c["neg"]
        assert O.field_op(field, "dbl", a).hex() == c["dbl"]
        assert O.field_op(field, "from_mont", a).hex() == c["a_canonical"]
        assert O.field_op(field, "to_mont", B(c["a_canonical"])).hex() == c["a"]
        if c["inv"] is not None:
            assert O.field_op(field, "inv", a).hex() == c["inv"]


@pytest.mark.parametrize("curve", ["bn254_g1", "bn254_g2", "bls12_381_g1", "bls12_381_g2"])
@pytest.mark.parametrize("method", ["parallel_term", "pippenger", "naive"])
def test_msm_golden(curve, method):
    g = load("msm.json")[curve]
    for c in g["cases"]:
        bases = b"".join(B(x) for x in c["bases"])
        scalars = b"".join(B(x) for x in c["scalars"])
        aff, _ = O.msm(curve, bases, scalars, method=method, threads=4)
        assert aff.hex() == c["expected"], (c["n"], c.get("label"))


@pytest.mark.parametrize("curve", ["bn254_g1", "bn254_g2", "bls12_381_g1", "bls12_381_g2"])
def test_input_generator_matches_golden(curve):
    """The synthetic-input scheme (splitmix64 scalars, k*G doubling chains) is
    reproduced bit-exactly by the oracle; the product's GPU generator is checked
    against the oracle in the gpu tests."""
    pb, sf = O.CURVE_INFO[curve]
    for c in load("msm.json")[curve]["cases"]:
        if c.get("seed") is None:
            continue
        s = O.gen_scalars(sf, c["seed"], c["n"]).tobytes()
        assert s == b"".join(B(x) for x in c["scalars"])
        bs = O.gen_bases(curve, c["seed"], c["n"], c["chunk"]).tobytes()
        assert bs == b"".join(B(x) for x in c["bases"])


@pytest.mark.parametrize("field", ["bn254_fr", "bls12_381_fr"])
def test_ntt_golden(field):
    g = load(f"ntt_{field}.json")
    for c in g["cases"]:
        n = 1 << c["log_n"]
        coeffs = b"".join(B(x) for x in c["coeffs"])
        off = B(c["offset_mont"]) if c["offset"] != 1 else None
        ev = O.fft(coeffs, n, off, field=field)
        assert ev.hex() == "".join(c["evals"]), c
        back = O.ifft(ev, n, off, field=field)
        assert back.hex() == "".join(c["ifft_of_evals"]), c


def test_bls12_381_fr_roots_of_unity():
    """BLS12-381 Fr: the BUILD subgroup generator 7
    (tachyon/math/elliptic_curves/bls12/bls12_381/BUILD.bazel:62-65) gives
    arkworks' two-adic root of unity (2-adicity 32), and the oracle's domain
    roots equal the golden file's w_(2^k)."""
    import ctypes
    g = load("ntt_bls12_381_fr.json")
    assert g["two_adic_root_of_unity"] == \
        "10238227357739495823651030575849232062558860180284477541189508159991286009131"
    r = pyref.Field("bls12_381_fr").p
    w32 = int(g["two_adic_root_of_unity"])
    assert pow(w32, 1 << 31, r) == r - 1  # a primitive 2^32-th root
    for k in range(1, 17):  # (a domain builds its twiddle cache: sizes up to 2^16 here)
        out = ctypes.create_string_buffer(96)
        assert O.lib().oracle_domain_info(3, 1 << k, out) == 0
        assert out.raw[:32].hex() == g["roots_of_unity_mont"][str(k)], k


def test_roots_of_unity():
    import ctypes
    g = load("ntt_bn254_fr.json")
    # arkworks-compatible BN254 Fr two-adic root
    assert g["two_adic_root_of_unity"] == \
        "19103219067921713944291392827692070036145651957329286315305642004821462161904"
    for k in range(1, 29):
        out = ctypes.create_string_buffer(96)
        assert O.lib().oracle_domain_info(1, 1 << k, out) == 0
        assert out.raw[:32].hex() == g["roots_of_unity_mont"][str(k)]


def test_zkey_points_and_msm():
    z = load("zkey_multiplier_3.json")
    for key, curve in (("g1", "bn254_g1"), ("g2", "bn254_g2")):
        pts = [B(x) for x in z[f"{key}_points"]]
        for p in pts:
            assert O.ec_op(curve, "on_curve", p)
        scalars = b"".join(B(x) for x in z[f"msm_{key}"]["scalars"])
        aff, _ = O.msm(curve, b"".join(pts), scalars)
        assert aff.hex() == z[f"msm_{key}"]["expected"]


def test_parallel_term_chunk_invariance():
    """pippenger_adapter_unittest.cc:31-48: every strategy / chunking gives the
    same point (this is the multi-GPU sharding contract)."""
    n = 1000
    bases = O.gen_bases("bn254_g1", 7, n, 37).tobytes()
    scalars = O.gen_scalars("bn254_fr", 7, n).tobytes()
    ref, _ = O.msm("bn254_g1", bases, scalars, method="pippenger")
    for t in (1, 2, 3, 8):
        aff, _ = O.msm("bn254_g1", bases, scalars, method="parallel_term", threads=t)
        assert aff == ref
    # shard sum: MSM(A) + MSM(B) == MSM(A||B)
    a, _ = O.msm("bn254_g1", bases[:64 * 300], scalars[:32 * 300])
    b, _ = O.msm("bn254_g1", bases[64 * 300:], scalars[32 * 300:])
    assert O.ec_op("bn254_g1", "add", a, b) == ref


def test_jacobian_return_matches_affine():
    n = 50
    bases = O.gen_bases("bn254_g1", 3, n, 5).tobytes()
    scalars = O.gen_scalars("bn254_fr", 3, n).tobytes()
    aff, jac = O.msm("bn254_g1", bases, scalars)
    assert O.ec_op("bn254_g1", "jac_to_affine", jac) == aff


@pytest.mark.parametrize("curve,sf", [("bn254_g1", "bn254_fr"), ("bn254_g2", "bn254_fr"),
                                      ("bls12_381_g1", "bls12_381_fr"), ("bls12_381_g2", "bls12_381_fr")])
def test_dlog_identity_pins_the_synthetic_msm(curve, sf):
    """oracle_dlog_dot: the synthetic bases are known multiples of G (chunk j
    starts at k_j G and doubles), so MSM(bases, s) = (sum s_i k_j 2^t mod r) G.
    The identity equals the oracle's Pippenger MSM and the pure-Python
    textbook MSM, for shards that start mid-chunk too -- it is the large-size
    answer of tests/test_gpu_full_size.py::test_msm_dlog_identity."""
    C = pyref.Curve(curve)
    for n, chunk, start in ((37, 8, 0), (29, 5, 13)):
        full = O.gen_bases(curve, 21, start + n, chunk).tobytes()
        pb = len(full) // (start + n)
        bases = full[start * pb:]
        sc = O.gen_scalars(sf, 22, n).tobytes()
        d = O.dlog_dot(sf, 21, chunk, sc, start=start)
        want = C.to_bytes(C.mul(C.G, d))
        assert want == O.msm(curve, bases, sc)[0]
        pts = [C.from_bytes(bases[i * pb:(i + 1) * pb]) for i in range(n)]
        ks = [pyref.Field(sf).from_bytes(sc[32 * i:32 * (i + 1)]) for i in range(n)]
        acc = None
        for P, k in zip(pts, ks):
            acc = C.add(acc, C.mul(P, k))
        assert C.to_bytes(acc) == want


@pytest.mark.parametrize("logn", [1, 6, 13, 17])
def test_direct_evaluation_equals_fft(logn):
    """oracle_eval_at_powers (sum_j c_j (w^i)^j, blocked Horner) equals the
    radix-2 FFT restatement at every sampled index, with w the pure-Python
    root of unity: the independent check the full-size GPU NTT tests use."""
    n = 1 << logn
    Fr = pyref.Field("bn254_fr")
    c = O.gen_scalars("bn254_fr", 40 + logn, n).tobytes()
    ev = O.fft(c, n)
    idx = sorted({0, 1, n - 1, n // 2, (5 * n) // 7})
    got = O.eval_at_powers(c, Fr.to_bytes(Fr.root_of_unity(n)), idx)
    assert got == [ev[32 * i:32 * (i + 1)] for i in idx]
