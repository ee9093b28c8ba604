"""Synthetic circom proving keys for the Groth16 parity tests and the bench
(test infrastructure; the reference's stand-in is ToxicWaste::RandomWithoutX,
vendors/circom/circomlib/circuit/circuit_test.h:34-49).

The points are seeded k*G doubling chains (oracle.gen_bases: valid curve
points, no trapdoor), the coefficients random, so the proofs are not
verifiable -- they pin the GPU prover to the CPU oracle bit for bit.  The
reference's multiplier_3.zkey covers verifiability (tests/test_groth16_oracle.py).
"""
import random

from oracle import oracle as O
from oracle.circom_format import CURVE_FIELDS, write_zkey

CURVE_NAMES = {"bn254": ("bn254_g1", "bn254_g2", "bn254_fr"),
               "bls12_381": ("bls12_381_g1", "bls12_381_g2", "bls12_381_fr")}


def synth_zkey(curve="bn254", log_n=6, num_vars=None, num_public=2, nnz_per_row=3, seed=1, empty_rows=0.1):
    """Returns (zkey bytes, full assignment as canonical ints)."""
    g1n, g2n, frn = CURVE_NAMES[curve]
    q, r, n8q, n8r = CURVE_FIELDS[curve]
    rng = random.Random(seed)
    n = 1 << log_n
    m = num_vars if num_vars is not None else max(num_public + 1, n - n // 4)
    pb1 = 2 * n8q

    def pts(c, k, s):
        if k == 0:
            return b""
        return O.gen_bases(c, s, k, max(1, k // 3)).tobytes()

    g1 = pts(g1n, 5 + num_public + 1 + 3 * m + n, seed * 7 + 1)
    g2 = pts(g2n, 3 + m, seed * 7 + 2)
    sp1 = [g1[i * pb1:(i + 1) * pb1] for i in range(len(g1) // pb1)]
    sp2 = [g2[i * 2 * pb1:(i + 1) * 2 * pb1] for i in range(len(g2) // (2 * pb1))]
    vk = dict(alpha_g1=sp1[0], beta_g1=sp1[1], delta_g1=sp1[2], beta_g2=sp2[0], gamma_g2=sp2[1], delta_g2=sp2[2])
    o = 5
    ic = sp1[o:o + num_public + 1]; o += num_public + 1
    a1 = sp1[o:o + m]; o += m
    b1 = sp1[o:o + m]; o += m
    c1 = sp1[o:o + m - num_public - 1]; o += m
    h1 = sp1[o:o + n]
    b2 = sp2[3:3 + m]
    # a couple of identity points in the queries (the zkey stores them as (0,0))
    if m > 3:
        a1[2] = b"\x00" * pb1
        b2[1] = b"\x00" * (2 * pb1)
    coefs = []
    for con in range(n):
        if rng.random() < empty_rows:
            continue
        for mat in (0, 1):
            for _ in range(rng.randint(1, nnz_per_row)):
                word = rng.randrange(r)
                coefs.append((mat, con, rng.randrange(m), word.to_bytes(n8r, "little")))
    rng.shuffle(coefs)
    full = [1] + [rng.randrange(r) for _ in range(m - 1)]
    if m > 4:
        full[3] = 0
    z = write_zkey(curve, m, num_public, n, vk, ic, coefs, a1, b1, b2, c1, h1)
    return z, full
