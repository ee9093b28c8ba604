"""Loader for tests/golden/halo2_circuits.json (written by
oracle/gen_halo2_golden.py from the reference's zk/plonk/examples/*_test_data.h).

Every value there was computed by the reference itself on the halo2 BN254 Fr
domain (math::halo2::OverrideSubgroupGenerator, bn/bn254/halo2/bn254.cc:7-30)
with KZG UnsafeSetup(kN, tau = 2) (zk/plonk/examples/circuit_test.h:66).
Values are canonical hex; helpers return the reference's in-memory layout
(Montgomery LE bytes, affine {x, y}).
"""
import json
import os

from oracle import pyref

PATH = os.path.join(os.path.dirname(__file__), "golden", "halo2_circuits.json")
FR = pyref.Field("bn254_fr")
G1 = pyref.Curve("bn254_g1")
TAU = 2


def load():
    with open(PATH) as f:
        return json.load(f)


def circuits():
    return load()["circuits"]


def case_id(c):
    return f"{c['file'].split('/')[-1].replace('_test_data.h', '')}#{c['index']}"


def fr_bytes(hex_list):
    return b"".join(FR.to_bytes(int(h, 16)) for h in hex_list)


def point_bytes(xy):
    return G1.to_bytes((int(xy[0], 16), int(xy[1], 16)))


def transform_pairs(c):
    """(evaluations, coefficients) pairs the reference holds for circuit c."""
    pairs = []
    for ev_key, poly_key in (("fixed_columns", "fixed_polys"), ("permutations_columns", "permutations_polys")):
        for ev, poly in zip(c.get(ev_key, []), c.get(poly_key, [])):
            pairs.append((fr_bytes(ev), fr_bytes(poly)))
    return pairs


def commitment_pairs(c):
    """(Lagrange column, expected commitment) pairs: fixed columns with
    fixed_commitments; permutation columns with the permutation VK's."""
    out = []
    for ev_key, com_key in (("fixed_columns", "fixed_commitments"),
                            ("permutations_columns", "permutation_commitments")):
        cols, coms = c.get(ev_key, []), c.get(com_key, [])
        if cols and len(cols) == len(coms):
            out += [(fr_bytes(col), point_bytes(com)) for col, com in zip(cols, coms)]
    return out


def indicator_polys(c):
    """l_first, l_last, l_active_row coefficient vectors (bytes) and the
    usable-row count u they imply: FFT(l_first) = [1, 0, ...],
    FFT(l_last) = delta_u, FFT(l_active_row) = [1]*u + [0]*(n-u)
    (zk/plonk/keys/proving_key.h:114-166)."""
    if not all(k in c for k in ("l_first", "l_last", "l_active_row")):
        return None
    n = c["n"]
    u = None
    act = [int(h, 16) for h in c["l_active_row"]]
    # u from the polynomial itself: sum of its evaluations at w^i is n * a_0
    u = act[0] * n % FR.p
    one, zero = FR.to_bytes(1), FR.to_bytes(0)
    return {
        "u": u,
        "l_first": (fr_bytes(c["l_first"]), one + zero * (n - 1)),
        "l_last": (fr_bytes(c["l_last"]), zero * u + one + zero * (n - u - 1)),
        "l_active_row": (fr_bytes(c["l_active_row"]), one * u + zero * (n - u)),
    }
