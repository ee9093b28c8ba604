"""CPU checks of the Groth16 oracle (oracle/groth16.py) and its pins:
  * the BN254 pairing (oracle/bn254_pairing.py) is bilinear and non-degenerate;
  * the oracle's proof for the reference's own fixtures
    (vendors/circom/examples/multiplier_3.zkey, circomlib/wtns/multiplier_3.wtns,
    committed as data under tests/golden/) passes the Groth16 pairing check,
    NoZK and ZK, and a proof for a wrong witness does not;
  * zkey/wtns parsing matches the reference's unit tests
    (zkey_unittest.cc:71-215 decimals, wtns_unittest.cc: {1, 60, 3, 4, 5, 12});
  * the committed golden proof (tests/golden/groth16_multiplier_3.json) is reproduced;
  * a second reference fixture, vendors/circom/examples/adder.zkey (97
    signals, 128-row domain; tests/golden/adder.zkey), with the witness of
    circomlib/circuit/adder_data.json {a: 3, b: 4} derived from the key's
    own constraints (adder_witness): its proofs verify, a wrong public output
    does not, and the 32-bit wrap-around case verifies too;
  * the numpy/C path used at BASELINE configs[4]'s size (prove_np) equals the
    step-by-step restatement on synthetic keys.
"""
import json
import os

import pytest

from oracle import bn254_pairing as BP
from oracle import circom_format as CF
from oracle import groth16 as OG
from oracle import pyref
from tachyon_amd import params as P

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
G1 = pyref.Curve("bn254_g1")
G2 = pyref.Curve("bn254_g2")


def load():
    zk = CF.parse_zkey(open(os.path.join(GOLDEN, "multiplier_3.zkey"), "rb").read())
    w = CF.parse_wtns(open(os.path.join(GOLDEN, "multiplier_3.wtns"), "rb").read(), P.BN254_FR)
    return zk, w


def verify(zk, public, proof):
    vk = {k: (G2 if k.endswith("g2") else G1).from_bytes(v) for k, v in zk["vk"].items()}
    ic = [G1.from_bytes(b) for b in zk["ic"]]
    A, B, C = proof
    return BP.groth16_verify(vk, ic, public, (G1.from_bytes(A), G2.from_bytes(B), G1.from_bytes(C)))


def test_pairing_bilinear():
    e = BP.pairing(G1.G, G2.G)
    assert e != BP.f12_one()
    assert BP.pairing(G1.mul(G1.G, 3), G2.G) == BP.pairing(G1.G, G2.mul(G2.G, 3)) == BP.f12_pow(e, 3)
    assert BP.f12_pow(e, P.BN254_FR) == BP.f12_one()


def test_parse_fixtures_match_reference_tests():
    zk, w = load()
    assert w == [1, 60, 3, 4, 5, 12]  # wtns_unittest.cc
    assert (zk["num_vars"], zk["num_public"], zk["domain_size"]) == (6, 1, 4)
    exp = json.load(open(os.path.join(GOLDEN, "zkey_multiplier_3.json")))["expected_decimal"]
    dec = lambda b: ["0", "0"] if G1.from_bytes(b) is None else [str(x) for x in G1.from_bytes(b)]
    assert dec(zk["vk"]["alpha_g1"]) == exp["alpha_g1"]
    assert [dec(b) for b in zk["a1"]] == exp["points_a1"]


def test_zkey_wtns_roundtrip():
    zk, w = load()
    again = CF.write_zkey("bn254", zk["num_vars"], zk["num_public"], zk["domain_size"], zk["vk"], zk["ic"],
                          zk["coefficients"], zk["a1"], zk["b1"], zk["b2"], zk["c1"], zk["h1"])
    assert CF.parse_zkey(again) == zk
    assert CF.parse_wtns(CF.write_wtns(w, P.BN254_FR), P.BN254_FR) == w


def test_oracle_proof_verifies_nozk_and_zk():
    zk, w = load()
    public = w[1:1 + zk["num_public"]]
    assert verify(zk, public, OG.prove(zk, w))
    assert verify(zk, public, OG.prove(zk, w, r_blind=0x1234567, s_blind=0xABCDEF))


def test_wrong_witness_fails():
    zk, w = load()
    bad = list(w)
    bad[5] = 13  # 3 * 4 != 13: the constraint no longer holds
    assert not verify(zk, bad[1:2], OG.prove(zk, bad))


def test_golden_proof_reproduced():
    zk, w = load()
    g = json.load(open(os.path.join(GOLDEN, "groth16_multiplier_3.json")))
    for case in g["cases"]:
        proof = OG.prove(zk, w, int(case["r"]), int(case["s"]))
        assert [x.hex() for x in proof] == case["proof"], case["label"]


def test_witness_map_golden():
    zk, w = load()
    g = json.load(open(os.path.join(GOLDEN, "groth16_multiplier_3.json")))
    Fr = pyref.Field("bn254_fr")
    assert [Fr.to_bytes(x).hex() for x in OG.witness_map(zk, w)] == g["h_evals"]


def adder_witness(a: int, b: int) -> list:
    """Full assignment of examples/adder.circom (Num2Bits(32) x2, BinSum(32, 2),
    Bits2Num(32); adder_circuit_unittest.cc feeds a, b from adder_data.json).
    Signal order read off adder.zkey's A/B rows: 0 = one, 1 = out (public),
    2 = a, 3 = b, 4..34 = bits 0..30 of out, 35..65 = bits 0..30 of a,
    66..96 = bits 0..30 of b; circom folded each top bit and the carry into
    linear combinations (rows 31, 63, 95, 96)."""
    out = (a + b) & 0xFFFFFFFF
    bits = lambda v: [(v >> i) & 1 for i in range(31)]
    return [1, out, a, b] + bits(out) + bits(a) + bits(b)


def load_adder():
    return CF.parse_zkey(open(os.path.join(GOLDEN, "adder.zkey"), "rb").read())


def test_adder_fixture_verifies():
    zk = load_adder()
    assert (zk["num_vars"], zk["num_public"], zk["domain_size"]) == (97, 1, 128)
    w = adder_witness(3, 4)  # circomlib/circuit/adder_data.json
    assert w[1] == 7  # adder_circuit_unittest.cc: public_inputs[0] == F(7)
    assert verify(zk, [7], OG.prove(zk, w))
    assert verify(zk, [7], OG.prove(zk, w, r_blind=99, s_blind=P.BN254_FR - 5))
    assert not verify(zk, [8], OG.prove(zk, w))
    wrap = adder_witness(0xFFFFFFF0, 0x20)  # carry out of bit 31 is dropped
    assert verify(zk, [0x10], OG.prove(zk, wrap, r_blind=3, s_blind=4))


@pytest.mark.parametrize("curve,log_n,seed", [("bn254", 6, 1), ("bn254", 10, 2), ("bls12_381", 7, 3)])
def test_prove_np_equals_restatement(curve, log_n, seed):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from groth16_synth import synth_zkey
    zb, full = synth_zkey(curve, log_n=log_n, num_public=2, seed=seed)
    zk = CF.parse_zkey(zb)
    Fr = pyref.Field("bn254_fr" if curve == "bn254" else "bls12_381_fr")
    fb = b"".join(Fr.to_bytes(v) for v in full)
    h = OG.witness_map(zk, full)
    assert OG.witness_map_np(zb, fb).tobytes() == b"".join(Fr.to_bytes(x) for x in h)
    assert OG.prove_np(zb, fb) == OG.prove(zk, full, h=h)
    assert OG.prove_np(zb, fb, 11, 13) == OG.prove(zk, full, 11, 13, h=h)
