"""CPU checks of the Groth16 oracle (oracle/groth16.py) and its pins:
  * the BN254 pairing (oracle/bn254_pairing.py) is bilinear and non-degenerate;
  * the oracle's proof for the reference's own fixtures
    (vendors/circom/examples/multiplier_3.zkey, circomlib/wtns/multiplier_3.wtns,
    committed as data under tests/golden/) passes the Groth16 pairing check,
    NoZK and ZK, and a proof for a wrong witness does not;
  * zkey/wtns parsing matches the reference's unit tests
    (zkey_unittest.cc:71-215 decimals, wtns_unittest.cc: {1, 60, 3, 4, 5, 12});
  * the committed golden proof (tests/golden/groth16_multiplier_3.json) is reproduced.
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
