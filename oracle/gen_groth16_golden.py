"""Writes tests/golden/groth16_multiplier_3.json: the oracle's proofs for the
reference's multiplier_3.zkey + multiplier_3.wtns fixtures (NoZK and two fixed
(r, s)), each checked with the pairing (oracle/bn254_pairing.py) before it is
written.  Run from the repo root:  python -m oracle.gen_groth16_golden
"""
import json
import os

from oracle import bn254_pairing as BP
from oracle import circom_format as CF
from oracle import groth16 as OG
from oracle import pyref
from tachyon_amd import params as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def main():
    zk = CF.parse_zkey(open(os.path.join(GOLDEN, "multiplier_3.zkey"), "rb").read())
    w = CF.parse_wtns(open(os.path.join(GOLDEN, "multiplier_3.wtns"), "rb").read(), P.BN254_FR)
    G1, G2 = pyref.Curve("bn254_g1"), pyref.Curve("bn254_g2")
    vk = {k: (G2 if k.endswith("g2") else G1).from_bytes(v) for k, v in zk["vk"].items()}
    ic = [G1.from_bytes(b) for b in zk["ic"]]
    cases = []
    for label, r, s in (("nozk", 0, 0), ("zk_a", 0x1234567, 0xABCDEF), ("zk_b", P.BN254_FR - 1, 2)):
        A, B, C = OG.prove(zk, w, r, s)
        assert BP.groth16_verify(vk, ic, w[1:2], (G1.from_bytes(A), G2.from_bytes(B), G1.from_bytes(C)))
        cases.append(dict(label=label, r=str(r), s=str(s), proof=[A.hex(), B.hex(), C.hex()]))
    out = dict(source="vendors/circom/examples/multiplier_3.zkey + circomlib/wtns/multiplier_3.wtns",
               public_inputs=[str(x) for x in w[1:2]], cases=cases,
               h_evals=[G1.Fr.to_bytes(x).hex() for x in OG.witness_map(zk, w)])
    with open(os.path.join(GOLDEN, "groth16_multiplier_3.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote tests/golden/groth16_multiplier_3.json")


if __name__ == "__main__":
    main()
