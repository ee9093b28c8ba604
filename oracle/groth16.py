"""ORACLE (test infrastructure only): CPU restatement of the circom Groth16 prover.

Follows the reference step by step:
  WitnessMapFromMatrices   vendors/circom/circomlib/circuit/quadratic_arithmetic_program.h:24-113
      a[c] += value * w[signal] over the A (matrix 0) / B coefficients (:38-63),
      c = a * b (:65-71), IFFT x3 (:77-82), DistributePowers by the 2n-th root
      of unity (:84-91), FFT x3 (:93-98), h = a * b - c (:100-108)
  CreateProofWithAssignment  tachyon/zk/r1cs/groth16/prove.h:52-165
      (CalculateCoeff :33-49; the circom driver passes instance = full[1:l],
      witness = full[l:], full[1:], vendors/circom/prover_main.cc:139-153)
  ToNativeProvingKey       vendors/circom/circomlib/zkey/proving_key.h:42-52
The FFTs and MSMs run in the C oracle (oracle/oracle.c: Radix2EvaluationDomain
and PippengerAdapter restated); field and point glue uses oracle/pyref.py.
Pinned by oracle/bn254_pairing.py: the proof for the reference's own
multiplier_3.zkey + multiplier_3.wtns fixtures passes the Groth16 pairing
check (tests/test_groth16_oracle.py).
"""
from oracle import oracle as O
from oracle import pyref
from oracle.circom_format import coefficient_value

CURVES = {"bn254": ("bn254_g1", "bn254_g2", "bn254_fr"),
          "bls12_381": ("bls12_381_g1", "bls12_381_g2", "bls12_381_fr")}


def witness_map(zk: dict, full: list) -> list:
    """h evaluations on the coset (canonical ints), full = canonical ints."""
    g1n, _, frn = CURVES[zk["curve"]]
    Fr = pyref.Field(frn)
    r = Fr.p
    n = zk["domain_size"]
    a = [0] * n
    b = [0] * n
    for m, con, sig, word in zk["coefficients"]:
        v = coefficient_value(word, r) * full[sig] % r
        if m == 0:
            a[con] = (a[con] + v) % r
        else:
            b[con] = (b[con] + v) % r
    c = [x * y % r for x, y in zip(a, b)]
    g = Fr.root_of_unity(2 * n)
    g_mont = Fr.to_bytes(g)
    evals = []
    for vec in (a, b, c):
        coeffs = O.ifft(b"".join(Fr.to_bytes(x) for x in vec), n, field=frn)
        ev = O.fft(coeffs, n, offset_mont=g_mont, field=frn)
        ev = ev + b"\x00" * (n * 32 - len(ev))
        evals.append([Fr.from_bytes(ev[i * 32:(i + 1) * 32]) for i in range(n)])
    return [(x * y - z) % r for x, y, z in zip(*evals)]


def prove(zk: dict, full: list, r_blind: int = 0, s_blind: int = 0, h: list = None):
    """Returns (A, B, C) as affine Montgomery byte strings (identity = zeros)."""
    g1n, g2n, frn = CURVES[zk["curve"]]
    G1, G2 = pyref.Curve(g1n), pyref.Curve(g2n)
    Fr = G1.Fr
    if h is None:
        h = witness_map(zk, full)
    m = zk["num_vars"]
    l_inst = zk["num_public"] + 1
    sc = [Fr.to_bytes(x) for x in full]

    def msm(curve, C, bases, scalars):
        if not bases:
            return None
        out, _ = O.msm(curve, b"".join(bases), b"".join(scalars))
        return C.from_bytes(out)

    pt1 = G1.from_bytes
    pt2 = G2.from_bytes
    vk = zk["vk"]
    delta1 = pt1(vk["delta_g1"])
    # [A]_1 = r delta + a_0 + sum_{i>=1} x_i a_i + alpha   (CalculateCoeff)
    r_delta1 = G1.mul(delta1, r_blind)
    A = G1.add(G1.add(G1.add(r_delta1, pt1(zk["a1"][0])), msm(g1n, G1, zk["a1"][1:], sc[1:])),
               pt1(vk["alpha_g1"]))
    B2 = G2.add(G2.add(G2.add(G2.mul(pt2(vk["delta_g2"]), s_blind), pt2(zk["b2"][0])),
                       msm(g2n, G2, zk["b2"][1:], sc[1:])), pt2(vk["beta_g2"]))
    witness_acc = msm(g1n, G1, zk["c1"], sc[l_inst:])
    h_acc = msm(g1n, G1, zk["h1"], [Fr.to_bytes(x) for x in h])
    C = G1.mul(A, s_blind)
    if r_blind % Fr.p:
        B1 = G1.add(G1.add(G1.add(G1.mul(delta1, s_blind), pt1(zk["b1"][0])),
                           msm(g1n, G1, zk["b1"][1:], sc[1:])), pt1(vk["beta_g1"]))
        C = G1.add(C, G1.mul(B1, r_blind))
        C = G1.add(C, G1.neg(G1.mul(r_delta1, s_blind)))
    C = G1.add(G1.add(C, witness_acc), h_acc)
    return G1.to_bytes(A), G2.to_bytes(B2), G1.to_bytes(C)
