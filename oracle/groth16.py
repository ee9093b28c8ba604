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
import struct

import numpy as np

from oracle import oracle as O
from oracle import pyref
from oracle.circom_format import CURVE_FIELDS, coefficient_value

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


# --- large keys: the same steps on numpy views of the zkey (no per-point lists) ---

def _zkey_sections(data: bytes) -> dict:
    secs, off = {}, 8
    (count,) = struct.unpack_from("<I", data, off)
    off += 4
    for _ in range(count):
        typ, size = struct.unpack_from("<IQ", data, off)
        off += 12
        secs.setdefault(typ, (off, size))
        off += size
    return secs


def witness_map_np(data: bytes, full: np.ndarray) -> np.ndarray:
    """WitnessMapFromMatrices in the C oracle (oracle_groth16_witness_map):
    full = m Montgomery elements (uint8/uint64 contiguous), returns the n
    h-evaluations as Montgomery bytes (uint8 array)."""
    secs = _zkey_sections(data)
    off, _ = secs[2]
    (n8q,) = struct.unpack_from("<I", data, off)
    q = int.from_bytes(data[off + 4:off + 4 + n8q], "little")
    o = off + 4 + n8q
    (n8r,) = struct.unpack_from("<I", data, o)
    r = int.from_bytes(data[o + 4:o + 4 + n8r], "little")
    curve = next(c for c, (qq, rr, _, _) in CURVE_FIELDS.items() if qq == q and rr == r)
    nvars, npub, n = struct.unpack_from("<III", data, o + 4 + n8r)
    coff, _ = secs[4]
    (ncoef,) = struct.unpack_from("<I", data, coff)
    coefs = np.frombuffer(data, dtype=np.uint8, count=ncoef * 44, offset=coff + 4)
    full = np.ascontiguousarray(full).view(np.uint8)
    assert full.nbytes == nvars * 32
    h = np.empty(n * 32, dtype=np.uint8)
    field = O.FIELDS[CURVES[curve][2]]
    rc = O.lib().oracle_groth16_witness_map(field, n, coefs.ctypes.data, ncoef, full.ctypes.data, nvars,
                                            h.ctypes.data)
    assert rc == 0, rc
    return h


def prove_np(data: bytes, full, r_blind: int = 0, s_blind: int = 0):
    """prove() for keys too large for per-point Python lists: the zkey's point
    sections are numpy views, the MSMs run in the C oracle on them, the few
    point additions of CreateProofWithAssignment (prove.h:52-165) in pyref.
    full: m Montgomery elements (bytes or numpy).  Returns (A, B, C) bytes."""
    secs = _zkey_sections(data)
    off, _ = secs[2]
    (n8q,) = struct.unpack_from("<I", data, off)
    q = int.from_bytes(data[off + 4:off + 4 + n8q], "little")
    o = off + 4 + n8q
    (n8r,) = struct.unpack_from("<I", data, o)
    r = int.from_bytes(data[o + 4:o + 4 + n8r], "little")
    curve = next(c for c, (qq, rr, _, _) in CURVE_FIELDS.items() if qq == q and rr == r)
    g1n, g2n, frn = CURVES[curve]
    G1, G2 = pyref.Curve(g1n), pyref.Curve(g2n)
    o += 4 + n8r
    m, npub, n = struct.unpack_from("<III", data, o)
    o += 12
    p1, p2 = 2 * n8q, 4 * n8q
    vk = {}
    for name, sz in (("alpha_g1", p1), ("beta_g1", p1), ("beta_g2", p2), ("gamma_g2", p2),
                     ("delta_g1", p1), ("delta_g2", p2)):
        vk[name] = data[o:o + sz]
        o += sz
    full = np.frombuffer(full, dtype=np.uint8) if isinstance(full, (bytes, bytearray)) else \
        np.ascontiguousarray(full).view(np.uint8)
    h = witness_map_np(data, full)

    def sec(i, size, count):
        so, _ = secs[i]
        return np.frombuffer(data, dtype=np.uint8, count=size * count, offset=so)

    a1, b1, b2 = sec(5, p1, m), sec(6, p1, m), sec(7, p2, m)
    c1, h1 = sec(8, p1, m - npub - 1), sec(9, p1, n)
    l_inst = npub + 1

    def msm(cname, C, bases, scalars):
        if scalars.nbytes == 0:
            return None
        return C.from_bytes(O.msm_np(cname, np.ascontiguousarray(bases), np.ascontiguousarray(scalars)))

    pt1, pt2 = G1.from_bytes, G2.from_bytes
    delta1 = pt1(vk["delta_g1"])
    r_delta1 = G1.mul(delta1, r_blind)
    A = G1.add(G1.add(G1.add(r_delta1, pt1(a1[:p1].tobytes())), msm(g1n, G1, a1[p1:], full[32:])),
               pt1(vk["alpha_g1"]))
    B2 = G2.add(G2.add(G2.add(G2.mul(pt2(vk["delta_g2"]), s_blind), pt2(b2[:p2].tobytes())),
                       msm(g2n, G2, b2[p2:], full[32:])), pt2(vk["beta_g2"]))
    witness_acc = msm(g1n, G1, c1, full[32 * l_inst:])
    h_acc = msm(g1n, G1, h1, h)
    C = G1.mul(A, s_blind)
    if r_blind % G1.Fr.p:
        B1 = G1.add(G1.add(G1.add(G1.mul(delta1, s_blind), pt1(b1[:p1].tobytes())),
                           msm(g1n, G1, b1[p1:], full[32:])), pt1(vk["beta_g1"]))
        C = G1.add(C, G1.mul(B1, r_blind))
        C = G1.add(C, G1.neg(G1.mul(r_delta1, s_blind)))
    C = G1.add(G1.add(C, witness_acc), h_acc)
    return G1.to_bytes(A), G2.to_bytes(B2), G1.to_bytes(C)
