"""GPU parity of the field and point arithmetic (the reference's
prime_field_correctness_gpu_test.cc and (non_)affine_point_correctness_gpu_test.cc:
device results must equal the CPU results bit for bit)."""
import ctypes
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
OPS = {"add": 0, "sub": 1, "mul": 2, "sqr": 3, "neg": 4, "inv": 5, "to_mont": 6, "from_mont": 7, "dbl": 8,
       "mul_const": 9, "mul_sub_zero": 10, "mul_sub_x2": 11}


def gpu_field_op(field, op, a: bytes, b: bytes) -> bytes:
    from tachyon_amd._lib import FIELD_BYTES, FIELDS, lib
    n = len(a) // FIELD_BYTES[field]
    out = ctypes.create_string_buffer(len(a))
    lib().tachyon_mi355x_field_op(FIELDS[field], OPS[op], a, b, out, n)
    return out.raw


@pytest.mark.parametrize("field", ["bn254_fq", "bn254_fr", "bls12_381_fq", "bls12_381_fr"])
def test_field_ops_golden(field):
    cases = json.load(open(os.path.join(GOLDEN, "field_ops.json")))[field]
    a = b"".join(bytes.fromhex(c["a"]) for c in cases)
    b = b"".join(bytes.fromhex(c["b"]) for c in cases)
    nb = len(bytes.fromhex(cases[0]["a"]))
    for op in ("add", "sub", "mul", "sqr", "neg", "dbl"):
        got = gpu_field_op(field, op, a, b)
        exp = b"".join(bytes.fromhex(c[op]) for c in cases)
        assert got == exp, op
    got = gpu_field_op(field, "from_mont", a, b)
    assert got == b"".join(bytes.fromhex(c["a_canonical"]) for c in cases)
    inv_cases = [c for c in cases if c["inv"] is not None]
    ai = b"".join(bytes.fromhex(c["a"]) for c in inv_cases)
    assert gpu_field_op(field, "inv", ai, ai) == b"".join(bytes.fromhex(c["inv"]) for c in inv_cases)
    assert nb in (32, 48)


@pytest.mark.parametrize("field", ["bn254_fq", "bn254_fr", "bls12_381_fq", "bls12_381_fr"])
def test_field_mul_random_vs_oracle(field):
    n = 1 << 14
    nb = O.FIELD_BYTES[field]
    rng = np.random.default_rng(1)
    raw = rng.integers(0, 2**63, size=(2, n * nb // 8), dtype=np.uint64)
    # reduce random limbs into the field through the oracle (canonical -> Montgomery)
    a = O.field_op(field, "to_mont", _reduce(field, raw[0].tobytes()))
    b = O.field_op(field, "to_mont", _reduce(field, raw[1].tobytes()))
    for op in ("mul", "add", "sub", "sqr"):
        assert gpu_field_op(field, op, a, b) == O.field_op(field, op, a, b), op


def _reduce(field, data: bytes) -> bytes:
    from tachyon_amd import params as P
    p = P.FIELDS[field][0]
    nb = O.FIELD_BYTES[field]
    out = bytearray()
    for i in range(0, len(data), nb):
        out += (int.from_bytes(data[i:i + nb], "little") % p).to_bytes(nb, "little")
    return bytes(out)


@pytest.mark.parametrize("curve", ["bn254_g1", "bn254_g2", "bls12_381_g1", "bls12_381_g2"])
def test_point_ops_vs_oracle(curve):
    from tachyon_amd._lib import CURVES, lib
    pb = O.CURVE_INFO[curve][0]
    n = 64
    P = O.gen_bases(curve, 5, n, 8).tobytes()
    Q = O.gen_bases(curve, 6, n, 8).tobytes()
    # include identity, P == Q and P == -Q lanes
    P = bytearray(P)
    Q = bytearray(Q)
    Q[0:pb] = b"\x00" * pb                      # P + O
    Q[pb:2 * pb] = P[pb:2 * pb]                 # P + P (doubling branch)
    neg = O.ec_op(curve, "mul", bytes(P[2 * pb:3 * pb]), _r_minus_1(curve))  # (r-1)P = -P
    Q[2 * pb:3 * pb] = neg                      # P + (-P) = O
    P, Q = bytes(P), bytes(Q)
    for op, name in ((0, "add"), (2, "madd")):
        out = ctypes.create_string_buffer(len(P))
        lib().tachyon_mi355x_ec_op(CURVES[curve], op, P, Q, out, n)
        for i in range(n):
            exp = O.ec_op(curve, "add", P[i * pb:(i + 1) * pb], Q[i * pb:(i + 1) * pb])
            assert out.raw[i * pb:(i + 1) * pb] == exp, (name, i)
    out = ctypes.create_string_buffer(len(P))
    lib().tachyon_mi355x_ec_op(CURVES[curve], 1, P, Q, out, n)
    for i in range(n):
        assert out.raw[i * pb:(i + 1) * pb] == O.ec_op(curve, "dbl", P[i * pb:(i + 1) * pb])


def _r_minus_1(curve):
    from tachyon_amd import params as P
    sf = O.CURVE_INFO[curve][1]
    r = P.FIELDS[sf][0]
    return (r - 1).to_bytes(32, "little")


def test_twiddle_product_shoup_bn254_fr():
    """Field op 9 = the NTT butterfly's twiddle product (Fp::mul_shoup on
    BN254 Fr): x * w mod p for ANY 256-bit x (the butterfly feeds it the
    unreduced lo - hi + 2p) and a plain canonical w.  The quotient estimate
    leaves out the low columns of x * floor(w 2^256 / p); the crafted x below
    make x * wq = t (mod 2^256) for small t, so the dropped columns carry into
    the kept ones and the estimate is one short -- the branch that maps
    [2p, 3p) back into the lazy range.  Pinned by Python big integers."""
    import random
    p = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    rnd = random.Random(7)
    xs, ws = [], []
    for _ in range(2000):
        xs.append(rnd.randrange(1 << 256))
        ws.append(rnd.randrange(p))
    for t in range(1, 2001):  # crafted: x * wq = t (mod 2^256)
        while True:
            w = rnd.randrange(p)
            wq = (w << 256) // p
            if wq & 1:
                break
        xs.append((t * pow(wq, -1, 1 << 256)) % (1 << 256))
        ws.append(w)
    xs += [0, (1 << 256) - 1, p, 4 * p - 1, 5 * p]
    ws += [p - 1, p - 1, 1, p - 1, 0]
    enc = lambda v: v.to_bytes(32, "little")
    got = gpu_field_op("bn254_fr", "mul_const", b"".join(map(enc, xs)), b"".join(map(enc, ws)))
    for k, (x, w) in enumerate(zip(xs, ws)):
        assert int.from_bytes(got[32 * k:32 * k + 32], "little") == x * w % p, (k, hex(x), hex(w))


@pytest.mark.parametrize("field", ["bn254_fq", "bn254_fr", "bls12_381_fq", "bls12_381_fr"])
def test_square_every_representative(field):
    """Field op 3 = Fp::sqr, the dedicated FIPS square (each cross product
    counted once, through the doubled limbs of x).  The device keeps the
    254- and 381-bit fields in [0, 2p), so the square must be right for every
    representative there, not only canonical ones: x^2 R^-1 mod p for x
    drawn over [0, 2p) (BLS12-381 Fr: [0, p)), limb patterns whose top bits
    carry into the next doubled limb, and the ends of the range.  Pinned by
    Python big integers and by the general product of x with itself."""
    import random
    from tachyon_amd import params as P
    p = P.FIELDS[field][0]
    nb = O.FIELD_BYTES[field]
    R = 1 << (8 * nb)
    top = 2 * p if field != "bls12_381_fr" else p
    rnd = random.Random(11)
    xs = [rnd.randrange(top) for _ in range(4000)]
    for _ in range(1000):  # limbs with the top bit set (the bit d_j takes from a_(j-1))
        v = sum((rnd.randrange(1 << 31) | (1 << 31) if rnd.random() < 0.7 else rnd.randrange(1 << 32)) << (32 * j)
                for j in range(nb // 4))
        xs.append(v % top)
    xs += [0, 1, p - 1, top - 1, (1 << 32) - 1, (1 << 64) - 1, R // 4 - 1 if R // 4 - 1 < top else top - 2]
    if top == 2 * p:
        xs += [p, p + 1]
    enc = lambda v: v.to_bytes(nb, "little")
    a = b"".join(map(enc, xs))
    got = gpu_field_op(field, "sqr", a, a)
    rinv = pow(R, -1, p)
    for k, x in enumerate(xs):
        assert int.from_bytes(got[nb * k:nb * k + nb], "little") == x * x * rinv % p, (k, hex(x))
    assert got == gpu_field_op(field, "mul", a, a)


@pytest.mark.parametrize("field", ["bn254_fq", "bn254_fr", "bls12_381_fq", "bls12_381_fr"])
def test_fused_mul_sub_every_representative(field):
    """Field ops 10 / 11 = Fp::mul_sub, a b - c d with one Montgomery
    reduction over the columns of a b + (2p - c) d (the y coordinate of every
    XYZZ addition).  Its REDC output reaches [2p, 3p) for the 254-bit fields,
    so the conditional subtraction after it is exercised by inputs drawn over
    the whole lazy range [0, 2p) and by the ends of the range.  Pinned by
    Python big integers (x y R^-1 - x^2 R^-1 mod p) and by op 10's zero."""
    import random
    from tachyon_amd import params as P
    p = P.FIELDS[field][0]
    nb = O.FIELD_BYTES[field]
    R = 1 << (8 * nb)
    top = 2 * p if field != "bls12_381_fr" else p
    rnd = random.Random(13)
    xs = [rnd.randrange(top) for _ in range(6000)]
    ys = [rnd.randrange(top) for _ in range(6000)]
    ends = [0, 1, p - 1, top - 1] + ([p, p + 1] if top == 2 * p else [])
    for u in ends:
        for v in ends:
            xs.append(u)
            ys.append(v)
    enc = lambda v: v.to_bytes(nb, "little")
    a = b"".join(map(enc, xs))
    b = b"".join(map(enc, ys))
    got = gpu_field_op(field, "mul_sub_x2", a, b)
    rinv = pow(R, -1, p)
    for k, (x, y) in enumerate(zip(xs, ys)):
        assert int.from_bytes(got[nb * k:nb * k + nb], "little") == (x * y - x * x) * rinv % p, (k, hex(x), hex(y))
    assert gpu_field_op(field, "mul_sub_zero", a, b) == bytes(len(a))
