"""ORACLE (test infrastructure only): circom zkey v1 / wtns v2 in Python.

Independent restatement of the reference readers, used by the Groth16 oracle
(oracle/groth16.py) and by tests that build synthetic proving keys:
  vendors/circom/circomlib/zkey/zkey.h:64-84 (magic "zkey", version 1),
    :89-100 (section ids), :114-123 (prover type 1), :147-153 (Groth header),
    :176-190 (point sections, Montgomery LE coordinates, (0,0) = identity),
    :211-223 (coefficients {u32 matrix, u32 constraint, u32 signal, value}
    with value re-read through FromMontgomery), :255-296 (element counts)
  vendors/circom/circomlib/zkey/verifying_key.h:33-36 (vk point order)
  vendors/circom/circomlib/wtns/wtns.h:75-117 (wtns v2: header {n8, modulus,
    count}, data = canonical LE values)
  vendors/circom/circomlib/base/sections.h (u32 count, {u32 type, u64 size})
Field elements and points stay as the raw Montgomery byte strings the C-ABI
exchanges; `coefficient_value` converts a coefficient word to the value the
reference computes with.
"""
import struct

from tachyon_amd import params as P

CURVE_FIELDS = {  # curve -> (base modulus, scalar modulus, n8q, n8r)
    "bn254": (P.BN254_FQ, P.BN254_FR, 32, 32),
    "bls12_381": (P.BLS12_381_FQ, P.BLS12_381_FR, 48, 32),
}


def _sections(data, off):
    (count,) = struct.unpack_from("<I", data, off)
    off += 4
    secs = {}
    for _ in range(count):
        typ, size = struct.unpack_from("<IQ", data, off)
        off += 12
        secs.setdefault(typ, (off, size))
        off += size
    return secs


def _split(blob, size, count):
    assert len(blob) >= size * count, "truncated section"
    return [bytes(blob[i * size:(i + 1) * size]) for i in range(count)]


def parse_zkey(data: bytes) -> dict:
    assert data[:4] == b"zkey", "bad magic"
    (version,) = struct.unpack_from("<I", data, 4)
    assert version == 1, f"unsupported zkey version {version}"
    secs = _sections(data, 8)

    def sec(i):
        off, size = secs[i]
        return data[off:off + size]

    assert struct.unpack_from("<I", sec(1), 0)[0] == 1, "not a Groth16 zkey"
    g = sec(2)
    (n8q,) = struct.unpack_from("<I", g, 0)
    q = int.from_bytes(g[4:4 + n8q], "little")
    o = 4 + n8q
    (n8r,) = struct.unpack_from("<I", g, o)
    r = int.from_bytes(g[o + 4:o + 4 + n8r], "little")
    o += 4 + n8r
    curve = next(c for c, (qq, rr, _, _) in CURVE_FIELDS.items() if qq == q and rr == r)
    nvars, npub, dsize = struct.unpack_from("<III", g, o)
    o += 12
    g1, g2 = 2 * n8q, 4 * n8q
    vk = {}
    for name, sz in (("alpha_g1", g1), ("beta_g1", g1), ("beta_g2", g2), ("gamma_g2", g2),
                     ("delta_g1", g1), ("delta_g2", g2)):
        vk[name] = bytes(g[o:o + sz])
        o += sz
    c = sec(4)
    (ncoef,) = struct.unpack_from("<I", c, 0)
    coefs = []
    step = 12 + n8r
    for i in range(ncoef):
        m, con, sig = struct.unpack_from("<III", c, 4 + i * step)
        coefs.append((m, con, sig, bytes(c[4 + i * step + 12:4 + (i + 1) * step])))
    nwit = nvars - npub - 1
    return dict(curve=curve, n8q=n8q, n8r=n8r, num_vars=nvars, num_public=npub, domain_size=dsize, vk=vk,
                ic=_split(sec(3), g1, npub + 1), coefficients=coefs,
                a1=_split(sec(5), g1, nvars), b1=_split(sec(6), g1, nvars), b2=_split(sec(7), g2, nvars),
                c1=_split(sec(8), g1, nwit), h1=_split(sec(9), g1, dsize))


def coefficient_value(word: bytes, r: int, n64: int = 4) -> int:
    """Canonical value of a zkey coefficient word B: the reference stores
    FromMontgomery(ToBigInt(B)), whose canonical value is B * R^-2 mod r."""
    R = 1 << (64 * n64)
    return int.from_bytes(word, "little") * pow(R, -2, r) % r


def write_zkey(curve, num_vars, num_public, domain_size, vk, ic, coefficients, a1, b1, b2, c1, h1) -> bytes:
    """Inverse of parse_zkey (synthetic proving keys for tests and the bench).
    coefficients: (matrix, constraint, signal, word bytes)."""
    q, r, n8q, n8r = CURVE_FIELDS[curve]
    header = struct.pack("<I", 1)
    groth = struct.pack("<I", n8q) + q.to_bytes(n8q, "little") + struct.pack("<I", n8r) + \
        r.to_bytes(n8r, "little") + struct.pack("<III", num_vars, num_public, domain_size) + \
        b"".join(vk[k] for k in ("alpha_g1", "beta_g1", "beta_g2", "gamma_g2", "delta_g1", "delta_g2"))
    coef = struct.pack("<I", len(coefficients)) + b"".join(
        struct.pack("<III", m, c, s) + w for (m, c, s, w) in coefficients)

    def blob(x):
        return x if isinstance(x, (bytes, bytearray)) else b"".join(x)

    sections = [(1, header), (2, groth), (3, blob(ic)), (4, coef), (5, blob(a1)), (6, blob(b1)),
                (7, blob(b2)), (8, blob(c1)), (9, blob(h1))]
    out = [b"zkey", struct.pack("<II", 1, len(sections))]
    for typ, body in sections:
        out.append(struct.pack("<IQ", typ, len(body)))
        out.append(body)
    return b"".join(out)


def parse_wtns(data: bytes, field_modulus: int) -> list:
    """Canonical ints of a wtns v2 file."""
    assert data[:4] == b"wtns", "bad magic"
    (version,) = struct.unpack_from("<I", data, 4)
    assert version == 2, f"unsupported wtns version {version}"
    secs = _sections(data, 8)
    off, size = secs[1]
    (n8,) = struct.unpack_from("<I", data, off)
    assert int.from_bytes(data[off + 4:off + 4 + n8], "little") == field_modulus, "wtns field mismatch"
    (count,) = struct.unpack_from("<I", data, off + 4 + n8)
    off, size = secs[2]
    return [int.from_bytes(data[off + i * n8:off + (i + 1) * n8], "little") for i in range(count)]


def write_wtns(values, field_modulus: int, n8: int = 32) -> bytes:
    hdr = struct.pack("<I", n8) + field_modulus.to_bytes(n8, "little") + struct.pack("<I", len(values))
    body = b"".join((v % field_modulus).to_bytes(n8, "little") for v in values)
    out = [b"wtns", struct.pack("<II", 2, 2), struct.pack("<IQ", 1, len(hdr)), hdr,
           struct.pack("<IQ", 2, len(body)), body]
    return b"".join(out)
