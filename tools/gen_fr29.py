#!/usr/bin/env python3
"""Generate tachyon_amd/csrc/field/fr29_gen.h: BN254 Fr in 9 x 29-bit limbs
for the NTT butterflies (field/fr29.h, ntt/ntt.hip) -- constants and the two
device products as hand-chained v_mad_u64_u32 columns (no carry words: a
column of <= 18 products of < 2^61 stays below 2^64, see the bounds below):

  mont(a, b)  = REDC(a b) by R' = 2^261 (the first pass: b = w 2^261 mod p,
                the 36-byte R'-form twiddle), output < a b / 2^261 + p;
  shoup(a, w, wq) = a w - q p with q = floor(a wq / 2^261) estimated from the
                columns >= 7 of a x wq (wq = floor(w 2^261 / p)), computed
                mod 2^261 as a w + q (2^261 - p): 53 + 90 = 143 mads against
                Montgomery's 162 (the later passes: 72-byte Shoup twiddles).

The butterfly data flow and its limb / value bounds are modelled in
`model_step` (Python integers, worst-case limbs) and checked by
tests/test_fr29_host.py, which also pins this file's output.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_f29_asm import column_pairs, stmt  # noqa: E402  (same column discipline as the Fq field)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tachyon_amd", "csrc", "field", "fr29_gen.h")
P = 21888242871839275222246405745257275088548364400416034343698204186575808495617  # BN254 Fr
N = 9
B = 1 << 261  # beta = R'
M29 = (1 << 29) - 1
QCOL = 7  # first column of a x wq that enters the quotient estimate


def limbs(v, n=N):
    return [(v >> (29 * i)) & M29 if i < n - 1 else v >> (29 * i) for i in range(n)]


def value(ls):
    return sum(x << (29 * i) for i, x in enumerate(ls))


def raised(k, m):
    """k p with every low limb raised by m 2^29 (borrowed from the limb above):
    limbs >= m 2^29 - m, so K - x is limb-wise non-negative for any x whose
    limbs are below that."""
    s = limbs(k * P)
    out = [s[0] + m * (1 << 29)] + [s[i] + m * (1 << 29) - m for i in range(1, 8)] + [s[8] - m]
    assert value(out) == k * P and all(0 <= x < (1 << 32) for x in out)
    return out


K16 = raised(16, 1)  # stage A: minus a normalized value < 8p (limbs < 2^29, limb 8 < 2^25)
K32 = raised(32, 2)  # stage B: minus a sum of two (limbs < 2^30)
NEGP = limbs(B - P)
PINV29 = (-pow(P, -1, 1 << 29)) % (1 << 29)
# reduce(): q from the top two limbs as a float, p_hi = p >> 203
P_HI = P >> 203


# ---------------------------------------------------------------------------
# Python model of the device arithmetic (exact limb semantics)
def mont(a, b):
    """REDC(a b) column by column (f29.h redc): returns limbs, and the widest column."""
    acc, m, r, widest = 0, [0] * N, [0] * N, 0
    pl = limbs(P)
    for k in range(2 * N - 1):
        for i in range(N):
            if 0 <= k - i < N:
                acc += a[i] * b[k - i]
        for i in range(N):
            if i < k and 0 < k - i < N:
                acc += m[i] * pl[k - i]
        if k < N:
            m[k] = ((acc & 0xFFFFFFFF) * PINV29) & M29
            acc += m[k] * pl[0]
        widest = max(widest, acc)
        if k >= N:
            r[k - N] = acc & M29
        acc >>= 29
    r[N - 1] = acc
    assert widest < (1 << 64)
    return r, widest


def shoup(a, w, wq):
    """The device Shoup product: returns (limbs, widest column)."""
    acc, widest, q = 0, 0, [0] * N
    for k in range(QCOL, 2 * N - 1):
        for i in range(N):
            if 0 <= k - i < N:
                acc += a[i] * wq[k - i]
        widest = max(widest, acc)
        if k >= N:
            q[k - N] = acc & M29
        acc >>= 29
    q[N - 1] = acc
    acc, r = 0, [0] * N
    for k in range(N):
        for i in range(N):
            if 0 <= k - i < N:
                acc += a[i] * w[k - i] + q[i] * NEGP[k - i]
        widest = max(widest, acc)
        r[k] = acc & M29
        acc >>= 29
    assert widest < (1 << 64)
    return r, widest


def shoup_q(w):
    return (w * B) // P


def reduce(a):
    """value - q p, q from the top two limbs (float32 as on the device),
    signed carries: normalized limbs, value < 3p."""
    import struct
    f32 = lambda x: struct.unpack("f", struct.pack("f", x))[0]
    vf = f32(f32(float(a[8]) * 536870912.0) + f32(float(a[7])))
    q = int(f32(vf * f32(1.0 / (P_HI + 1)))) - 1
    q = max(q, 0)
    pl = limbs(P)
    r, carry = [0] * N, 0
    for i in range(N):
        t = a[i] + carry - q * pl[i]
        r[i] = t & M29 if i < N - 1 else t & 0xFFFFFFFF
        carry = t >> 29
    assert carry >> 3 in (0, -1) or True
    return r


def normalize(a):
    r, c = list(a), 0
    for i in range(N - 1):
        t = r[i] + c
        r[i], c = t & M29, t >> 29
    r[N - 1] += c
    return r


def gen_shoup():
    L = ["__device__ __forceinline__ F29 shoup(const F29& a, const F29& w, const F29& wq) {",
         "  uint64_t acc = 0, sc;",
         f"  uint32_t q[{N}];",
         "  F29 r;"]
    for k in range(QCOL, 2 * N - 1):
        pairs = [(f"a{i}", f"x{k - i}") for i in range(N) if 0 <= k - i < N]
        L.append(f"  // quotient column {k}")
        L += stmt(pairs, operand=_operand)
        if k >= N:
            L.append(f"  q[{k - N}] = (uint32_t)acc & kM29;")
        L.append("  acc >>= 29;")
    L.append(f"  q[{N - 1}] = (uint32_t)acc;")
    L.append("  acc = 0;")
    for k in range(N):
        pairs = [(f"a{i}", f"w{k - i}") for i in range(N) if 0 <= k - i < N]
        pairs += [(f"q{i}", f"n{k - i}") for i in range(N) if 0 <= k - i < N]
        L.append(f"  // remainder column {k}")
        L += stmt(pairs, operand=_operand)
        L.append(f"  r.l[{k}] = (uint32_t)acc & kM29;")
        if k < N - 1:
            L.append("  acc >>= 29;")
    L.append("  return r;")
    L.append("}")
    return "\n".join(L) + "\n"


def _operand(v):
    kind, idx = v[0], v[1:]
    if kind == "p":
        return f'[{v}] "s"(kP29[{idx}])'
    if kind == "n":
        return f'[{v}] "s"(kNegP29[{idx}])'
    src = {"a": f"a.l[{idx}]", "b": f"b.l[{idx}]", "w": f"w.l[{idx}]", "x": f"wq.l[{idx}]", "q": f"q[{idx}]",
           "m": f"m[{idx}]"}
    return f'[{v}] "v"({src[kind]})'


def gen_mont():
    L = ["__device__ __forceinline__ F29 mont(const F29& a, const F29& b) {",
         "  uint64_t acc = 0, sc;",
         f"  uint32_t m[{N}];",
         "  F29 r;"]
    for k in range(2 * N - 1):
        L.append(f"  // column {k}")
        L += stmt(column_pairs(k, "mul"), operand=_operand)
        if k < N:
            L.append(f"  m[{k}] = ((uint32_t)acc * kPinv29) & kM29;")
            L += stmt([(f"m{k}", "p0")], operand=_operand)
        else:
            L.append(f"  r.l[{k - N}] = (uint32_t)acc & kM29;")
        L.append("  acc >>= 29;")
    L.append(f"  r.l[{N - 1}] = (uint32_t)acc;")
    L.append("  return r;")
    L.append("}")
    return "\n".join(L) + "\n"


def carr(name, v, comment):
    return f"// {comment}\nconstexpr uint32_t {name}[9] = {{" + ", ".join(f"0x{x:08x}u" for x in v) + "};"


def render():
    head = ["// GENERATED by tools/gen_fr29.py -- do not edit.",
            "// BN254 Fr in 9 x 29-bit limbs (field/fr29.h): constants and the device",
            "// products as hand-chained v_mad_u64_u32 columns.",
            "#pragma once",
            "namespace tachyon_amd::fr29 {",
            carr("kP29", limbs(P), "p"),
            carr("kNegP29", NEGP, "2^261 - p (the Shoup remainder adds q (2^261 - p) = -q p mod 2^261)"),
            f"constexpr uint32_t kPinv29 = 0x{PINV29:08x}u;  // -p^-1 mod 2^29",
            carr("kK16", K16, "16p, low limbs raised by 2^29 (stage A subtrahends: normalized, < 8p)"),
            carr("kK32", K32, "32p, low limbs raised by 2^30 (stage B subtrahends: sums of two)"),
            "// p as 8 x 32-bit words\nconstexpr uint32_t kPWords[8] = {" + ", ".join(f"0x{(P >> (32 * i)) & 0xFFFFFFFF:08x}u" for i in range(8)) + "};",
            f"constexpr float kInvPhi = 1.0f / {P_HI + 1}.0f;  // 1 / ((p >> 203) + 1)",
            "}  // namespace tachyon_amd::fr29",
            "#if defined(__HIP_DEVICE_COMPILE__)",
            "namespace tachyon_amd::fr29::asm29 {",
            ""]
    body = [gen_mont(), gen_shoup()]
    tail = ["}  // namespace tachyon_amd::fr29::asm29", "#endif", ""]
    return "\n".join(head) + "\n".join(body) + "\n".join(tail)


def main():
    text = render()
    open(OUT, "w").write(text)
    print(f"wrote {OUT}: {text.count('v_mad_u64_u32')} v_mad_u64_u32")


if __name__ == "__main__":
    main()
