"""The 9 x 29-bit BN254 Fq field of the G1 bucket accumulation
(tachyon_amd/csrc/field/f29.h), host build: every operation checked against
Python integers -- values mod p, the N-form limb shape and the value bounds
the madd bound analysis relies on -- and the point formulas built on it
(msm/acc29.h: the accumulation's madd, the reductions' add and dbl, the run
start) on operands at the top of their bounds.  The device
products (field/f29_asm.h) are the generator's output of the same columns;
they are pinned here against tools/gen_f29_asm.py and on the GPU by the MSM
golden tests (tests/test_gpu_msm.py, variant 8192)."""
import importlib.util
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
R1 = pow(2, 261, P)  # R' = 2^261
M29 = (1 << 29) - 1

HARNESS = r"""
#include <cstdio>
#include <cstring>
#include "f29.h"
using namespace tachyon_amd::f29;
static void rd(F29& x) { for (int i = 0; i < 9; ++i) scanf("%u", &x.l[i]); }
static void wr(const F29& x) { for (int i = 0; i < 9; ++i) printf("%u ", x.l[i]); printf("\n"); }
int main() {
  char op[32];
  while (scanf("%31s", op) == 1) {
    F29 a, b, c, d;
    if (!strcmp(op, "from32")) { uint32_t w[8]; for (int i = 0; i < 8; ++i) scanf("%u", &w[i]); wr(from32(w)); }
    else if (!strcmp(op, "to32")) { rd(a); uint32_t w[8]; to32(a, w); for (int i = 0; i < 8; ++i) printf("%u ", w[i]); printf("\n"); }
    else if (!strcmp(op, "mul")) { rd(a); rd(b); wr(mul(a, b)); }
    else if (!strcmp(op, "mul_add")) { rd(a); rd(b); rd(c); wr(mul_add(a, b, c)); }
    else if (!strcmp(op, "mul2_add")) { rd(a); rd(b); rd(c); rd(d); wr(mul2_add(a, b, c, d)); }
    else if (!strcmp(op, "sqr")) { rd(a); wr(sqr(a)); }
    else if (!strcmp(op, "sqr_add")) { rd(a); rd(b); wr(sqr_add(a, b)); }
    else if (!strcmp(op, "iszero")) { rd(a); printf("%d\n", (int)is_zero_mod_p(a)); }
  }
  return 0;
}
"""


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("f29")
    src, exe = d / "h.cpp", d / "h"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "tachyon_amd", "csrc", "field"),
                    str(src), "-o", str(exe)], check=True)

    def run(lines):
        out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
        return [[int(t) for t in ln.split()] for ln in out[:len(lines)]]
    return run


def limbs(v):
    """N-form limbs of v (limbs 0..7 exact, limb 8 the rest)."""
    return [(v >> (29 * i)) & M29 for i in range(8)] + [v >> 232]


def value(ls):
    return sum(x << (29 * i) for i, x in enumerate(ls))


def words(v):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def n_form(ls):
    return all(x <= M29 for x in ls[:8]) and ls[8] < (1 << 32)


def fmt(op, *xs):
    return " ".join([op] + [str(t) for x in xs for t in x])


def test_from32_to32(harness):
    rng = random.Random(1)
    xs = [0, 1, P - 1, P, 2 * P - 1, (1 << 254) - 1] + [rng.randrange(2 * P) for _ in range(300)]
    out = harness([fmt("from32", words(x)) for x in xs])
    for x, r in zip(xs, out):
        assert n_form(r)
        v = value(r)
        assert v < 3 * P and v % P == (x << 5) % P
    ys = [0, 1, P, 16 * P - 1] + [rng.randrange(16 * P) for _ in range(300)]
    ys += [value(limbs(y)) | ((1 << 29) - 1) for y in ys[:20]]  # all-ones low limbs
    ys = [y for y in ys if y < 16 * P]
    out = harness([fmt("to32", limbs(y)) for y in ys])
    for y, w in zip(ys, out):
        v = sum(t << (32 * i) for i, t in enumerate(w))
        assert v < 2 * P and v % P == (y * pow(2, -5, P)) % P


def test_products(harness):
    rng = random.Random(2)
    inv = pow(R1, -1, P)
    cases = []
    for _ in range(200):
        a, b, c, d, e = (rng.randrange(10 * P) for _ in range(5))
        cases.append((a, b, c, d, e))
    cases.append((0, 0, 0, 0, 0))
    cases.append((10 * P - 1,) * 5)
    lines = []
    for a, b, c, d, e in cases:
        A, B, C, D, E = map(limbs, (a, b, c, d, e))
        lines += [fmt("mul", A, B), fmt("mul_add", A, B, E), fmt("mul2_add", A, B, C, D), fmt("sqr", A),
                  fmt("sqr_add", A, E)]
    out = harness(lines)
    for i, (a, b, c, d, e) in enumerate(cases):
        want = [a * b * inv, a * b * inv + e, (a * b + c * d) * inv, a * a * inv, a * a * inv + e]
        bound = [a * b / 2**261 + P, a * b / 2**261 + P + e, (a * b + c * d) / 2**261 + P,
                 a * a / 2**261 + P, a * a / 2**261 + P + e]
        for k in range(5):
            r = out[5 * i + k]
            assert n_form(r), (i, k)
            assert value(r) % P == want[k] % P, (i, k)
            assert value(r) < bound[k], (i, k)


def test_is_zero(harness):
    rng = random.Random(3)
    xs = [k * P for k in range(64)] + [k * P + 1 for k in range(64)] + [rng.randrange(64 * P) for _ in range(100)]
    out = harness([fmt("iszero", limbs(x)) for x in xs])
    for x, r in zip(xs, out):
        assert r[0] == int(x % P == 0)


def test_asm_header_matches_generator():
    spec = importlib.util.spec_from_file_location("gen_f29_asm", os.path.join(ROOT, "tools", "gen_f29_asm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with open(os.path.join(ROOT, "tachyon_amd", "csrc", "field", "f29_asm.h")) as f:
        text = f.read()
    assert text == mod.render()
    # 9 x 9 products + 9 x 9 reduction mads per column set; mul2 has 81 more
    per = {"mul": 162, "mul_add": 162, "mul2": 243, "mul2_add": 243, "sqr": 126, "sqr_add": 126}
    for fn, n in per.items():
        body = text.split(f"F29 {fn}(", 1)[1].split("\n}\n", 1)[0]
        assert body.count("v_mad_u64_u32") == n, fn


POINT_HARNESS = r"""
#include <cstdio>
#include <cstring>
#include "acc29.h"
using namespace tachyon_amd::f29;
using namespace tachyon_amd::msm::acc29_core;
static void rd(F29& x) { for (int i = 0; i < 9; ++i) scanf("%u", &x.l[i]); }
static void rda(Acc& a) { rd(a.x); rd(a.y); rd(a.zz); rd(a.zzz); }
static void wr(const F29& x) { for (int i = 0; i < 9; ++i) printf("%u ", x.l[i]); }
static void wra(int special, const Acc& a) { printf("%d ", special); wr(a.x); wr(a.y); wr(a.zz); wr(a.zzz); printf("\n"); }
int main() {
  char op[32];
  while (scanf("%31s", op) == 1) {
    Acc a, b;
    F29 x2, y2;
    int special = 0;
    if (!strcmp(op, "madd")) { rda(a); rd(x2); rd(y2); Acc c = madd(a, x2, y2, &special); wra(special, c); }
    else if (!strcmp(op, "add")) { rda(a); rda(b); Acc c = add(a, b, &special); wra(special, c); }
    else if (!strcmp(op, "dbl")) { rda(a); wra(0, dbl(a)); }
    else if (!strcmp(op, "start")) { rd(x2); rd(y2); wra(0, from_shifted(x2, y2)); }
  }
  return 0;
}
"""


@pytest.fixture(scope="module")
def point_harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("acc29")
    src, exe = d / "p.cpp", d / "p"
    src.write_text(POINT_HARNESS)
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "tachyon_amd", "csrc", "msm"),
                    "-I", os.path.join(ROOT, "tachyon_amd", "csrc", "field"), str(src), "-o", str(exe)], check=True)

    def run(lines):
        out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
        return [[int(t) for t in ln.split()] for ln in out[:len(lines)]]
    return run


def _affine_add(P, Q):
    if P is None:
        return Q
    if Q is None:
        return P
    (x1, y1), (x2, y2) = P, Q
    if x1 == x2:
        if (y1 + y2) % P_MOD == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, P_MOD) % P_MOD
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P_MOD) % P_MOD
    x3 = (lam * lam - x1 - x2) % P_MOD
    return x3, (lam * (x1 - x3) - y1) % P_MOD


P_MOD = P


def _mul(k, Pt):
    R = None
    while k:
        if k & 1:
            R = _affine_add(R, Pt)
        Pt = _affine_add(Pt, Pt)
        k >>= 1
    return R


def _top_rep(v, bound):
    """The representative v + k p below bound * p with the largest low limbs
    (the widest columns), as N-form limbs."""
    best = None
    for k in range(bound):
        w = v + k * P
        if w >= bound * P:
            break
        s = sum(limbs(w)[:8])
        if best is None or s > best[0]:
            best = (s, w)
    return limbs(best[1])


def _acc(pt, z, bx=10, by=3, bz=3):
    """XYZZ accumulator of affine pt with Z = z, R' form, representatives at the
    top of the invariant X < bx p, Y < by p, ZZ, ZZZ < bz p."""
    x, y = pt
    zz, zzz = z * z % P, z * z * z % P
    m = lambda v: v * R1 % P  # noqa: E731
    return (_top_rep(m(x * zz % P), bx) + _top_rep(m(y * zzz % P), by) + _top_rep(m(zz), bz)
            + _top_rep(m(zzz), bz))


def _point_of(res):
    """(special, affine point or None, component values) of a harness result."""
    sp, v = res[0], res[1:]
    X, Y, ZZ, ZZZ = (value(v[9 * i:9 * i + 9]) for i in range(4))
    inv = pow(R1, -1, P)
    if ZZ % P == 0:
        return sp, None, (X, Y, ZZ, ZZZ), v
    x = X * inv * pow(ZZ * inv, -1, P) % P
    y = Y * inv * pow(ZZZ * inv, -1, P) % P
    return sp, (x, y), (X, Y, ZZ, ZZZ), v


def _check_bounds(vals, v, bx, by, bz):
    X, Y, ZZ, ZZZ = vals
    assert X < bx * P and Y < by * P and ZZ < bz * P and ZZZ < bz * P
    for i in range(4):
        assert n_form(v[9 * i:9 * i + 9])


def test_point_formulas_at_bounds(point_harness):
    """msm/acc29.h's madd / add / dbl / run start on operands at the top of
    their bounds (largest representatives below 10p / 3p / 32p), against affine
    arithmetic in Python: results, the output bounds the invariant needs (X <
    10p, Y, ZZ, ZZZ < 3p), N-form limbs, and the special cases (P = acc ->
    doubling, P = -acc -> identity)."""
    rng = random.Random(7)
    G = (1, 2)
    pts = [_mul(rng.randrange(1, 1 << 64), G) for _ in range(24)]
    lines, want = [], []
    for i in range(0, 24, 2):
        A, B = pts[i], pts[i + 1]
        za, zb = rng.randrange(1, P), rng.randrange(1, P)
        acc_a, acc_b = _acc(A, za), _acc(B, zb)
        # base B for madd: R-form x~ = x 2^256 mod p (canonical), shifted by 5
        xt, yt = B[0] * 2**256 % P, B[1] * 2**256 % P
        lines.append(" ".join(map(str, ["madd"] + acc_a + limbs(xt << 5) + limbs(yt << 5))))
        want.append(("madd", _affine_add(A, B), 0))
        # the negated base (the kernel's p - y~ for a negative digit)
        lines.append(" ".join(map(str, ["madd"] + acc_a + limbs(xt << 5) + limbs((P - yt) << 5))))
        want.append(("madd", _affine_add(A, (B[0], P - B[1])), 0))
        xa, ya = A[0] * 2**256 % P, A[1] * 2**256 % P
        # the kernel's negation in 29-bit limbs (msm_impl.h Pol29::repack_y): 33p - y~ << 5 with
        # kK33's raised limbs, at the top of its bound (y~ = 0 gives 33p itself)
        k33 = [0x281ca627, 0x2190778e, 0x2ac70d2f, 0x3d797cec, 0x26410879, 0x3e4358d5, 0x35830962,
               0x39e0ecb3, 0x063cee1b]
        assert value(k33) == 33 * P
        lines.append(" ".join(map(str, ["madd"] + acc_a + limbs(xt << 5) +
                                  [k - l for k, l in zip(k33, limbs(yt << 5))])))
        want.append(("madd", _affine_add(A, (B[0], P - B[1])), 0))
        lines.append(" ".join(map(str, ["madd"] + acc_a + limbs(xa << 5) +
                                  [k - l for k, l in zip(k33, limbs(ya << 5))])))
        want.append(("madd", None, 1))
        # specials: base = acc point (double in the caller), base = -acc (identity)
        xa, ya = A[0] * 2**256 % P, A[1] * 2**256 % P
        lines.append(" ".join(map(str, ["madd"] + acc_a + limbs(xa << 5) + limbs(ya << 5))))
        want.append(("madd", None, 2))
        lines.append(" ".join(map(str, ["madd"] + acc_a + limbs(xa << 5) + limbs((P - ya) << 5))))
        want.append(("madd", None, 1))
        lines.append(" ".join(map(str, ["add"] + acc_a + acc_b)))
        want.append(("add", _affine_add(A, B), 0))
        lines.append(" ".join(map(str, ["add"] + acc_a + _acc(A, zb))))
        want.append(("add", None, 2))
        lines.append(" ".join(map(str, ["add"] + acc_a + _acc((A[0], P - A[1]), zb))))
        want.append(("add", None, 1))
        lines.append(" ".join(map(str, ["dbl"] + acc_a)))
        want.append(("dbl", _affine_add(A, A), 0))
        lines.append(" ".join(map(str, ["start"] + limbs(xt << 5) + limbs(yt << 5))))
        want.append(("start", B, 0))
    out = point_harness(lines)
    for (op, expect, special), res in zip(want, out):
        sp, pt, vals, v = _point_of(res)
        assert sp == special, (op, sp, special)
        if special:
            continue
        assert pt == expect, op
        _check_bounds(vals, v, 10, 3, 3)
