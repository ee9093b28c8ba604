"""The lane-pair BN254 G2 formulas over the 9 x 29-bit Fq
(tachyon_amd/csrc/msm/pair29.h) on the exact limb model of the device products
(field/f29.h's columns, every column asserted below 2^64): both lanes of every
operation evaluated as the kernel does (lane 0: a0 b0 + a1 (K - b1), lane 1:
a0 b1 + a1 b0; squares as (a0 + a1)(a0 + K - a1) and a0 (2 a1)), the
accumulator at the top of madd's input invariant (X, Y < 32p, ZZ, ZZZ < 3p,
largest low limbs -- a run's first point comes in unreduced as x~ << 5) and
bases x~ << 5 < 32p -- outputs equal madd-2008-s / dbl-2008-s-1 over Fq2 mod p
and stay inside the invariant.  R' / p = 2^7.4 is small for the pair's
two-product reductions, so P and R are brought under 3p (f29::reduce_shl5)
before the products that square them.  The device code is checked on the GPU
by the BN254 G2 MSM golden and parity tests."""
import os
import random
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_f29_constants as C  # noqa: E402

P, N, W = C.P, 9, 29
M29 = (1 << W) - 1
RP = pow(2, 261, P)  # R'
INV = pow(RP, -1, P)
limbs = C.limbs
PINV = (-pow(P, -1, 1 << W)) % (1 << W)
PL = limbs(P)


def value(ls):
    return sum(x << (W * i) for i, x in enumerate(ls))


def u32(ls):
    """the device's 32-bit limb registers: a limb-wise result must not wrap"""
    assert all(0 <= x < (1 << 32) for x in ls), "limb wrapped"
    return ls


def _redc(pairs, e=None):
    """f29::redc: columns of the products, the FIPS digits, e added to the output columns"""
    acc, m, r = 0, [0] * N, [0] * N
    for k in range(2 * N - 1):
        for a, b in pairs:
            for i in range(N):
                if 0 <= k - i < N:
                    acc += a[i] * b[k - i]
        for i in range(N):
            if i < k and 0 < k - i < N:
                acc += m[i] * PL[k - i]
        if k < N:
            m[k] = ((acc & 0xFFFFFFFF) * PINV) & M29
            acc += m[k] * PL[0]
        else:
            if e is not None:
                acc += e[k - N]
            r[k - N] = acc & M29
        assert acc < (1 << 64), "column overflow"
        acc >>= W
    r[N - 1] = acc + (e[N - 1] if e is not None else 0)
    return u32(r)


def reduce(v):
    """f29::reduce_shl5 (float32 quotient as on the device)"""
    f32 = lambda x: struct.unpack("f", struct.pack("f", x))[0]  # noqa: E731
    vf = f32(f32(float(v[N - 1]) * 536870912.0) + f32(float(v[N - 2])))
    q = max(int(f32(vf * f32(1.0 / 1702635872462389.0))) - 1, 0)
    r, carry = [0] * N, 0
    for i in range(N):
        t = v[i] + carry - q * PL[i]
        r[i] = t & M29 if i < N - 1 else t
        carry = t >> W
    assert r[N - 1] >= 0
    return r


def normalize(a):
    r, c = list(a), 0
    for i in range(N - 1):
        t = r[i] + c
        r[i], c = t & M29, t >> W
    r[N - 1] += c
    return r


K4, K8, K16 = C.raised(4, 1), C.raised(8, 4), C.raised(16, 1)
K32R3 = C.raised(32, 3)
K33 = C.raised(33, 1)


def ksub(K, x):
    return u32([k - v for k, v in zip(K, x)])


def add(a, b):
    return u32([x + y for x, y in zip(a, b)])


def times(a, k):
    return u32([x * k for x in a])


def is_zero(a):
    return value(a) % P == 0


# lane-pair values: (c0 limbs, c1 limbs)
def pmul(a, b, K, e=None):
    (a0, a1), (b0, b1) = a, b
    return (_redc([(a0, b0), (a1, ksub(K, b1))], e[0] if e else None), _redc([(a0, b1), (a1, b0)], e[1] if e else None))


def psqr(a, K, e=None):
    a0, a1 = a
    return (_redc([(add(a0, a1), add(a0, ksub(K, a1)))], e[0] if e else None),
            _redc([(a0, times(a1, 2))], e[1] if e else None))


def pksub(K, x):
    return (ksub(K, x[0]), ksub(K, x[1]))


def pksub2(K, a, b):
    return (u32([k - x - 2 * y for k, x, y in zip(K, a[0], b[0])]), u32([k - x - 2 * y for k, x, y in zip(K, a[1], b[1])]))


def padd_ksub(a, K, x):
    return (add(a[0], ksub(K, x[0])), add(a[1], ksub(K, x[1])))


def pred(a):
    return (reduce(a[0]), reduce(a[1]))


def madd(A, x2, y2):
    X, Y, ZZ, ZZZ = A
    Pv = pred(pmul(x2, ZZ, K4, pksub(K33, X)))
    R = pred(pmul(y2, ZZZ, K4, pksub(K33, Y)))
    if is_zero(Pv[0]) and is_zero(Pv[1]):
        return (2 if is_zero(R[0]) and is_zero(R[1]) else 1), A
    PP = psqr(Pv, K4)
    PPP = pmul(Pv, PP, K4)
    Q = pmul(X, PP, K4)
    Wv = pmul(Y, PPP, K4)
    X3 = psqr(R, K4, pksub2(K8, PPP, Q))
    T = padd_ksub(Q, K16, X3)
    Y3 = pmul(R, T, K32R3, pksub(K4, Wv))
    return 0, (X3, Y3, pmul(ZZ, PP, K4), pmul(ZZZ, PPP, K4))


def dbl(A):
    """the rare doubling (P = acc) under the same input invariant: X and Y
    reduced first (< 3p), 2Y and 3X normalized"""
    X, Y, ZZ, ZZZ = A
    Xr, Yr = pred(X), pred(Y)
    U = (normalize(times(Yr[0], 2)), normalize(times(Yr[1], 2)))
    V = psqr(U, K4)
    Wv = pmul(U, V, K4)
    S = pmul(Xr, V, K4)
    M = pmul(Xr, (normalize(times(Xr[0], 3)), normalize(times(Xr[1], 3))), K16)
    WY = pmul(Wv, Yr, K4)
    zero = [0] * N
    X3 = psqr(M, K4, pksub2(K8, (zero, zero), S))
    Y3 = pmul(M, padd_ksub(S, K16, X3), K32R3, pksub(K4, WY))
    return X3, Y3, pmul(V, ZZ, K4), pmul(Wv, ZZZ, K4)


# exact Fq2 algebra (u^2 = -1), values mod p of the R'-form components
def f2(v):
    return (value(v[0]) * INV % P, value(v[1]) * INV % P)


def fm(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def fs(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def fa(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def madd_ref(A, x2, y2):
    X, Y, ZZ, ZZZ = A
    Pv = fs(fm(x2, ZZ), X)
    R = fs(fm(y2, ZZZ), Y)
    PP = fm(Pv, Pv)
    PPP = fm(Pv, PP)
    Q = fm(X, PP)
    X3 = fs(fs(fm(R, R), PPP), fa(Q, Q))
    Y3 = fs(fm(R, fs(Q, X3)), fm(Y, PPP))
    return X3, Y3, fm(ZZ, PP), fm(ZZZ, PPP)


def dbl_ref(A):
    X, Y, ZZ, ZZZ = A
    U = fa(Y, Y)
    V = fm(U, U)
    Wv = fm(U, V)
    S = fm(X, V)
    XX = fm(X, X)
    M = fa(fa(XX, XX), XX)
    X3 = fs(fm(M, M), fa(S, S))
    Y3 = fs(fm(M, fs(S, X3)), fm(Wv, Y))
    return X3, Y3, fm(V, ZZ), fm(Wv, ZZZ)


def top_rep(v, bound):
    """largest-low-limb representative of v (an R'-form residue) below bound * p"""
    best = None
    for k in range(bound):
        w = v + k * P
        if w >= bound * P:
            break
        s = sum(limbs(w)[:N - 1])
        if best is None or s > best[0]:
            best = (s, w)
    return limbs(best[1])


IN_BOUNDS = (32, 32, 3, 3)   # madd's input invariant (a run's first point: x~ << 5 as it is)
OUT_BOUNDS = (10, 6, 3, 3)   # what madd and dbl leave (inside IN_BOUNDS)


def rand_acc(rng, bounds=IN_BOUNDS):
    comps = [(rng.randrange(P), rng.randrange(P)) for _ in range(4)]
    return tuple((top_rep(c[0] * RP % P, b), top_rep(c[1] * RP % P, b)) for c, b in zip(comps, bounds))


def base(rng, x=None):
    """a base component pair x~ << 5 with x~ (R-form, R = 2^256) canonical"""
    x = x if x is not None else (rng.randrange(P), rng.randrange(P))
    return tuple(limbs(((c * 2**256) % P) << 5) for c in x), x


def check_out(A, want, bounds=OUT_BOUNDS):
    got = tuple(f2(c) for c in A)
    assert got == want
    for (c0, c1), b in zip(A, bounds):
        for c in (c0, c1):
            assert all(x <= M29 for x in c[:N - 1]) and value(c) < b * P


def test_pair29_madd_and_dbl_at_bounds():
    rng = random.Random(21)
    for _ in range(60):
        A = rand_acc(rng)
        (x2, xv), (y2, yv) = base(rng), base(rng)
        sp, out = madd(A, x2, y2)
        assert sp == 0
        # the base as an Fq2 value: x~ 2^5 in R' form = x 2^261 -> value x
        check_out(out, madd_ref(tuple(f2(c) for c in A), xv, yv))
        check_out(dbl(A), dbl_ref(tuple(f2(c) for c in A)))


def test_pair29_run_start_then_madd():
    """a run's first point as from_shifted leaves it (x~ << 5, Z = 1) and the next madd"""
    rng = random.Random(22)
    one = limbs(RP % P)
    for _ in range(30):
        (x2, xv), (y2, yv) = base(rng), base(rng)
        A = (x2, y2, (one, [0] * N), (one, [0] * N))
        (bx, bxv), (by, byv) = base(rng), base(rng)
        sp, out = madd(A, bx, by)
        assert sp == 0
        check_out(out, madd_ref((xv, yv, (1, 0), (1, 0)), bxv, byv))


def test_pair29_madd_specials():
    rng = random.Random(23)
    for _ in range(10):
        A = rand_acc(rng)
        Af = tuple(f2(c) for c in A)
        inv = lambda a: fm((a[0], (-a[1]) % P), (pow((a[0] ** 2 + a[1] ** 2) % P, -1, P), 0))  # noqa: E731
        xv = fm(Af[0], inv(Af[2]))
        yv = fm(Af[1], inv(Af[3]))
        (x2, _), (y2, _) = base(rng, xv), base(rng, yv)
        assert madd(A, x2, y2)[0] == 2
        (y2n, _) = base(rng, ((-yv[0]) % P, (-yv[1]) % P))
        assert madd(A, x2, y2n)[0] == 1


def test_pair29_mutant_detected():
    """the model notices a too-small site constant (16p for X, as before the
    unreduced run start): a limb wraps or a bound breaks"""
    rng = random.Random(24)
    global K33
    keep = K33
    try:
        K33 = K16
        failed = False
        for _ in range(20):
            A = rand_acc(rng)
            (x2, xv), (y2, yv) = base(rng), base(rng)
            try:
                sp, out = madd(A, x2, y2)
                check_out(out, madd_ref(tuple(f2(c) for c in A), xv, yv))
            except AssertionError:
                failed = True
                break
        assert failed
    finally:
        K33 = keep


def point_add(A, B):
    """add-2008-s for the G2 reductions (pair29.h add): inputs and outputs X <
    10p, Y < 6p, ZZ, ZZZ < 3p (from32 loads give < 3p); R reduced before its
    square, P squared as it is (5.4p, the 8p negation constant)"""
    X1, Y1, ZZ1, ZZZ1 = A
    X2, Y2, ZZ2, ZZZ2 = B
    U1 = pmul(X1, ZZ2, K4)
    S1 = pmul(Y1, ZZZ2, K4)
    Pv = pmul(X2, ZZ1, K4, pksub(K4, U1))
    R = pred(pmul(Y2, ZZZ1, K4, pksub(K4, S1)))
    if is_zero(Pv[0]) and is_zero(Pv[1]):
        return (2 if is_zero(R[0]) and is_zero(R[1]) else 1), A
    PP = psqr(Pv, K8)
    PPP = pmul(Pv, PP, K4)
    Q = pmul(U1, PP, K4)
    Wv = pmul(S1, PPP, K4)
    X3 = psqr(R, K4, pksub2(K8, PPP, Q))
    T = padd_ksub(Q, K16, X3)
    Y3 = pmul(R, T, K32R3, pksub(K4, Wv))
    return 0, (X3, Y3, pmul(pmul(ZZ1, ZZ2, K4), PP, K4), pmul(pmul(ZZZ1, ZZZ2, K4), PPP, K4))


def add_ref(A, B):
    X1, Y1, ZZ1, ZZZ1 = A
    X2, Y2, ZZ2, ZZZ2 = B
    U1, S1 = fm(X1, ZZ2), fm(Y1, ZZZ2)
    Pv = fs(fm(X2, ZZ1), U1)
    R = fs(fm(Y2, ZZZ1), S1)
    PP = fm(Pv, Pv)
    PPP = fm(Pv, PP)
    Q = fm(U1, PP)
    X3 = fs(fs(fm(R, R), PPP), fa(Q, Q))
    Y3 = fs(fm(R, fs(Q, X3)), fm(S1, PPP))
    return X3, Y3, fm(fm(ZZ1, ZZ2), PP), fm(fm(ZZZ1, ZZZ2), PPP)


def test_pair29_add_at_bounds():
    """the reductions' addition at the top of X < 10p, Y < 6p, ZZ, ZZZ < 3p"""
    rng = random.Random(25)
    for _ in range(60):
        A, B = rand_acc(rng, OUT_BOUNDS), rand_acc(rng, OUT_BOUNDS)
        sp, out = point_add(A, B)
        assert sp == 0
        check_out(out, add_ref(tuple(f2(c) for c in A), tuple(f2(c) for c in B)))
