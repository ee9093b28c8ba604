"""The lane-pair BLS12-381 G2 formulas over the 14 x 28-bit Fq
(tachyon_amd/csrc/msm/pair28.h) on the exact limb model of the device products
(tools/gen_f28.py: every column asserted below 2^64): both lanes of every
operation evaluated as the kernel does (lane 0: a0 b0 + a1 (K - b1), lane 1:
a0 b1 + a1 b0; squares as (a0 + a1)(a0 + K - a1) and a0 (2 a1)), with the
accumulator at the top of its invariant (X < 10p, Y < 6p, ZZ, ZZZ < 3p, largest
low limbs) and bases x~ << 8 up to 256p -- outputs equal madd-2008-s /
dbl-2008-s-1 over Fq2 mod p and stay inside the invariant.  The device code
is checked on the GPU by the BLS12-381 G2 MSM golden and parity tests."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_f28 as G  # noqa: E402

P, N, M28 = G.P, G.N, G.M
RR = pow(2, 392, P)
INV = pow(RR, -1, P)
limbs, value = G.limbs, G.value


def u32(ls):
    """the device's 32-bit limb registers: a limb-wise result must not wrap"""
    assert all(0 <= x < (1 << 32) for x in ls), "limb wrapped"
    return ls


def ksub(K, x):
    return u32([k - v for k, v in zip(K, x)])


def add(a, b):
    return u32([x + y for x, y in zip(a, b)])


def times(a, k):
    return u32([x * k for x in a])


def normalize(a):
    r, c = list(a), 0
    for i in range(N - 1):
        t = r[i] + c
        r[i], c = t & M28, t >> 28
    r[N - 1] += c
    return r


def reduce(v):
    """f28::reduce (float32 quotient as on the device)"""
    import struct
    f32 = lambda x: struct.unpack("f", struct.pack("f", x))[0]  # noqa: E731
    vf = f32(f32(float(v[N - 1]) * 268435456.0) + f32(float(v[N - 2])))
    q = max(int(f32(vf * f32(1.0 / (G.P_HI + 1)))) - 1, 0)
    pl = limbs(P)
    r, carry = [0] * N, 0
    for i in range(N):
        t = v[i] + carry - q * pl[i]
        r[i] = t & M28 if i < N - 1 else t
        carry = t >> 28
    return r


def is_zero(a):
    return value(a) % P == 0


# lane-pair values: (c0 limbs, c1 limbs)
def pmul(a, b, K, e=None):
    (a0, a1), (b0, b1) = a, b
    return (G.mul2(a0, b0, a1, ksub(K, b1), e[0] if e else None), G.mul2(a0, b1, a1, b0, e[1] if e else None))


def psqr(a, K, e=None):
    a0, a1 = a
    return (G.mul(add(a0, a1), add(a0, ksub(K, a1)), e[0] if e else None),
            G.mul(a0, times(a1, 2), e[1] if e else None))


def pksub(K, x):
    return (ksub(K, x[0]), ksub(K, x[1]))


def pksub2(K, a, b):
    return (u32([k - x - 2 * y for k, x, y in zip(K, a[0], b[0])]), u32([k - x - 2 * y for k, x, y in zip(K, a[1], b[1])]))


def padd_ksub(a, K, x):
    return (add(a[0], ksub(K, x[0])), add(a[1], ksub(K, x[1])))


def madd(A, x2, y2):
    X, Y, ZZ, ZZZ = A
    Pv = pmul(x2, ZZ, G.K4, pksub(G.K16, X))
    R = pmul(y2, ZZZ, G.K4, pksub(G.K8, Y))
    if is_zero(Pv[0]) and is_zero(Pv[1]):
        return (2 if is_zero(R[0]) and is_zero(R[1]) else 1), A
    PP = psqr(Pv, G.K32)
    PPP = pmul(Pv, PP, G.K4)
    Q = pmul(X, PP, G.K4)
    W = pmul(Y, PPP, G.K4)
    X3 = psqr(R, G.K16, pksub2(G.K8, PPP, Q))
    T = padd_ksub(Q, G.K16, X3)
    Y3 = pmul(R, T, G.K32R3, pksub(G.K4, W))
    return 0, (X3, Y3, pmul(ZZ, PP, G.K4), pmul(ZZZ, PPP, G.K4))


def dbl(A):
    X, Y, ZZ, ZZZ = A
    U = (normalize(times(Y[0], 2)), normalize(times(Y[1], 2)))
    V = psqr(U, G.K16)
    W = pmul(U, V, G.K4)
    S = pmul(X, V, G.K4)
    M = pmul(X, (normalize(times(X[0], 3)), normalize(times(X[1], 3))), G.K32)
    WY = pmul(W, Y, G.K8)
    zero = [0] * N
    X3 = psqr(M, G.K4, pksub2(G.K8, (zero, zero), S))
    Y3 = pmul(M, padd_ksub(S, G.K16, X3), G.K32R3, pksub(G.K4, WY))
    return X3, Y3, pmul(V, ZZ, G.K4), pmul(W, ZZZ, G.K4)


# exact Fq2 algebra (u^2 = -1), values mod p of the R''-form components
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
    W = fm(U, V)
    S = fm(X, V)
    XX = fm(X, X)
    M = fa(fa(XX, XX), XX)
    X3 = fs(fm(M, M), fa(S, S))
    Y3 = fs(fm(M, fs(S, X3)), fm(W, Y))
    return X3, Y3, fm(V, ZZ), fm(W, ZZZ)


def top_rep(v, bound):
    """largest-low-limb representative of v (an R''-form residue) below bound * p"""
    best = None
    for k in range(bound):
        w = v + k * P
        if w >= bound * P:
            break
        s = sum(limbs(w)[:N - 1])
        if best is None or s > best[0]:
            best = (s, w)
    return limbs(best[1])


def rand_acc(rng):
    comps = [(rng.randrange(P), rng.randrange(P)) for _ in range(4)]
    bounds = (10, 6, 3, 3)
    return tuple((top_rep(c[0] * RR % P, b), top_rep(c[1] * RR % P, b)) for c, b in zip(comps, bounds))


def base(rng, x=None):
    """a base component pair x~ << 8 with x~ (R-form, R = 2^384) canonical or lazy < 2p"""
    x = x if x is not None else (rng.randrange(P), rng.randrange(P))
    lazy = rng.random() < 0.5
    return tuple(limbs(((c * 2**384) % P + (P if lazy else 0)) << 8) for c in x), x


def check_out(A, want):
    got = tuple(f2(c) for c in A)
    assert got == want
    for (c0, c1), b in zip(A, (10, 6, 3, 3)):
        for c in (c0, c1):
            assert all(x <= M28 for x in c[:N - 1]) and value(c) < b * P


def test_pair_madd_and_dbl_at_bounds():
    rng = random.Random(11)
    for _ in range(60):
        A = rand_acc(rng)
        (x2, xv), (y2, yv) = base(rng), base(rng)
        sp, out = madd(A, x2, y2)
        assert sp == 0
        # the base as an Fq2 value: x~ 2^8 in R'' form = x 2^392 -> value x
        check_out(out, madd_ref(tuple(f2(c) for c in A), xv, yv))
        check_out(dbl(A), dbl_ref(tuple(f2(c) for c in A)))


def test_pair_madd_specials():
    rng = random.Random(12)
    for _ in range(10):
        A = rand_acc(rng)
        Af = tuple(f2(c) for c in A)
        # base = the accumulator's affine point: x2 ZZ = X, y2 ZZZ = Y -> special 2 (double)
        inv = lambda a: fm((a[0], (-a[1]) % P), (pow((a[0] ** 2 + a[1] ** 2) % P, -1, P), 0))  # noqa: E731
        xv = fm(Af[0], inv(Af[2]))
        yv = fm(Af[1], inv(Af[3]))
        (x2, _), (y2, _) = base(rng, xv), base(rng, yv)
        assert madd(A, x2, y2)[0] == 2
        (y2n, _) = base(rng, ((-yv[0]) % P, (-yv[1]) % P))
        assert madd(A, x2, y2n)[0] == 1


def test_run_start_bounds():
    rng = random.Random(13)
    for _ in range(50):
        (x2, xv), (y2, yv) = base(rng), base(rng)
        for c, want in ((x2[0], xv[0]), (x2[1], xv[1]), (y2[0], yv[0]), (y2[1], yv[1])):
            r = reduce(c)
            assert value(r) < 3 * P and value(r) * INV % P == want and all(x <= M28 for x in r[:N - 1])


def point_add(A, B):
    """add-2008-s for the G2 reductions (pair28.h add): inputs and outputs X <
    10p, Y < 6p, ZZ, ZZZ < 3p (from32 loads give < 3p)"""
    X1, Y1, ZZ1, ZZZ1 = A
    X2, Y2, ZZ2, ZZZ2 = B
    U1 = pmul(X1, ZZ2, G.K4)
    S1 = pmul(Y1, ZZZ2, G.K4)
    Pv = pmul(X2, ZZ1, G.K4, pksub(G.K4, U1))
    R = pmul(Y2, ZZZ1, G.K4, pksub(G.K4, S1))
    if is_zero(Pv[0]) and is_zero(Pv[1]):
        return (2 if is_zero(R[0]) and is_zero(R[1]) else 1), A
    PP = psqr(Pv, G.K16)
    PPP = pmul(Pv, PP, G.K4)
    Q = pmul(U1, PP, G.K4)
    Wv = pmul(S1, PPP, G.K4)
    X3 = psqr(R, G.K16, pksub2(G.K8, PPP, Q))
    T = padd_ksub(Q, G.K16, X3)
    Y3 = pmul(R, T, G.K32R3, pksub(G.K4, Wv))
    return 0, (X3, Y3, pmul(pmul(ZZ1, ZZ2, G.K4), PP, G.K4), pmul(pmul(ZZZ1, ZZZ2, G.K4), PPP, G.K4))


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


def test_pair28_add_at_bounds():
    """the reductions' addition at the top of the invariant"""
    rng = random.Random(14)
    for _ in range(60):
        A, B = rand_acc(rng), rand_acc(rng)
        sp, out = point_add(A, B)
        assert sp == 0
        check_out(out, add_ref(tuple(f2(c) for c in A), tuple(f2(c) for c in B)))
