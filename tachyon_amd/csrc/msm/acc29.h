// The 29-bit-limb BN254 G1 point arithmetic of the MSM (field/f29.h): the
// accumulation's mixed addition and the reductions' addition and doubling,
// with the value bounds they rely on.  Host and device (the host build runs
// f29.h's C++ columns; tests/test_f29_host.py checks these formulas against
// Python integers with operands at the top of their bounds).
#pragma once
#include "../field/f29.h"

namespace tachyon_amd::msm::acc29_core {
using namespace ::tachyon_amd::f29;
struct Acc {
  F29 x, y, zz, zzz;
};

// the first point of a run, from its coordinates already shifted for madd
TA_HD Acc from_shifted(const F29& x2, const F29& y2) {
  return {reduce_shl5(x2), reduce_shl5(y2), konst(kOne29), konst(kOne29)};
}

// acc + (x2, y2): madd-2008-s (point_xyzz_impl.h:129-176) with every
// subtraction folded into a product's output columns (limb-wise K - x, K a
// raised multiple of p) and Y3 = R (Q - X3) - Y1 PPP as one reduction of
// R T + (4p - Y1) PPP.  Value bounds (in units of p; a product of A and B
// leaves < A B / 128 + 1 + addend), invariant acc X < 10, Y, ZZ, ZZZ < 3 (a
// run's first point and the doubling's output come in through from32, < 3p);
// base coordinates x~ << 5 < 32, y2 < 33 (a negative digit's y is 33p - y~ << 5
// in kK33's raised limbs, limbs < 2^30):
//   P   = x2 ZZ1 + (16p - X1)  < 17.75    R  = y2 ZZZ1 + (4p - Y1) < 5.78
//   PP  = P^2 < 3.47  PPP = P PP < 1.49   Q  = X1 PP < 1.28
//   X3  = R^2 + (8p - PPP - 2Q) < 9.26    T  = Q + (16p - X3) < 17.3
//   Y3  = R T + (4p - Y1) PPP < 1.83      ZZ3, ZZZ3 < 1.09
// Column sums stay below 2^64: the widest, R T + (4p - Y1) PPP + m p, is
// < 13.5 2^60 (T's limbs < 1.41 2^30, 4p - Y1's < 2^30).
// *special = 1: the sum is the identity (P = -acc), 2: P = acc (the caller
// doubles); acc is returned unchanged then.
TA_HD Acc madd(const Acc& A, const F29& x2, const F29& y2, int* special) {
  const F29 P = mul_add(x2, A.zz, ksub(kK16, A.x));
  const F29 R = mul_add(y2, A.zzz, ksub(kK4, A.y));
  if (is_zero_mod_p(P)) {
    *special = is_zero_mod_p(R) ? 2 : 1;
    return A;
  }
  const F29 PP = sqr(P);
  const F29 PPP = mul(P, PP);
  const F29 Q = mul(A.x, PP);
  Acc C;
  C.x = sqr_add(R, ksub2(kK8, PPP, Q));
  const F29 T = add_ksub(Q, kK16, C.x);
  C.y = mul2_add(R, T, ksub(kK4, A.y), PPP);
  C.zz = mul(A.zz, PP);
  C.zzz = mul(A.zzz, PPP);
  return C;
}

// The bucket-sum reductions over the same field (chain join, window sums).
// Invariant of their points: X < 10p, Y, ZZ, ZZZ < 3p (from32 of R-form
// values gives < 3p).  add-2008-s (point_xyzz_impl.h:45-97), both operands
// not the identity; *special as madd's:
//   U1 = X1 ZZ2 < 1.24   S1 = Y1 ZZZ2 < 1.08
//   P  = X2 ZZ1 + (4p - U1) < 5.24       R = Y2 ZZZ1 + (4p - S1) < 5.08
//   PP < 1.22  PPP < 1.05  Q = U1 PP < 1.02
//   X3 = R^2 + (8p - PPP - 2Q) < 9.21    T = Q + (16p - X3) < 17.1
//   Y3 = R T + (4p - S1) PPP < 1.72      ZZ3 = (ZZ1 ZZ2) PP, ZZZ3 < 1.02
TA_HD Acc add(const Acc& A, const Acc& B, int* special) {
  const F29 U1 = mul(A.x, B.zz), S1 = mul(A.y, B.zzz);
  const F29 P = mul_add(B.x, A.zz, ksub(kK4, U1));
  const F29 R = mul_add(B.y, A.zzz, ksub(kK4, S1));
  if (is_zero_mod_p(P)) {
    *special = is_zero_mod_p(R) ? 2 : 1;
    return A;
  }
  const F29 PP = sqr(P);
  const F29 PPP = mul(P, PP);
  const F29 Q = mul(U1, PP);
  Acc C;
  C.x = sqr_add(R, ksub2(kK8, PPP, Q));
  const F29 T = add_ksub(Q, kK16, C.x);
  C.y = mul2_add(R, T, ksub(kK4, S1), PPP);
  C.zz = mul(mul(A.zz, B.zz), PP);
  C.zzz = mul(mul(A.zzz, B.zzz), PPP);
  return C;
}
// dbl-2008-s-1 (a = 0; point_xyzz_impl.h:199-236) under the same invariant:
//   U = 2 Y1 < 6   V = U^2 < 1.29   W = U V < 1.07   S = X1 V < 1.11
//   M = X1 (3 X1) < 3.35 (3 X1's limbs < 1.5 2^30)
//   X3 = M^2 + (8p - 2S) < 9.09      Y3 = M (S + 16p - X3) + (4p - W) Y1 < 1.55
//   ZZ3 = V ZZ1, ZZZ3 = W ZZZ1 < 1.04
// (the widest column, M T + (4p - W) Y1 + m p, < 10.2 2^60)
TA_HD Acc dbl(const Acc& A) {
  const F29 U = times(A.y, 2);
  const F29 V = sqr(U);
  const F29 W = mul(U, V);
  const F29 S = mul(A.x, V);
  const F29 M = mul(A.x, times(A.x, 3));
  F29 zero{};
  Acc C;
  C.x = sqr_add(M, ksub2(kK8, zero, S));
  C.y = mul2_add(M, add_ksub(S, kK16, C.x), ksub(kK4, W), A.y);
  C.zz = mul(V, A.zz);
  C.zzz = mul(W, A.zzz);
  return C;
}
}  // namespace tachyon_amd::msm::acc29_core
