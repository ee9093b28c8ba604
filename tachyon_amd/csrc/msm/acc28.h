// The 28-bit-limb BLS12-381 G1 point arithmetic of the MSM (field/f28.h): the
// accumulation's mixed addition, the run start and the doubling of the rare
// P = acc case -- msm/acc29.h's formulas over the 14 x 28-bit field.  Host and
// device (tests/test_f28_host.py checks them against affine arithmetic with
// operands at the top of their bounds).
#pragma once
#include "../field/f28.h"

namespace tachyon_amd::msm::acc28_core {
using namespace ::tachyon_amd::f28;
struct Acc {
  F28 x, y, zz, zzz;
};

// the first point of a run, from its coordinates already shifted for madd
TA_HD Acc from_shifted(const F28& x2, const F28& y2) {
  return {reduce(x2), reduce(y2), konst(kOne28), konst(kOne28)};
}

// acc + (x2, y2): madd-2008-s (point_xyzz_impl.h:129-176), every subtraction
// folded into a product's output columns, Y3 = R (Q - X3) - Y1 PPP as one
// reduction.  Value bounds in units of p (a product of A and B leaves
// < A B / 2520 + 1 + addend; R'' / p > 2520), invariant acc X < 10, Y, ZZ,
// ZZZ < 3; base coordinates x~ << 8 < 512 (lazy R-form inputs < 2p):
//   P   = x2 ZZ1 + (16p - X1) < 17.61   R  = y2 ZZZ1 + (4p - Y1) < 5.61
//   PP  < 1.13  PPP < 1.008  Q = X1 PP < 1.005
//   X3  = R^2 + (8p - PPP - 2Q) < 9.02  T  = Q + (16p - X3) < 17.01
//   Y3  = R T + (4p - Y1) PPP < 1.05    ZZ3, ZZZ3 < 1.002
// Column sums: the widest, R T + (4p - Y1) PPP + m p, has 42 products of
// < 2^28 x 2^29.6 -- < 2^62.
// *special = 1: the sum is the identity (P = -acc), 2: P = acc (the caller
// doubles); acc is returned unchanged then.
TA_HD Acc madd(const Acc& A, const F28& x2, const F28& y2, int* special) {
  const F28 P = mul_add(x2, A.zz, ksub(kK16, A.x));
  const F28 R = mul_add(y2, A.zzz, ksub(kK4, A.y));
  if (is_zero_mod_p(P)) {
    *special = is_zero_mod_p(R) ? 2 : 1;
    return A;
  }
  const F28 PP = sqr(P);
  const F28 PPP = mul(P, PP);
  const F28 Q = mul(A.x, PP);
  Acc C;
  C.x = sqr_add(R, ksub2(kK8, PPP, Q));
  const F28 T = add_ksub(Q, kK16, C.x);
  C.y = mul2_add(R, T, ksub(kK4, A.y), PPP);
  C.zz = mul(A.zz, PP);
  C.zzz = mul(A.zzz, PPP);
  return C;
}

// The bucket-sum reductions over the same field: add-2008-s
// (point_xyzz_impl.h:45-97), both operands not the identity, invariant X <
// 10p, Y, ZZ, ZZZ < 3p (from32 gives < 3p); *special as madd's:
//   U1 = X1 ZZ2, S1 = Y1 ZZZ2 < 1.02   P = X2 ZZ1 + (4p - U1) < 5.02
//   R = Y2 ZZZ1 + (4p - S1) < 5.01     PP < 1.02  PPP, Q < 1.003
//   X3 = R^2 + (8p - PPP - 2Q) < 9.02  Y3 = R T + (4p - S1) PPP < 1.04
//   ZZ3 = (ZZ1 ZZ2) PP, ZZZ3 < 1.002
TA_HD Acc add(const Acc& A, const Acc& B, int* special) {
  const F28 U1 = mul(A.x, B.zz), S1 = mul(A.y, B.zzz);
  const F28 ZZ12 = mul(A.zz, B.zz), ZZZ12 = mul(A.zzz, B.zzz);
  const F28 P = mul_add(B.x, A.zz, ksub(kK4, U1));
  const F28 R = mul_add(B.y, A.zzz, ksub(kK4, S1));
  if (is_zero_mod_p(P)) {
    *special = is_zero_mod_p(R) ? 2 : 1;
    return A;
  }
  const F28 PP = sqr(P);
  const F28 PPP = mul(P, PP);
  const F28 Q = mul(U1, PP);
  Acc C;
  C.x = sqr_add(R, ksub2(kK8, PPP, Q));
  const F28 T = add_ksub(Q, kK16, C.x);
  C.y = mul2_add(R, T, ksub(kK4, S1), PPP);
  C.zz = mul(ZZ12, PP);
  C.zzz = mul(ZZZ12, PPP);
  return C;
}

// dbl-2008-s-1 (a = 0; point_xyzz_impl.h:199-236) under the same invariant:
//   U = 2 Y1 < 6   V = U^2 < 1.02   W = U V < 1.003   S = X1 V < 1.005
//   M = X1 (3 X1) < 1.12
//   X3 = M^2 + (8p - 2S) < 9.01     Y3 = M (S + 16p - X3) + (4p - W) Y1 < 1.02
//   ZZ3 = V ZZ1, ZZZ3 = W ZZZ1 < 1.002
TA_HD Acc dbl(const Acc& A) {
  const F28 U = times(A.y, 2);
  const F28 V = sqr(U);
  const F28 W = mul(U, V);
  const F28 S = mul(A.x, V);
  const F28 M = mul(A.x, times(A.x, 3));
  F28 zero{};
  Acc C;
  C.x = sqr_add(M, ksub2(kK8, zero, S));
  C.y = mul2_add(M, add_ksub(S, kK16, C.x), ksub(kK4, W), A.y);
  C.zz = mul(V, A.zz);
  C.zzz = mul(W, A.zzz);
  return C;
}
}  // namespace tachyon_amd::msm::acc28_core
