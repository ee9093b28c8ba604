// BN254 G2 bucket accumulation with a lane pair per point (msm/acc_pair.h)
// over the 9 x 29-bit Fq (field/f29.h): lane 2v holds the c0 and lane 2v + 1
// the c1 component of every Fq2 value, the partner's components come in by
// DPP, and every Fq2 product is ONE 29-bit two-product reduction per lane,
//   lane h: a0 b_h + a1 s_h,  s_0 = K - b1 (-b1), s_1 = b0,
// with the subtraction that follows it in madd-2008-s folded into the same
// columns (the reduction's addend) -- msm/pair28.h's layout on BN254.
//
// R' / p = 2^7.4 only (BLS12-381's 28-bit field has 2^11.3), and a pair
// product's second term doubles its output bound, so P and R are brought
// under 3p (reduce_shl5: a float quotient and 9 multiply-adds) before the
// products that square them.  Value bounds (units of p, per component; a
// product leaves < (A B + A S) / 170 + 1 + addend), madd's input invariant X,
// Y < 32, ZZ, ZZZ < 3 (a run's first point comes in as x~ << 5, unreduced),
// its outputs X < 10, Y < 6, ZZ, ZZZ < 3; bases x~ << 5 < 32:
//   P   = x2 ZZ + (33p - X) < 35.3 -> < 3    R = y2 ZZZ + (33p - Y) -> < 3
//   PP  = P^2 (lane 0: (P0 + P1)(P0 + 4p - P1))  < 1.25
//   PPP = P PP < 1.09        Q = X PP < 1.98     W = Y PPP < 1.95
//   X3  = R^2 + (8p - PPP - 2Q) < 9.25          T = Q + 16p - X3 < 18
//   Y3  = R T + (4p - W)  < 5.9   (T negated as 32p - T, limbs < 3 2^29)
//   ZZ3 = ZZ PP, ZZZ3 = ZZZ PPP < 1.09
// tests/test_pair29_model.py runs these formulas on the exact limb model with
// operands at the top of their bounds (values, 32-bit limbs, 64-bit columns).
#pragma once
#include "../field/f29.h"
#include "acc_pair.h"

namespace tachyon_amd::msm::pair29 {
using namespace ::tachyon_amd::f29;
using pair::dpp;
using pair::kEven;
using pair::kOdd;
using pair::kSwap;

__device__ __forceinline__ F29 even(const F29& a) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = dpp<kEven>(a.l[i]);
  return r;
}
__device__ __forceinline__ F29 odd(const F29& a) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = dpp<kOdd>(a.l[i]);
  return r;
}
// s_h: lane 0 gets K - b1 from its partner, lane 1 gets b0
template <const uint32_t (&K)[9]>
__device__ __forceinline__ F29 partner_s(const F29& b, bool h) {
  const F29 nb = ksub(K, b);
  F29 s;
#pragma unroll
  for (int i = 0; i < 9; ++i) s.l[i] = dpp<kSwap>(h ? nb.l[i] : b.l[i]);
  return s;
}
// this lane's component of a b (+ e): one two-product reduction
template <const uint32_t (&K)[9]>
__device__ __forceinline__ F29 pmul(const F29& a, const F29& b, bool h) {
  return mul2_add(even(a), b, odd(a), partner_s<K>(b, h));
}
template <const uint32_t (&K)[9]>
__device__ __forceinline__ F29 pmul_add(const F29& a, const F29& b, const F29& e, bool h) {
#if defined(__HIP_DEVICE_COMPILE__)
  return asm29::mul2_add(even(a), b, odd(a), partner_s<K>(b, h), e);
#else
  return redc<true, true>(even(a), b, odd(a), partner_s<K>(b, h), e);
#endif
}
// this lane's component of a^2 (+ e): lane 0 (a0 + a1)(a0 + K - a1), lane 1 a0 (2 a1)
template <const uint32_t (&K)[9]>
__device__ __forceinline__ F29 psqr_operands(const F29& a, bool h, F29* y) {
  const F29 a0 = even(a), a1 = odd(a);
  F29 x;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    x.l[i] = h ? a0.l[i] : a0.l[i] + a1.l[i];
    y->l[i] = h ? (a1.l[i] << 1) : a0.l[i] + (K[i] - a1.l[i]);
  }
  return x;
}
template <const uint32_t (&K)[9]>
__device__ __forceinline__ F29 psqr(const F29& a, bool h) {
  F29 y;
  const F29 x = psqr_operands<K>(a, h, &y);
  return mul(x, y);
}
template <const uint32_t (&K)[9]>
__device__ __forceinline__ F29 psqr_add(const F29& a, const F29& e, bool h) {
  F29 y;
  const F29 x = psqr_operands<K>(a, h, &y);
  return mul_add(x, y, e);
}
// zero of the whole Fq2 value (both lanes agree)
__device__ __forceinline__ bool pzero(const F29& a) {
  const uint32_t z = is_zero_mod_p(a) ? 1u : 0u;
  return (z & dpp<kSwap>(z)) != 0;
}

struct Acc {
  F29 x, y, zz, zzz;
};

// the first point of a run as it comes (lane h: its components; (1, 0) for Z)
__device__ __forceinline__ Acc from_shifted(const F29& x2, const F29& y2, bool h) {
  const F29 one = h ? F29{} : konst(kOne29);
  return {x2, y2, one, one};
}

// madd-2008-s (point_xyzz_impl.h:129-176); *special as acc29::madd
__device__ __forceinline__ Acc madd(const Acc& A, const F29& x2, const F29& y2, bool h, int* special) {
  const F29 P = reduce_shl5(pmul_add<kK4>(x2, A.zz, ksub(kK33, A.x), h));
  const F29 R = reduce_shl5(pmul_add<kK4>(y2, A.zzz, ksub(kK33, A.y), h));
  if (pzero(P)) {
    *special = pzero(R) ? 2 : 1;
    return A;
  }
  const F29 PP = psqr<kK4>(P, h);
  const F29 PPP = pmul<kK4>(P, PP, h);
  const F29 Q = pmul<kK4>(A.x, PP, h);
  const F29 W = pmul<kK4>(A.y, PPP, h);
  Acc C;
  C.x = psqr_add<kK4>(R, ksub2(kK8, PPP, Q), h);
  const F29 T = add_ksub(Q, kK16, C.x);
  C.y = pmul_add<kK32r3>(R, T, ksub(kK4, W), h);
  C.zz = pmul<kK4>(A.zz, PP, h);
  C.zzz = pmul<kK4>(A.zzz, PPP, h);
  return C;
}

// dbl-2008-s-1 (a = 0; point_xyzz_impl.h:199-236), the rare P = acc case
// (performance does not matter): X, Y reduced under 3p first, 2Y and 3X
// normalized (tests/test_pair29_model.py's dbl)
__device__ __forceinline__ Acc dbl(const Acc& A, bool h) {
  const F29 X = reduce_shl5(A.x), Y = reduce_shl5(A.y);
  const F29 U = normalize(times(Y, 2));
  const F29 V = psqr<kK4>(U, h);
  const F29 W = pmul<kK4>(U, V, h);
  const F29 S = pmul<kK4>(X, V, h);
  const F29 M = pmul<kK16>(X, normalize(times(X, 3)), h);
  const F29 WY = pmul<kK4>(W, Y, h);
  F29 zero{};
  Acc C;
  C.x = psqr_add<kK4>(M, ksub2(kK8, zero, S), h);
  C.y = pmul_add<kK32r3>(M, add_ksub(S, kK16, C.x), ksub(kK4, WY), h);
  C.zz = pmul<kK4>(V, A.zz, h);
  C.zzz = pmul<kK4>(W, A.zzz, h);
  return C;
}

// add-2008-s (point_xyzz_impl.h:45-97) for the G2 reductions, both operands
// not the identity (the caller keeps identity flags); inputs and outputs
// X < 10p, Y < 6p, ZZ, ZZZ < 3p (from32 loads give < 3p), R reduced before its
// square, P squared as it is with the 8p negation constant; *special as madd's
// (tests/test_pair29_model.py point_add)
__device__ __forceinline__ Acc add(const Acc& A, const Acc& B, bool h, int* special) {
  // ZZ1 ZZ2 and ZZZ1 ZZZ2 first: the operands' Z coordinates die early (register pressure)
  const F29 U1 = pmul<kK4>(A.x, B.zz, h), S1 = pmul<kK4>(A.y, B.zzz, h);
  const F29 ZZ12 = pmul<kK4>(A.zz, B.zz, h), ZZZ12 = pmul<kK4>(A.zzz, B.zzz, h);
  const F29 P = pmul_add<kK4>(B.x, A.zz, ksub(kK4, U1), h);
  const F29 R = reduce_shl5(pmul_add<kK4>(B.y, A.zzz, ksub(kK4, S1), h));
  if (pzero(P)) {
    *special = pzero(R) ? 2 : 1;
    return A;
  }
  const F29 PP = psqr<kK8>(P, h);
  const F29 PPP = pmul<kK4>(P, PP, h);
  const F29 Q = pmul<kK4>(U1, PP, h);
  const F29 W = pmul<kK4>(S1, PPP, h);
  Acc C;
  C.x = psqr_add<kK4>(R, ksub2(kK8, PPP, Q), h);
  const F29 T = add_ksub(Q, kK16, C.x);
  C.y = pmul_add<kK32r3>(R, T, ksub(kK4, W), h);
  C.zz = pmul<kK4>(ZZ12, PP, h);
  C.zzz = pmul<kK4>(ZZZ12, PPP, h);
  return C;
}

}  // namespace tachyon_amd::msm::pair29
