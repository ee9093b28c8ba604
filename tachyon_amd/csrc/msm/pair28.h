// BLS12-381 G2 bucket accumulation with a lane pair per point (msm/acc_pair.h)
// over the 14 x 28-bit Fq (field/f28.h): lane 2v holds the c0 and lane 2v + 1
// the c1 component of every Fq2 value, the partner's components come in by
// DPP, and every Fq2 product is ONE 28-bit two-product reduction per lane,
//   lane h: a0 b_h + a1 s_h,  s_0 = K - b1 (-b1), s_1 = b0,
// with the subtraction that follows it in madd-2008-s folded into the same
// columns (the reduction's addend), as in the G1 28-bit field (msm/acc28.h).
//
// Value bounds (units of p, per component; a product leaves < (A B + A S) /
// 2520 + 1 + addend, R'' / p > 2520), invariant of the accumulator: X < 10,
// Y < 6, ZZ, ZZZ < 3, normalized limbs; base components x~ << 8 < 256:
//   P   = x2 ZZ + (16p - X)   < 17.71    R   = y2 ZZZ + (8p - Y)  < 9.71
//   PP  = P^2 (lane 0: (P0 + P1)(P0 + 32p - P1))  < 1.70
//   PPP = P PP < 1.04        Q = X PP < 1.03     W = Y PPP < 1.02
//   X3  = R^2 + (8p - PPP - 2Q) < 9.20          T = Q + 16p - X3 < 17.03
//   Y3  = R T + (4p - W)  < 5.2   (T negated as 32p - T, limbs < 3 2^28)
//   ZZ3 = ZZ PP, ZZZ3 = ZZZ PPP < 1.01
// tests/test_pair28_model.py runs these formulas on the exact limb model with
// operands at the top of their bounds (values, limbs, 64-bit columns).
#pragma once
#include "../field/f28.h"
#include "acc_pair.h"

namespace tachyon_amd::msm::pair28 {
using namespace ::tachyon_amd::f28;
using pair::dpp;
using pair::kEven;
using pair::kOdd;
using pair::kSwap;

__device__ __forceinline__ F28 even(const F28& a) {
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) r.l[i] = dpp<kEven>(a.l[i]);
  return r;
}
__device__ __forceinline__ F28 odd(const F28& a) {
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) r.l[i] = dpp<kOdd>(a.l[i]);
  return r;
}
// s_h: lane 0 gets K - b1 from its partner, lane 1 gets b0
template <const uint32_t (&K)[kN]>
__device__ __forceinline__ F28 partner_s(const F28& b, bool h) {
  const F28 nb = ksub(K, b);
  F28 s;
#pragma unroll
  for (int i = 0; i < kN; ++i) s.l[i] = dpp<kSwap>(h ? nb.l[i] : b.l[i]);
  return s;
}
// this lane's component of a b (+ e): one two-product reduction
template <const uint32_t (&K)[kN]>
__device__ __forceinline__ F28 pmul(const F28& a, const F28& b, bool h) {
  return mul2_add(even(a), b, odd(a), partner_s<K>(b, h));
}
template <const uint32_t (&K)[kN]>
__device__ __forceinline__ F28 pmul_add(const F28& a, const F28& b, const F28& e, bool h) {
#if defined(__HIP_DEVICE_COMPILE__)
  return asm28::mul2_add(even(a), b, odd(a), partner_s<K>(b, h), e);
#else
  return redc<true, true>(even(a), b, odd(a), partner_s<K>(b, h), e);
#endif
}
// this lane's component of a^2 (+ e): lane 0 (a0 + a1)(a0 + K - a1), lane 1 a0 (2 a1)
template <const uint32_t (&K)[kN]>
__device__ __forceinline__ F28 psqr_operands(const F28& a, bool h, F28* y) {
  const F28 a0 = even(a), a1 = odd(a);
  F28 x;
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    x.l[i] = h ? a0.l[i] : a0.l[i] + a1.l[i];
    y->l[i] = h ? (a1.l[i] << 1) : a0.l[i] + (K[i] - a1.l[i]);
  }
  return x;
}
template <const uint32_t (&K)[kN]>
__device__ __forceinline__ F28 psqr(const F28& a, bool h) {
  F28 y;
  const F28 x = psqr_operands<K>(a, h, &y);
  return mul(x, y);
}
template <const uint32_t (&K)[kN]>
__device__ __forceinline__ F28 psqr_add(const F28& a, const F28& e, bool h) {
  F28 y;
  const F28 x = psqr_operands<K>(a, h, &y);
  return mul_add(x, y, e);
}
// zero of the whole Fq2 value (both lanes agree)
__device__ __forceinline__ bool pzero(const F28& a) {
  const uint32_t z = is_zero_mod_p(a) ? 1u : 0u;
  return (z & dpp<kSwap>(z)) != 0;
}

struct Acc {
  F28 x, y, zz, zzz;
};

// the first point of a run (lane h: its components; (1, 0) for Z)
__device__ __forceinline__ Acc from_shifted(const F28& x2, const F28& y2, bool h) {
  const F28 one = h ? F28{} : konst(kOne28);
  return {reduce(x2), reduce(y2), one, one};
}

// madd-2008-s (point_xyzz_impl.h:129-176); *special as acc28::madd
__device__ __forceinline__ Acc madd(const Acc& A, const F28& x2, const F28& y2, bool h, int* special) {
  const F28 P = pmul_add<kK4>(x2, A.zz, ksub(kK16, A.x), h);
  const F28 R = pmul_add<kK4>(y2, A.zzz, ksub(kK8, A.y), h);
  if (pzero(P)) {
    *special = pzero(R) ? 2 : 1;
    return A;
  }
  const F28 PP = psqr<kK32>(P, h);
  const F28 PPP = pmul<kK4>(P, PP, h);
  const F28 Q = pmul<kK4>(A.x, PP, h);
  const F28 W = pmul<kK4>(A.y, PPP, h);
  Acc C;
  C.x = psqr_add<kK16>(R, ksub2(kK8, PPP, Q), h);
  const F28 T = add_ksub(Q, kK16, C.x);
  C.y = pmul_add<kK32r3>(R, T, ksub(kK4, W), h);
  C.zz = pmul<kK4>(A.zz, PP, h);
  C.zzz = pmul<kK4>(A.zzz, PPP, h);
  return C;
}

// dbl-2008-s-1 (a = 0; point_xyzz_impl.h:199-236), the rare P = acc case
// (performance does not matter; the limb-wise multiples are normalized first):
//   U = 2Y < 12   V = U^2 < 1.2   W = U V < 1.03   S = X V < 1.03
//   M = X (3X) < 1.25             X3 = M^2 + (8p - 2S) < 9.01
//   Y3 = M (S + 16p - X3) + (4p - W Y) < 5.1     ZZ3, ZZZ3 < 1.01
__device__ __forceinline__ Acc dbl(const Acc& A, bool h) {
  const F28 U = normalize(times(A.y, 2));
  const F28 V = psqr<kK16>(U, h);
  const F28 W = pmul<kK4>(U, V, h);
  const F28 S = pmul<kK4>(A.x, V, h);
  const F28 M = pmul<kK32>(A.x, normalize(times(A.x, 3)), h);
  const F28 WY = pmul<kK8>(W, A.y, h);
  F28 zero{};
  Acc C;
  C.x = psqr_add<kK4>(M, ksub2(kK8, zero, S), h);
  C.y = pmul_add<kK32r3>(M, add_ksub(S, kK16, C.x), ksub(kK4, WY), h);
  C.zz = pmul<kK4>(V, A.zz, h);
  C.zzz = pmul<kK4>(W, A.zzz, h);
  return C;
}

// add-2008-s (point_xyzz_impl.h:45-97) for the G2 reductions, both operands
// not the identity (the caller keeps identity flags); inputs and outputs
// X < 10p, Y < 6p, ZZ, ZZZ < 3p (from32 loads give < 3p); *special as madd's
// (tests/test_pair28_model.py point_add)
__device__ __forceinline__ Acc add(const Acc& A, const Acc& B, bool h, int* special) {
  // ZZ1 ZZ2 and ZZZ1 ZZZ2 first: the operands' Z coordinates die early (register pressure)
  const F28 U1 = pmul<kK4>(A.x, B.zz, h), S1 = pmul<kK4>(A.y, B.zzz, h);
  const F28 ZZ12 = pmul<kK4>(A.zz, B.zz, h), ZZZ12 = pmul<kK4>(A.zzz, B.zzz, h);
  const F28 P = pmul_add<kK4>(B.x, A.zz, ksub(kK4, U1), h);
  const F28 R = pmul_add<kK4>(B.y, A.zzz, ksub(kK4, S1), h);
  if (pzero(P)) {
    *special = pzero(R) ? 2 : 1;
    return A;
  }
  const F28 PP = psqr<kK16>(P, h);
  const F28 PPP = pmul<kK4>(P, PP, h);
  const F28 Q = pmul<kK4>(U1, PP, h);
  const F28 W = pmul<kK4>(S1, PPP, h);
  Acc C;
  C.x = psqr_add<kK16>(R, ksub2(kK8, PPP, Q), h);
  const F28 T = add_ksub(Q, kK16, C.x);
  C.y = pmul_add<kK32r3>(R, T, ksub(kK4, W), h);
  C.zz = pmul<kK4>(ZZ12, PP, h);
  C.zzz = pmul<kK4>(ZZZ12, PPP, h);
  return C;
}

}  // namespace tachyon_amd::msm::pair28
