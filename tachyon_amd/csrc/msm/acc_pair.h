// G2 bucket accumulation with a LANE PAIR per point: lane 2v holds the c0
// and lane 2v + 1 the c1 component of every Fq2 value of virtual thread v.
//
// Why: an Fq2 XYZZ accumulator, the gathered point and the madd's temporaries
// are ~10 Fq2 values -- 240 VGPRs for BLS12-381 (12-limb Fq), 160 for BN254 --
// so the one-lane-per-point kernels run at a 2-wave cap, and BLS12-381's Fq
// products are out-of-line calls whose argument marshalling and register
// saves cost ~1,250 moves and ~550 B of scratch writes per addition
// (profiles/r03a: 36.8 GB of WRITE_SIZE per 2^22 accumulation).  Split by
// component, a lane holds one Fq per value; additions and subtractions are
// component-wise, and a product needs the partner's components, fetched with
// one DPP quad_perm per word:
//   (a0 + a1 u)(b0 + b1 u) = (a0 b0 - a1 b1) + (a0 b1 + a1 b0) u   (u^2 = -1)
//   lane h: a0 * b_h + a1 * s_h,  s_0 = -b1, s_1 = b0
// -- one fused two-product Montgomery reduction per lane (mul_add_inline),
// the same multiply count as the Karatsuba product on one lane (3 N^2 per
// lane pair... 2 x 3N^2 / 2), with no calls and every value in registers.
//   a^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u: lane h multiplies X_h Y_h with
// X_0 = a0 + a1, Y_0 = a0 - a1, X_1 = a0, Y_1 = 2 a1 (one plain product).
// Both lanes of a pair follow the same entries, so every branch is
// pair-uniform; zero tests AND the two lanes' results.
#pragma once
#include "msm.h"

namespace tachyon_amd::msm::pair {

// DPP quad_perm controls: [1,0,3,2] swap partners, [0,0,2,2] even lane's
// value to both, [1,1,3,3] odd lane's value to both
constexpr int kSwap = 0xB1, kEven = 0xA0, kOdd = 0xF5;

template <int kCtrl>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, kCtrl, 0xF, 0xF, false);
}

// The lane's component of a b (a0 b_h + a1 s_h) and of a^2, given its own
// components; the partner's come in by DPP.  Inline for 8-limb fields; for
// 12-limb fields an out-of-line call with the operands as 24 register
// arguments (the ~900-instruction fused product inlined ~10 times per madd
// would overflow the instruction cache), result in 12 registers.
template <class F>
__device__ __forceinline__ F perm_even(const F& a) {
  F r;
#pragma unroll
  for (int i = 0; i < F::N; ++i) r.v[i] = dpp<kEven>(a.v[i]);
  return r;
}
template <class F>
__device__ __forceinline__ F perm_odd(const F& a) {
  F r;
#pragma unroll
  for (int i = 0; i < F::N; ++i) r.v[i] = dpp<kOdd>(a.v[i]);
  return r;
}
template <class F>
__device__ __forceinline__ F pair_mul(const F& a, const F& b, bool h) {
  const F a0 = perm_even(a), a1 = perm_odd(a);
  // the partner's b with the sign this lane needs: lane 1 offers -b1 to
  // lane 0 (a lazy 2p - b1), lane 0 offers b0 to lane 1
  const F nb = -b;
  F s;
#pragma unroll
  for (int i = 0; i < F::N; ++i) s.v[i] = dpp<kSwap>(h ? nb.v[i] : b.v[i]);
  return a0.mul_add_inline(b, a1, s);
}
template <class F>
__device__ __forceinline__ F pair_sqr(const F& a, bool h) {
  const F a0 = perm_even(a), a1 = perm_odd(a);
  const F s = a0 + a1, d = a0 - a1, t = a1.dbl();
  F x, y;
#pragma unroll
  for (int i = 0; i < F::N; ++i) {
    x.v[i] = h ? a0.v[i] : s.v[i];
    y.v[i] = h ? t.v[i] : d.v[i];
  }
  return x.mul_inline(y);
}
template <class F>
__device__ __noinline__ F pair_mul_regs(TA_LIMBS12(a), TA_LIMBS12(b), uint32_t h) {
  const F x{TA_UNPACK12(a)}, y{TA_UNPACK12(b)};
  return pair_mul(x, y, h != 0);
}
template <class F>
__device__ __noinline__ F pair_sqr_regs(TA_LIMBS12(a), uint32_t h) {
  const F x{TA_UNPACK12(a)};
  return pair_sqr(x, h != 0);
}

template <class F, bool kCall = (F::N == 12)>
struct Half {  // this lane's component of an Fq2 value (kCall: 12-limb products out of line)
  F v;
  __device__ __forceinline__ Half operator+(const Half& o) const { return {v + o.v}; }
  __device__ __forceinline__ Half operator-(const Half& o) const { return {v - o.v}; }
  __device__ __forceinline__ Half dbl() const { return {v.dbl()}; }
  __device__ __forceinline__ Half mul(const Half& b, bool h) const {
    if constexpr (kCall) return {pair_mul_regs<F>(TA_PASS12(v), TA_PASS12(b.v), h ? 1u : 0u)};
    else return {pair_mul(v, b.v, h)};
  }
  __device__ __forceinline__ Half sqr(bool h) const {
    if constexpr (kCall) return {pair_sqr_regs<F>(TA_PASS12(v), h ? 1u : 0u)};
    else return {pair_sqr(v, h)};
  }
  // zero of the whole Fq2 value (both lanes agree)
  __device__ __forceinline__ bool is_zero() const {
    const uint32_t z = v.is_zero() ? 1u : 0u;
    return (z & dpp<kSwap>(z)) != 0;
  }
};

template <class H>
struct Acc {
  H x, y, zz, zzz;
};

// madd-2008-s (point_xyzz_impl.h:129-176) on lane-pair Fq2 values, with the
// identity accumulator kept as a flag by the caller.  *special: 1 = the sum is
// the identity (P = -acc), 2 = P = acc (the caller doubles); acc unchanged then.
template <class H>
__device__ __forceinline__ Acc<H> madd(const Acc<H>& A, const H& x2, const H& y2, bool h, int* special) {
  const H p = x2.mul(A.zz, h) - A.x;
  const H r = y2.mul(A.zzz, h) - A.y;
  if (p.is_zero()) {
    *special = r.is_zero() ? 2 : 1;
    return A;
  }
  const H pp = p.sqr(h);
  const H ppp = p.mul(pp, h);
  const H q = A.x.mul(pp, h);
  Acc<H> c;
  c.x = r.sqr(h) - ppp - q.dbl();
  c.y = r.mul(q - c.x, h) - A.y.mul(ppp, h);
  c.zz = A.zz.mul(pp, h);
  c.zzz = A.zzz.mul(ppp, h);
  return c;
}

// dbl-2008-s-1 (a = 0; point_xyzz_impl.h:199-236): the P = acc case.  Inline
// (an out-of-line call taking the accumulator's address would keep it in
// scratch for the whole loop); its 12-limb products are calls anyway.
template <class H>
__device__ __forceinline__ Acc<H> dbl(const Acc<H>& A, bool h) {
  const H u = A.y.dbl();
  const H v = u.sqr(h);
  const H w = u.mul(v, h);
  const H s = A.x.mul(v, h);
  H m = A.x.sqr(h);
  m = m + m.dbl();
  Acc<H> c;
  c.x = m.sqr(h) - s.dbl();
  c.y = m.mul(s - c.x, h) - w.mul(A.y, h);
  c.zz = v.mul(A.zz, h);
  c.zzz = w.mul(A.zzz, h);
  return c;
}

// The identity (1, 1, 0, 0): this lane's components (Fq2 one = 1 + 0 u)
template <class H>
__device__ __forceinline__ Acc<H> zero(bool h) {
  using F = decltype(H{}.v);
  const H one{h ? F::zero() : F::one()}, nil{F::zero()};
  return {one, one, nil, nil};
}

// add-2008-s (point_xyzz_impl.h:45-97) on lane-pair values, identities
// (zz = 0) handled: the bucket / window reduction's point sum
template <class H>
__device__ __forceinline__ Acc<H> add(const Acc<H>& A, const Acc<H>& B, bool h) {
  if (A.zz.is_zero()) return B;
  if (B.zz.is_zero()) return A;
  const H u1 = A.x.mul(B.zz, h), s1 = A.y.mul(B.zzz, h);
  const H p = B.x.mul(A.zz, h) - u1;
  const H r = B.y.mul(A.zzz, h) - s1;
  if (p.is_zero()) return r.is_zero() ? dbl(A, h) : zero<H>(h);
  const H pp = p.sqr(h);
  const H ppp = p.mul(pp, h);
  const H q = u1.mul(pp, h);
  Acc<H> c;
  c.x = r.sqr(h) - ppp - q.dbl();
  c.y = r.mul(q - c.x, h) - s1.mul(ppp, h);
  c.zz = A.zz.mul(B.zz, h).mul(pp, h);
  c.zzz = A.zzz.mul(B.zzz, h).mul(ppp, h);
  return c;
}

// m P for a small m (double-and-add from the top bit)
template <class H>
__device__ __forceinline__ Acc<H> small_mul(const Acc<H>& P, uint32_t m, bool h) {
  if (m == 0 || P.zz.is_zero()) return zero<H>(h);
  Acc<H> r = P;
  for (int bit = 30 - __builtin_clz(m); bit >= 0; --bit) {
    r = dbl(r, h);
    if ((m >> bit) & 1) r = add(r, P, h);
  }
  return r;
}

// point i of an XYZZ<Fq2> array: this lane's components (x0 x1 y0 y1 zz0 ...)
template <class H, class Fb>
__device__ __forceinline__ Acc<H> load(const Fb* pts, size_t i, uint32_t h) {
  const Fb* o = pts + 8 * i;
  return {H{o[h]}, H{o[2 + h]}, H{o[4 + h]}, H{o[6 + h]}};
}
template <class H, class Fb>
__device__ __forceinline__ void store(Fb* pts, size_t i, uint32_t h, const Acc<H>& a) {
  Fb* o = pts + 8 * i;
  o[h] = a.x.v;
  o[2 + h] = a.y.v;
  o[4 + h] = a.zz.v;
  o[6 + h] = a.zzz.v;
}

}  // namespace tachyon_amd::msm::pair
