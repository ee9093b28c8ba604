// BN254 Fq in 9 x 29-bit limbs: the carry-free Montgomery product of the
// G1 bucket accumulation (seg_acc_kernel, MSM).
//
// Why: with 32-bit limbs every v_mad_u64_u32 of a product column can carry out
// of the 64-bit accumulator, so each one needs a v_addc_co_u32 to collect it
// (128 of the 256 VALU instructions of an 8-limb product, mont_asm.h).  With
// 29-bit limbs a product is < 2^58 and a whole column -- at most 9 a_i b_j,
// 9 m_i p_j and the carry -- stays below 2^64: no carries to collect; the
// column ends with a shift and a mask.  The price is 9 x 9 instead of 8 x 8
// limb products, paid back by the carry adds and by additions that need no
// carry propagation at all (limb-wise, the limbs have 3 bits of headroom).
//
// Representation: x is held as any x' = x * 2^261 (mod p) (Montgomery with
// R' = 2^261 = 2^(29 * 9)), value = sum_i l_i 2^(29 i).  "N-form" (every
// product's output): limbs 0..7 < 2^29, limb 8 the rest.  A product's inputs
// may have wider limbs as long as every column stays below 2^64 (the bounds
// are derived at each use in msm_impl.h, seg_acc29 / madd29).
//
// Conversions to the 8 x 32-bit R = 2^256 form of the rest of the library:
//   in : x' = x~ << 5 repacked (x~ the R-form value: x~ 2^5 = x 2^261), then
//        one product by 1' to bring the value below 2p (from32);
//   out: mont29(x', 2^256) = x 2^256 (R form), < 2p, repacked (to32).
// Constants: tools/gen_f29_constants.py.
#pragma once
#include <cstdint>

#ifndef TA_HD
#if defined(__HIPCC__)
#define TA_HD __host__ __device__ __forceinline__
#else
#define TA_HD inline
#endif
#endif

namespace tachyon_amd::f29 {

constexpr uint32_t kM29 = (1u << 29) - 1;
// p
constexpr uint32_t kP29[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                              0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
constexpr uint32_t kPinv29 = 0x04866389u;  // -p^-1 mod 2^29
constexpr uint32_t kPinv32 = 0x1b799c77u;  // p^-1 mod 2^32 (zero test)
// 4p, low limbs raised by 2^29 (>= 2^29 - 1)
constexpr uint32_t kK4[9] = {0x21f3f51cu, 0x241182dau, 0x31ca8d3bu, 0x2b548b42u, 0x361765dfu,
                             0x2b6d0301u, 0x229b8503u, 0x397098cfu, 0x00c19138u};
// 8p, low limbs raised by 2^31 (>= 2^31 - 4)
constexpr uint32_t kK8[9] = {0x83e7ea38u, 0x882305b2u, 0x83951a74u, 0x96a91683u, 0x8c2ecbbcu,
                             0x96da0601u, 0x85370a04u, 0x92e1319cu, 0x0183226fu};
// 16p, low limbs raised by 2^29
constexpr uint32_t kK16[9] = {0x27cfd470u, 0x30460b6bu, 0x272a34efu, 0x2d522d0du, 0x385d9780u,
                              0x2db40c09u, 0x2a6e1410u, 0x25c2633fu, 0x030644e6u};
// 33p, low limbs raised by 2^29 (minus a normalized value < 32p: msm/pair29.h)
constexpr uint32_t kK33[9] = {0x281ca627u, 0x2190778eu, 0x2ac70d2fu, 0x3d797cecu, 0x26410879u,
                              0x3e4358d5u, 0x35830962u, 0x39e0ecb3u, 0x063cee1bu};
// 32p, low limbs raised by 3 2^29 (the lane-pair G2 products negate T = Q + 16p - X3,
// limbs < 3 2^29 - 2, msm/pair29.h)
constexpr uint32_t kK32r3[9] = {0x6f9fa8e0u, 0x608c16d5u, 0x6e5469deu, 0x7aa45a19u, 0x70bb2effu,
                                0x7b681812u, 0x74dc281fu, 0x6b84c67du, 0x060c89cbu};
// 1 in R' form (2^261 mod p)
constexpr uint32_t kOne29[9] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u,
                                0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};

struct F29 {
  uint32_t l[9];
};

TA_HD F29 konst(const uint32_t (&k)[9]) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = k[i];
  return r;
}

// REDC(a b [+ c d]) [+ e]: one Montgomery reduction by 2^261 of the column
// sums of a b (and c d), the addend e added into the output columns.  FIPS:
// the digit m_k = (column mod 2^29) (-p^-1) mod 2^29 is folded in as column k
// ends, so columns 0..8 end divisible by 2^29 and columns 9..16 are the
// output limbs 0..7; limb 8 is what is left.  Output: N-form, value
// < (A B [+ C D]) / 2^261 + p [+ E].
template <bool kPair, bool kAdd>
TA_HD F29 redc(const F29& a, const F29& b, const F29& c, const F29& d, const F29& e) {
  uint64_t acc = 0;
  uint32_t m[9];
  F29 r;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
      if (k - i >= 0 && k - i < 9) acc += (uint64_t)a.l[i] * b.l[k - i];
    if constexpr (kPair) {
#pragma unroll
      for (int i = 0; i < 9; ++i)
        if (k - i >= 0 && k - i < 9) acc += (uint64_t)c.l[i] * d.l[k - i];
    }
#pragma unroll
    for (int i = 0; i < 9; ++i)
      if (i < k && k - i < 9) acc += (uint64_t)m[i] * kP29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * kPinv29) & kM29;
      acc += (uint64_t)m[k] * kP29[0];
    } else {
      if constexpr (kAdd) acc += e.l[k - 9];
      r.l[k - 9] = (uint32_t)acc & kM29;
    }
    acc >>= 29;
  }
  if constexpr (kAdd) acc += e.l[8];
  r.l[8] = (uint32_t)acc;
  return r;
}

// a^2 [+ e]: the cross products once through the doubled limbs
template <bool kAdd>
TA_HD F29 sqr_redc(const F29& a, const F29& e) {
  uint64_t acc = 0;
  uint32_t m[9], d[9];
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = a.l[i] << 1;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
      if (k - i > i && k - i < 9) acc += (uint64_t)a.l[i] * d[k - i];
    if ((k & 1) == 0 && k / 2 < 9) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = 0; i < 9; ++i)
      if (i < k && k - i < 9) acc += (uint64_t)m[i] * kP29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * kPinv29) & kM29;
      acc += (uint64_t)m[k] * kP29[0];
    } else {
      if constexpr (kAdd) acc += e.l[k - 9];
      r.l[k - 9] = (uint32_t)acc & kM29;
    }
    acc >>= 29;
  }
  if constexpr (kAdd) acc += e.l[8];
  r.l[8] = (uint32_t)acc;
  return r;
}

}  // namespace tachyon_amd::f29
#include "f29_asm.h"  // device: the same columns as hand-chained v_mad_u64_u32 (tools/gen_f29_asm.py)
namespace tachyon_amd::f29 {

// mul2_add(a, b, c, d) = REDC(a b + c d); mul_add / sqr_add add e to the output
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TA_F29_CXX)
TA_HD F29 mul(const F29& a, const F29& b) { return asm29::mul(a, b); }
TA_HD F29 mul_add(const F29& a, const F29& b, const F29& e) { return asm29::mul_add(a, b, e); }
TA_HD F29 mul2_add(const F29& a, const F29& b, const F29& c, const F29& d) { return asm29::mul2(a, b, c, d); }
TA_HD F29 sqr(const F29& a) { return asm29::sqr(a); }
TA_HD F29 sqr_add(const F29& a, const F29& e) { return asm29::sqr_add(a, e); }
#else
TA_HD F29 mul(const F29& a, const F29& b) { return redc<false, false>(a, b, a, b, a); }
TA_HD F29 mul_add(const F29& a, const F29& b, const F29& e) { return redc<false, true>(a, b, a, b, e); }
TA_HD F29 mul2_add(const F29& a, const F29& b, const F29& c, const F29& d) { return redc<true, false>(a, b, c, d, a); }
TA_HD F29 sqr(const F29& a) { return sqr_redc<false>(a, a); }
TA_HD F29 sqr_add(const F29& a, const F29& e) { return sqr_redc<true>(a, e); }
#endif

// limb-wise (no carries): K - x, K + a - x, K - a - b (K a raised multiple of p
// whose limbs are at least the subtrahends' limbs)
TA_HD F29 ksub(const uint32_t (&k)[9], const F29& x) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = k[i] - x.l[i];
  return r;
}
TA_HD F29 add_ksub(const F29& a, const uint32_t (&k)[9], const F29& x) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = a.l[i] + (k[i] - x.l[i]);
  return r;
}
// k a limb-wise (a small k: k times the limb bound)
TA_HD F29 times(const F29& a, uint32_t k) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = a.l[i] * k;
  return r;
}
TA_HD F29 ksub2(const uint32_t (&k)[9], const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = k[i] - a.l[i] - (b.l[i] << 1);
  return r;
}

// carries propagated: limbs 0..7 < 2^29 (a limb-wise sum of small multiples)
TA_HD F29 normalize(const F29& a) {
  F29 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t t = a.l[i] + c;
    r.l[i] = t & kM29;
    c = t >> 29;
  }
  r.l[8] = a.l[8] + c;
  return r;
}

// x' = x~ << 5 as 29-bit limbs, from the 8 x 32-bit R-form words w (x~ < 2^254
// or lazy < 2p: the shifted value has < 261 bits, limbs exact)
TA_HD F29 shl5_repack(const uint32_t* w) {
  F29 r;
  r.l[0] = (w[0] << 5) & kM29;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    const int bit = 29 * i - 5;  // first bit of limb i in x~
    const int word = bit >> 5, sh = bit & 31;
    const uint32_t lo = w[word];
    const uint32_t hi = word + 1 < 8 ? w[word + 1] : 0u;
    const uint32_t v = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
    r.l[i] = i < 8 ? (v & kM29) : v;
  }
  return r;
}

// bits kOff .. kOff + 255 of a limb-exact value (limbs 0..7 < 2^29) -> 8 x 32-bit words
template <int kOff = 0>
TA_HD void repack32(const F29& x, uint32_t* w) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int bit = 32 * j + kOff;
    const int i = bit / 29, sh = bit % 29;
    uint64_t v = (uint64_t)(x.l[i] >> sh);
    int got = 29 - sh;
    if (i + 1 < 9) v |= (uint64_t)x.l[i + 1] << got;
    got += 29;
    if (got < 32 && i + 2 < 9) v |= (uint64_t)x.l[i + 2] << got;
    w[j] = (uint32_t)v;
  }
}

// R-form words (x~ < 2^255) -> R' form x' = x~ 2^5 - q p, value < 3p: no
// product, the quotient estimated from the top two limbs.  With v = x~ << 5
// and v_hi = v >> 203, v_hi / (p_hi + 1) <= v / p < v_hi / (p_hi + 1) + 2^-40,
// so the float estimate (relative error < 2^-21, times q < 64) minus one is
// q* - 2 .. q*, q* = floor(v / p): 0 <= v - q p < 3p.
constexpr float kInvPhi = 1.0f / 1702635872462389.0f;  // 1 / (p >> 203 + 1)
TA_HD F29 reduce_shl5(const F29& v) {
  const float vf = (float)v.l[8] * 536870912.0f + (float)v.l[7];
  int q = (int)(vf * kInvPhi) - 1;
  q = q < 0 ? 0 : q;
  F29 r;
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int64_t t = (int64_t)(-q) * (int64_t)(int32_t)kP29[i] + ((int64_t)v.l[i] + carry);  // v_mad_i64_i32
    r.l[i] = i < 8 ? (uint32_t)t & kM29 : (uint32_t)t;
    carry = t >> 29;  // arithmetic: the borrow
  }
  return r;
}
TA_HD F29 from32(const uint32_t* w) { return reduce_shl5(shl5_repack(w)); }
// R' form (N-form, value < 16p) -> R-form words, value < 2p: x' 2^-5 =
// (x' + k p) / 32 with k = -x' p^-1 mod 32 (p = 7 mod 32, -7^-1 = 9 mod 32):
// < (16 + 31) p / 32.  One digit of a Montgomery reduction by 2^5.
TA_HD void to32(const F29& x, uint32_t* w) {
  const uint32_t k = (x.l[0] * 9u) & 31u;
  F29 v;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t t = (uint64_t)x.l[i] + (uint64_t)k * kP29[i] + carry;
    v.l[i] = i < 8 ? (uint32_t)t & kM29 : (uint32_t)t;
    carry = t >> 29;
  }
  repack32<5>(v, w);
}

// x = 0 (mod p) for an N-form x < 64p: x = k p exactly for some k < 64, so
// (x mod 2^32) p^-1 mod 2^32 = k -- a one-multiply filter; the full limb
// compare runs only when it passes (a true zero, or 64 in 2^32 others).
TA_HD bool is_zero_mod_p(const F29& x) {
  const uint32_t lo = x.l[0] | (x.l[1] << 29);
  const uint32_t k = lo * kPinv32;
  if (k >= 64) return false;
  uint64_t carry = 0;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {  // k p in N-form limbs, compared with x
    const uint64_t t = (uint64_t)k * kP29[i] + carry;
    const uint32_t limb = i < 8 ? (uint32_t)t & kM29 : (uint32_t)t;
    carry = i < 8 ? t >> 29 : 0;
    diff |= limb ^ x.l[i];
  }
  return diff == 0;
}

}  // namespace tachyon_amd::f29
