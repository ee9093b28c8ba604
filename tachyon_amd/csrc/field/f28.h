// BLS12-381 Fq in 14 x 28-bit limbs: the carry-free Montgomery product of the
// BLS12-381 G1 bucket accumulation (msm/acc28.h, seg_acc28_kernel) -- the
// BN254 29-bit field (f29.h) carried to the 381-bit modulus.
//
// Why: the 12 x 32-bit FIPS product issues 144 + 144 v_mad_u64_u32, 288
// v_addc_co_u32 carry collections, 12 digits and ~30 moves (~620 VALU); with
// 28-bit limbs a column of at most 14 a_i b_j, 14 m_i p_j (and 14 c_i d_j for
// a two-product reduction) and the carry stays below 2^62 -- no carry words,
// the column ends with a digit, a mask and a 64-bit shift: 392 mads + ~70
// others (~460).  R'' / p = 2^11.3: the representation has 2520 multiples of p
// of headroom, so sums and differences need no reduction between products.
//
// Representation: x is held as any x'' = x 2^392 (mod p), value = sum_i l_i
// 2^(28 i).  "N-form" (every product's output): limbs 0..12 < 2^28, limb 13
// the rest.  Conversions to the 12 x 32-bit R = 2^384 form of the library:
//   in : x'' = x~ << 8 repacked (x~ the R-form value), then a quotient
//        estimate brings it below 3p (from32);
//   out: (x'' + k p) / 2^8 with k = -x'' p^-1 mod 2^8 (one 8-bit Montgomery
//        digit), < 2p for x'' < 16p, repacked (to32).
// Constants and device asm: tools/gen_f28.py.
#pragma once
#include <cstdint>

#ifndef TA_HD
#if defined(__HIPCC__)
#define TA_HD __host__ __device__ __forceinline__
#else
#define TA_HD inline
#endif
#endif

#include "f28_asm.h"

namespace tachyon_amd::f28 {

constexpr int kN = 14;

TA_HD F28 konst(const uint32_t (&k)[kN]) {
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) r.l[i] = k[i];
  return r;
}

// REDC(a b [+ c d]) [+ e] by 2^392, FIPS columns (the host reference of the
// generated device products): output N-form, < (A B [+ C D]) / 2^392 + p [+ E]
template <bool kPair, bool kAdd>
TA_HD F28 redc(const F28& a, const F28& b, const F28& c, const F28& d, const F28& e) {
  uint64_t acc = 0;
  uint32_t m[kN];
  F28 r;
#pragma unroll
  for (int k = 0; k < 2 * kN - 1; ++k) {
#pragma unroll
    for (int i = 0; i < kN; ++i)
      if (k - i >= 0 && k - i < kN) acc += (uint64_t)a.l[i] * b.l[k - i];
    if constexpr (kPair) {
#pragma unroll
      for (int i = 0; i < kN; ++i)
        if (k - i >= 0 && k - i < kN) acc += (uint64_t)c.l[i] * d.l[k - i];
    }
#pragma unroll
    for (int i = 0; i < kN; ++i)
      if (i < k && k - i < kN) acc += (uint64_t)m[i] * kP28[k - i];
    if (k < kN) {
      m[k] = ((uint32_t)acc * kPinv28) & kM28;
      acc += (uint64_t)m[k] * kP28[0];
    } else {
      if constexpr (kAdd) acc += e.l[k - kN];
      r.l[k - kN] = (uint32_t)acc & kM28;
    }
    acc >>= 28;
  }
  if constexpr (kAdd) acc += e.l[kN - 1];
  r.l[kN - 1] = (uint32_t)acc;
  return r;
}
template <bool kAdd>
TA_HD F28 sqr_redc(const F28& a, const F28& e) {
  uint64_t acc = 0;
  uint32_t m[kN], d[kN];
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) d[i] = a.l[i] << 1;
#pragma unroll
  for (int k = 0; k < 2 * kN - 1; ++k) {
#pragma unroll
    for (int i = 0; i < kN; ++i)
      if (k - i > i && k - i < kN) acc += (uint64_t)a.l[i] * d[k - i];
    if ((k & 1) == 0 && k / 2 < kN) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = 0; i < kN; ++i)
      if (i < k && k - i < kN) acc += (uint64_t)m[i] * kP28[k - i];
    if (k < kN) {
      m[k] = ((uint32_t)acc * kPinv28) & kM28;
      acc += (uint64_t)m[k] * kP28[0];
    } else {
      if constexpr (kAdd) acc += e.l[k - kN];
      r.l[k - kN] = (uint32_t)acc & kM28;
    }
    acc >>= 28;
  }
  if constexpr (kAdd) acc += e.l[kN - 1];
  r.l[kN - 1] = (uint32_t)acc;
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
TA_HD F28 mul(const F28& a, const F28& b) { return asm28::mul(a, b); }
TA_HD F28 mul_add(const F28& a, const F28& b, const F28& e) { return asm28::mul_add(a, b, e); }
TA_HD F28 mul2_add(const F28& a, const F28& b, const F28& c, const F28& d) { return asm28::mul2(a, b, c, d); }
TA_HD F28 sqr(const F28& a) { return asm28::sqr(a); }
TA_HD F28 sqr_add(const F28& a, const F28& e) { return asm28::sqr_add(a, e); }
#else
TA_HD F28 mul(const F28& a, const F28& b) { return redc<false, false>(a, b, a, b, a); }
TA_HD F28 mul_add(const F28& a, const F28& b, const F28& e) { return redc<false, true>(a, b, a, b, e); }
TA_HD F28 mul2_add(const F28& a, const F28& b, const F28& c, const F28& d) { return redc<true, false>(a, b, c, d, a); }
TA_HD F28 sqr(const F28& a) { return sqr_redc<false>(a, a); }
TA_HD F28 sqr_add(const F28& a, const F28& e) { return sqr_redc<true>(a, e); }
#endif

// limb-wise (no carries): K - x, a + (K - x), K - a - 2b
TA_HD F28 ksub(const uint32_t (&k)[kN], const F28& x) {
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) r.l[i] = k[i] - x.l[i];
  return r;
}
TA_HD F28 add_ksub(const F28& a, const uint32_t (&k)[kN], const F28& x) {
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) r.l[i] = a.l[i] + (k[i] - x.l[i]);
  return r;
}
TA_HD F28 times(const F28& a, uint32_t k) {
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) r.l[i] = a.l[i] * k;
  return r;
}
TA_HD F28 ksub2(const uint32_t (&k)[kN], const F28& a, const F28& b) {
  F28 r;
#pragma unroll
  for (int i = 0; i < kN; ++i) r.l[i] = k[i] - a.l[i] - (b.l[i] << 1);
  return r;
}

// carry propagation: limbs 0..12 < 2^28, the value unchanged (for limb-wise
// sums whose limbs would overflow a product's columns)
TA_HD F28 normalize(const F28& a) {
  F28 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < kN - 1; ++i) {
    const uint32_t t = a.l[i] + c;
    r.l[i] = t & kM28;
    c = t >> 28;
  }
  r.l[kN - 1] = a.l[kN - 1] + c;
  return r;
}

// x'' = x~ << 8 as 28-bit limbs, from the 12 x 32-bit R-form words w (x~ <
// 2^384 - 2^? : lazy < 2p < 2^382, so the shifted value has < 390 bits)
TA_HD F28 shl8_repack(const uint32_t* w) {
  F28 r;
  r.l[0] = (w[0] << 8) & kM28;
#pragma unroll
  for (int i = 1; i < kN; ++i) {
    const int bit = 28 * i - 8;  // first bit of limb i in x~
    const int word = bit >> 5, sh = bit & 31;
    const uint32_t lo = w[word];
    const uint32_t hi = word + 1 < 12 ? w[word + 1] : 0u;
    const uint32_t v = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
    r.l[i] = i < kN - 1 ? (v & kM28) : v;
  }
  return r;
}

// value - q p, q = floor(v / p) - 0..2 from the top two limbs in float
// (v_hi = l13 2^28 + l12, p_hi = p >> 336 ~ 2^44.7): N-form, < 3p, for
// N-form inputs below 2^400.  Signed carries (v_mad_i64_i32 chains).
TA_HD F28 reduce(const F28& v) {
  const float vf = (float)v.l[kN - 1] * 268435456.0f + (float)v.l[kN - 2];
  int q = (int)(vf * kInvPhi) - 1;
  q = q < 0 ? 0 : q;
  F28 r;
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    const int64_t t = (int64_t)(-q) * (int64_t)(int32_t)kP28[i] + ((int64_t)v.l[i] + carry);
    r.l[i] = i < kN - 1 ? (uint32_t)t & kM28 : (uint32_t)t;
    carry = t >> 28;
  }
  return r;
}
TA_HD F28 from32(const uint32_t* w) { return reduce(shl8_repack(w)); }

// bits kOff .. kOff + 383 of a limb-exact value (limbs 0..12 < 2^28) -> 12 words
template <int kOff = 0>
TA_HD void repack32(const F28& x, uint32_t* w) {
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    const int bit = 32 * j + kOff;
    const int i = bit / 28, sh = bit % 28;
    uint64_t v = (uint64_t)(x.l[i] >> sh);
    int got = 28 - sh;
    if (i + 1 < kN) v |= (uint64_t)x.l[i + 1] << got;
    got += 28;
    if (got < 32 && i + 2 < kN) v |= (uint64_t)x.l[i + 2] << got;
    w[j] = (uint32_t)v;
  }
}
// R'' form (N-form, value < 16p) -> R-form words, value < 2p: x'' 2^-8 =
// (x'' + k p) / 2^8 with k = -x'' p^-1 mod 2^8 (kPinv28 mod 2^8).
TA_HD void to32(const F28& x, uint32_t* w) {
  const uint32_t k = (x.l[0] * kPinv28) & 0xFFu;
  F28 v;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    const uint64_t t = (uint64_t)x.l[i] + (uint64_t)k * kP28[i] + carry;
    v.l[i] = i < kN - 1 ? (uint32_t)t & kM28 : (uint32_t)t;
    carry = t >> 28;
  }
  repack32<8>(v, w);
}

// x = 0 (mod p) for an N-form x < 32p: x = k p for some k < 32, so
// (x mod 2^32) p^-1 mod 2^32 = k -- a one-multiply filter before the full compare
TA_HD bool is_zero_mod_p(const F28& x) {
  const uint32_t lo = x.l[0] | (x.l[1] << 28);
  const uint32_t k = lo * kPinv32;
  if (k >= 32) return false;
  uint64_t carry = 0;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    const uint64_t t = (uint64_t)k * kP28[i] + carry;
    const uint32_t limb = i < kN - 1 ? (uint32_t)t & kM28 : (uint32_t)t;
    carry = i < kN - 1 ? t >> 28 : 0;
    diff |= limb ^ x.l[i];
  }
  return diff == 0;
}

}  // namespace tachyon_amd::f28
