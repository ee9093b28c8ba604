// Montgomery prime-field arithmetic for CDNA4 (gfx950), 32-bit limbs.
//
// Same values as the reference's PrimeField (tachyon/math/finite_fields/
// prime_field_fallback.h): Montgomery form with R = 2^(64*N64), canonical in
// [0, p), little-endian limbs -- so a tachyon_bn254_fq {uint64_t limbs[4]} is
// bit-identical to an Fp<bn254_fq> {uint32_t v[8]}.
//
// Device multiplication is Finely Integrated Product Scanning with generated
// v_mad_u64_u32 carry chains (mont_asm.h, tools/gen_mont_asm.py); the host
// keeps the reference's CIOS "no-carry" DoFastMul (prime_field_fallback.h:331-355)
// restated on 32-bit limbs.
//
// Lazy reduction (device only): when 4p < 2^(32N) (BN254 Fq/Fr, BLS12-381 Fq)
// device values live in [0, 2p): the FIPS product of two such values is < 2p
// without the final conditional subtraction, add/sub/neg wrap by 2p, and
// zero/equality tests compare canonical forms.  Every value that leaves a
// kernel as a result is canonicalised (canonical()); host code always works
// on canonical values.  BLS12-381 Fr (1 spare bit) stays canonical.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#include "constants.h"
#include "mont_asm.h"

#define TA_HD __host__ __device__ __forceinline__
// Rarely-executed or very large bodies stay out of line: inlining every
// 12-limb (BLS12-381 Fq) product and every exceptional-case doubling made
// single kernels tens of thousands of instructions long and compile for
// minutes.
#define TA_HD_NOINLINE __host__ __device__ __noinline__
// device add/sub/conditional-subtract as hand-written VCC carry chains
// (mont_asm.h); 0 = hipcc's code from the portable C below
#ifndef TA_FIELD_ASM
#define TA_FIELD_ASM 1
#endif
// device squares by the dedicated FIPS square (mont_asm.h mont_sqr_fips_N);
// 0 = a general product of the value with itself
#ifndef TA_FIELD_SQR
#define TA_FIELD_SQR 1
#endif
// a b - c d with one reduction (mont_asm.h mont_mul_sub_fips_N); 0 = two
// products and a modular subtraction
#ifndef TA_FIELD_MULSUB
#define TA_FIELD_MULSUB 1
#endif
// Fq2 a b - c d as three fused base a b - c d (Fp2::mul_sub)
#ifndef TA_FQ2_MULSUB
#define TA_FQ2_MULSUB 1
#endif
// Fq2 products over the inline 8-limb field as two fused products
#ifndef TA_FQ2_FUSED_MUL
#define TA_FQ2_FUSED_MUL 1
#endif

namespace tachyon_amd {

TA_HD uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
}

TA_HD uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
}

template <class Cfg>
struct Fp {
  static constexpr int N = Cfg::N32;
  using Config = Cfg;
  // [0, 2p) representation is sound when 4p < 2^(32N)
  static constexpr bool kLazyCapable = Cfg::kModulusBits <= 32 * N - 2;
  // Fp2 over this field multiplies inline (else through one out-of-line call)
  static constexpr bool kExtInline = N <= 8;
#if defined(__HIP_DEVICE_COMPILE__)
  static constexpr bool kLazy = kLazyCapable;
#else
  static constexpr bool kLazy = false;
#endif
  uint32_t v[N];

  TA_HD static Fp zero() {
    Fp r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = 0;
    return r;
  }
  TA_HD static Fp one() {
    Fp r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = Cfg::kR32[i];
    return r;
  }
  TA_HD static Fp modulus() {
    Fp r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = Cfg::kP32[i];
    return r;
  }

  // r = a - m if a >= m else a, with m = p or 2p given as limbs
  TA_HD static void cond_sub(uint32_t* a, const uint32_t* m) {
    uint32_t t[N];
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = subb(a[i], m[i], br, &br);
#pragma unroll
    for (int i = 0; i < N; ++i) a[i] = br ? a[i] : t[i];
  }
  TA_HD static void reduce_once(uint32_t* a) {
#if defined(__HIP_DEVICE_COMPILE__) && TA_FIELD_ASM
    if constexpr (N == 8) return detail::cond_sub_8<Cfg, false>(a);
    else if constexpr (N == 12) return detail::cond_sub_12<Cfg, false>(a);
#endif
    cond_sub(a, Cfg::kP32);
  }

  // canonical representative in [0, p); also applied on the host to values
  // copied back from the device
  TA_HD Fp canonical() const {
    Fp r = *this;
    if constexpr (kLazyCapable) reduce_once(r.v);
    return r;
  }

  TA_HD bool is_zero() const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) acc |= v[i];
    if constexpr (kLazy) {
      uint32_t accp = 0;  // x == p is the other representative of zero
#pragma unroll
      for (int i = 0; i < N; ++i) accp |= v[i] ^ Cfg::kP32[i];
      return acc == 0 || accp == 0;
    }
    return acc == 0;
  }
  // zero test of a value known to be canonical (< p), e.g. an input point
  TA_HD bool is_zero_canonical() const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) acc |= v[i];
    return acc == 0;
  }
  // -x for a canonical x as p - x: no borrow test, a lazy representative in
  // (0, p] (p stands for zero); device fields with the [0, 2p) representation
  TA_HD Fp neg_canonical() const {
    if constexpr (!kLazy) {
      return -*this;
    } else {
      Fp r;
      uint32_t br = 0;
#pragma unroll
      for (int i = 0; i < N; ++i) r.v[i] = subb(Cfg::kP32[i], v[i], br, &br);
      return r;
    }
  }
  // x or -x by a run-time flag, as limb selects (no branch)
  TA_HD Fp cond_neg_canonical(bool neg) const {
    const Fp m = neg_canonical();
    Fp r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = neg ? m.v[i] : v[i];
    return r;
  }
  TA_HD bool operator==(const Fp& o) const {
    Fp a = canonical(), b = o.canonical();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) acc |= a.v[i] ^ b.v[i];
    return acc == 0;
  }
  TA_HD bool operator!=(const Fp& o) const { return !(*this == o); }
  TA_HD bool is_one() const { return *this == one(); }

  // prime_field_fallback.h:199-214 (Add + Clamp); lazy: wrap at 2p
  TA_HD Fp operator+(const Fp& o) const {
    Fp r;
#if defined(__HIP_DEVICE_COMPILE__) && TA_FIELD_ASM
    if constexpr (N == 8) { detail::add_mod_8<Cfg, kLazy>(r.v, v, o.v); return r; }
    else if constexpr (N == 12) { detail::add_mod_12<Cfg, kLazy>(r.v, v, o.v); return r; }
#endif
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = addc(v[i], o.v[i], c, &c);
    // spare top bits: no carry out of the top limb
    if constexpr (kLazy) cond_sub(r.v, Cfg::kP232);
    else reduce_once(r.v);
    return r;
  }
  TA_HD Fp dbl() const { return *this + *this; }

  // a - b + 2p without the borrow test: in [0, 4p) for lazy a, b.  Only as
  // the left factor of a product whose other factor is canonical (< p): the
  // lazy product is then (x y + m p) / R < 4p^2/R + p < 2p since 4p < R.
  TA_HD Fp sub_unreduced(const Fp& o) const {
    if constexpr (!kLazy) {
      return *this - o;
    } else {
      Fp r;
#if defined(__HIP_DEVICE_COMPILE__) && TA_FIELD_ASM
      if constexpr (N == 8) { detail::sub_unreduced_8<Cfg, true>(r.v, v, o.v); return r; }
      else if constexpr (N == 12) { detail::sub_unreduced_12<Cfg, true>(r.v, v, o.v); return r; }
#endif
      uint32_t br = 0;
#pragma unroll
      for (int i = 0; i < N; ++i) r.v[i] = subb(v[i], o.v[i], br, &br);
      uint32_t c = 0;  // the borrow of a - b cancels against the carry of + 2p
#pragma unroll
      for (int i = 0; i < N; ++i) r.v[i] = addc(r.v[i], Cfg::kP232[i], c, &c);
      return r;
    }
  }

  // prime_field_fallback.h:234-251 (Sub: add p back on borrow); lazy: add 2p
  TA_HD Fp operator-(const Fp& o) const {
    Fp r;
#if defined(__HIP_DEVICE_COMPILE__) && TA_FIELD_ASM
    if constexpr (N == 8) { detail::sub_mod_8<Cfg, kLazy>(r.v, v, o.v); return r; }
    else if constexpr (N == 12) { detail::sub_mod_12<Cfg, kLazy>(r.v, v, o.v); return r; }
#endif
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = subb(v[i], o.v[i], br, &br);
    uint32_t mask = 0u - br;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint32_t m = kLazy ? Cfg::kP232[i] : Cfg::kP32[i];
      r.v[i] = addc(r.v[i], m & mask, c, &c);
    }
    return r;
  }
  TA_HD Fp operator-() const { return zero() - *this; }

  TA_HD Fp operator*(const Fp& b) const {
    if constexpr (N <= 8) return mul_inline(b);
    else return mul_outline(b);
  }
  TA_HD_NOINLINE Fp mul_outline(const Fp& b) const { return mul_inline(b); }

  TA_HD Fp mul_inline(const Fp& b) const {
#if defined(__HIP_DEVICE_COMPILE__)
    // device: FIPS with hand-scheduled v_mad_u64_u32 carry chains (mont_asm.h);
    // the product is < 2p for inputs < 2p (4p < R)
    Fp r;
    if constexpr (N == 8) detail::mont_mul_fips_8<Cfg>(r.v, v, b.v);
    else detail::mont_mul_fips_12<Cfg>(r.v, v, b.v);
    if constexpr (!kLazy) reduce_once(r.v);
    return r;
#else
    return mul_cios64(b);
#endif
  }

  // Host product: CIOS on 64-bit limbs with 128-bit intermediates (the
  // reference's 64-bit-limb Montgomery multiplication, prime_field_fallback.h
  // :296-329); a quarter of the multiplies of the 32-bit CIOS below -- the
  // host window Horner of every MSM is (W-1)*c doublings, ~2.5K products.
  Fp mul_cios64(const Fp& b) const {
    constexpr int M = N / 2;
    uint64_t x[M], y[M], t[M + 2] = {};
    for (int i = 0; i < M; ++i) {
      x[i] = v[2 * i] | (uint64_t)v[2 * i + 1] << 32;
      y[i] = b.v[2 * i] | (uint64_t)b.v[2 * i + 1] << 32;
    }
    for (int i = 0; i < M; ++i) {
      unsigned __int128 c = 0;
      for (int j = 0; j < M; ++j) {
        c += (unsigned __int128)x[j] * y[i] + t[j];
        t[j] = (uint64_t)c;
        c >>= 64;
      }
      unsigned __int128 s = (unsigned __int128)t[M] + c;
      t[M] = (uint64_t)s;
      t[M + 1] = (uint64_t)(s >> 64);
      const uint64_t m = t[0] * Cfg::kInv64;
      c = ((unsigned __int128)m * Cfg::kP64[0] + t[0]) >> 64;
      for (int j = 1; j < M; ++j) {
        c += (unsigned __int128)m * Cfg::kP64[j] + t[j];
        t[j - 1] = (uint64_t)c;
        c >>= 64;
      }
      s = (unsigned __int128)t[M] + c;
      t[M - 1] = (uint64_t)s;
      t[M] = t[M + 1] + (uint64_t)(s >> 64);
    }
    Fp r;
    for (int i = 0; i < M; ++i) {
      r.v[2 * i] = (uint32_t)t[i];
      r.v[2 * i + 1] = (uint32_t)(t[i] >> 32);
    }
    reduce_once(r.v);  // t < 2p
    return r;
  }

  // Product by a constant w given as (w canonical plain, wq = floor(w 2^(32N)
  // / p)): the Shoup product of mont_asm.h (8 limbs: 115 v_mad_u64_u32 + 99
  // carry adds vs 128 + 128 + 8 v_mul_lo_u32 Montgomery digits in
  // mul_inline).  For a Montgomery-form *this
  // (any value < 2^(32N), e.g. an unreduced difference) it is the Montgomery
  // form of a * w, lazy in [0, 2p).  Device: 8-limb fields with 3p < 2^256.
  TA_HD Fp mul_shoup(const Fp& w, const Fp& wq) const {
#if defined(__HIP_DEVICE_COMPILE__)
    static_assert(N == 8 && kLazy, "Shoup products: 8-limb lazy fields only");
    Fp r;
    detail::shoup_mul_8<Cfg>(r.v, v, w.v, wq.v);
    // r < 3p; r >= 2p only when the quotient estimate came out one short
    // (probability ~2^-30 per product; the top-limb test rarely passes)
    if (r.v[N - 1] >= Cfg::kP232[N - 1]) detail::cond_sub_8<Cfg, true>(r.v);
    return r;
#else
    (void)wq;
    return mul_cios(w.to_mont());
#endif
  }

  // The Shoup quotient floor(w 2^(32N) / p) of a canonical w < p (2p <
  // 2^(32N)): long division, one quotient bit per step (table setup only)
  TA_HD static Fp shoup_quotient(const Fp& w) {
    uint32_t rem[N], q[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      rem[i] = w.v[i];
      q[i] = 0;
    }
    for (int bit = 32 * N - 1; bit >= 0; --bit) {
      uint32_t carry = 0;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const uint32_t nc = rem[i] >> 31;
        rem[i] = (rem[i] << 1) | carry;
        carry = nc;
      }
      uint32_t t[N], br = 0;
#pragma unroll
      for (int i = 0; i < N; ++i) t[i] = subb(rem[i], Cfg::kP32[i], br, &br);
      if (!br) {
#pragma unroll
        for (int i = 0; i < N; ++i) rem[i] = t[i];
        q[bit >> 5] |= 1u << (bit & 31);
      }
    }
    Fp r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = q[i];
    return r;
  }

  // CIOS no-carry Montgomery product (DoFastMul, prime_field_fallback.h:331-355);
  // the host path (final Horner step, conversions).
  TA_HD Fp mul_cios(const Fp& b) const {
    uint32_t t[N];
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint32_t bi = b.v[i];
      uint64_t s = (uint64_t)v[0] * bi + t[0];
      t[0] = (uint32_t)s;
      uint32_t hi1 = (uint32_t)(s >> 32);
      const uint32_t k = t[0] * Cfg::kInv32;
      uint64_t s2 = (uint64_t)k * Cfg::kP32[0] + t[0];
      uint32_t hi2 = (uint32_t)(s2 >> 32);
#pragma unroll
      for (int j = 1; j < N; ++j) {
        s = (uint64_t)v[j] * bi + ((uint64_t)t[j] + hi1);
        t[j] = (uint32_t)s;
        hi1 = (uint32_t)(s >> 32);
        s2 = (uint64_t)k * Cfg::kP32[j] + ((uint64_t)t[j] + hi2);
        t[j - 1] = (uint32_t)s2;
        hi2 = (uint32_t)(s2 >> 32);
      }
      t[N - 1] = hi1 + hi2;
    }
    Fp r;
    reduce_once(t);
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = t[i];
    return r;
  }
  // (*this) b - c d with one Montgomery reduction (mont_asm.h gen_mulsub):
  // the y coordinate of the XYZZ additions.  Device, lazy fields: the
  // columns sum a b + (2p - c) d; the REDC output is < 3p (p < 2^254), one
  // conditional subtraction of 2p puts it back in [0, 2p)
  TA_HD Fp mul_sub(const Fp& b, const Fp& c, const Fp& d) const {
    if constexpr (N <= 8) return mul_sub_inline(b, c, d);
    else return (*this) * b - c * d;
  }
  TA_HD Fp mul_sub_inline(const Fp& b, const Fp& c, const Fp& d) const {
#if defined(__HIP_DEVICE_COMPILE__) && TA_FIELD_MULSUB
    if constexpr (N == 8 && kLazy) {
      static_assert(Cfg::kModulusBits <= 32 * N - 2, "mul_sub: 8p^2/R + p < 3p");
      Fp r;
      detail::mont_mul_sub_fips_8<Cfg>(r.v, v, b.v, c.v, d.v);
      detail::cond_sub_8<Cfg, true>(r.v);
      return r;
    } else if constexpr (N == 12 && kLazy) {
      static_assert(Cfg::kModulusBits <= 32 * N - 3, "mul_sub: 8p^2/R + p < 2p");
      Fp r;  // BLS12-381 Fq: already below 2p
      detail::mont_mul_sub_fips_12<Cfg>(r.v, v, b.v, c.v, d.v);
      return r;
    }
#endif
    return mul_inline(b) - c.mul_inline(d);
  }

  // (*this) b + c d with one Montgomery reduction (mont_mul_add_fips_8; the
  // Fq2 product's imaginary part), < 3p before one conditional subtraction
  TA_HD Fp mul_add_inline(const Fp& b, const Fp& c, const Fp& d) const {
#if defined(__HIP_DEVICE_COMPILE__) && TA_FIELD_MULSUB
    if constexpr (N == 8 && kLazy) {
      Fp r;
      detail::mont_mul_add_fips_8<Cfg>(r.v, v, b.v, c.v, d.v);
      detail::cond_sub_8<Cfg, true>(r.v);
      return r;
    } else if constexpr (N == 12 && kLazy) {
      Fp r;  // BLS12-381 Fq: < 2p already
      detail::mont_mul_add_fips_12<Cfg>(r.v, v, b.v, c.v, d.v);
      return r;
    }
#endif
    return mul_inline(b) + c.mul_inline(d);
  }

  // Squares count each cross product once (mont_asm.h gen_sqr: 100 instead
  // of 128 v_mad_u64_u32 for 8 limbs); the device square needs a value below
  // 2^(32N-1), which every representation here keeps (lazy < 2p of a 254- or
  // 381-bit field, canonical < p of BLS12-381 Fr)
  static_assert(Cfg::kModulusBits + (kLazyCapable ? 1 : 0) <= 32 * N - 1, "mont_sqr_fips: top bit must be clear");
  TA_HD Fp sqr() const {
    if constexpr (N <= 8) return sqr_inline();
    else return sqr_outline();
  }
  TA_HD_NOINLINE Fp sqr_outline() const { return sqr_inline(); }
  TA_HD Fp sqr_inline() const {
#if defined(__HIP_DEVICE_COMPILE__) && TA_FIELD_SQR
    Fp r;
    if constexpr (N == 8) detail::mont_sqr_fips_8<Cfg>(r.v, v);
    else detail::mont_sqr_fips_12<Cfg>(r.v, v);
    if constexpr (!kLazy) reduce_once(r.v);
    return r;
#else
    return mul_inline(*this);
#endif
  }

  // Montgomery -> canonical integer (ToBigInt, prime_field_fallback.h:166-169)
  TA_HD Fp from_mont() const {
#if defined(__HIP_DEVICE_COMPILE__)
    // device: the Montgomery reduction alone (N rounds of one digit and N
    // multiply-adds: 64 v_mad_u64_u32 for 8 limbs, against 128 for the
    // product by 1 through the asm multiply, whose zero limbs it cannot
    // skip) -- the MSM recode runs this once per scalar in each of its two
    // passes.  For x < 2p: (x + m p) / 2^(32N) <= p, and = p only for x = p.
    uint32_t t[N];
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = v[i];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint32_t k = t[0] * Cfg::kInv32;
      uint64_t s = (uint64_t)k * Cfg::kP32[0] + t[0];
#pragma unroll
      for (int j = 1; j < N; ++j) {
        s = (uint64_t)k * Cfg::kP32[j] + ((uint64_t)t[j] + (s >> 32));
        t[j - 1] = (uint32_t)s;
      }
      t[N - 1] = (uint32_t)(s >> 32);
    }
    Fp r;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = t[i];
    reduce_once(r.v);
    return r;
#else
    Fp one_plain = zero();
    one_plain.v[0] = 1;
    return ((*this) * one_plain).canonical();
#endif
  }
  // canonical integer (< p) -> Montgomery (lazy on device)
  TA_HD Fp to_mont() const {
    Fp r2;
#pragma unroll
    for (int i = 0; i < N; ++i) r2.v[i] = Cfg::kR232[i];
    return (*this) * r2;
  }

  TA_HD_NOINLINE Fp pow(const uint32_t* e, int nlimbs) const {
    Fp r = one();
    for (int i = nlimbs - 1; i >= 0; --i)
      for (int bit = 31; bit >= 0; --bit) {
        r = r.sqr();
        if ((e[i] >> bit) & 1) r = r * (*this);
      }
    return r;
  }
  // Fermat inverse (same canonical value as the reference's BY inverter)
  TA_HD_NOINLINE Fp inverse() const {
    // e = p - 2 with borrow (BLS12-381 Fr's low 32-bit limb is 1)
    uint32_t e[N];
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = subb(Cfg::kP32[i], i == 0 ? 2u : 0u, br, &br);
    return pow(e, N);
  }
};

// Fq2 = Fq[u]/(u^2 + 1)  (non-residue -1 for BN254 and BLS12-381;
// quadratic_extension_field.h:315-360 Karatsuba).
template <class F>
struct Fp2 {
  using Base = F;
  F c0, c1;
  TA_HD static Fp2 zero() { return {F::zero(), F::zero()}; }
  TA_HD static Fp2 one() { return {F::one(), F::zero()}; }
  TA_HD Fp2 canonical() const { return {c0.canonical(), c1.canonical()}; }
  TA_HD bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  TA_HD bool is_zero_canonical() const { return c0.is_zero_canonical() && c1.is_zero_canonical(); }
  TA_HD Fp2 cond_neg_canonical(bool neg) const { return {c0.cond_neg_canonical(neg), c1.cond_neg_canonical(neg)}; }
  TA_HD bool is_one() const { return c0.is_one() && c1.is_zero(); }
  TA_HD bool operator==(const Fp2& o) const { return c0 == o.c0 && c1 == o.c1; }
  TA_HD bool operator!=(const Fp2& o) const { return !(*this == o); }
  TA_HD Fp2 operator+(const Fp2& o) const { return {c0 + o.c0, c1 + o.c1}; }
  TA_HD Fp2 operator-(const Fp2& o) const { return {c0 - o.c0, c1 - o.c1}; }
  TA_HD Fp2 operator-() const { return {-c0, -c1}; }
  TA_HD Fp2 dbl() const { return {c0.dbl(), c1.dbl()}; }
  TA_HD Fp2 operator*(const Fp2& o) const {
    if constexpr (F::kExtInline) return mul_inline(o);
    else return mul_outline(o);
  }
  TA_HD_NOINLINE Fp2 mul_outline(const Fp2& o) const { return mul_inline(o); }
  TA_HD Fp2 mul_inline(const Fp2& o) const {
#if TA_FQ2_FUSED_MUL
    // inline 8-limb base field (BN254 Fq2): schoolbook as two fused
    // products -- a0 b0 - a1 b1 and a0 b1 + a1 b0, two reductions instead of
    // Karatsuba's three and no Karatsuba sums/differences (the same 384
    // v_mad_u64_u32)
    // (BLS12-381 Fq2 keeps Karatsuba: the same pair as two register-argument
    // calls with 48 words in each spilled at the G2 kernel's 2-wave cap, 2^22
    // 52.2 -> 54.8 ms)
    if constexpr (F::kLazy && F::kExtInline && F::N == 8)
      return {c0.mul_sub(o.c0, c1, o.c1), c0.mul_add_inline(o.c1, c1, o.c0)};
#endif
    F v0 = c0 * o.c0;
    F v1 = c1 * o.c1;
    F m = (c0 + c1) * (o.c0 + o.c1);
    return {v0 - v1, m - v0 - v1};
  }
  // a b - c d: over the inline 8-limb base field (BN254 Fq2) each Karatsuba
  // term pairs with its counterpart in one fused base product (three
  // reductions instead of six; BN254 G2 2^22 22.1 -> 21.5 ms); otherwise two
  // products and a subtraction (BLS12-381 Fq2: the 12-limb fused product as
  // a register-argument call measured neutral, 2^22 52.2 vs 52.1 ms, with 30
  // more VGPR spills at the 2-wave cap)
  TA_HD Fp2 mul_sub(const Fp2& b, const Fp2& c, const Fp2& d) const {
#if TA_FQ2_MULSUB
    if constexpr (F::kLazy && F::kExtInline && F::N == 8) {
      const F u0 = c0.mul_sub(b.c0, c.c0, d.c0);
      const F u1 = c1.mul_sub(b.c1, c.c1, d.c1);
      const F um = (c0 + c1).mul_sub(b.c0 + b.c1, c.c0 + c.c1, d.c0 + d.c1);
      return {u0 - u1, um - u0 - u1};
    }
#endif
    return (*this) * b - c * d;
  }
  TA_HD Fp2 sqr() const {
    F ab = c0 * c1;
    return {(c0 + c1) * (c0 - c1), ab.dbl()};
  }
  TA_HD_NOINLINE Fp2 inverse() const {
    F t = (c0.sqr() + c1.sqr()).inverse();
    return {c0 * t, -(c1 * t)};
  }
};

// The same field with every product inlined.  Wide fields (BLS12-381 Fq, and
// Fq2 through Fp2<HotFp<Fq>>) multiply out of line by default to bound code
// size and compile time; the one hot kernel of a curve (the MSM bucket
// accumulation) views its data through this type instead, which has the same
// layout.
template <class F>
struct HotFp : F {
  HotFp() = default;
  TA_HD HotFp(const F& f) : F(f) {}
  TA_HD static HotFp zero() { return F::zero(); }
  TA_HD static HotFp one() { return F::one(); }
  TA_HD HotFp operator+(const HotFp& o) const { return F::operator+(o); }
  TA_HD HotFp operator-(const HotFp& o) const { return F::operator-(o); }
  TA_HD HotFp operator-() const { return F::operator-(); }
  TA_HD HotFp sub_unreduced(const HotFp& o) const { return F::sub_unreduced(o); }
  TA_HD HotFp operator*(const HotFp& o) const { return F::mul_inline(o); }
  TA_HD HotFp dbl() const { return F::dbl(); }
  TA_HD HotFp sqr() const { return F::sqr_inline(); }
  TA_HD HotFp mul_sub(const HotFp& b, const HotFp& c, const HotFp& d) const { return F::mul_sub_inline(b, c, d); }
  TA_HD HotFp mul_add_inline(const HotFp& b, const HotFp& c, const HotFp& d) const { return F::mul_add_inline(b, c, d); }
  TA_HD HotFp inverse() const { return F::inverse(); }
  TA_HD HotFp cond_neg_canonical(bool neg) const { return F::cond_neg_canonical(neg); }
  TA_HD HotFp mul_shoup(const HotFp& w, const HotFp& wq) const { return F::mul_shoup(w, wq); }
  TA_HD HotFp canonical() const { return F::canonical(); }
};

// 12-limb products as calls whose operands travel in registers.  An
// out-of-line Fq2 product takes `this` and its operand by address (48 words
// exceed the registers clang passes arguments in), so every call went
// through scratch memory: the caller stores both operands, the callee loads
// them back with flat loads, and its wide register footprint forces the
// caller to spill the accumulator around it.  One Fq product takes 24 words
// in v0..v23 and returns 12 in v0..v11, and its small footprint leaves the
// caller's live point in registers.
#define TA_LIMBS12(x) uint32_t x##0, uint32_t x##1, uint32_t x##2, uint32_t x##3, uint32_t x##4, uint32_t x##5, \
                      uint32_t x##6, uint32_t x##7, uint32_t x##8, uint32_t x##9, uint32_t x##10, uint32_t x##11
#define TA_UNPACK12(x) {x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11}
#define TA_PASS12(f) f.v[0], f.v[1], f.v[2], f.v[3], f.v[4], f.v[5], f.v[6], f.v[7], f.v[8], f.v[9], f.v[10], f.v[11]
namespace detail {
template <class F>
__device__ __noinline__ F mul_in_regs(TA_LIMBS12(a), TA_LIMBS12(b)) {
  const F x{TA_UNPACK12(a)}, y{TA_UNPACK12(b)};
  return x.mul_inline(y);
}
template <class F>
__device__ __noinline__ F sqr_in_regs(TA_LIMBS12(a)) {
  const F x{TA_UNPACK12(a)};
  return x.sqr_inline();
}
}  // namespace detail

template <class F>
struct CallFp : F {
  static_assert(F::N == 12, "register-argument products: 12-limb fields");
  static constexpr bool kExtInline = true;
  CallFp() = default;
  TA_HD CallFp(const F& f) : F(f) {}
  TA_HD static CallFp zero() { return F::zero(); }
  TA_HD static CallFp one() { return F::one(); }
  TA_HD CallFp operator+(const CallFp& o) const { return F::operator+(o); }
  TA_HD CallFp operator-(const CallFp& o) const { return F::operator-(o); }
  TA_HD CallFp operator-() const { return F::operator-(); }
  TA_HD CallFp sub_unreduced(const CallFp& o) const { return F::sub_unreduced(o); }
  TA_HD CallFp dbl() const { return F::dbl(); }
  TA_HD CallFp operator*(const CallFp& o) const {
#if defined(__HIP_DEVICE_COMPILE__)
    return detail::mul_in_regs<F>(TA_PASS12((*this)), TA_PASS12(o));
#else
    return F::mul_inline(o);
#endif
  }
  TA_HD CallFp sqr() const {
#if defined(__HIP_DEVICE_COMPILE__)
    return detail::sqr_in_regs<F>(TA_PASS12((*this)));
#else
    return F::sqr_inline();
#endif
  }
  TA_HD CallFp mul_sub(const CallFp& b, const CallFp& c, const CallFp& d) const { return (*this) * b - c * d; }
  TA_HD CallFp inverse() const { return F::inverse(); }
  TA_HD CallFp cond_neg_canonical(bool neg) const { return F::cond_neg_canonical(neg); }
  TA_HD CallFp canonical() const { return F::canonical(); }
};

template <class F>
struct HotOf {
  using type = F;
};
template <class Cfg>
struct HotOf<Fp<Cfg>> {
  using type = HotFp<Fp<Cfg>>;
};
template <class Cfg>
struct HotOf<Fp2<Fp<Cfg>>> {
  using type = std::conditional_t<(Fp<Cfg>::N > 8), Fp2<CallFp<Fp<Cfg>>>, Fp2<HotFp<Fp<Cfg>>>>;
};

using Bn254Fq = Fp<consts::bn254_fq>;
using Bn254Fr = Fp<consts::bn254_fr>;
using Bls381Fq = Fp<consts::bls12_381_fq>;
using Bls381Fr = Fp<consts::bls12_381_fr>;
using Bn254Fq2 = Fp2<Bn254Fq>;
using Bls381Fq2 = Fp2<Bls381Fq>;

}  // namespace tachyon_amd
