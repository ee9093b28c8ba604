/* ORACLE -- test infrastructure only.
 *
 * CPU restatement of the reference's MSM + radix-2 NTT path (Tachyon,
 * /root/reference, 2025-01-31 snapshot) in plain C.  It is the parity checker
 * for the HIP product path and the `cpu_baseline` of bench.py; nothing in the
 * product (tachyon_amd/, include/) links, imports or calls it.
 *
 * Pinning: the restatement is checked against (1) golden vectors written by an
 * independent pure-Python big-int restatement (oracle/pyref.py ->
 * tests/golden/), (2) the reference's own known-answer tests -- the "Easy" MSM
 * set sum_{i=1..n} i*G = n(n+1)/2*G (msm/test/variable_base_msm_test_set.h:55-68),
 * the curve generators of the BUILD files, and the real BN254 G1/G2 points of
 * vendors/circom/examples/multiplier_3.zkey whose decimal coordinates the
 * reference's zkey_unittest.cc:71-140 states, and (3) the arkworks-compatible
 * BN254 Fr two-adic root of unity.  The reference itself
 * cannot be built here (bazel + absl/glog/gtest + genrule constants).
 *
 * Build: `make -C oracle` -> oracle/liboracle.so (gcc -O3 -march=native -fopenmp).
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "oracle_constants.h"

/* ---- fields -------------------------------------------------------------- */
#define FF bn254_fq
#define FF_N 4
#define FF_P BN254_FQ_P
#define FF_R BN254_FQ_R
#define FF_R2 BN254_FQ_R2
#define FF_INV BN254_FQ_INV
#include "ff_impl.h"
#undef FF
#undef FF_N
#undef FF_P
#undef FF_R
#undef FF_R2
#undef FF_INV

#define FF bn254_fr
#define FF_N 4
#define FF_P BN254_FR_P
#define FF_R BN254_FR_R
#define FF_R2 BN254_FR_R2
#define FF_INV BN254_FR_INV
#include "ff_impl.h"
#undef FF
#undef FF_N
#undef FF_P
#undef FF_R
#undef FF_R2
#undef FF_INV

#define FF bls12_381_fq
#define FF_N 6
#define FF_P BLS12_381_FQ_P
#define FF_R BLS12_381_FQ_R
#define FF_R2 BLS12_381_FQ_R2
#define FF_INV BLS12_381_FQ_INV
#include "ff_impl.h"
#undef FF
#undef FF_N
#undef FF_P
#undef FF_R
#undef FF_R2
#undef FF_INV

#define FF bls12_381_fr
#define FF_N 4
#define FF_P BLS12_381_FR_P
#define FF_R BLS12_381_FR_R
#define FF_R2 BLS12_381_FR_R2
#define FF_INV BLS12_381_FR_INV
#include "ff_impl.h"
#undef FF
#undef FF_N
#undef FF_P
#undef FF_R
#undef FF_R2
#undef FF_INV

#define F2 bn254_fq2
#define F1 bn254_fq
#include "fp2_impl.h"
#undef F2
#undef F1
#define F2 bls12_381_fq2
#define F1 bls12_381_fq
#include "fp2_impl.h"
#undef F2
#undef F1

/* ---- curves -------------------------------------------------------------- */
#define EC bn254_g1
#define EF bn254_fq
#include "ec_impl.h"
#undef EC
#undef EF
#define EC bn254_g2
#define EF bn254_fq2
#include "ec_impl.h"
#undef EC
#undef EF
#define EC bls12_381_g1
#define EF bls12_381_fq
#include "ec_impl.h"
#undef EC
#undef EF
#define EC bls12_381_g2
#define EF bls12_381_fq2
#include "ec_impl.h"
#undef EC
#undef EF

/* ---- MSM ------------------------------------------------------------------ */
#define EC bn254_g1
#define EF bn254_fq
#define SF bn254_fr
#define SF_N 4
#define SF_BITS BN254_FR_BITS
#include "msm_impl.h"
#undef EC
#undef EF
#define EC bn254_g2
#define EF bn254_fq2
#include "msm_impl.h"
#undef EC
#undef EF
#undef SF
#undef SF_BITS
#define SF bls12_381_fr
#define SF_BITS BLS12_381_FR_BITS
#define EC bls12_381_g1
#define EF bls12_381_fq
#include "msm_impl.h"
#undef EC
#undef EF
#define EC bls12_381_g2
#define EF bls12_381_fq2
#include "msm_impl.h"
#undef EC
#undef EF
#undef SF
#undef SF_N
#undef SF_BITS

/* ---- NTT ------------------------------------------------------------------ */
/* math::halo2::OverrideSubgroupGenerator() (bn/bn254/halo2/bn254.cc:7-30)
 * replaces BN254 Fr's kSubgroupGenerator (5 -> 7), kTwoAdicRootOfUnity and
 * kLargeSubgroupRootOfUnity with halo2curves' values (Montgomery limbs, as
 * the reference writes them).  GetRootOfUnity (prime_field_base.h:90-130)
 * takes the large-subgroup branch for BN254 Fr: w = large^(3^2) squared
 * (28 - log n) times; large^9 equals the two-adic root for both constant
 * sets (checked by tests/test_halo2_golden.py), so the two-adic root below
 * is that same w.  Domains capture the root when they are created. */
static const uint64_t BN254_FR_HALO2_TWO_ADIC_ROOT_MONT[4] = {
    10822932506504462008ULL, 10978899855858987673ULL, 12888607242213977304ULL, 2119232853909229097ULL};
static const uint64_t BN254_FR_HALO2_LARGE_SUBGROUP_ROOT_MONT[4] = {
    9055134861510678988ULL, 3166494206591041163ULL, 11983946130272577941ULL, 1690279781341100183ULL};
static int g_bn254_fr_halo2 = 0;
#define FF bn254_fr
#define FF_TWO_ADICITY BN254_FR_TWO_ADICITY
#define FF_TWO_ADIC_ROOT (g_bn254_fr_halo2 ? BN254_FR_HALO2_TWO_ADIC_ROOT_MONT : BN254_FR_TWO_ADIC_ROOT_MONT)
#include "ntt_impl.h"
#undef FF
#undef FF_TWO_ADICITY
#undef FF_TWO_ADIC_ROOT
#define FF bls12_381_fr
#define FF_TWO_ADICITY BLS12_381_FR_TWO_ADICITY
#define FF_TWO_ADIC_ROOT BLS12_381_FR_TWO_ADIC_ROOT_MONT
#include "ntt_impl.h"
#undef FF
#undef FF_TWO_ADICITY
#undef FF_TWO_ADIC_ROOT

/* ========================================================================== */
/* Exported API (ctypes).  Field ids: 0 bn254_fq, 1 bn254_fr, 2 bls12_381_fq,
 * 3 bls12_381_fr.  Curve ids: 0 bn254_g1, 1 bn254_g2, 2 bls12_381_g1,
 * 3 bls12_381_g2.  All field data is Montgomery-form 64-bit LE limbs unless a
 * function says "canonical". */
#define EXPORT __attribute__((visibility("default")))

EXPORT int oracle_field_limbs(int field) {
  switch (field) {
    case 0: case 1: case 3: return 4;
    case 2: return 6;
  }
  return 0;
}

#define FIELD_OP_CASE(F, NL)                                                     \
  {                                                                               \
    const F##_t* A = (const F##_t*)a;                                             \
    const F##_t* B = (const F##_t*)b;                                             \
    F##_t* O = (F##_t*)out;                                                       \
    for (size_t i = 0; i < count; ++i) {                                          \
      switch (op) {                                                               \
        case 0: O[i] = F##_add(A[i], B[i]); break;                                \
        case 1: O[i] = F##_sub(A[i], B[i]); break;                                \
        case 2: O[i] = F##_mul(A[i], B[i]); break;                                \
        case 3: O[i] = F##_sqr(A[i]); break;                                      \
        case 4: O[i] = F##_neg(A[i]); break;                                      \
        case 5: O[i] = F##_inv(A[i]); break;                                      \
        case 6: O[i] = F##_from_bigint(A[i].l); break;                            \
        case 7: F##_to_bigint(&A[i], O[i].l); break;                              \
        case 8: O[i] = F##_dbl(A[i]); break;                                      \
        default: return -1;                                                       \
      }                                                                           \
    }                                                                             \
    return 0;                                                                     \
  }

/* op: 0 add, 1 sub, 2 mul, 3 square, 4 negate, 5 inverse, 6 canonical->Montgomery,
 *     7 Montgomery->canonical, 8 double. */
EXPORT int oracle_field_op(int field, int op, const void* a, const void* b, void* out, size_t count) {
  switch (field) {
    case 0: FIELD_OP_CASE(bn254_fq, 4)
    case 1: FIELD_OP_CASE(bn254_fr, 4)
    case 2: FIELD_OP_CASE(bls12_381_fq, 6)
    case 3: FIELD_OP_CASE(bls12_381_fr, 4)
  }
  return -1;
}

/* ---- deterministic synthetic inputs ---------------------------------------
 * Counter-based splitmix64: u64(seed, ctr) = mix(seed + (ctr+1)*gamma), i.e.
 * the ctr-th output of a splitmix64 stream seeded with `seed`.  The product's
 * GPU input generator implements the identical scheme, so parity tests can
 * cross-check it.
 *   scalar i : limbs u64(seed, i*4 + k), k<4, halved until < r (BigInt::Random,
 *              big_int.h:107-115), then FromBigInt (Montgomery).
 *   bases    : chunks of `chunk` points; chunk j starts at k_j*G with
 *              k_j = scalar(seed ^ BASE_SEED_XOR, j) and continues by doubling
 *              (CreatePseudoRandomPoints, test/random.h:12-28). */
#define SM_GAMMA UINT64_C(0x9E3779B97F4A7C15)
#define BASE_SEED_XOR UINT64_C(0xBA5E5EEDBA5E5EED)

static inline uint64_t sm_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * UINT64_C(0xBF58476D1CE4E5B9);
  z = (z ^ (z >> 27)) * UINT64_C(0x94D049BB133111EB);
  return z ^ (z >> 31);
}
EXPORT uint64_t oracle_rand_u64(uint64_t seed, uint64_t ctr) { return sm_mix(seed + (ctr + 1) * SM_GAMMA); }

static inline int geq_limbs(const uint64_t* a, const uint64_t* b, int n) {
  for (int i = n - 1; i >= 0; --i) {
    if (a[i] > b[i]) return 1;
    if (a[i] < b[i]) return 0;
  }
  return 1;
}

/* canonical random scalar (4 limbs) below modulus m */
static inline void rand_scalar_canonical(uint64_t seed, uint64_t i, const uint64_t* m, uint64_t* out) {
  for (int k = 0; k < 4; ++k) out[k] = oracle_rand_u64(seed, i * 4 + k);
  while (geq_limbs(out, m, 4)) {
    for (int k = 0; k < 3; ++k) out[k] = (out[k] >> 1) | (out[k + 1] << 63);
    out[3] >>= 1;
  }
}

/* scalar_field: 1 bn254_fr, 3 bls12_381_fr.  Writes Montgomery scalars
 * [start, start+n). */
EXPORT int oracle_gen_scalars(int scalar_field, uint64_t seed, size_t start, size_t n, void* out) {
  const uint64_t* m = scalar_field == 1 ? BN254_FR_P : BLS12_381_FR_P;
  if (scalar_field != 1 && scalar_field != 3) return -1;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (size_t i = 0; i < n; ++i) {
    uint64_t c[4];
    rand_scalar_canonical(seed, start + i, m, c);
    if (scalar_field == 1) ((bn254_fr_t*)out)[i] = bn254_fr_from_bigint(c);
    else ((bls12_381_fr_t*)out)[i] = bls12_381_fr_from_bigint(c);
  }
  return 0;
}

#define GEN_BASES(EC, EF, GX, GY)                                                      \
  {                                                                                     \
    EC##_affine_t* O = (EC##_affine_t*)out;                                             \
    EC##_affine_t G;                                                                    \
    memcpy(&G.x, GX, sizeof G.x);                                                       \
    memcpy(&G.y, GY, sizeof G.y);                                                       \
    size_t nchunks = (n + chunk - 1) / chunk;                                           \
    int failed = 0;                                                                     \
    _Pragma("omp parallel for schedule(dynamic)")                                       \
    for (size_t j = 0; j < nchunks; ++j) {                                              \
      size_t s = j * chunk, len = (s + chunk <= n) ? chunk : n - s;                     \
      EC##_xyzz_t* tmp = (EC##_xyzz_t*)malloc(sizeof(EC##_xyzz_t) * len);               \
      EF##_t* scr = (EF##_t*)malloc(sizeof(EF##_t) * len);                              \
      if (!tmp || !scr) { failed = 1; free(tmp); free(scr); continue; }                 \
      uint64_t k[4];                                                                    \
      rand_scalar_canonical(seed ^ BASE_SEED_XOR, j, sm, k);                            \
      EC##_xyzz_t r = EC##_scalar_mul(&G, k, 4);                                        \
      for (size_t i = 0; i < len; ++i) { tmp[i] = r; r = EC##_xyzz_dbl(&r); }          \
      EC##_batch_to_affine(tmp, O + s, len, scr);                                       \
      free(tmp);                                                                        \
      free(scr);                                                                        \
    }                                                                                   \
    return failed ? -2 : 0;                                                             \
  }

EXPORT int oracle_gen_bases(int curve, uint64_t seed, size_t n, size_t chunk, void* out) {
  if (chunk == 0) return -1;
  const uint64_t* sm = (curve <= 1) ? BN254_FR_P : BLS12_381_FR_P;
  switch (curve) {
    case 0: GEN_BASES(bn254_g1, bn254_fq, BN254_G1_X_MONT, BN254_G1_Y_MONT)
    case 1: GEN_BASES(bn254_g2, bn254_fq2, BN254_G2_X_MONT, BN254_G2_Y_MONT)
    case 2: GEN_BASES(bls12_381_g1, bls12_381_fq, BLS12_381_G1_X_MONT, BLS12_381_G1_Y_MONT)
    case 3: GEN_BASES(bls12_381_g2, bls12_381_fq2, BLS12_381_G2_X_MONT, BLS12_381_G2_Y_MONT)
  }
  return -1;
}

/* ---- direct polynomial evaluation -------------------------------------------
 * out[q] = sum_j coeffs[j] x_q^j with x_q = w^idx[q] (Montgomery in/out): the
 * FFT's output idx[q] computed without the butterfly network, so large
 * transforms are checked at sampled indices independently of the radix-2
 * restatement.  Blocks of 2^16 coefficients run Horner on OpenMP threads; the
 * block sums are scaled by x^(block start). */
#define EVAL_POINTS(FRN)                                                                   \
  {                                                                                        \
    const FRN##_t* c = (const FRN##_t*)coeffs;                                             \
    FRN##_t w;                                                                             \
    memcpy(&w, w_mont, sizeof w);                                                          \
    const size_t B = (size_t)1 << 16, nb = (n + B - 1) / B;                                \
    for (size_t q = 0; q < nidx; ++q) {                                                    \
      uint64_t e = idx[q];                                                                 \
      const FRN##_t x = FRN##_pow(w, &e, 1);                                               \
      FRN##_t total = FRN##_zero();                                                        \
      _Pragma("omp parallel")                                                              \
      {                                                                                    \
        FRN##_t part = FRN##_zero();                                                       \
        _Pragma("omp for schedule(static) nowait")                                         \
        for (size_t b = 0; b < nb; ++b) {                                                  \
          const size_t lo = b * B, hi = lo + B < n ? lo + B : n;                           \
          FRN##_t h = FRN##_zero();                                                        \
          for (size_t j = hi; j-- > lo;) h = FRN##_add(FRN##_mul(h, x), c[j]);             \
          uint64_t eb = (uint64_t)lo;                                                      \
          part = FRN##_add(part, FRN##_mul(h, FRN##_pow(x, &eb, 1)));                      \
        }                                                                                  \
        _Pragma("omp critical")                                                            \
        total = FRN##_add(total, part);                                                    \
      }                                                                                    \
      ((FRN##_t*)out)[q] = total;                                                          \
    }                                                                                      \
    return 0;                                                                              \
  }

EXPORT int oracle_eval_at_powers(int field, const void* coeffs, size_t n, const void* w_mont, const uint64_t* idx,
                                 size_t nidx, void* out) {
  if (field == 1) EVAL_POINTS(bn254_fr)
  if (field == 3) EVAL_POINTS(bls12_381_fr)
  return -1;
}

/* ---- discrete-log identity of the synthetic inputs ---------------------------
 * The generated bases are known multiples of G: point i (global index start+i)
 * = k_j 2^t G with j = (start+i) / chunk, t = (start+i) mod chunk.  So for any
 * scalars s_i, MSM(bases, s) = (sum_i s_i k_j 2^t mod r) G: one inner product
 * over Fr and one scalar multiplication -- an answer for full-size MSMs that
 * shares nothing with the Pippenger restatement (the test multiplies G in
 * pure Python, oracle/pyref.py).  scalars: Montgomery Fr; out: canonical
 * 4 limbs of the sum. */
#define DLOG_DOT(FRN)                                                                      \
  {                                                                                        \
    const FRN##_t* S = (const FRN##_t*)scalars;                                            \
    const size_t first = start / chunk, last = (start + n + chunk - 1) / chunk;            \
    FRN##_t total = FRN##_zero();                                                          \
    _Pragma("omp parallel")                                                                \
    {                                                                                      \
      FRN##_t part = FRN##_zero();                                                         \
      _Pragma("omp for schedule(static) nowait")                                           \
      for (size_t j = first; j < last; ++j) {                                              \
        uint64_t k[4];                                                                     \
        rand_scalar_canonical(seed ^ BASE_SEED_XOR, j, m, k);                              \
        FRN##_t d = FRN##_from_bigint(k);                                                  \
        size_t g0 = j * chunk, g1 = g0 + chunk;                                            \
        for (size_t g = g0; g < g1; ++g) {                                                 \
          if (g >= start && g < start + n) part = FRN##_add(part, FRN##_mul(S[g - start], d)); \
          d = FRN##_add(d, d);                                                             \
        }                                                                                  \
      }                                                                                    \
      _Pragma("omp critical")                                                              \
      total = FRN##_add(total, part);                                                      \
    }                                                                                      \
    FRN##_to_bigint(&total, (uint64_t*)out);                                               \
    return 0;                                                                              \
  }

EXPORT int oracle_dlog_dot(int scalar_field, uint64_t seed, size_t start, size_t n, size_t chunk,
                           const void* scalars, void* out) {
  if (chunk == 0) return -1;
  const uint64_t* m = scalar_field == 1 ? BN254_FR_P : BLS12_381_FR_P;
  if (scalar_field == 1) DLOG_DOT(bn254_fr)
  if (scalar_field == 3) DLOG_DOT(bls12_381_fr)
  return -1;
}

/* ---- MSM ------------------------------------------------------------------ */
/* method: 0 PippengerAdapter kParallelTerm (reference default), 1 single
 * Pippenger (kNone), 2 naive double-and-add.  Writes the affine result (x, y)
 * and, if out_jac != NULL, the Jacobian the reference C-ABI would return
 * (ConvertPoint<Jacobian>(XYZZ), point_xyzz.h:228-237). */
#define MSM_CASE(EC)                                                                     \
  {                                                                                      \
    const EC##_affine_t* B = (const EC##_affine_t*)bases;                                \
    EC##_xyzz_t r;                                                                       \
    if (method == 0) r = EC##_msm_parallel_term(B, S, n, threads);                       \
    else if (method == 1) r = EC##_pippenger(B, S, n);                                   \
    else r = EC##_msm_naive(B, S, n);                                                    \
    *(EC##_affine_t*)out_affine = EC##_xyzz_to_affine(&r);                               \
    if (out_jac) *(EC##_jacobian_t*)out_jac = EC##_xyzz_to_jacobian(&r);                 \
    return 0;                                                                            \
  }

EXPORT int oracle_msm(int curve, const void* bases, const void* scalars, size_t n, int method,
                      int threads, void* out_affine, void* out_jac) {
  switch (curve) {
    case 0: { const bn254_fr_t* S = (const bn254_fr_t*)scalars; MSM_CASE(bn254_g1) }
    case 1: { const bn254_fr_t* S = (const bn254_fr_t*)scalars; MSM_CASE(bn254_g2) }
    case 2: { const bls12_381_fr_t* S = (const bls12_381_fr_t*)scalars; MSM_CASE(bls12_381_g1) }
    case 3: { const bls12_381_fr_t* S = (const bls12_381_fr_t*)scalars; MSM_CASE(bls12_381_g2) }
  }
  return -1;
}

/* Point helpers for tests.  op: 0 P+Q (affine,affine -> affine), 1 2P,
 * 2 is_on_curve(P) -> return value, 3 k*P (k canonical 4 limbs in `q`),
 * 4 jacobian -> affine (p = jacobian). */
#define EC_OP_CASE(EC, BCONST)                                                           \
  {                                                                                      \
    const EC##_affine_t* A = (const EC##_affine_t*)p;                                    \
    switch (op) {                                                                        \
      case 0: {                                                                          \
        EC##_xyzz_t t = EC##_affine_to_xyzz(A);                                          \
        t = EC##_xyzz_madd(&t, (const EC##_affine_t*)q);                                 \
        *(EC##_affine_t*)out = EC##_xyzz_to_affine(&t);                                  \
        return 0;                                                                        \
      }                                                                                  \
      case 1: {                                                                          \
        EC##_xyzz_t t = EC##_affine_to_xyzz(A);                                          \
        t = EC##_xyzz_dbl(&t);                                                           \
        *(EC##_affine_t*)out = EC##_xyzz_to_affine(&t);                                  \
        return 0;                                                                        \
      }                                                                                  \
      case 2: {                                                                          \
        __typeof__(((EC##_affine_t*)0)->x) b;                                                            \
        memcpy(&b, BCONST, sizeof b);                                                    \
        return EC##_affine_is_on_curve(A, &b);                                           \
      }                                                                                  \
      case 3: {                                                                          \
        EC##_xyzz_t t = EC##_scalar_mul(A, (const uint64_t*)q, 4);                       \
        *(EC##_affine_t*)out = EC##_xyzz_to_affine(&t);                                  \
        return 0;                                                                        \
      }                                                                                  \
      case 4: {                                                                          \
        *(EC##_affine_t*)out = EC##_jacobian_to_affine((const EC##_jacobian_t*)p);       \
        return 0;                                                                        \
      }                                                                                  \
    }                                                                                    \
    return -1;                                                                           \
  }

EXPORT int oracle_ec_op(int curve, int op, const void* p, const void* q, void* out) {
  switch (curve) {
    case 0: EC_OP_CASE(bn254_g1, BN254_G1_B_MONT)
    case 1: EC_OP_CASE(bn254_g2, BN254_G2_B_MONT)
    case 2: EC_OP_CASE(bls12_381_g1, BLS12_381_G1_B_MONT)
    case 3: EC_OP_CASE(bls12_381_g2, BLS12_381_G2_B_MONT)
  }
  return -1;
}

/* ---- NTT ------------------------------------------------------------------ */
/* field: 1 bn254_fr, 3 bls12_381_fr.  v has room for the domain size
 * (bit_ceil(domain_num_coeffs)); `len` input elements.  offset (Montgomery) may
 * be NULL for the plain domain.  Returns the output length (FFT: domain size
 * or 0; IFFT: length after RemoveHighDegreeZeros), or -1. */
#define NTT_CASE(F, FN)                                                                  \
  {                                                                                      \
    F##_domain_t* d = F##_domain_create(domain_num_coeffs);                              \
    if (!d) return -1;                                                                   \
    if (offset) { F##_t o; memcpy(&o, offset, sizeof o); F##_domain_set_offset(d, o); }  \
    long r = (long)F##_domain_##FN(d, (F##_t*)v, len);                                   \
    F##_domain_destroy(d);                                                               \
    return r;                                                                            \
  }

EXPORT long oracle_fft(int field, size_t domain_num_coeffs, const void* offset, void* v, size_t len) {
  if (field == 1) NTT_CASE(bn254_fr, fft)
  if (field == 3) NTT_CASE(bls12_381_fr, fft)
  return -1;
}

EXPORT long oracle_ifft(int field, size_t domain_num_coeffs, const void* offset, void* v, size_t len) {
  if (field == 1) NTT_CASE(bn254_fr, ifft)
  if (field == 3) NTT_CASE(bls12_381_fr, ifft)
  return -1;
}

/* 1: install the halo2 generator / roots (OverrideSubgroupGenerator), 0: restore
 * (~ScopedSubgroupGeneratorOverrider).  Returns the previous state. */
EXPORT int oracle_bn254_fr_set_halo2(int on) {
  int prev = g_bn254_fr_halo2;
  g_bn254_fr_halo2 = on != 0;
  return prev;
}

/* out: kLargeSubgroupRootOfUnity of the active constant set (Montgomery limbs) */
EXPORT void oracle_bn254_fr_large_subgroup_root(void* out) {
  if (g_bn254_fr_halo2) {
    memcpy(out, BN254_FR_HALO2_LARGE_SUBGROUP_ROOT_MONT, 32);
  } else {
    /* generator 5: 5^(t / 3^2), t = (p - 1) / 2^28 (prime_field_generator.cc:292-316) */
    uint64_t t[4];
    memcpy(t, BN254_FR_P, sizeof t);
    t[0] -= 1;
    for (int i = 0; i < 4; ++i) t[i] = (t[i] >> 28) | (i < 3 ? t[i + 1] << 36 : 0);
    unsigned __int128 rem = 0;
    for (int i = 3; i >= 0; --i) {
      unsigned __int128 cur = (rem << 64) | t[i];
      t[i] = (uint64_t)(cur / 9);
      rem = cur % 9;
    }
    bn254_fr_t r = bn254_fr_pow(bn254_fr_from_u64(5), t, 4);
    memcpy(out, r.l, 32);
  }
}

/* Domain scalars for tests: writes group_gen, group_gen_inv, size_inv. */
EXPORT int oracle_domain_info(int field, size_t num_coeffs, void* out3) {
  if (field == 1) {
    bn254_fr_domain_t* d = bn254_fr_domain_create(num_coeffs);
    if (!d) return -1;
    bn254_fr_t* o = (bn254_fr_t*)out3;
    o[0] = d->group_gen; o[1] = d->group_gen_inv; o[2] = d->size_inv;
    bn254_fr_domain_destroy(d);
    return 0;
  }
  if (field == 3) {
    bls12_381_fr_domain_t* d = bls12_381_fr_domain_create(num_coeffs);
    if (!d) return -1;
    bls12_381_fr_t* o = (bls12_381_fr_t*)out3;
    o[0] = d->group_gen; o[1] = d->group_gen_inv; o[2] = d->size_inv;
    bls12_381_fr_domain_destroy(d);
    return 0;
  }
  return -1;
}

/* QuadraticArithmeticProgram::WitnessMapFromMatrices
 * (vendors/circom/circomlib/circuit/quadratic_arithmetic_program.h:24-113):
 *   a[c] += value * full[s] (matrix 0) / b[c] likewise (:38-63, serial here:
 *   field addition is exact, so the reference's lock order does not matter);
 *   c = a * b (:65-71); a, b, c = IFFT (:77-82); DistributePowers by the
 *   2n-th root of unity (:84-91); FFT (:93-98); h = a * b - c (:100-108).
 * coefs: ncoef packed zkey records {u32 matrix, u32 constraint, u32 signal,
 * 32-byte word}; the value is FromMontgomery(word) as the zkey reader stores
 * it (zkey.h:211-223).  full: m Montgomery elements.  h_out: n elements. */
#define WITNESS_MAP(F)                                                                      \
  {                                                                                         \
    F##_t* abc = (F##_t*)calloc(3 * n, sizeof(F##_t));                                      \
    if (!abc) return -1;                                                                    \
    F##_t *a = abc, *b = abc + n, *c = abc + 2 * n;                                         \
    const F##_t* w = (const F##_t*)full;                                                    \
    const uint8_t* rec = (const uint8_t*)coefs;                                             \
    for (size_t i = 0; i < ncoef; ++i, rec += 44) {                                         \
      uint32_t mc[3];                                                                       \
      memcpy(mc, rec, 12);                                                                  \
      if (mc[1] >= n || mc[2] >= m) { free(abc); return -2; }                               \
      F##_t word, val;                                                                      \
      memcpy(word.l, rec + 12, 32);                                                         \
      F##_to_bigint(&word, val.l);                                                          \
      F##_t t = F##_mul(val, w[mc[2]]);                                                     \
      F##_t* dst = mc[0] == 0 ? &a[mc[1]] : &b[mc[1]];                                      \
      *dst = F##_add(*dst, t);                                                              \
    }                                                                                       \
    for (size_t i = 0; i < n; ++i) c[i] = F##_mul(a[i], b[i]);                              \
    F##_domain_t* d = F##_domain_create(n);                                                 \
    F##_domain_t* d2 = F##_domain_create(2 * n);                                            \
    if (!d || !d2) { free(abc); return -3; }                                                \
    F##_domain_set_offset(d, d2->group_gen); /* DistributePowers(g_2n) + FFT = coset FFT */ \
    F##_t one = F##_one();                                                                  \
    for (int k = 0; k < 3; ++k) {                                                           \
      F##_t* v = abc + (size_t)k * n;                                                       \
      F##_domain_t tmp = *d;                                                                \
      tmp.has_offset = 0; tmp.offset = one; tmp.offset_inv = one;                           \
      size_t len = F##_domain_ifft(&tmp, v, n);                                             \
      if (F##_domain_fft(d, v, len) == 0)                                                   \
        for (size_t i = 0; i < n; ++i) v[i] = F##_zero();                                   \
    }                                                                                       \
    F##_t* h = (F##_t*)h_out;                                                               \
    for (size_t i = 0; i < n; ++i) h[i] = F##_sub(F##_mul(a[i], b[i]), c[i]);               \
    F##_domain_destroy(d);                                                                  \
    F##_domain_destroy(d2);                                                                 \
    free(abc);                                                                              \
    return 0;                                                                               \
  }

EXPORT int oracle_groth16_witness_map(int field, size_t n, const void* coefs, size_t ncoef, const void* full,
                                      size_t m, void* h_out) {
  if (field == 1) WITNESS_MAP(bn254_fr)
  if (field == 3) WITNESS_MAP(bls12_381_fr)
  return -1;
}

EXPORT int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
