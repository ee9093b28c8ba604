/* ORACLE (test infrastructure only -- never linked into the product path).
 *
 * CPU variable-base MSM, restating the reference's default CPU path:
 *   VariableBaseMSM<Point>::Run                         variable_base_msm.h:20-36
 *   -> PippengerAdapter::RunWithStrategy(kParallelTerm)  pippenger_adapter.h:38-116 (default :34)
 *   -> Pippenger::Run                                    pippenger.h:78-109
 *        MSMCtx::CreateDefault                           msm_ctx.h:22-48
 *        FillDigits                                      pippenger.h:28-51
 *        AccumulateWindowNAFSums / SingleWindowNAFSum    pippenger.h:113-170
 *        PippengerBase::AccumulateBuckets                pippenger_base.h:36-57
 *        PippengerBase::AccumulateWindowSums             pippenger_base.h:59-77
 * Bucket type is PointXYZZ for affine bases (pippenger_base.h:24-28).
 *
 * Define EC (point prefix), EF (base-field prefix), SF (scalar-field prefix),
 * SF_N (scalar limbs) and SF_BITS (kModulusBits) before including.
 */
#include <math.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MS_CAT2(a, b) a##_##b
#define MS_CAT(a, b) MS_CAT2(a, b)
#define EC_FN(name) MS_CAT(EC, name)
#define SF_FN(name) MS_CAT(SF, name)
#define SF_T MS_CAT(SF, t)
#define EC_AFF MS_CAT(EC, affine_t)
#define EC_XYZZ MS_CAT(EC, xyzz_t)

/* msm_ctx.h:22-48 */
static inline unsigned EC_FN(msm_window_bits)(size_t n) {
  if (n < 32) return 3;
  return (unsigned)(log2((double)n) * 69 / 100) + 2;
}
static inline unsigned EC_FN(msm_window_count)(unsigned c) { return (SF_BITS + c - 1) / c; }

/* BigInt::ExtractBits64 (big_int.h:338-341) on a canonical scalar. */
static inline uint64_t EC_FN(extract_bits)(const uint64_t* s, size_t bit_offset, size_t count) {
  size_t limb = bit_offset / 64, sh = bit_offset % 64;
  if (limb >= SF_N) return 0;
  uint64_t v = s[limb] >> sh;
  if (sh && limb + 1 < SF_N) v |= s[limb + 1] << (64 - sh);
  return count >= 64 ? v : (v & ((UINT64_C(1) << count) - 1));
}

/* pippenger.h:28-51 */
static inline void EC_FN(fill_digits)(const uint64_t* s, unsigned c, unsigned windows, int64_t* digits) {
  uint64_t radix = UINT64_C(1) << c;
  uint64_t carry = 0;
  size_t bit_offset = 0;
  for (unsigned i = 0; i < windows; ++i) {
    uint64_t bits = EC_FN(extract_bits)(s, bit_offset, c);
    uint64_t coeff = carry + bits;
    carry = (coeff + radix / 2) >> c;
    digits[i] = (int64_t)coeff - (int64_t)(carry << c);
    bit_offset += c;
  }
  digits[windows - 1] += (int64_t)(carry << c);
}

/* pippenger_base.h:36-57 */
static inline EC_XYZZ EC_FN(accumulate_buckets)(const EC_XYZZ* buckets, size_t nb) {
  EC_XYZZ running = EC_FN(xyzz_zero)(), window = EC_FN(xyzz_zero)();
  for (size_t i = nb; i-- > 0;) {
    running = EC_FN(xyzz_add)(&running, &buckets[i]);
    window = EC_FN(xyzz_add)(&window, &running);
  }
  return window;
}

/* Pippenger::Run with use_msm_window_naf_ = true, serial windows. */
static EC_XYZZ EC_FN(pippenger)(const EC_AFF* bases, const SF_T* scalars, size_t n) {
  unsigned c = EC_FN(msm_window_bits)(n);
  unsigned windows = EC_FN(msm_window_count)(c);
  int64_t* digits = (int64_t*)malloc(sizeof(int64_t) * windows * (n ? n : 1));
  for (size_t i = 0; i < n; ++i) {
    uint64_t s[SF_N];
    SF_FN(to_bigint)(&scalars[i], s);
    EC_FN(fill_digits)(s, c, windows, digits + i * windows);
  }
  EC_XYZZ* window_sums = (EC_XYZZ*)malloc(sizeof(EC_XYZZ) * windows);
  EC_XYZZ* buckets = (EC_XYZZ*)malloc(sizeof(EC_XYZZ) * ((size_t)1 << c));
  for (unsigned w = 0; w < windows; ++w) {
    size_t nb = (w == windows - 1) ? ((size_t)1 << c) : ((size_t)1 << (c - 1));
    for (size_t b = 0; b < nb; ++b) buckets[b] = EC_FN(xyzz_zero)();
    for (size_t j = 0; j < n; ++j) {
      int64_t d = digits[j * windows + w];
      if (d > 0) {
        buckets[d - 1] = EC_FN(xyzz_madd)(&buckets[d - 1], &bases[j]);
      } else if (d < 0) {
        EC_AFF nb_ = EC_FN(affine_neg)(&bases[j]);
        buckets[-d - 1] = EC_FN(xyzz_madd)(&buckets[-d - 1], &nb_);
      }
    }
    window_sums[w] = EC_FN(accumulate_buckets)(buckets, nb);
  }
  /* pippenger_base.h:59-77 */
  EC_XYZZ total = EC_FN(xyzz_zero)();
  for (unsigned w = windows; w-- > 1;) {
    total = EC_FN(xyzz_add)(&total, &window_sums[w]);
    for (unsigned k = 0; k < c; ++k) total = EC_FN(xyzz_dbl)(&total);
  }
  total = EC_FN(xyzz_add)(&window_sums[0], &total);
  free(buckets);
  free(window_sums);
  free(digits);
  return total;
}

/* PippengerAdapter kParallelTerm: ceil(n/T) chunks, one Pippenger each, summed
 * in chunk order (pippenger_adapter.h:82-113). `threads` <= 0 means
 * omp_get_max_threads(). */
static EC_XYZZ EC_FN(msm_parallel_term)(const EC_AFF* bases, const SF_T* scalars, size_t n, int threads) {
  if (n == 0) return EC_FN(xyzz_zero)();
  int T = 1;
#ifdef _OPENMP
  T = threads > 0 ? threads : omp_get_max_threads();
#else
  (void)threads;
#endif
  size_t chunk = (n + T - 1) / T;
  size_t nchunks = (n + chunk - 1) / chunk;
  EC_XYZZ* parts = (EC_XYZZ*)malloc(sizeof(EC_XYZZ) * nchunks);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(T)
#endif
  for (size_t k = 0; k < nchunks; ++k) {
    size_t start = k * chunk;
    size_t len = (start + chunk <= n) ? chunk : n - start;
    parts[k] = EC_FN(pippenger)(bases + start, scalars + start, len);
  }
  EC_XYZZ total = EC_FN(xyzz_zero)();
  for (size_t k = 0; k < nchunks; ++k) total = EC_FN(xyzz_add)(&total, &parts[k]);
  free(parts);
  return total;
}

/* Naive sum_i s_i * P_i (the expectation of pippenger_unittest.cc / msm_gpu_unittest.cc). */
static EC_XYZZ EC_FN(msm_naive)(const EC_AFF* bases, const SF_T* scalars, size_t n) {
  EC_XYZZ total = EC_FN(xyzz_zero)();
  for (size_t i = 0; i < n; ++i) {
    uint64_t s[SF_N];
    SF_FN(to_bigint)(&scalars[i], s);
    EC_XYZZ t = EC_FN(scalar_mul)(&bases[i], s, SF_N);
    total = EC_FN(xyzz_add)(&total, &t);
  }
  return total;
}

#undef MS_CAT2
#undef MS_CAT
#undef EC_FN
#undef SF_FN
#undef SF_T
#undef EC_AFF
#undef EC_XYZZ
