/* ORACLE (test infrastructure only -- never linked into the product path).
 *
 * Radix-2 evaluation domain over a two-adic prime field FF, restating
 *   UnivariateEvaluationDomain ctor / FFT / IFFT      univariate_evaluation_domain.h:55-69,141-232
 *   GetCoset                                          univariate_evaluation_domain.h:102-117
 *   DistributePowersAndMulByConst                     univariate_evaluation_domain.h:464-489
 *   ButterflyFnInOut / ButterflyFnOutIn               univariate_evaluation_domain.h:518-524,558-566
 *   Radix2EvaluationDomain::Create / DoFFT / DoIFFT /
 *     DegreeAwareFFTInPlace / InOrderIFFTInPlace /
 *     IFFTHelperInPlace / ApplyButterfly /
 *     InOutHelper / OutInHelper                       radix2_evaluation_domain.h:83-89,213-333
 *   Radix2TwiddleCache::Item                          radix2_twiddle_cache.h:57-121
 *   SwapBitRevElementsInPlace                         evaluations_utils.h:26-36
 *   PrimeFieldBase::GetRootOfUnity                    prime_field_base.h:90-130
 * Define FF (field prefix), FF_TWO_ADICITY, FF_TWO_ADIC_ROOT (Montgomery limbs).
 */
#include <stdlib.h>

#define NT_CAT2(a, b) a##_##b
#define NT_CAT(a, b) NT_CAT2(a, b)
#define FF_FN(name) NT_CAT(FF, name)
#define FF_T NT_CAT(FF, t)
#define DOM_T NT_CAT(FF, domain_t)
#define DOM_FN(name) NT_CAT(FF, NT_CAT(domain, name))

typedef struct {
  size_t size;
  uint32_t log_size;
  FF_T size_inv, group_gen, group_gen_inv;
  FF_T offset, offset_inv;
  int has_offset;
  /* roots_vec[s] has 2^s entries (s = 0..log-1), inv_roots_vec[i] has n/2^(i+1). */
  FF_T** roots_vec;
  FF_T** inv_roots_vec;
} DOM_T;

static inline uint32_t FF_FN(log2_ceil)(size_t n) {
  uint32_t l = 0;
  while (((size_t)1 << l) < n) ++l;
  return l;
}

static inline size_t FF_FN(reverse_bits)(size_t x, uint32_t bits) {
  size_t r = 0;
  for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

/* evaluations_utils.h:26-36 */
static inline void FF_FN(swap_bitrev)(FF_T* v, size_t size, uint32_t log_len) {
  if (size <= 1) return;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (size_t idx = 1; idx < size; ++idx) {
    size_t r = FF_FN(reverse_bits)(idx, log_len);
    if (idx < r) { FF_T t = v[idx]; v[idx] = v[r]; v[r] = t; }
  }
}

/* prime_field_base.h:90-130 (two-adic branch; for BN254 Fr the large-subgroup
 * branch reduces to the same g^((p-1)/n) for power-of-two n). */
static inline int FF_FN(root_of_unity)(size_t n, FF_T* out) {
  uint32_t l = FF_FN(log2_ceil)(n);
  if (((size_t)1 << l) != n || l > FF_TWO_ADICITY) return 0;
  FF_T w;
  memcpy(w.l, FF_TWO_ADIC_ROOT, sizeof w.l);
  for (uint32_t i = l; i < FF_TWO_ADICITY; ++i) w = FF_FN(sqr)(w);
  *out = w;
  return 1;
}

/* F::GetSuccessivePowers(size, g), out[i] = c * g^i.  Blocks of 2^16 run on
 * OpenMP threads, each starting from c * g^start (field arithmetic is exact, so
 * the values equal the serial running product's). */
static inline void FF_FN(scaled_powers)(FF_T* out, size_t n, FF_T g, FF_T c, int mul_into) {
  const size_t blk = (size_t)1 << 16;
  const long nb = (long)((n + blk - 1) / blk);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (long b = 0; b < nb; ++b) {
    size_t i0 = (size_t)b * blk, i1 = i0 + blk < n ? i0 + blk : n;
    uint64_t e = (uint64_t)i0;
    FF_T p = FF_FN(mul)(c, FF_FN(pow)(g, &e, 1));
    for (size_t i = i0; i < i1; ++i) {
      out[i] = mul_into ? FF_FN(mul)(out[i], p) : p;
      p = FF_FN(mul)(p, g);
    }
  }
}
static inline void FF_FN(powers)(FF_T* out, size_t n, FF_T g) { FF_FN(scaled_powers)(out, n, g, FF_FN(one)(), 0); }

static DOM_T* DOM_FN(create)(size_t num_coeffs) {
  DOM_T* d = (DOM_T*)calloc(1, sizeof(DOM_T));
  d->log_size = FF_FN(log2_ceil)(num_coeffs);
  d->size = (size_t)1 << d->log_size;
  d->size_inv = FF_FN(inv)(FF_FN(from_u64)(d->size));
  if (!FF_FN(root_of_unity)(d->size, &d->group_gen)) { free(d); return NULL; }
  d->group_gen_inv = FF_FN(inv)(d->group_gen);
  d->offset = FF_FN(one)();
  d->offset_inv = FF_FN(one)();
  d->has_offset = 0;
  uint32_t L = d->log_size;
  if (L == 0) return d;
  d->roots_vec = (FF_T**)calloc(L, sizeof(FF_T*));
  d->inv_roots_vec = (FF_T**)calloc(L, sizeof(FF_T*));
  size_t half = d->size / 2;
  d->roots_vec[L - 1] = (FF_T*)malloc(sizeof(FF_T) * half);
  d->inv_roots_vec[0] = (FF_T*)malloc(sizeof(FF_T) * half);
  FF_FN(powers)(d->roots_vec[L - 1], half, d->group_gen);
  FF_FN(powers)(d->inv_roots_vec[0], half, d->group_gen_inv);
  for (uint32_t i = 1; i < L; ++i) {
    size_t sz = d->size >> (i + 1);
    d->roots_vec[L - i - 1] = (FF_T*)malloc(sizeof(FF_T) * sz);
    d->inv_roots_vec[i] = (FF_T*)malloc(sizeof(FF_T) * sz);
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (size_t j = 0; j < sz; ++j) {
      d->roots_vec[L - i - 1][j] = d->roots_vec[L - 1][j << i];
      d->inv_roots_vec[i][j] = d->inv_roots_vec[0][j << i];
    }
  }
  return d;
}

static void DOM_FN(destroy)(DOM_T* d) {
  if (!d) return;
  for (uint32_t i = 0; i < d->log_size; ++i) {
    free(d->roots_vec[i]);
    free(d->inv_roots_vec[i]);
  }
  free(d->roots_vec);
  free(d->inv_roots_vec);
  free(d);
}

/* GetCoset: same domain, offset set. */
static void DOM_FN(set_offset)(DOM_T* d, FF_T offset) {
  d->offset = offset;
  d->offset_inv = FF_FN(inv)(offset);
  d->has_offset = !FF_FN(is_one)(&offset);
}

/* DistributePowersAndMulByConst: v[i] *= c * g^i */
static void FF_FN(distribute_powers)(FF_T* v, size_t n, FF_T g, FF_T c) { FF_FN(scaled_powers)(v, n, g, c, 1); }

/* ApplyButterfly, radix2_evaluation_domain.h:290-312 */
static void FF_FN(apply_butterfly)(FF_T* v, size_t n, const FF_T* roots, size_t gap, int in_out) {
  /* one loop over all n/2 butterflies (i = chunk base, j = offset in the
   * chunk), so the large-gap stages spread over the threads too */
  size_t chunk = 2 * gap;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (size_t b = 0; b < n / 2; ++b) {
    {
      size_t i = (b / gap) * chunk, j = b % gap;
      FF_T* lo = &v[i + j];
      FF_T* hi = &v[i + j + gap];
      if (in_out) { /* ButterflyFnInOut :518-524 */
        FF_T neg = FF_FN(sub)(*lo, *hi);
        *lo = FF_FN(add)(*lo, *hi);
        *hi = FF_FN(mul)(neg, roots[j]);
      } else { /* ButterflyFnOutIn :558-566 */
        FF_T h = FF_FN(mul)(*hi, roots[j]);
        FF_T neg = FF_FN(sub)(*lo, h);
        *lo = FF_FN(add)(*lo, h);
        *hi = neg;
      }
    }
  }
}

/* FFT(DensePoly) -> Evals. `v` holds num_coeffs coefficients and must have
 * room for d->size elements. Returns the number of evaluations (0 for the
 * zero polynomial, which the reference returns as empty Evals). */
static size_t DOM_FN(fft)(const DOM_T* d, FF_T* v, size_t num_coeffs) {
  if (num_coeffs == 0) return 0;
  /* DegreeAwareFFTInPlace :226-261 */
  if (d->has_offset) FF_FN(distribute_powers)(v, num_coeffs, d->offset, FF_FN(one)());
  size_t n = d->size;
  uint32_t log_n = d->log_size;
  uint32_t log_d = FF_FN(log2_ceil)(num_coeffs);
  size_t dup = (size_t)1 << (log_n - log_d);
  for (size_t i = num_coeffs; i < n; ++i) v[i] = FF_FN(zero)();
  FF_FN(swap_bitrev)(v, num_coeffs, log_n);
  size_t start_gap = 1;
  if (dup >= 4) { /* kDegreeAwareFFTThresholdFactor = 1 << 2 */
    for (size_t c = 0; c < n; c += dup)
      for (size_t j = 1; j < dup; ++j) v[c + j] = v[c];
    start_gap = dup;
  }
  /* OutInHelper :326-333 */
  size_t gap = start_gap;
  uint32_t idx = FF_FN(log2_ceil)(start_gap);
  while (gap < n) {
    FF_FN(apply_butterfly)(v, n, d->roots_vec[idx++], gap, 0);
    gap *= 2;
  }
  return n;
}

/* IFFT(Evals) -> DensePoly, in place on d->size elements (num_evals <= size,
 * zero-padded). Returns the coefficient count after RemoveHighDegreeZeros. */
static size_t DOM_FN(ifft)(const DOM_T* d, FF_T* v, size_t num_evals) {
  if (num_evals == 0) return 0;
  size_t n = d->size;
  for (size_t i = num_evals; i < n; ++i) v[i] = FF_FN(zero)();
  /* InOutHelper :316-324 */
  size_t gap = n / 2;
  uint32_t idx = 0;
  while (gap > 0) {
    FF_FN(apply_butterfly)(v, n, d->inv_roots_vec[idx++], gap, 1);
    gap /= 2;
  }
  FF_FN(swap_bitrev)(v, n, d->log_size);
  if (!d->has_offset) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (size_t i = 0; i < n; ++i) v[i] = FF_FN(mul)(v[i], d->size_inv);
  } else {
    FF_FN(distribute_powers)(v, n, d->offset_inv, d->size_inv);
  }
  size_t len = n;
  while (len > 0 && FF_FN(is_zero)(&v[len - 1])) --len;
  return len;
}

#undef NT_CAT2
#undef NT_CAT
#undef FF_FN
#undef FF_T
#undef DOM_T
#undef DOM_FN
