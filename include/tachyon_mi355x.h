/*
 * tachyon_mi355x.h -- C-ABI of the MI355X MSM + NTT backend.
 *
 * The entry points in the "reference C-ABI" sections keep the names, argument
 * meaning, ownership and error behaviour of Tachyon's tachyon/c API
 * (reference snapshot /root/reference, cited per declaration) so a binary
 * linked against libtachyon.so's MSM / univariate-domain symbols can link
 * against libtachyon_mi355x.so instead.  Entry points prefixed
 * tachyon_mi355x_ are extensions (device-resident buffers, G2 MSM, multi-GPU
 * helpers, synthetic inputs, timings); they have no reference counterpart.
 *
 * Data layout (identical to the reference, msm_input_provider.h:23-29
 * bit-casts these structs to its native types):
 *   field elements: Montgomery form, R = 2^(64*N), little-endian 64-bit limbs
 *   affine / point2: {x, y}, identity = (0, 0) (affine_point.h:39,125)
 *   jacobian / projective: {x, y, z};  xyzz: {x, y, zz, zzz}
 *
 * Ownership: returned points / containers are allocated with C++ operator
 * new (as msm.h:45 / msm_gpu.h:81 / bn254_univariate_evaluation_domain.cc:50-85
 * do); free them with delete (C++) or the matching *_destroy / free helper.
 * Errors: like the reference's CHECK, any failure prints a message and aborts.
 * There is no CPU fallback: every compute entry point needs a HIP device.
 */
#ifndef TACHYON_MI355X_H_
#define TACHYON_MI355X_H_

#include <stddef.h>
#include <stdint.h>

#define TACHYON_C_EXPORT __attribute__((visibility("default")))

#ifdef __cplusplus
extern "C" {
#endif

/* ---- field and point types (prime_field.h.tpl / point.h.tpl:22-94) -------- */
typedef struct tachyon_bn254_fq { uint64_t limbs[4]; } tachyon_bn254_fq;
typedef struct tachyon_bn254_fr { uint64_t limbs[4]; } tachyon_bn254_fr;
typedef struct tachyon_bn254_fq2 { tachyon_bn254_fq c0, c1; } tachyon_bn254_fq2;
typedef struct tachyon_bls12_381_fq { uint64_t limbs[6]; } tachyon_bls12_381_fq;
typedef struct tachyon_bls12_381_fr { uint64_t limbs[4]; } tachyon_bls12_381_fr;
typedef struct tachyon_bls12_381_fq2 { tachyon_bls12_381_fq c0, c1; } tachyon_bls12_381_fq2;

#define TACHYON_MI355X_POINT_TYPES(C, G, F)                                   \
  typedef struct tachyon_##C##_##G##_affine { F x, y; } tachyon_##C##_##G##_affine;             \
  typedef struct tachyon_##C##_##G##_point2 { F x, y; } tachyon_##C##_##G##_point2;             \
  typedef struct tachyon_##C##_##G##_jacobian { F x, y, z; } tachyon_##C##_##G##_jacobian;      \
  typedef struct tachyon_##C##_##G##_projective { F x, y, z; } tachyon_##C##_##G##_projective;  \
  typedef struct tachyon_##C##_##G##_xyzz { F x, y, zz, zzz; } tachyon_##C##_##G##_xyzz;

TACHYON_MI355X_POINT_TYPES(bn254, g1, tachyon_bn254_fq)
TACHYON_MI355X_POINT_TYPES(bn254, g2, tachyon_bn254_fq2)
TACHYON_MI355X_POINT_TYPES(bls12_381, g1, tachyon_bls12_381_fq)
TACHYON_MI355X_POINT_TYPES(bls12_381, g2, tachyon_bls12_381_fq2)
#undef TACHYON_MI355X_POINT_TYPES

/* ========================================================================== */
/* Reference C-ABI: MSM (generated per curve from                              */
/* tachyon/c/math/elliptic_curves/generator/msm{,_gpu}.h.tpl; G1 only there)   */
/* ========================================================================== */
typedef struct tachyon_bn254_g1_msm* tachyon_bn254_g1_msm_ptr;               /* msm.h.tpl:21 */
typedef struct tachyon_bn254_g1_msm_gpu* tachyon_bn254_g1_msm_gpu_ptr;       /* msm_gpu.h.tpl:17 */
typedef struct tachyon_bls12_381_g1_msm* tachyon_bls12_381_g1_msm_ptr;
typedef struct tachyon_bls12_381_g1_msm_gpu* tachyon_bls12_381_g1_msm_gpu_ptr;

/* point.cc.tpl:7-9 -- curve constant initialisation; constants are compiled in here, so a no-op. */
TACHYON_C_EXPORT void tachyon_bn254_g1_init(void);
TACHYON_C_EXPORT void tachyon_bls12_381_g1_init(void);
TACHYON_C_EXPORT void tachyon_bn254_g2_init(void);
TACHYON_C_EXPORT void tachyon_bls12_381_g2_init(void);

/* msm.h.tpl:30-58 (CPU-named entry points; served by the MI355X backend). */
TACHYON_C_EXPORT tachyon_bn254_g1_msm_ptr tachyon_bn254_g1_create_msm(uint8_t degree);
TACHYON_C_EXPORT void tachyon_bn254_g1_destroy_msm(tachyon_bn254_g1_msm_ptr ptr);
TACHYON_C_EXPORT tachyon_bn254_g1_jacobian* tachyon_bn254_g1_point2_msm(
    tachyon_bn254_g1_msm_ptr ptr, const tachyon_bn254_g1_point2* bases, const tachyon_bn254_fr* scalars,
    size_t size);
TACHYON_C_EXPORT tachyon_bn254_g1_jacobian* tachyon_bn254_g1_affine_msm(
    tachyon_bn254_g1_msm_ptr ptr, const tachyon_bn254_g1_affine* bases, const tachyon_bn254_fr* scalars,
    size_t size);

/* msm_gpu.h.tpl:26-54 -> tachyon/c/math/elliptic_curves/msm/msm_gpu.h:23-122. */
TACHYON_C_EXPORT tachyon_bn254_g1_msm_gpu_ptr tachyon_bn254_g1_create_msm_gpu(uint8_t degree);
TACHYON_C_EXPORT void tachyon_bn254_g1_destroy_msm_gpu(tachyon_bn254_g1_msm_gpu_ptr ptr);
TACHYON_C_EXPORT tachyon_bn254_g1_jacobian* tachyon_bn254_g1_point2_msm_gpu(
    tachyon_bn254_g1_msm_gpu_ptr ptr, const tachyon_bn254_g1_point2* bases, const tachyon_bn254_fr* scalars,
    size_t size);
TACHYON_C_EXPORT tachyon_bn254_g1_jacobian* tachyon_bn254_g1_affine_msm_gpu(
    tachyon_bn254_g1_msm_gpu_ptr ptr, const tachyon_bn254_g1_affine* bases, const tachyon_bn254_fr* scalars,
    size_t size);

TACHYON_C_EXPORT tachyon_bls12_381_g1_msm_ptr tachyon_bls12_381_g1_create_msm(uint8_t degree);
TACHYON_C_EXPORT void tachyon_bls12_381_g1_destroy_msm(tachyon_bls12_381_g1_msm_ptr ptr);
TACHYON_C_EXPORT tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_point2_msm(
    tachyon_bls12_381_g1_msm_ptr ptr, const tachyon_bls12_381_g1_point2* bases,
    const tachyon_bls12_381_fr* scalars, size_t size);
TACHYON_C_EXPORT tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_affine_msm(
    tachyon_bls12_381_g1_msm_ptr ptr, const tachyon_bls12_381_g1_affine* bases,
    const tachyon_bls12_381_fr* scalars, size_t size);
TACHYON_C_EXPORT tachyon_bls12_381_g1_msm_gpu_ptr tachyon_bls12_381_g1_create_msm_gpu(uint8_t degree);
TACHYON_C_EXPORT void tachyon_bls12_381_g1_destroy_msm_gpu(tachyon_bls12_381_g1_msm_gpu_ptr ptr);
TACHYON_C_EXPORT tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_point2_msm_gpu(
    tachyon_bls12_381_g1_msm_gpu_ptr ptr, const tachyon_bls12_381_g1_point2* bases,
    const tachyon_bls12_381_fr* scalars, size_t size);
TACHYON_C_EXPORT tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_affine_msm_gpu(
    tachyon_bls12_381_g1_msm_gpu_ptr ptr, const tachyon_bls12_381_g1_affine* bases,
    const tachyon_bls12_381_fr* scalars, size_t size);

/* ========================================================================== */
/* Reference C-ABI: univariate evaluation domain over BN254 Fr                 */
/* (tachyon/c/math/polynomials/univariate/bn254_univariate_*.h)               */
/* ========================================================================== */
typedef struct tachyon_bn254_univariate_evaluation_domain tachyon_bn254_univariate_evaluation_domain;
typedef struct tachyon_bn254_univariate_evaluations tachyon_bn254_univariate_evaluations;
typedef struct tachyon_bn254_univariate_dense_polynomial tachyon_bn254_univariate_dense_polynomial;
typedef struct tachyon_bn254_univariate_rational_evaluations tachyon_bn254_univariate_rational_evaluations;

/* bn254_univariate_evaluation_domain.h:38-136 */
TACHYON_C_EXPORT tachyon_bn254_univariate_evaluation_domain* tachyon_bn254_univariate_evaluation_domain_create(
    size_t num_coeffs);
TACHYON_C_EXPORT void tachyon_bn254_univariate_evaluation_domain_destroy(
    tachyon_bn254_univariate_evaluation_domain* domain);
TACHYON_C_EXPORT tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluation_domain_empty_evals(
    const tachyon_bn254_univariate_evaluation_domain* domain);
TACHYON_C_EXPORT tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_evaluation_domain_empty_poly(
    const tachyon_bn254_univariate_evaluation_domain* domain);
/* size() rational zeros 0/1 (bn254_univariate_evaluation_domain.h:70-79) */
TACHYON_C_EXPORT tachyon_bn254_univariate_rational_evaluations*
tachyon_bn254_univariate_evaluation_domain_empty_rational_evals(const tachyon_bn254_univariate_evaluation_domain* domain);
TACHYON_C_EXPORT tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluation_domain_fft(
    const tachyon_bn254_univariate_evaluation_domain* domain, const tachyon_bn254_univariate_dense_polynomial* poly);
TACHYON_C_EXPORT tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluation_domain_fft_inplace(
    const tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_univariate_dense_polynomial* poly);
TACHYON_C_EXPORT tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_evaluation_domain_ifft(
    const tachyon_bn254_univariate_evaluation_domain* domain, const tachyon_bn254_univariate_evaluations* evals);
TACHYON_C_EXPORT tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_evaluation_domain_ifft_inplace(
    const tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_univariate_evaluations* evals);

/* bn254_univariate_evaluations.h:36-79 */
TACHYON_C_EXPORT tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluations_create(void);
TACHYON_C_EXPORT tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluations_clone(
    const tachyon_bn254_univariate_evaluations* evals);
TACHYON_C_EXPORT void tachyon_bn254_univariate_evaluations_destroy(tachyon_bn254_univariate_evaluations* evals);
TACHYON_C_EXPORT size_t tachyon_bn254_univariate_evaluations_len(const tachyon_bn254_univariate_evaluations* evals);
TACHYON_C_EXPORT void tachyon_bn254_univariate_evaluations_set_value(tachyon_bn254_univariate_evaluations* evals,
                                                                     size_t i, const tachyon_bn254_fr* value);

/* bn254_univariate_rational_evaluations.h: UnivariateEvaluations<RationalField<bn254::Fr>>
 * (numerator / denominator pairs, zero = 0/1; boundary checks are the caller's).
 * _evaluate: numerator / denominator of element i (aborts on a zero
 * denominator, like RationalField::Evaluate's unwrap); _batch_evaluate: a new
 * evaluations container of every quotient, zero where the denominator is zero
 * (RationalField::BatchEvaluate + DoBatchInverse, groups.h:124-180), computed
 * on the GPU (Montgomery's batch-inversion trick). */
TACHYON_C_EXPORT tachyon_bn254_univariate_rational_evaluations* tachyon_bn254_univariate_rational_evaluations_create(
    void);
TACHYON_C_EXPORT tachyon_bn254_univariate_rational_evaluations* tachyon_bn254_univariate_rational_evaluations_clone(
    const tachyon_bn254_univariate_rational_evaluations* evals);
TACHYON_C_EXPORT void tachyon_bn254_univariate_rational_evaluations_destroy(
    tachyon_bn254_univariate_rational_evaluations* evals);
TACHYON_C_EXPORT size_t tachyon_bn254_univariate_rational_evaluations_len(
    const tachyon_bn254_univariate_rational_evaluations* evals);
TACHYON_C_EXPORT void tachyon_bn254_univariate_rational_evaluations_set_zero(
    tachyon_bn254_univariate_rational_evaluations* evals, size_t i);
TACHYON_C_EXPORT void tachyon_bn254_univariate_rational_evaluations_set_trivial(
    tachyon_bn254_univariate_rational_evaluations* evals, size_t i, const tachyon_bn254_fr* numerator);
TACHYON_C_EXPORT void tachyon_bn254_univariate_rational_evaluations_set_rational(
    tachyon_bn254_univariate_rational_evaluations* evals, size_t i, const tachyon_bn254_fr* numerator,
    const tachyon_bn254_fr* denominator);
TACHYON_C_EXPORT void tachyon_bn254_univariate_rational_evaluations_evaluate(
    const tachyon_bn254_univariate_rational_evaluations* evals, size_t i, tachyon_bn254_fr* value);
TACHYON_C_EXPORT tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_rational_evaluations_batch_evaluate(
    const tachyon_bn254_univariate_rational_evaluations* evals);

/* bn254_univariate_dense_polynomial.h (create/clone/destroy) */
TACHYON_C_EXPORT tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_dense_polynomial_create(void);
TACHYON_C_EXPORT tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_dense_polynomial_clone(
    const tachyon_bn254_univariate_dense_polynomial* poly);
TACHYON_C_EXPORT void tachyon_bn254_univariate_dense_polynomial_destroy(
    tachyon_bn254_univariate_dense_polynomial* poly);

/* ========================================================================== */
/* Extensions (no reference counterpart)                                       */
/* ========================================================================== */
/* Container access the reference performs through C++ native_cast. */
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluations_get_value(
    const tachyon_bn254_univariate_evaluations* evals, size_t i, tachyon_bn254_fr* value);
TACHYON_C_EXPORT tachyon_bn254_fr* tachyon_mi355x_bn254_univariate_evaluations_data(
    tachyon_bn254_univariate_evaluations* evals);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluations_resize(tachyon_bn254_univariate_evaluations* evals,
                                                                         size_t len);
TACHYON_C_EXPORT size_t tachyon_mi355x_bn254_univariate_dense_polynomial_len(
    const tachyon_bn254_univariate_dense_polynomial* poly);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_dense_polynomial_resize(
    tachyon_bn254_univariate_dense_polynomial* poly, size_t len);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_dense_polynomial_set_value(
    tachyon_bn254_univariate_dense_polynomial* poly, size_t i, const tachyon_bn254_fr* value);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_dense_polynomial_get_value(
    const tachyon_bn254_univariate_dense_polynomial* poly, size_t i, tachyon_bn254_fr* value);
TACHYON_C_EXPORT tachyon_bn254_fr* tachyon_mi355x_bn254_univariate_dense_polynomial_data(
    tachyon_bn254_univariate_dense_polynomial* poly);

/* rational container access the reference performs through native_cast */
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_rational_evaluations_resize(
    tachyon_bn254_univariate_rational_evaluations* evals, size_t len);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_rational_evaluations_get(
    const tachyon_bn254_univariate_rational_evaluations* evals, size_t i, tachyon_bn254_fr* numerator,
    tachyon_bn254_fr* denominator);

/* halo2 BN254 Fr generator set (math::halo2, bn/bn254/halo2/bn254.h:9-17):
 * _override = OverrideSubgroupGenerator() (bn254.cc:7-30: generator 7 and
 * halo2curves' two-adic / large-subgroup roots of unity), _restore = the
 * ScopedSubgroupGeneratorOverrider destructor (bn254.cc:40-44, back to the
 * arkworks-compatible generator 5).  Process-wide; domains, four-step plans
 * and KZG setups created afterwards use the active set (Domain::Create
 * captures the root).  _active returns 1 while the halo2 set is installed. */
TACHYON_C_EXPORT void tachyon_mi355x_bn254_halo2_override_subgroup_generator(void);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_halo2_restore_subgroup_generator(void);
TACHYON_C_EXPORT int tachyon_mi355x_bn254_halo2_subgroup_generator_active(void);

/* Domain queries and the coset hook (UnivariateEvaluationDomain::GetCoset,
 * univariate_evaluation_domain.h:102-117): set_offset turns the domain into
 * its coset h*<w>; offset 1 restores it. */
TACHYON_C_EXPORT size_t tachyon_mi355x_bn254_univariate_evaluation_domain_size(
    const tachyon_bn254_univariate_evaluation_domain* domain);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluation_domain_group_gen(
    const tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_fr* out);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluation_domain_set_offset(
    tachyon_bn254_univariate_evaluation_domain* domain, const tachyon_bn254_fr* offset);
/* Device-resident in-place transform of size() elements at d_data (HBM),
 * enqueued on the domain's stream (see _stream).  inverse = 0: FFT,
 * 1: IFFT (no trimming).  Not synchronised.  _batch_device transforms `batch`
 * consecutive arrays of size() elements. */
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluation_domain_transform_device(
    tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_fr* d_data, int inverse);
/* Host-resident in-place transform (IcicleNTT<bn254::Fr>::Run on a host
 * pointer, icicle_ntt.h:53-142 / icicle_ntt_bn254.cc:31-116: natural order in
 * and out, the domain's coset offset): inout holds exactly size() Montgomery
 * elements; synchronous.  The C++ hook over it is
 * include/tachyon_mi355x_ntt_holder.h (IcicleNTTHolder's shape). */
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluation_domain_transform_host(
    tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_fr* inout, size_t len, int inverse);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluation_domain_transform_batch_device(
    tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_fr* d_data, size_t batch, int inverse);
TACHYON_C_EXPORT void* tachyon_mi355x_bn254_univariate_evaluation_domain_stream(
    tachyon_bn254_univariate_evaluation_domain* domain);
/* per-pass device time (ms) of the last transform when profiling is on;
 * returns the number of passes written. */
TACHYON_C_EXPORT void tachyon_mi355x_bn254_univariate_evaluation_domain_set_profile(
    tachyon_bn254_univariate_evaluation_domain* domain, int on);
/* Kernel variant of the domain's transforms (no reference counterpart):
 * 0 = the 8 x 32-bit-limb passes, 1 = the 9 x 29-bit-limb passes, 3 = the
 * 29-bit passes with XOR-swizzled LDS positions; a new domain uses 1 up to
 * 2^20 elements and 0 above (the faster of the two at each size).  All compute
 * the same canonical outputs.  Returns 0 (nothing changed) for other values. */
TACHYON_C_EXPORT int tachyon_mi355x_bn254_univariate_evaluation_domain_set_variant(
    tachyon_bn254_univariate_evaluation_domain* domain, int variant);
/* One process, several GPUs: later transforms of the plain domain (offset 1;
 * a coset keeps the single device) through the fft/ifft entry points above,
 * transform_host and transform_device run the four-step NTT over `count`
 * devices (ids may repeat: logical devices sharing a GPU) -- part g on ids[g],
 * the all-to-all as peer copies over xGMI, input and output in natural order
 * on the device the domain was created on (transform_device: a buffer there).
 * The four-step splits by a power of two: the first 2^k ids are used, the
 * largest 2^k <= count with 2^k <= 2^floor(log n / 2) (_devices reports
 * them); count <= 1 restores the single device, and so does 2^k = 2: two
 * parts exchange n/4 elements over ONE xGMI link, which takes longer than
 * the whole transform on one MI355X (2^24: 134 MB at <= 153 GB/s >= 0.9 ms
 * plus 2 x 0.55 ms of local stages, against 1.84 ms) -- from four parts the
 * all-to-all spreads over 3+ links and the split pays.  Returns 1, or 0 (nothing
 * changed) for a bad id, a domain too small for two parts, or when the
 * generator set active now differs from the domain's (the plans would use
 * another root).  Same results as one device. */
TACHYON_C_EXPORT int tachyon_mi355x_bn254_univariate_evaluation_domain_set_devices(
    tachyon_bn254_univariate_evaluation_domain* domain, const int* ids, size_t count);
/* the device list of set_devices (0 = single device); writes up to cap ids */
TACHYON_C_EXPORT size_t tachyon_mi355x_bn254_univariate_evaluation_domain_devices(
    const tachyon_bn254_univariate_evaluation_domain* domain, int* ids, size_t cap);
TACHYON_C_EXPORT int tachyon_mi355x_bn254_univariate_evaluation_domain_last_timings(
    const tachyon_bn254_univariate_evaluation_domain* domain, float* total_ms, float* pass_ms, int max_passes);

/* Distributed four-step NTT over 2^log_world ranks (no
 * reference counterpart -- icicle's NTT is single-GPU).  One plan per rank;
 * rank r holds the columns c in [r C/G, (r+1) C/G) of the R x C view of the
 * input (R = 2^floor(log_n/2)), column-major: in[c_l R + r'] = x[C r' + c],
 * and produces rows k1 in [r R/G, (r+1) R/G) of the output, row-major:
 * out[k1_l C + k2] = X[k1 + R k2].  A transform is
 *   stage(1, in -> send); all-to-all(send -> recv) by the caller; stage(2, recv -> out)
 * with send/recv = G chunks of local_size/G elements (chunk h to/from rank h).
 * The inverse maps the output layout back to the input layout (n^-1 included).
 *
 * Ordering contract.  Every stage is enqueued on the plan's stream (`stream`
 * at create, a hipStream_t; NULL = a non-blocking stream the plan owns;
 * _stream returns it) and returns without synchronising.  The stages wait for
 * nothing else: the caller (1) makes the plan's stream wait for whatever
 * produced d_in (hipEventRecord on the producer + hipStreamWaitEvent, or
 * produce it on the plan's stream), (2) runs its all-to-all on the plan's
 * stream -- e.g. ncclAllToAll / RCCL with that stream -- or orders it after
 * stage 1 with an event, and (3) does the same before reading d_out.  A
 * non-blocking stream does not order against the legacy NULL stream, so
 * "same stream" must be meant literally.  tachyon_amd.dist.sharded_ntt keeps
 * the contract (tests/test_gpu_dist.py produces the input on another stream). */
typedef struct tachyon_mi355x_bn254_ntt4 tachyon_mi355x_bn254_ntt4;
TACHYON_C_EXPORT tachyon_mi355x_bn254_ntt4* tachyon_mi355x_bn254_ntt4_create(uint32_t log_n, uint32_t log_world,
                                                                            uint32_t rank, void* stream);
/* The same plan with R = 2^log_r (1 <= log_r < log_n, R and C = n / R >= G):
 * the layouts above with that R.  _split_log_r returns the split with the
 * fewest pass launches (passes of <= 8 stages; ties: the larger R up to C),
 * e.g. 2^24 -> R = 2^8, C = 2^16: one pass for the column NTTs (several
 * columns per workgroup) and two for the rows, against 2 + 2 for 2^12 x 2^12.
 * _log_rows returns a plan's log R. */
TACHYON_C_EXPORT tachyon_mi355x_bn254_ntt4* tachyon_mi355x_bn254_ntt4_create_split(uint32_t log_n, uint32_t log_r,
                                                                                  uint32_t log_world, uint32_t rank,
                                                                                  void* stream);
TACHYON_C_EXPORT uint32_t tachyon_mi355x_bn254_ntt4_log_rows(const tachyon_mi355x_bn254_ntt4* plan);
TACHYON_C_EXPORT uint32_t tachyon_mi355x_ntt4_split_log_r(uint32_t log_n, uint32_t log_world);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_ntt4_destroy(tachyon_mi355x_bn254_ntt4* plan);
TACHYON_C_EXPORT size_t tachyon_mi355x_bn254_ntt4_local_size(const tachyon_mi355x_bn254_ntt4* plan);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_ntt4_stage(tachyon_mi355x_bn254_ntt4* plan, int stage, int inverse,
                                                      const tachyon_bn254_fr* d_in, tachyon_bn254_fr* d_out);
TACHYON_C_EXPORT void tachyon_mi355x_bn254_ntt4_synchronize(tachyon_mi355x_bn254_ntt4* plan);
TACHYON_C_EXPORT void* tachyon_mi355x_bn254_ntt4_stream(const tachyon_mi355x_bn254_ntt4* plan);
/* A/B (every variant gives the same bytes): bit 0 = the round-4 stages (an
 * input copy, the passes, a separate twiddle kernel) instead of the exchange's
 * twiddle and packing fused into the sub-transforms' passes; bit 1 = the
 * sub-transforms on the 8 x 32-bit-limb passes instead of their size's
 * default (29-bit up to 2^20); bit 2 = one column per workgroup in one-pass
 * sub-transforms (no packing); bit 3 = the exchange twiddles computed in the
 * pass instead of read from the plan's precomputed table.  Returns 0 for other
 * values. */
TACHYON_C_EXPORT int tachyon_mi355x_bn254_ntt4_set_variant(tachyon_mi355x_bn254_ntt4* plan, int variant);

/* ---- field-generic radix-2 NTT domains --------------------------------------
 * Radix2EvaluationDomain<F> FFT / IFFT on the GPU for the scalar fields the
 * reference's icicle backend covers: field 1 = bn254 Fr (IcicleNTT<bn254::Fr>,
 * icicle_ntt_bn254.cc:31-116), 3 = bls12_381 Fr (IcicleNTT<bls12_381::Fr>,
 * icicle_ntt_bls12_381.cc:31-115).  Elements are the field's 4 x uint64
 * Montgomery limbs (tachyon_bn254_fr / tachyon_bls12_381_fr).  size =
 * bit_ceil(num_coeffs); the root is the field's two-adic root squared down
 * (bn254 Fr: the generator set active at creation, halo2 override included).
 * _set_offset: the coset h * <w> of later transforms (NULL or 1 = the plain
 * domain; GetCoset, univariate_evaluation_domain.h:102-117).
 * _transform_host: IcicleNTT::Run -- in place on a host vector of exactly
 * size() elements, natural order, forward (coefficients -> evaluations) or
 * inverse (n^-1 and the coset included); synchronous.  _transform_device:
 * `batch` consecutive device arrays in place, enqueued on _stream.  Returns
 * NULL from _create for another field id; failures abort. */
typedef struct tachyon_mi355x_ntt_domain tachyon_mi355x_ntt_domain;
TACHYON_C_EXPORT tachyon_mi355x_ntt_domain* tachyon_mi355x_ntt_domain_create(int field, size_t num_coeffs);
TACHYON_C_EXPORT void tachyon_mi355x_ntt_domain_destroy(tachyon_mi355x_ntt_domain* d);
TACHYON_C_EXPORT size_t tachyon_mi355x_ntt_domain_size(const tachyon_mi355x_ntt_domain* d);
TACHYON_C_EXPORT int tachyon_mi355x_ntt_domain_field(const tachyon_mi355x_ntt_domain* d);
TACHYON_C_EXPORT void tachyon_mi355x_ntt_domain_group_gen(const tachyon_mi355x_ntt_domain* d, void* out);
TACHYON_C_EXPORT void tachyon_mi355x_ntt_domain_set_offset(tachyon_mi355x_ntt_domain* d, const void* offset);
TACHYON_C_EXPORT void tachyon_mi355x_ntt_domain_transform_host(tachyon_mi355x_ntt_domain* d, void* inout, size_t len,
                                                              int inverse);
TACHYON_C_EXPORT void tachyon_mi355x_ntt_domain_transform_device(tachyon_mi355x_ntt_domain* d, void* d_data,
                                                                size_t batch, int inverse);
TACHYON_C_EXPORT void* tachyon_mi355x_ntt_domain_stream(tachyon_mi355x_ntt_domain* d);

/* ---- communicators and library-level sharded entry points ------------------
 * One process per MI355X: a multi-process C/C++ caller (benchmark/msm/
 * msm_benchmark_gpu.cc:57-69 or vendors/circom/prover_main.cc:116-128 under a
 * launcher) hands the library a communicator and the library does the
 * exchange itself.  Backends:
 *   rccl -- RCCL over xGMI: _comm_init_rccl (ncclCommInitRank on the current
 *     device from a 128-byte ncclUniqueId that rank 0 got from
 *     _comm_unique_id and shared) or _comm_from_rccl (wrap the caller's
 *     ncclComm_t, not owned).  All-gathers are ncclAllGather, the NTT
 *     all-to-all one ncclGroupStart/End of ncclSend/ncclRecv pairs on the
 *     plan's stream.
 *   host -- the HOST-STAGED FALLBACK (_comm_create_host): two callbacks
 *     exchange host buffers (all_gather: every rank's `bytes` in rank order;
 *     all_to_all: world blocks of `bytes`, block h to / from rank h); device
 *     data are staged through the host.  For ranks RCCL refuses (two ranks on
 *     one GPU: "Duplicate GPU detected") and CPU rehearsal backends (gloo). */
typedef struct tachyon_mi355x_comm tachyon_mi355x_comm;
typedef int (*tachyon_mi355x_all_gather_fn)(void* user, const void* send, void* recv, size_t bytes);
typedef int (*tachyon_mi355x_all_to_all_fn)(void* user, const void* send, void* recv, size_t bytes);
/* writes the 128-byte ncclUniqueId to out (cap >= 128); returns its size or 0 */
TACHYON_C_EXPORT int tachyon_mi355x_comm_unique_id(void* out, size_t cap);
TACHYON_C_EXPORT tachyon_mi355x_comm* tachyon_mi355x_comm_init_rccl(const void* unique_id, int world, int rank);
TACHYON_C_EXPORT tachyon_mi355x_comm* tachyon_mi355x_comm_from_rccl(void* nccl_comm);
TACHYON_C_EXPORT tachyon_mi355x_comm* tachyon_mi355x_comm_create_host(int world, int rank,
                                                                     tachyon_mi355x_all_gather_fn all_gather,
                                                                     tachyon_mi355x_all_to_all_fn all_to_all,
                                                                     void* user);
TACHYON_C_EXPORT void tachyon_mi355x_comm_destroy(tachyon_mi355x_comm* comm);
/* every rank's `bytes` of host memory, gathered in rank order into recv
 * (world x bytes): the exchange the sharded entries use, for callers that
 * combine their own partial results */
TACHYON_C_EXPORT void tachyon_mi355x_comm_all_gather(tachyon_mi355x_comm* comm, const void* send, void* recv,
                                                    size_t bytes);
TACHYON_C_EXPORT int tachyon_mi355x_comm_world(const tachyon_mi355x_comm* comm);
TACHYON_C_EXPORT int tachyon_mi355x_comm_rank(const tachyon_mi355x_comm* comm);
TACHYON_C_EXPORT const char* tachyon_mi355x_comm_backend(const tachyon_mi355x_comm* comm);
/* The four-step NTT of this rank's slab: stage 1, the all-to-all over `comm`,
 * stage 2 (layouts as _ntt4_stage; plan world/rank must be comm's).  Ordered
 * on the plan's stream; d_out is ready there (the host backend returns with
 * the exchange done and stage 2 enqueued). */
TACHYON_C_EXPORT void tachyon_mi355x_bn254_ntt4_run(tachyon_mi355x_bn254_ntt4* plan, tachyon_mi355x_comm* comm,
                                                   int inverse, const tachyon_bn254_fr* d_in,
                                                   tachyon_bn254_fr* d_out);

/* G2 MSM contexts (Groth16's B-in-G2, BLS12-381 config 4); same semantics as
 * the G1 *_msm_gpu entry points. */
typedef struct tachyon_bn254_g2_msm_gpu* tachyon_bn254_g2_msm_gpu_ptr;
typedef struct tachyon_bls12_381_g2_msm_gpu* tachyon_bls12_381_g2_msm_gpu_ptr;
TACHYON_C_EXPORT tachyon_bn254_g2_msm_gpu_ptr tachyon_bn254_g2_create_msm_gpu(uint8_t degree);
TACHYON_C_EXPORT void tachyon_bn254_g2_destroy_msm_gpu(tachyon_bn254_g2_msm_gpu_ptr ptr);
TACHYON_C_EXPORT tachyon_bn254_g2_jacobian* tachyon_bn254_g2_affine_msm_gpu(
    tachyon_bn254_g2_msm_gpu_ptr ptr, const tachyon_bn254_g2_affine* bases, const tachyon_bn254_fr* scalars,
    size_t size);
TACHYON_C_EXPORT tachyon_bls12_381_g2_msm_gpu_ptr tachyon_bls12_381_g2_create_msm_gpu(uint8_t degree);
TACHYON_C_EXPORT void tachyon_bls12_381_g2_destroy_msm_gpu(tachyon_bls12_381_g2_msm_gpu_ptr ptr);
TACHYON_C_EXPORT tachyon_bls12_381_g2_jacobian* tachyon_bls12_381_g2_affine_msm_gpu(
    tachyon_bls12_381_g2_msm_gpu_ptr ptr, const tachyon_bls12_381_g2_affine* bases,
    const tachyon_bls12_381_fr* scalars, size_t size);

/* Curve-generic extension API.  curve: 0 bn254_g1, 1 bn254_g2, 2 bls12_381_g1,
 * 3 bls12_381_g2.  A context is any *_msm_gpu_ptr / *_msm_ptr of that curve. */
/* Affine result written to out_affine (identity = all zero bytes). */
TACHYON_C_EXPORT void tachyon_mi355x_msm_gpu_affine(int curve, void* ctx, const void* bases, const void* scalars,
                                                    size_t size, void* out_affine);
/* The windows [w_begin, w_end) of the MSM only (window bits: the context's
 * set_window_bits, else the size's default; W = ceil((bits + 1) / c)):
 * sum over them of 2^(c w) * S_w, S_w = window w's bucket sum
 * (pippenger_base.h:59-77 restricted to the range).  Ranges that tile
 * [0, W) sum to the full MSM -- the multi-GPU window split, every rank
 * holding all points.  Affine result as in _msm_gpu_affine. */
TACHYON_C_EXPORT void tachyon_mi355x_msm_gpu_window_range_affine(int curve, void* ctx, const void* bases,
                                                                 const void* scalars, size_t size,
                                                                 unsigned w_begin, unsigned w_end,
                                                                 void* out_affine);
/* `count` MSMs over the same `len` bases (device memory of the current
 * device, e.g. a KZG SRS) in one recode / sort / accumulation / reduction:
 * MSM g takes scalars[g len, (g+1) len) (host or device; zero scalars pad
 * shorter ones) and writes its affine result to out_affine[g].  Runs on the
 * context's own device even after set_devices (the bases live there).  Window
 * bits: set_window_bits if forced, else 8 up to 2^13 points per MSM and 10
 * from 2^14 (or one MSM's default where larger).  Returns 1, or 0 (nothing
 * written) when the bases are not device memory; count x len must stay below
 * 2^31 and count at most 4096 (else the call aborts with a message, as
 * every failure of this library does). */
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_batch_affine(int curve, void* ctx, const void* bases, size_t len,
                                                        const void* scalars, size_t count, void* out_affine);
/* Fixed-base folding (bases known ahead, e.g. a proving key; an extension,
 * no reference counterpart -- the result is the same MSM).  _plan_windows:
 * W for `size` points under the context's window bits.  _fold_bases: from
 * `size` device-resident affine bases, `fold` x `size` affine points into
 * out_bases (device): copy k = 2^(k c W / fold) * P_i.  _folded_affine: the
 * MSM of `size` device scalars over such a table (same size, same window
 * bits), with W / fold window sums instead of W.  Both return 1, or 0
 * (nothing written) when fold does not divide W or a pointer is not device
 * memory. */
TACHYON_C_EXPORT unsigned tachyon_mi355x_msm_gpu_plan_windows(int curve, const void* ctx, size_t size);
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_fold_bases(int curve, void* ctx, const void* bases, size_t size,
                                                      unsigned fold, void* out_bases);
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_folded_affine(int curve, void* ctx, const void* folded_bases,
                                                         const void* scalars, size_t size, unsigned fold,
                                                         void* out_affine);
/* Contexts for the C++ plugin boundary (include/tachyon_mi355x_msm.h):
 * VariableBaseMSMGpu<Point>(mem_pool, stream) (variable_base_msm_gpu.h:16-18)
 * over any of the four groups, its work on `stream` (hipStream_t; NULL = a
 * stream the context owns; the call returns with the stream synchronised).
 * _run: the MSM of bases[0..n) and scalars[0..n) (host or device pointers)
 * written as `form` -- 0 affine {x,y}; 1 projective / 2 jacobian {x,y,z},
 * identity (1,1,0); 3 xyzz {x,y,zz,zzz}, identity (1,1,0,0).  Returns 1, or
 * 0 (out untouched) when bases_size != scalars_size, as IcicleMSM::Run
 * (icicle_msm_bn254_g1.cc:30-33) and PippengerAdapter (:55-59) return false. */
TACHYON_C_EXPORT void* tachyon_mi355x_msm_gpu_create(int curve, void* stream);
TACHYON_C_EXPORT void tachyon_mi355x_msm_gpu_destroy(int curve, void* ctx);
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_run(int curve, void* ctx, const void* bases, size_t bases_size,
                                               const void* scalars, size_t scalars_size, int form, void* out);
/* _run_points: the same with bases given in `base_form` -- 0 affine {x,y}, 1
 * projective {x,y,z} (x/z, y/z), 2 jacobian {x,y,z} (x/z^2, y/z^3), 3 xyzz
 * {x,y,zz,zzz} (x/zz, y/zzz); z (zz) = 0 is the identity -- normalised to
 * affine on the device by batch inversion first: VariableBaseMSM<Point> for
 * the non-affine point types the reference instantiates
 * (variable_base_msm_unittest.cc:30-33; Bucket = the point's own add type,
 * pippenger_base.h:18-28).  Returns 1, or 0 (out untouched) on a size
 * mismatch. */
/* _sharded_affine: this rank's shard (bases / scalars of `size` points, host
 * or device; 0 allowed) over `comm`: the local partial, one all-gather of
 * every rank's partial, the group sum in rank order -- every rank writes the
 * whole MSM's affine result (the kParallelTerm split, pippenger_adapter.h:82-113,
 * across processes). */
TACHYON_C_EXPORT void tachyon_mi355x_msm_gpu_sharded_affine(int curve, void* ctx, tachyon_mi355x_comm* comm,
                                                           const void* bases, const void* scalars, size_t size,
                                                           void* out_affine);
/* The partition of an n_total-point MSM over `world` ranks that this library
 * runs fastest (measured on MI355X): point shards, or the
 * hybrid of P = world / Q point groups x Q window groups -- rank r takes
 * point group r / Q ([start, start + count) of the global input) over window
 * range r % Q ([w_begin, w_end) of the W windows at window_bits).  Point
 * shards: window_groups 1, window_bits 0 (the shard's own default), w_begin 0,
 * w_end 0 (all windows).  Returns 1, or 0 for a rank outside [0, world). */
typedef struct tachyon_mi355x_msm_shard {
  size_t start, count;
  unsigned point_groups, window_groups, window_bits, w_begin, w_end;
} tachyon_mi355x_msm_shard;
TACHYON_C_EXPORT int tachyon_mi355x_msm_shard_plan(int curve, size_t n_total, int world, int rank,
                                                  tachyon_mi355x_msm_shard* out);
/* _sharded_plan_affine: this rank's part of `plan` (its point group's
 * bases / scalars, `plan->count` points, host or device) over `comm`: the
 * windows [w_begin, w_end) at window_bits (all windows and the shard's
 * default bits for a point shard), one all-gather of every rank's partial
 * and their group sum -- every rank writes the whole MSM's affine result and
 * returns 1.  A rank whose local part fails still enters the exchange with a
 * failure flag, so no rank is left waiting in the collective: then EVERY rank
 * returns 0 (out untouched, the message on stderr) instead of aborting. */
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_sharded_plan_affine(int curve, void* ctx, tachyon_mi355x_comm* comm,
                                                                const tachyon_mi355x_msm_shard* plan,
                                                                const void* bases, const void* scalars,
                                                                void* out_affine);
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_run_points(int curve, void* ctx, const void* bases, size_t bases_size,
                                                      int base_form, const void* scalars, size_t scalars_size,
                                                      int form, void* out);
TACHYON_C_EXPORT void tachyon_mi355x_msm_gpu_set_window_bits(int curve, void* ctx, unsigned c);
TACHYON_C_EXPORT void tachyon_mi355x_msm_gpu_set_profile(int curve, void* ctx, int on);
/* kernel-variant bits for A/B tuning in one process (0 = default schedule).
 * Every accepted variant computes the same MSM; returns 0 (nothing changed)
 * for bits outside 0x3FFFFBF (bits 0-25 but 6; bit 23: two-level window sums
 * for the G2 / BLS12-381 G1 / FIPS reductions, measured slower; bit 24: the
 * G2 window segment sums in two passes; bit 25: the limb-field G1
 * accumulations read their entries by 8-byte loads, not LDS-staged chunks). */
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_set_variant(int curve, void* ctx, int variant);
/* device ms of the last run with profiling on: h2d, recode, sort, prep (bounds +
 * chunk scan), acc (the bucket-accumulation kernel alone), reduce, total,
 * accumulation launches (8 floats; of the last point chunk when the run was divided) */
TACHYON_C_EXPORT void tachyon_mi355x_msm_gpu_last_timings(int curve, const void* ctx, float* out8);
/* Point chunks the last run was split into: > 1 when the working set did not
 * fit the free device memory (DetermineMsmDivisionsForMemory,
 * icicle_msm_utils.cc:10-68; TACHYON_MSM_MEM_LIMIT caps the free bytes) or when
 * host-resident inputs were uploaded chunk by chunk under the kernels. */
TACHYON_C_EXPORT size_t tachyon_mi355x_msm_gpu_last_divisions(int curve, const void* ctx);
/* Schedule of the last run (of its last point chunk): bit 0 the recode fused
 * with the first radix pass, bit 1 onesweep passes fed by the recode's digit
 * counts, bit 2 7-byte LDS staging in the recode scatter, bit 3 an
 * accumulation over the 29-bit-limb field (BN254 G1; BN254 G2's lane pair),
 * bit 4 the lane-pair G2 accumulation, bit 5 over the 28-bit-limb field
 * (BLS12-381 G1 / G2), bit 6 the chain-flag debug check ran, bit 7 the
 * limb-field accumulation read its sorted entries through LDS (64-byte chunks
 * by LDS-DMA; BN254 / BLS12-381 G1, BLS12-381 G2). */
TACHYON_C_EXPORT unsigned tachyon_mi355x_msm_gpu_last_schedule(int curve, const void* ctx);
/* Diagnostic: mixed additions per second (G/s) of the curve's bucket
 * accumulation field code in registers on the current device (no gathers, no
 * bucket runs; ~0.1 s): the VALU ceiling the bench prices the accumulation
 * against.  field_bits: BN254 G1 29 (its 29-bit-limb field) or 32 (FIPS);
 * BLS12-381 G1 28 (14 x 28-bit limbs); BN254 G2 29 / BLS12-381 G2 28 (the
 * lane-pair Fq2 of the G2 accumulation, whole G2 additions, two lanes each);
 * returns 0 for other widths. */
TACHYON_C_EXPORT double tachyon_mi355x_msm_madd_ceiling(int curve, int field_bits);
/* One process, several MI355X: every later MSM of this context splits its
 * points into `count` contiguous shards, shard k on device device_ids[k]
 * (its own host thread and stream; host inputs are uploaded per shard over
 * that device's link, device inputs owned by another device are copied
 * peer-to-peer), and adds the shard results on the host -- the reference's
 * kParallelTerm chunk-and-sum (pippenger_adapter.h:82-113) and its GPU
 * divisions loop (icicle_msm_bn254_g1.cc:50-73), across devices.  The
 * reference pins device 0 (msm_gpu.h:54-56); with this, benchmark/msm and the
 * scroll_halo2 bridge reach every GPU without torch.  Ids may repeat (several
 * shards on one GPU).  count <= 1 returns to the context's own device.
 * Returns 1, or 0 (nothing changed) for an id outside [0, device count).
 * Environment: TACHYON_MSM_GPU_DEVICES="0,1,2,3" applies it to every new
 * context (the C-ABI create functions included). */
TACHYON_C_EXPORT int tachyon_mi355x_msm_gpu_set_devices(int curve, void* ctx, const int* device_ids, size_t count);
/* The shards of the last multi-device run: for each (up to cap) its wall ms
 * (upload or peer copy + MSM), point count and device; returns the number of
 * shards (0 for a single-device context).  Any output pointer may be NULL. */
TACHYON_C_EXPORT size_t tachyon_mi355x_msm_gpu_last_shards(int curve, const void* ctx, float* shard_ms,
                                                           size_t* shard_points, int* shard_devices, size_t cap);
/* window bits / windows the planner picks for `size` points */
TACHYON_C_EXPORT void tachyon_mi355x_msm_plan(int curve, size_t size, unsigned* c, unsigned* windows);
/* Host-side group arithmetic on affine points (multi-GPU partial sums):
 * out = sum of `count` affine points. */
TACHYON_C_EXPORT void tachyon_mi355x_affine_sum(int curve, const void* points, size_t count, void* out_affine);
/* Jacobian -> affine. */
TACHYON_C_EXPORT void tachyon_mi355x_jacobian_to_affine(int curve, const void* jacobian, void* out_affine);

/* Synthetic inputs generated on the device (bench / tests):
 *   scalars: splitmix64 counter stream, BigInt::Random halving, Montgomery
 *   bases:   chunks of `chunk` points, chunk j = k_j * G, 2 k_j * G, 4 k_j * G ...
 * field: 1 bn254_fr, 3 bls12_381_fr.  d_out is device memory. stream may be NULL. */
TACHYON_C_EXPORT void tachyon_mi355x_gen_scalars(int field, uint64_t seed, size_t start, size_t n, void* d_out,
                                                 void* stream);
TACHYON_C_EXPORT void tachyon_mi355x_gen_bases(int curve, uint64_t seed, size_t n, size_t chunk, void* d_out,
                                               void* stream);
/* points [start, start + n) of that same sequence (any start; the chunk that
 * holds `start` is advanced by doublings): a rank's shard of the global input, so N ranks compute the N = 1 MSM. */
TACHYON_C_EXPORT void tachyon_mi355x_gen_bases_at(int curve, uint64_t seed, size_t start, size_t n, size_t chunk,
                                                  void* d_out, void* stream);

/* Elementwise device parity kernels (prime_field_correctness_gpu_test.cc,
 * (non_)affine_point_correctness_gpu_test.cc).  field: 0 bn254_fq, 1 bn254_fr,
 * 2 bls12_381_fq, 3 bls12_381_fr; op: 0 add 1 sub 2 mul 3 sqr 4 neg 5 inv
 * 6 to_mont 7 from_mont 8 dbl 9 a times the plain constant b (the NTT's
 * twiddle product: Shoup on BN254 Fr/Fq, a any 256-bit value) 10 a b - b a
 * and 11 a b - a^2 through the fused one-reduction a b - c d of the XYZZ
 * y coordinates.  Host buffers in, host buffer out. */
TACHYON_C_EXPORT void tachyon_mi355x_field_op(int field, int op, const void* a, const void* b, void* out,
                                              size_t count);
/* point op: 0 add (affine + affine), 1 double, 2 add-mixed into xyzz of a. Affine in/out. */
TACHYON_C_EXPORT void tachyon_mi355x_ec_op(int curve, int op, const void* a, const void* b, void* out, size_t count);

/* Groth16 prover over a circom zkey (no reference C-ABI --
 * the reference drives this path from C++: vendors/circom/prover_main.cc:82-160,
 * QuadraticArithmeticProgram::WitnessMapFromMatrices
 * (quadratic_arithmetic_program.h:24-113), CreateProofWithAssignment(NoZK)
 * (tachyon/zk/r1cs/groth16/prove.h:52-186)).  The zkey bytes (v1, BN254 or
 * BLS12-381) are parsed and the proving key uploaded once at create; a proof
 * uploads only the witness.  Field elements are Montgomery form.
 *   info: out4 = {curve (0 bn254, 1 bls12_381), num_vars, num_public, domain_size}
 *   prove: full = num_vars assignments (full[0] = 1; host or device pointer),
 *          r, s = blinding scalars or NULL for zero (the NoZK proof);
 *          out_a: G1 affine, out_b: G2 affine, out_c: G1 affine (canonical).
 *   witness_map: the h evaluations on the coset (domain_size Fr) to host memory.
 *   last_timings (profiling on): upload, qap, msm_a, msm_b2, msm_b1, msm_l,
 *          msm_h, total -- ms, 8 floats (msm_l: the witness and h MSMs, run as
 *          one MSM over C1 | H1 since the proof only uses their sum; msm_h 0).
 * Multi-GPU split of prove (one process per GPU):
 *   prove_partials: this rank's shard (contiguous ceil(count / world) chunk
 *          `rank` of every MSM's points, the kParallelTerm split of
 *          pippenger_adapter.h:82-113) of the proof's MSMs, after the full
 *          witness map; writes partials_size() bytes (an opaque blob of
 *          XYZZ sums, identical layout on every rank of one build).
 *          with_b1 != 0 runs the B-in-G1 MSM (required when r != 0).
 *   assemble: `world` blobs (one per rank, any order, concatenated -- the
 *          result of one all-gather) -> the proof, as prove() would return.
 *   prove(full, r, s) == assemble(prove_partials(full, r != 0, 0, 1), 1, r, s). */
typedef struct tachyon_mi355x_groth16_prover tachyon_mi355x_groth16_prover;
TACHYON_C_EXPORT tachyon_mi355x_groth16_prover* tachyon_mi355x_groth16_prover_create(const uint8_t* zkey,
                                                                                     size_t len);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_prover_destroy(tachyon_mi355x_groth16_prover* prover);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_prover_info(const tachyon_mi355x_groth16_prover* prover,
                                                         uint32_t* out4);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_prove(tachyon_mi355x_groth16_prover* prover, const void* full,
                                                   size_t count, const void* r, const void* s, void* out_a,
                                                   void* out_b, void* out_c);
/* One-process multi-device proofs (no reference counterpart; the reference's
 * prover_main.cc:116-128 runs one process on one GPU): every later
 * tachyon_mi355x_groth16_prove runs the multi-rank split on these devices --
 * one host thread per entry runs the witness map and its 1/count chunk of
 * every MSM (_prove_partials with rank = entry, world = count), and the
 * partials are added on the host (_assemble); the proof equals the
 * single-device one.  Ids may repeat (provers sharing a GPU on separate
 * streams); count <= 1 returns to the single-device prover.  Returns 0 and
 * changes nothing when an id is out of range. */
TACHYON_C_EXPORT int tachyon_mi355x_groth16_set_devices(tachyon_mi355x_groth16_prover* prover, const int* device_ids,
                                                        size_t count);
TACHYON_C_EXPORT size_t tachyon_mi355x_groth16_partials_size(const tachyon_mi355x_groth16_prover* prover);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_prove_partials(tachyon_mi355x_groth16_prover* prover, const void* full,
                                                            size_t count, int with_b1, uint32_t rank,
                                                            uint32_t world, void* out);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_assemble(tachyon_mi355x_groth16_prover* prover, const void* parts,
                                                      size_t world, const void* r, const void* s, void* out_a,
                                                      void* out_b, void* out_c);
/* The proof across the ranks of `comm` (one process per GPU): every rank runs
 * the witness map and its chunk of every MSM (_prove_partials with the
 * comm's rank / world), one all-gather of the partials blobs, and the same
 * assembly -- every rank writes the same proof, equal to the single-GPU one. */
TACHYON_C_EXPORT void tachyon_mi355x_groth16_prove_sharded(tachyon_mi355x_groth16_prover* prover,
                                                          tachyon_mi355x_comm* comm, const void* full, size_t count,
                                                          const void* r, const void* s, void* out_a, void* out_b,
                                                          void* out_c);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_witness_map(tachyon_mi355x_groth16_prover* prover, const void* full,
                                                         size_t count, void* out_h);
/* Proving-key setup (no reference counterpart: the reference keeps no
 * per-key device state): builds the fixed-base fold tables the proofs of
 * shard (rank, world) use -- B in G2, the grouped A + witness/h G1 MSM (one
 * device) or A / B1 / witness+h (shards) -- each at the largest fold up to
 * the variant's that fits the device next to the MSM's working set
 * (TACHYON_MSM_MEM_LIMIT caps the free bytes, as for the MSM); no table
 * (fold 1) runs plain MSMs, and a grouped MSM that does not fit runs as
 * separate MSMs.  Proofs without it prepare themselves on first use.  After
 * set_devices it prepares every device's prover for its entry of the split.
 * Returns the table bytes held (summed over devices); _prover_folds writes
 * the folds chosen by the last prepare: B2, grouped G1 (0 = separate MSMs),
 * A, B1 (0 = not built), witness + h (0 = grouped). */
TACHYON_C_EXPORT size_t tachyon_mi355x_groth16_prepare(tachyon_mi355x_groth16_prover* prover, uint32_t rank,
                                                       uint32_t world, int with_b1);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_prover_folds(const tachyon_mi355x_groth16_prover* prover,
                                                          uint32_t* out5);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_set_profile(tachyon_mi355x_groth16_prover* prover, int on);
/* A/B: variant bit 0 runs A and the witness + h MSM as two MSMs (round 4);
 * clear (default) as one grouped MSM over their own bases (one recode / sort
 * / accumulation / reduction; single-device proofs).  Bits 1-3 pick the fold
 * of the G2 B query (a table of its points times 2^(k c W / F), built on the
 * first proof; _msm_gpu_fold_bases), bits 4-6 the fold of the grouped G1
 * MSM's bases: 0 the default (B2 16 copies, G1 4), k = 1..5 2^(k-1) copies (1 =
 * none), each lowered to the largest power of two dividing the MSM's window
 * count.  Same proof for every variant; returns 0 for other values. */
TACHYON_C_EXPORT int tachyon_mi355x_groth16_set_variant(tachyon_mi355x_groth16_prover* prover, int variant);
/* Window bits of the proof's MSMs (0 = each MSM's size default): A (and B in
 * G1), the merged witness + h MSM, B in G2.  Tuning / A/B; the proof is the
 * same for every choice. */
TACHYON_C_EXPORT void tachyon_mi355x_groth16_set_msm_window_bits(tachyon_mi355x_groth16_prover* prover, unsigned c_a,
                                                               unsigned c_lh, unsigned c_b2);
TACHYON_C_EXPORT void tachyon_mi355x_groth16_last_timings(const tachyon_mi355x_groth16_prover* prover,
                                                          float* out8);
/* zkey curve (0 bn254, 1 bls12_381) without building a prover. */
TACHYON_C_EXPORT int tachyon_mi355x_zkey_curve(const uint8_t* zkey, size_t len);
/* wtns v2 -> Montgomery field elements of the curve's scalar field
 * (wtns.h:99-117).  Writes min(count, cap) elements to out (may be NULL);
 * returns the witness count. */
TACHYON_C_EXPORT size_t tachyon_mi355x_wtns_parse(int curve, const uint8_t* wtns, size_t len, void* out,
                                                  size_t cap);

/* KZG commitments with a device-resident SRS (the reference's
 * tachyon/crypto/commitments/kzg/kzg.h is C++ only).  curve: 0 bn254_g1,
 * 2 bls12_381_g1.  Field elements Montgomery form, points affine.
 *   unsafe_setup: size a power of two; SRS = [tau^i] G and [L_i(tau)] G over
 *     the size-n domain (UnsafeSetup :173-207), built and kept on the device;
 *   downsize: returns 0 if n >= N (Downsize :210-215);
 *   get_srs: the N points (lagrange = 0 powers of tau, 1 Lagrange) to host;
 *   commit: MSM of the first len SRS points with `scalars` (host or device
 *     pointer) -- Commit (lagrange = 0) / CommitLagrange (1), :217-258.
 *     Returns 1, or 0 with out_affine untouched when len > N (the reference
 *     returns false: DoMSM trims the bases to min(N, len), then the MSM
 *     refuses bases/scalars of different sizes, :267-290). */
typedef struct tachyon_mi355x_kzg tachyon_mi355x_kzg;
TACHYON_C_EXPORT tachyon_mi355x_kzg* tachyon_mi355x_kzg_create(int curve);
TACHYON_C_EXPORT void tachyon_mi355x_kzg_destroy(tachyon_mi355x_kzg* kzg);
TACHYON_C_EXPORT void tachyon_mi355x_kzg_unsafe_setup(tachyon_mi355x_kzg* kzg, size_t size, const void* tau);
TACHYON_C_EXPORT size_t tachyon_mi355x_kzg_n(const tachyon_mi355x_kzg* kzg);
TACHYON_C_EXPORT int tachyon_mi355x_kzg_downsize(tachyon_mi355x_kzg* kzg, size_t n);
TACHYON_C_EXPORT void tachyon_mi355x_kzg_get_srs(const tachyon_mi355x_kzg* kzg, int lagrange, void* out);
TACHYON_C_EXPORT int tachyon_mi355x_kzg_commit(tachyon_mi355x_kzg* kzg, int lagrange, const void* scalars,
                                               size_t len, void* out_affine);
/* Batch commitments (ResizeBatchCommitments / Commit(v, state, index) /
 * GetBatchCommitments, kzg.h:116-165,296-307): `count` polynomials,
 * scalars[i] of lens[i] elements (host or device), their commitments written
 * affine to out_affine[i], normalised together with one field inversion
 * (BatchNormalize).  Polynomials of similar length run as batched MSMs
 * (groups closed when zero-padding would more than double their work or at
 * the batched MSM's size limits), the rest as single MSMs: any count and any
 * mix of lengths <= N is accepted.  Returns 1, or 0 (nothing written) when
 * any lens[i] > N. */
TACHYON_C_EXPORT int tachyon_mi355x_kzg_commit_batch(tachyon_mi355x_kzg* kzg, int lagrange,
                                                     const void* const* scalars, const size_t* lens, size_t count,
                                                     void* out_affine);

/* delete a Jacobian returned by an *_msm / *_msm_gpu entry point (for callers
 * that cannot use C++ delete, e.g. ctypes). */
TACHYON_C_EXPORT void tachyon_mi355x_jacobian_destroy(int curve, void* jacobian);
TACHYON_C_EXPORT const char* tachyon_mi355x_version(void);
TACHYON_C_EXPORT int tachyon_mi355x_device_count(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* TACHYON_MI355X_H_ */
