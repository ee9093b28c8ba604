/* C++ plugin boundary of the MI355X MSM backend: Tachyon's
 * tachyon::math::VariableBaseMSMGpu<Point> and VariableBaseMSM<Point>, header-
 * only over the C-ABI of libtachyon_mi355x.so.
 *
 * Replaces (same shape and semantics):
 *   VariableBaseMSMGpu<Point>   tachyon/math/elliptic_curves/msm/variable_base_msm_gpu.h:11-30
 *     ctor(gpuMemPool_t, gpuStream_t); Run(bases, cpu_scalars, ProjectivePoint<Curve>*) -> bool
 *     (IcicleMSM<Point>::Run, algorithms/icicle/icicle_msm.h:35-100 and
 *     icicle_msm_bn254_g1.cc:22-77: false when |bases| != |scalars|; bases may
 *     be host or device memory -- detected with hipPointerGetAttributes, as
 *     :37-45 does; memory divisions when the MSM does not fit, :47-72)
 *     instantiated for bn254 G1/G2 and bls12_381 G1/G2 (icicle_msm.h:78-100).
 *   VariableBaseMSM<Point>      tachyon/math/elliptic_curves/msm/variable_base_msm.h:14-38
 *     Run(bases_first, bases_last, scalars_first, scalars_last, Bucket*) and
 *     Run(const BaseContainer&, const ScalarContainer&, Bucket*) -> bool, with
 *     Bucket = PointXYZZ<Curve> for affine input and the point's own type for
 *     ProjectivePoint / JacobianPoint / PointXYZZ input (pippenger_base.h:18-28;
 *     the four base types of variable_base_msm_unittest.cc:30-33 -- non-affine
 *     bases are normalised to affine on the device by batch inversion);
 *     served by the GPU here (the reference's PippengerAdapter is the CPU
 *     oracle the tests compare against).
 *
 * Callers that keep working unchanged: Groth16 (tachyon/zk/r1cs/groth16/prove.h:
 * 64-147 builds two VariableBaseMSMGpu objects, G1 and G2, and calls Run on
 * std::vector / absl::Span arguments) and KZG (tachyon/crypto/commitments/kzg/
 * kzg.h:90-114,267-313, device-resident SRS bases).  INTEGRATION.md shows the
 * three-line change to variable_base_msm_gpu.h that routes them here.
 *
 * Types.  Point is any point type with the layout of a C-ABI struct of its
 * group (Montgomery limbs): affine {x, y} (identity (0, 0)), projective or
 * Jacobian {x, y, z} (identity z = 0) or XYZZ {x, y, zz, zzz} (identity
 * zz = 0).  The group comes from tachyon_mi355x::GroupOf<Point> and the
 * coordinate system from tachyon_mi355x::PointFormOf<Point> (affine unless
 * specialised), both specialised below for the C-ABI structs.  A Tachyon
 * build adds one line per native type, e.g.
 *   template <> struct tachyon_mi355x::GroupOf<tachyon::math::bn254::G1AffinePoint>
 *       : std::integral_constant<int, tachyon_mi355x::kBn254G1> {};
 * and for the non-affine ones also
 *   template <> struct tachyon_mi355x::PointFormOf<tachyon::math::bn254::G1JacobianPoint>
 *       : std::integral_constant<int, tachyon_mi355x::kFormJacobian> {};
 * VariableBaseMSMGpu takes affine bases only, as the reference's does.
 * Scalars: any type with the layout of tachyon_bn254_fr / tachyon_bls12_381_fr.
 * Results: any type of 3 (projective) or 4 (XYZZ) base-field coordinates.
 * Containers: anything std::data / std::size accept (std::vector, absl::Span,
 * arrays); the iterator form needs contiguous iterators.
 * Errors other than the size mismatch abort inside the library, like the
 * reference's CHECKs. */
#ifndef TACHYON_MI355X_MSM_H_
#define TACHYON_MI355X_MSM_H_

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <iterator>
#include <memory>
#include <type_traits>

#include "tachyon_mi355x.h"

namespace tachyon_mi355x {

/* group ids of the curve-generic C-ABI */
enum : int { kBn254G1 = 0, kBn254G2 = 1, kBls12_381G1 = 2, kBls12_381G2 = 3 };

/* bytes of one base-field coordinate per group (Fq or Fq2) */
constexpr size_t kCoordBytes[4] = {32, 64, 48, 96};

/* coordinate systems (the C-ABI's point forms) */
enum : int { kFormAffine = 0, kFormProjective = 1, kFormJacobian = 2, kFormXYZZ = 3 };

template <typename Point>
struct GroupOf;
template <typename Point>
struct PointFormOf : std::integral_constant<int, kFormAffine> {};
template <>
struct GroupOf<tachyon_bn254_g1_affine> : std::integral_constant<int, kBn254G1> {};
template <>
struct GroupOf<tachyon_bn254_g2_affine> : std::integral_constant<int, kBn254G2> {};
template <>
struct GroupOf<tachyon_bls12_381_g1_affine> : std::integral_constant<int, kBls12_381G1> {};
template <>
struct GroupOf<tachyon_bls12_381_g2_affine> : std::integral_constant<int, kBls12_381G2> {};
template <>
struct GroupOf<tachyon_bn254_g1_point2> : std::integral_constant<int, kBn254G1> {};
template <>
struct GroupOf<tachyon_bls12_381_g1_point2> : std::integral_constant<int, kBls12_381G1> {};
#define TACHYON_MI355X_NON_AFFINE(C, G, GROUP)                                                       \
  template <>                                                                                        \
  struct GroupOf<tachyon_##C##_##G##_projective> : std::integral_constant<int, GROUP> {};            \
  template <>                                                                                        \
  struct GroupOf<tachyon_##C##_##G##_jacobian> : std::integral_constant<int, GROUP> {};              \
  template <>                                                                                        \
  struct GroupOf<tachyon_##C##_##G##_xyzz> : std::integral_constant<int, GROUP> {};                  \
  template <>                                                                                        \
  struct PointFormOf<tachyon_##C##_##G##_projective> : std::integral_constant<int, kFormProjective> {}; \
  template <>                                                                                        \
  struct PointFormOf<tachyon_##C##_##G##_jacobian> : std::integral_constant<int, kFormJacobian> {};  \
  template <>                                                                                        \
  struct PointFormOf<tachyon_##C##_##G##_xyzz> : std::integral_constant<int, kFormXYZZ> {};
TACHYON_MI355X_NON_AFFINE(bn254, g1, kBn254G1)
TACHYON_MI355X_NON_AFFINE(bn254, g2, kBn254G2)
TACHYON_MI355X_NON_AFFINE(bls12_381, g1, kBls12_381G1)
TACHYON_MI355X_NON_AFFINE(bls12_381, g2, kBls12_381G2)
#undef TACHYON_MI355X_NON_AFFINE

namespace internal {

/* coordinates per point of each form */
constexpr size_t kCoords[4] = {2, 3, 3, 4};

/* One MSM context of the library (curve-generic C-ABI). */
template <typename Point>
class MsmContext {
 public:
  static constexpr int kGroup = GroupOf<Point>::value;
  static constexpr int kBaseForm = PointFormOf<Point>::value;
  static constexpr size_t kCoord = kCoordBytes[kGroup];
  static_assert(kBaseForm >= kFormAffine && kBaseForm <= kFormXYZZ, "unknown point form");
  static_assert(sizeof(Point) == kCoords[kBaseForm] * kCoord,
                "Point must have the layout of the group's C-ABI struct of its form");

  explicit MsmContext(hipStream_t stream) : ctx_(tachyon_mi355x_msm_gpu_create(kGroup, stream)) {}
  ~MsmContext() { tachyon_mi355x_msm_gpu_destroy(kGroup, ctx_); }
  MsmContext(const MsmContext&) = delete;
  MsmContext& operator=(const MsmContext&) = delete;

  template <typename Scalar, typename Out>
  bool Run(const Point* bases, size_t bases_size, const Scalar* scalars, size_t scalars_size, int form, Out* out) {
    static_assert(sizeof(Scalar) == 32, "Scalar must have the layout of the group's Fr");
    if constexpr (kBaseForm == kFormAffine)
      return tachyon_mi355x_msm_gpu_run(kGroup, ctx_, bases, bases_size, scalars, scalars_size, form, out) != 0;
    else
      return tachyon_mi355x_msm_gpu_run_points(kGroup, ctx_, bases, bases_size, kBaseForm, scalars, scalars_size,
                                              form, out) != 0;
  }

 private:
  void* ctx_ = nullptr;
};

}  // namespace internal

/* VariableBaseMSMGpu<Point> (variable_base_msm_gpu.h:11-30). */
template <typename Point>
class VariableBaseMSMGpu {
 public:
  /* mem_pool: accepted for signature compatibility; the context keeps its own
   * device buffers (grown once, reused).  stream: where the MSM runs. */
  VariableBaseMSMGpu(hipMemPool_t mem_pool, hipStream_t stream) : impl_(std::make_unique<Impl>(stream)) {
    (void)mem_pool;
  }
  VariableBaseMSMGpu(const VariableBaseMSMGpu& other) = delete;
  VariableBaseMSMGpu& operator=(const VariableBaseMSMGpu& other) = delete;

  /* ProjectiveResult: 3 base-field coordinates {x, y, z} (ProjectivePoint<Curve>). */
  template <typename BaseContainer, typename ScalarContainer, typename ProjectiveResult>
  [[nodiscard]] bool Run(const BaseContainer& bases, const ScalarContainer& cpu_scalars,
                         ProjectiveResult* cpu_result) {
    static_assert(Impl::kBaseForm == kFormAffine, "VariableBaseMSMGpu takes affine bases (icicle_msm.h:35-100)");
    static_assert(sizeof(ProjectiveResult) == 3 * Impl::kCoord, "result must be a projective point {x, y, z}");
    return impl_->Run(std::data(bases), std::size(bases), std::data(cpu_scalars), std::size(cpu_scalars),
                      kFormProjective, cpu_result);
  }

 private:
  using Impl = internal::MsmContext<Point>;
  std::unique_ptr<Impl> impl_;
};

/* VariableBaseMSM<Point> (variable_base_msm.h:14-38): Bucket = PointXYZZ for
 * affine bases, else the base's own form (PippengerTraits,
 * pippenger_base.h:18-28).  Results are normalised (z = 1, or the identity). */
template <typename Point>
class VariableBaseMSM {
 public:
  VariableBaseMSM() : impl_(std::make_unique<Impl>(nullptr)) {}

  template <typename BaseInputIterator, typename ScalarInputIterator, typename Bucket>
  [[nodiscard]] bool Run(BaseInputIterator bases_first, BaseInputIterator bases_last,
                         ScalarInputIterator scalars_first, ScalarInputIterator scalars_last, Bucket* ret) {
    const size_t nb = static_cast<size_t>(std::distance(bases_first, bases_last));
    const size_t ns = static_cast<size_t>(std::distance(scalars_first, scalars_last));
    return RunRaw(nb ? &*bases_first : nullptr, nb, ns ? &*scalars_first : nullptr, ns, ret);
  }

  /* Bucket: {x, y, zz, zzz} (PointXYZZ<Curve>) for affine bases; {x, y, z}
   * for projective / Jacobian bases; {x, y, zz, zzz} for XYZZ bases. */
  template <typename BaseContainer, typename ScalarContainer, typename Bucket>
  [[nodiscard]] bool Run(const BaseContainer& bases, const ScalarContainer& scalars, Bucket* ret) {
    return RunRaw(std::data(bases), std::size(bases), std::data(scalars), std::size(scalars), ret);
  }

 private:
  using Impl = internal::MsmContext<Point>;

  static constexpr int kBucketForm = Impl::kBaseForm == kFormAffine ? kFormXYZZ : Impl::kBaseForm;

  template <typename Scalar, typename Bucket>
  bool RunRaw(const Point* bases, size_t nb, const Scalar* scalars, size_t ns, Bucket* ret) {
    static_assert(sizeof(Bucket) == internal::kCoords[kBucketForm] * Impl::kCoord,
                  "Bucket must be the base's add type (PointXYZZ for affine bases)");
    return impl_->Run(bases, nb, scalars, ns, kBucketForm, ret);
  }

  std::unique_ptr<Impl> impl_;
};

}  // namespace tachyon_mi355x

#endif  // TACHYON_MI355X_MSM_H_
