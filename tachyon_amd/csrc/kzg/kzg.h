// KZG commitments with a device-resident SRS on MI355X.
//
// Reference: tachyon/crypto/commitments/kzg/kzg.h
//   :90-114   SetupForGpu -- the SRS lives in device memory next to the GPU MSM
//   :173-207  UnsafeSetup(size, tau): g1_powers_of_tau = [tau^i] G and
//             g1_powers_of_tau_lagrange = [L_i(tau)] G over the size-n domain
//             (BatchMapScalarFieldToPoint, affine_point.h:184-206;
//             EvaluateAllLagrangeCoefficients, univariate_evaluation_domain.h:279-360)
//   :210-215  Downsize(n): false if n >= N
//   :217-258  Commit / CommitLagrange = MSM over the first min(N, |v|) SRS points
//   :267-313  DoMSM (batch commitments: one MSM per polynomial into a slot)
// Both SRS vectors are built on the GPU: per-element tau^i and L_i(tau)
// (Fermat inverse per element), then a fixed-base double-and-add per point.
#pragma once
#include <hip/hip_runtime.h>

#include <memory>

#include "../common/hip_util.h"
#include "../msm/msm.h"

namespace tachyon_amd::kzg {

template <class Curve>
class Kzg {
 public:
  using F = typename Curve::F;
  using Fr = typename Curve::Fr;
  using Aff = Affine<F>;

  explicit Kzg(hipStream_t stream = nullptr);
  ~Kzg();
  Kzg(const Kzg&) = delete;
  Kzg& operator=(const Kzg&) = delete;

  // size must be a power of two (the Lagrange basis is over the radix-2 domain)
  void unsafe_setup(size_t size, const Fr& tau);
  size_t n() const { return n_; }
  bool downsize(size_t n);

  // MSM of the first len SRS points with `scalars` (host or device).  False,
  // with *out untouched, when len > N (the reference's DoMSM trims the bases
  // to min(|bases|, |scalars|) and PippengerAdapter then refuses unequal
  // sizes, so Commit / CommitLagrange return false, kzg.h:217-258,267-290).
  bool commit(const Fr* scalars, size_t len, bool lagrange, Aff* out);
  // Batch mode (ResizeBatchCommitments / Commit(v, state, index) /
  // GetBatchCommitments, kzg.h:116-165,296-307): one MSM per polynomial, the
  // results kept projective (XYZZ) and normalised together with ONE field
  // inversion (BatchNormalize's Montgomery trick, projective_point.h).  False,
  // with out untouched, when any len > N.
  bool commit_batch(const Fr* const* scalars, const size_t* lens, size_t count, bool lagrange, Aff* out);

  const Aff* d_srs(bool lagrange) const { return lagrange ? lagrange_.as<Aff>() : powers_.as<Aff>(); }
  void copy_srs(bool lagrange, Aff* host_out) const;
  hipStream_t stream() const { return stream_; }

 private:
  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  size_t n_ = 0;
  DeviceBuffer powers_, lagrange_, scratch_;
  DeviceBuffer batch_;  // commit_batch: the zero-padded count x len scalars
  std::unique_ptr<msm::MsmGpu<Curve>> msm_;
};

extern template class Kzg<Bn254G1>;
extern template class Kzg<Bls381G1>;

}  // namespace tachyon_amd::kzg
