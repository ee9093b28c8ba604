// Radix-2 NTT over a two-adic prime field on MI355X: host driver interface.
//
// Drop-in for the GPU hook of tachyon::math::UnivariateEvaluationDomain
// (set_icicle / IcicleNTT::Run, univariate_evaluation_domain.h:99,169-178,
// icicle_ntt_bn254.cc:68-101): natural-order input and output, Montgomery form
// end to end, optional coset offset h (GetCoset, univariate_evaluation_domain.h:102-117).
//
//   forward:  e_i = sum_j c_j (h w^i)^j
//   inverse:  c_j = n^-1 h^-j sum_i e_i w^-ij
//
// Both run the decimation-in-frequency network (the reference's
// ButterflyFnInOut form, univariate_evaluation_domain.h:518-524) in passes of
// up to 8 stages held in LDS, with the bit-reversal permutation and the
// n^-1 / coset scaling fused into the last pass.  Results are canonical field
// elements, so they equal the reference's DIT (FFT) / DIF (IFFT) CPU output
// byte for byte.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#include "../common/hip_util.h"
#include "../field/ff.h"

namespace tachyon_amd::ntt {

struct NttTimings {
  float total = 0;
  std::vector<float> passes;
};

// The four-step's exchange fused into a domain's passes (Ntt4Step): element
// k of batch entry b (the rank's local column c_l) is multiplied by
// w_N^(+-(c0 + b) k) (two-level power tables lo / hi of N = 2^log_n, split at
// `bits`) and read from / written to its packed position
// ((k >> log_rg) << log_cg + b) << log_rg | (k mod 2^log_rg).
template <class Fr>
struct FourStepTw {
  const Fr* lo = nullptr;
  const Fr* hi = nullptr;
  uint32_t bits = 0, log_n = 0, log_rg = 0, log_cg = 0, c0 = 0;
  // BN254 Fr 29-bit passes: the rank's twiddles w_N^(+-(c0 + c_l) k1)
  // precomputed in R'-form (fr29::TwMont29, entry c_l << log_r | k1): one
  // 36-byte read and one product per element instead of two table reads and
  // two Montgomery products (nullptr: computed in the pass)
  const void* tab29 = nullptr;
  uint32_t log_r = 0;
  // 1: the row NTTs of the exchange (forward stage 2 reads, inverse stage 1
  // writes the exchange layout directly: no transpose); 0: the column NTTs
  uint32_t rows = 0;
};

template <class Fr>
class NttDomain {
 public:
  // size = bit_ceil(num_coeffs) (Radix2EvaluationDomain::Create, radix2_evaluation_domain.h:83-89)
  explicit NttDomain(size_t num_coeffs, hipStream_t stream = nullptr);
  ~NttDomain();
  NttDomain(const NttDomain&) = delete;
  NttDomain& operator=(const NttDomain&) = delete;

  size_t size() const { return n_; }
  uint32_t log_size() const { return log_n_; }
  const Fr& group_gen() const { return omega_; }
  const Fr& group_gen_inv() const { return omega_inv_; }
  const Fr& size_inv() const { return size_inv_; }
  hipStream_t stream() const { return stream_; }

  // Coset offset h (Montgomery).  h == 1 restores the plain domain.
  void set_offset(const Fr& h);
  const Fr& offset() const { return offset_; }

  // In-place transform of `batch` consecutive arrays of n device-resident
  // elements (d_data), enqueued on stream(); scratch is owned by the domain.
  // Not synchronised.
  void forward_device(Fr* d_data, size_t batch = 1);
  void inverse_device(Fr* d_data, size_t batch = 1);
  // Out of place (`src` read by the first pass, `dst` written by the last;
  // dst may equal src) with the four-step's twiddle and packed layout fused
  // (fs: forward -> into the last pass's store, inverse -> into the first
  // pass's load; null = plain batched layout).
  void transform_device(const Fr* src, Fr* dst, bool inverse, size_t batch, const FourStepTw<Fr>* fs);

  // Host vector in/out: `len` <= n input elements, zero-padded to n; writes n
  // outputs to `out` (may alias `in`).  Synchronises.
  void forward_host(const Fr* in, size_t len, Fr* out);
  void inverse_host(const Fr* in, size_t len, Fr* out);

  void set_profile(bool on) { profile_ = on; }
  const NttTimings& timings() const { return timings_; }
  // Kernel variants (BN254 Fr): bit 0 = the 9 x 29-bit-limb passes
  // (dif29_pass_kernel), 0 = the 8 x 32-bit ones (dif_pass_kernel); the
  // default is 1 up to 2^20 and 0 above (DESIGN.md NTT round 4: fewer
  // instructions win while the clock holds, more multiplies per butterfly
  // lower it at 2^22+); bit 1 (with bit 0) swizzles their LDS positions;
  // bit 2 (any field) keeps one batch entry per workgroup in one-pass
  // transforms (no packing, pack_log).  Unknown values (or bits 0-1 on other
  // fields): refused.
  bool set_variant(int v);
  int variant() const { return variant_; }

  struct Pass {
    uint32_t s0, k, log_m;
    bool final_pass;
  };
  const std::vector<Pass>& plan() const { return plan_; }

 private:
  void run(Fr* d_data, bool inverse, size_t batch, const Fr* src = nullptr, const FourStepTw<Fr>* fs = nullptr);
  void run29(Fr* d_data, bool inverse, size_t batch, const Fr* src = nullptr, const FourStepTw<Fr>* fs = nullptr);
  uint32_t pack_log(size_t batch) const;
  void build_twiddles();
  void build_tables29();
  void ensure_tables32();
  void build_powers(const Fr& base, const Fr& scale, Fr* d_lo, Fr* d_hi);

  size_t n_ = 0;
  uint32_t log_n_ = 0;
  Fr omega_, omega_inv_, size_inv_, offset_, offset_inv_;
  bool has_offset_ = false;
  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  bool profile_ = false;
  std::vector<Pass> plan_;
  uint32_t pow_bits_ = 0;  // split point of the two-level power tables
  int radix_ = 2;          // DIF stages per register step of the pass kernel (see kMaxLdsElems)
  DeviceBuffer tw_fwd_, tw_inv_, scratch_, io_;
  DeviceBuffer twm_fwd_, twm_inv_;  // Montgomery twiddles when tw_* hold Shoup entries (BN254 Fr)
  int shoup_mode_ = 2;              // Shoup twiddles: 0 never, 1 every pass, 2 all but the first pass
  int ntt_variant_ = 0;             // A/B kernel variants (TACHYON_NTT_VARIANT, see run())
  // BN254 Fr: the 29-bit-limb passes and their tables -- R'-form entries for
  // the first pass's stages [0, k0), Shoup entries for the later stages
  int variant_ = 0;
  bool tables32_ = false;  // the 32-bit Shoup tables (built with the domain)
  bool tables29_ = false;  // the 29-bit tables (built with the domain up to 2^20, else on first use of bit 0)
  size_t split29_ = 0;     // = n - (n >> k0): stage-table entries before the Shoup part
  DeviceBuffer t29m_fwd_, t29m_inv_, t29s_fwd_, t29s_inv_, scratch29_;
  DeviceBuffer coset_lo_, coset_hi_, icoset_lo_, icoset_hi_;
  NttTimings timings_;
  std::vector<hipEvent_t> ev_;
};

extern template class NttDomain<Bn254Fr>;
extern template class NttDomain<Bls381Fr>;

// w_(2^log_n), Montgomery form: the two-adic root squared down
// (PrimeFieldBase::GetRootOfUnity, prime_field_base.h:90-130).  For BN254 Fr
// the root comes from the active generator set (below).
template <class Fr>
Fr root_of_unity(uint32_t log_n);

// BN254 Fr generator set used by domains created from now on:
// math::halo2::OverrideSubgroupGenerator() (bn/bn254/halo2/bn254.cc:7-30)
// installs halo2curves' generator 7 and its two-adic / large-subgroup roots
// in place of the arkworks-compatible generator 5; the scoped overrider's
// destructor (bn254.cc:32-44) restores them.  A domain, a four-step plan and a
// KZG setup capture the root when they are built, as the reference's
// Domain::Create does.  Returns the previous state.
bool set_bn254_fr_halo2_generator(bool on);
bool bn254_fr_halo2_generator();
// n as a field element (Montgomery form)
template <class Fr>
Fr field_from_u64(uint64_t v);

}  // namespace tachyon_amd::ntt

namespace tachyon_amd::ntt {

// Distributed four-step NTT (Bailey) over G = 2^log_world ranks, one process
// per GPU: n = R * C with R = 2^floor(L/2) (or 2^log_r when
// given: ntt4_split_log_r picks the split with the fewest passes), C = n / R,
// both >= G.  Rank g owns
//   input   the columns c in [g C/G, (g+1) C/G) of the R x C row-major view
//           of x, stored column by column: in[c_l * R + r] = x[C r + c]
//   output  the rows k1 in [g R/G, (g+1) R/G) of X, stored row by row:
//           out[k1_l * C + k2] = X[k1 + R k2]
// forward = stage1 (R-point NTTs on the local columns, twiddles w_n^(c k1),
// pack per destination rank), one all-to-all of n/G elements, stage2
// (transpose, C-point NTTs on the local rows).  inverse mirrors it and maps
// the output layout back to the input layout (n^-1 included).  The
// all-to-all is the caller's (torch.distributed / RCCL): send and recv are
// G equal chunks of n/G^2 elements, chunk h going to / coming from rank h.
template <class Fr>
class Ntt4Step {
 public:
  Ntt4Step(uint32_t log_n, uint32_t log_world, uint32_t rank, hipStream_t stream, uint32_t log_r = 0);
  ~Ntt4Step();
  Ntt4Step(const Ntt4Step&) = delete;
  Ntt4Step& operator=(const Ntt4Step&) = delete;

  size_t local_size() const { return n_ >> log_g_; }
  uint32_t world() const { return 1u << log_g_; }
  uint32_t rank() const { return rank_; }
  uint32_t log_rows() const { return log_r_; }
  const Fr& root() const { return w_; }  // w_n of the plan (the generator set active at construction)
  hipStream_t stream() const { return stream_; }

  void forward_stage1(const Fr* in, Fr* send);
  void forward_stage2(const Fr* recv, Fr* out);
  void inverse_stage1(const Fr* in, Fr* send);
  void inverse_stage2(const Fr* recv, Fr* out);
  // A/B: bit 0 = the round-4 stages (copies, separate twiddle kernel), bit 1
  // = the sub-transforms on the 32-bit passes, bit 2 = no packing of one-pass
  // sub-transforms (NttDomain variant bit 2), bit 3 = the exchange twiddles
  // computed in the pass (no tab29)
  void set_variant(int v) {
    fused_ = !(v & 1);
    no_table_ = (v & 8) != 0;
    const int nopack = (v & 4) ? 4 : 0;
    if (v & 2) {
      dom_r_->set_variant(nopack);
      dom_c_->set_variant(nopack);
    } else {
      dom_r_->set_variant((dom_r_->log_size() <= 20 ? 1 : 0) | nopack);
      dom_c_->set_variant((dom_c_->log_size() <= 20 ? 1 : 0) | nopack);
    }
  }

 private:
  bool fused_ = true;
  bool no_table_ = false;
  uint32_t log_n_, log_g_, rank_, log_r_, log_c_;
  size_t n_;
  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  NttDomain<Fr>* dom_r_ = nullptr;
  NttDomain<Fr>* dom_c_ = nullptr;
  uint32_t pow_bits_ = 0;
  Fr w_;
  DeviceBuffer work_, w_lo_, w_hi_, wi_lo_, wi_hi_;
  DeviceBuffer tab29_fwd_, tab29_inv_;  // FourStepTw::tab29 of the two directions (built on first use)
  const void* exchange_table(bool inverse);
};

extern template class Ntt4Step<Bn254Fr>;

// The R x C split with the fewest pass launches (ceil(log R / 8) + ceil(log C
// / 8), passes of <= 8 stages) with R, C >= 2^log_world, ties to the larger R
// up to C: 2^24 -> 2^8 x 2^16 (1 + 2 passes instead of 2 + 2 for 2^12 x
// 2^12).  One-pass R-point transforms pack several columns per workgroup.
uint32_t ntt4_split_log_r(uint32_t log_n, uint32_t log_world);

// One process, several GPUs (round 4): the four-step plan above with one part
// per entry of `devices` (ids may repeat -- logical devices sharing a GPU on
// their own streams), the all-to-all as G x G peer copies (hipMemcpyPeerAsync:
// xGMI between GPUs, a device copy within one), and the natural-order input
// and output on the primary device: x is transposed there (R x C -> C x R) so
// that part g's input columns are one contiguous chunk, and the parts' output
// rows come back as one R x C matrix transposed to natural order.  Everything
// is enqueued on the primary stream and the parts' streams (events between
// them).  G = |devices| is a power of two, R x C = ntt4_split_log_r's split, R, C >= G.
template <class Fr>
class NttMultiDevice {
 public:
  NttMultiDevice(uint32_t log_n, const std::vector<int>& devices, int primary, hipStream_t primary_stream);
  ~NttMultiDevice();
  NttMultiDevice(const NttMultiDevice&) = delete;
  NttMultiDevice& operator=(const NttMultiDevice&) = delete;

  size_t size() const { return n_; }
  const std::vector<int>& device_ids() const { return ids_; }
  const Fr& root() const { return parts_[0]->plan->root(); }
  // x -> y, n elements each on the primary device (may alias); not synchronised
  void forward_device(const Fr* x, Fr* y) { run(x, y, false); }
  void inverse_device(const Fr* x, Fr* y) { run(x, y, true); }
  // host vectors: len <= n inputs, zero-padded; n outputs (may alias); synchronises
  void forward_host(const Fr* in, size_t len, Fr* out) { host(in, len, out, false); }
  void inverse_host(const Fr* in, size_t len, Fr* out) { host(in, len, out, true); }

 private:
  struct Part {
    int device = 0;
    hipStream_t stream = nullptr;
    std::unique_ptr<Ntt4Step<Fr>> plan;
    DeviceBuffer in, send, recv, out;
    hipEvent_t ev1 = nullptr, ev2 = nullptr;
  };
  void run(const Fr* x, Fr* y, bool inverse);
  void host(const Fr* in, size_t len, Fr* out, bool inverse);

  uint32_t log_n_, log_g_, log_r_, log_c_;
  size_t n_;
  int primary_;
  hipStream_t s0_;
  hipEvent_t ev0_ = nullptr;
  std::vector<int> ids_;
  std::vector<std::unique_ptr<Part>> parts_;
  DeviceBuffer stage_, io_;
};

extern template class NttMultiDevice<Bn254Fr>;

}  // namespace tachyon_amd::ntt
