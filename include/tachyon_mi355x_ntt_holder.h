/* C++ GPU-NTT hook for Tachyon's UnivariateEvaluationDomain, header-only over
 * the C-ABI of libtachyon_mi355x.so.
 *
 * Replaces (same shape and semantics):
 *   IcicleNTTHolder<F>   tachyon/math/polynomials/univariate/icicle/icicle_ntt_holder.h:15-63
 *                        (Create(), operator->, owns the NTT object)
 *   IcicleNTT<F>::FFT / IFFT / Run
 *                        icicle_ntt.h:53-142, icicle_ntt_bn254.cc:31-116
 *                        (in place on the host vector, natural order in and out,
 *                        the coset offset given per call; CHECK-abort on failure)
 *   UnivariateEvaluationDomain::set_icicle / FFT / IFFT dispatch
 *                        univariate_evaluation_domain.h:99,141-232 (the caller
 *                        resizes the evaluations to size() first)
 *
 * A Tachyon build with this backend keeps its set_icicle call sites and swaps
 * the holder type ("set_gpu_backend"):
 *
 *   auto holder = tachyon_mi355x::NTTHolder::Create(domain->size());
 *   // FFT: evals.evaluations_ resized to size(), then
 *   holder->FFT(evals.evaluations_, offset);      // offset: bn254::Fr, 1 = no coset
 *   holder->IFFT(poly.coefficients_, offset);
 *
 * F is any type with the layout of tachyon_bn254_fr (4 x uint64 Montgomery
 * limbs): bn254::Fr itself, or tachyon_bn254_fr.  NTT / NTTHolder go through
 * the reference's BN254 C-ABI domain (its multi-device split included).
 *
 * The other scalar field the reference's icicle backend covers,
 * IcicleNTT<bls12_381::Fr> (icicle_ntt_bls12_381.cc:31-115), is
 * FieldNTT<kBls12_381Fr> / FieldNTTHolder<kBls12_381Fr> over the
 * field-generic domain (tachyon_mi355x_ntt_domain_*, bn254 Fr too):
 *
 *   auto holder = tachyon_mi355x::FieldNTTHolder<tachyon_mi355x::kBls12_381Fr>::Create(size);
 *   holder->FFT(evals, &offset);   // bls12_381::Fr, nullptr = no coset */
#ifndef TACHYON_MI355X_NTT_HOLDER_H_
#define TACHYON_MI355X_NTT_HOLDER_H_

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "tachyon_mi355x.h"

namespace tachyon_mi355x {

class NTT {
 public:
  explicit NTT(size_t size) : domain_(tachyon_bn254_univariate_evaluation_domain_create(size)) {
    size_ = tachyon_mi355x_bn254_univariate_evaluation_domain_size(domain_);
  }
  NTT(const NTT&) = delete;
  NTT& operator=(const NTT&) = delete;
  ~NTT() { tachyon_bn254_univariate_evaluation_domain_destroy(domain_); }

  size_t size() const { return size_; }

  /* IcicleNTT::FFT: evaluations (size() elements, coefficients in) in place. */
  template <class F>
  bool FFT(std::vector<F>& evals, const F* coset = nullptr) {
    return Run(evals.data(), evals.size(), coset, 0);
  }
  /* IcicleNTT::IFFT: coefficients (size() elements, evaluations in) in place. */
  template <class F>
  bool IFFT(std::vector<F>& coeffs, const F* coset = nullptr) {
    return Run(coeffs.data(), coeffs.size(), coset, 1);
  }

  /* IcicleNTT::Run on a raw host pointer; size must equal size(). */
  template <class F>
  bool Run(F* inout, size_t size, const F* coset, int inverse) {
    static_assert(sizeof(F) == sizeof(tachyon_bn254_fr), "F must have the layout of tachyon_bn254_fr");
    SetCoset(coset);
    tachyon_mi355x_bn254_univariate_evaluation_domain_transform_host(
        domain_, reinterpret_cast<tachyon_bn254_fr*>(inout), size, inverse);
    return true;  // failures abort inside the library, like the reference's CHECKs
  }

  tachyon_bn254_univariate_evaluation_domain* domain() { return domain_; }

 private:
  template <class F>
  void SetCoset(const F* coset) {
    tachyon_bn254_fr want;
    if (coset) {
      std::memcpy(&want, coset, sizeof(want));
    } else {
      want = One();
    }
    if (have_coset_ && std::memcmp(&want, &coset_, sizeof(want)) == 0) return;
    tachyon_mi355x_bn254_univariate_evaluation_domain_set_offset(domain_, &want);
    coset_ = want;
    have_coset_ = true;
  }
  static tachyon_bn254_fr One() {
    /* 1 in Montgomery form = R mod r for BN254 Fr */
    tachyon_bn254_fr one = {{0xac96341c4ffffffbULL, 0x36fc76959f60cd29ULL, 0x666ea36f7879462eULL,
                             0x0e0a77c19a07df2fULL}};
    return one;
  }

  tachyon_bn254_univariate_evaluation_domain* domain_ = nullptr;
  size_t size_ = 0;
  tachyon_bn254_fr coset_ = {};
  bool have_coset_ = false;
};

/* Field ids of tachyon_mi355x_ntt_domain_create. */
enum NttField : int { kBn254Fr = 1, kBls12_381Fr = 3 };

/* IcicleNTT<F> over the field-generic domain: the same FFT / IFFT / Run as
 * NTT above for the field kField (F: 4 x uint64 Montgomery limbs). */
template <int kField>
class FieldNTT {
 public:
  explicit FieldNTT(size_t size) : domain_(tachyon_mi355x_ntt_domain_create(kField, size)) {
    size_ = tachyon_mi355x_ntt_domain_size(domain_);
  }
  FieldNTT(const FieldNTT&) = delete;
  FieldNTT& operator=(const FieldNTT&) = delete;
  ~FieldNTT() { tachyon_mi355x_ntt_domain_destroy(domain_); }

  size_t size() const { return size_; }
  template <class F>
  bool FFT(std::vector<F>& evals, const F* coset = nullptr) {
    return Run(evals.data(), evals.size(), coset, 0);
  }
  template <class F>
  bool IFFT(std::vector<F>& coeffs, const F* coset = nullptr) {
    return Run(coeffs.data(), coeffs.size(), coset, 1);
  }
  template <class F>
  bool Run(F* inout, size_t size, const F* coset, int inverse) {
    static_assert(sizeof(F) == 4 * sizeof(uint64_t), "F must be 4 x uint64 Montgomery limbs");
    uint64_t want[4] = {0, 0, 0, 0};
    if (coset) std::memcpy(want, coset, sizeof(want));
    if (!have_coset_ || std::memcmp(want, coset_, sizeof(want)) != 0) {
      /* (all-zero = no coset: the offset 0 is not a coset of the domain) */
      tachyon_mi355x_ntt_domain_set_offset(domain_, coset ? static_cast<const void*>(want) : nullptr);
      std::memcpy(coset_, want, sizeof(want));
      have_coset_ = true;
    }
    tachyon_mi355x_ntt_domain_transform_host(domain_, inout, size, inverse);
    return true;  // failures abort inside the library, like the reference's CHECKs
  }
  tachyon_mi355x_ntt_domain* domain() { return domain_; }

 private:
  tachyon_mi355x_ntt_domain* domain_ = nullptr;
  size_t size_ = 0;
  uint64_t coset_[4] = {0, 0, 0, 0};
  bool have_coset_ = false;
};

/* IcicleNTTHolder<F> for FieldNTT<kField>. */
template <int kField>
class FieldNTTHolder {
 public:
  static FieldNTTHolder Create(size_t size) { return FieldNTTHolder(std::make_unique<FieldNTT<kField>>(size)); }
  FieldNTT<kField>* operator->() { return ntt_.get(); }
  const FieldNTT<kField>* operator->() const { return ntt_.get(); }
  FieldNTT<kField>* get() { return ntt_.get(); }

 private:
  explicit FieldNTTHolder(std::unique_ptr<FieldNTT<kField>> ntt) : ntt_(std::move(ntt)) {}
  std::unique_ptr<FieldNTT<kField>> ntt_;
};

/* IcicleNTTHolder<bn254::Fr>: owns one NTT; Create() + operator->. */
class NTTHolder {
 public:
  static NTTHolder Create(size_t size) { return NTTHolder(std::make_unique<NTT>(size)); }
  NTT* operator->() { return ntt_.get(); }
  const NTT* operator->() const { return ntt_.get(); }
  NTT* get() { return ntt_.get(); }

 private:
  explicit NTTHolder(std::unique_ptr<NTT> ntt) : ntt_(std::move(ntt)) {}
  std::unique_ptr<NTT> ntt_;
};

}  // namespace tachyon_mi355x

#endif  // TACHYON_MI355X_NTT_HOLDER_H_
