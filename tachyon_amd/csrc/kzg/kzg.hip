// KZG with a device-resident SRS (see kzg.h for the reference mapping).
#include "kzg.h"

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "../field/curve_constants.h"
#include "../ntt/ntt.h"

namespace tachyon_amd::kzg {

namespace {

constexpr unsigned kBlock = 256;

template <class Curve>
struct Generator;
template <>
struct Generator<Bn254G1> {
  static constexpr const uint64_t* x = consts::bn254_g1::kXMont64;
  static constexpr const uint64_t* y = consts::bn254_g1::kYMont64;
};
template <>
struct Generator<Bls381G1> {
  static constexpr const uint64_t* x = consts::bls12_381_g1::kXMont64;
  static constexpr const uint64_t* y = consts::bls12_381_g1::kYMont64;
};

template <class F>
F from_words(const uint64_t* w) {
  F r;
  for (int i = 0; i < F::N; ++i) r.v[i] = (uint32_t)(w[i / 2] >> (32 * (i & 1)));
  return r;
}

// s_i = tau^i; l_i = L_i(tau) = (Z_H(tau) / n) * w^i / (tau - w^i)
// (EvaluatePartialLagrangeCoefficients, univariate_evaluation_domain.h:308-360,
// offset 1), one Fermat inverse per element
template <class Fr>
__global__ __launch_bounds__(kBlock) void srs_scalars_kernel(Fr tau, Fr omega, Fr z_over_n, uint32_t n,
                                                             Fr* __restrict__ s, Fr* __restrict__ l) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Fr ti = tau.pow(&i, 1);
  s[i] = ti.canonical();
  if (l) {
    const Fr wi = omega.pow(&i, 1);
    l[i] = (z_over_n * wi * (tau - wi).inverse()).canonical();
  }
}

// out_i = k_i * G (BatchMapScalarFieldToPoint), double-and-add from the top bit
template <class Curve>
__global__ __launch_bounds__(kBlock) void fixed_base_kernel(Affine<typename Curve::F> g,
                                                            const typename Curve::Fr* __restrict__ k, uint32_t n,
                                                            Affine<typename Curve::F>* __restrict__ out) {
  using F = typename Curve::F;
  using Fr = typename Curve::Fr;
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Fr c = k[i].from_mont();
  XYZZ<F> r = XYZZ<F>::zero();
  for (int b = Fr::N * 32 - 1; b >= 0; --b) {
    r = r.dbl();
    if ((c.v[b / 32] >> (b % 32)) & 1) r = r.madd(g);
  }
  out[i] = r.to_affine();
}

}  // namespace

template <class Curve>
Kzg<Curve>::Kzg(hipStream_t stream) : stream_(stream) {
  require_gpu();
  if (!stream_) {
    TA_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    own_stream_ = true;
  }
  msm_ = std::make_unique<msm::MsmGpu<Curve>>(stream_);
}

template <class Curve>
Kzg<Curve>::~Kzg() {
  msm_.reset();
  if (own_stream_) (void)hipStreamDestroy(stream_);
}

template <class Curve>
void Kzg<Curve>::unsafe_setup(size_t size, const Fr& tau) {
  if (size == 0 || (size & (size - 1)) || size > (size_t(1) << 30))
    throw std::runtime_error("tachyon_mi355x: KZG setup size must be a power of two <= 2^30");
  uint32_t log_n = 0;
  while ((size_t(1) << log_n) < size) ++log_n;
  const Fr omega = ntt::root_of_unity<Fr>(log_n);
  const uint32_t n = (uint32_t)size;
  const uint32_t e = n;
  const Fr z = tau.pow(&e, 1) - Fr::one();  // Z_H(tau) = tau^n - 1
  Fr* d_s = static_cast<Fr*>(scratch_.ensure(2 * size * sizeof(Fr)));
  Fr* d_l = d_s + size;
  const unsigned grid = ceil_div(size, kBlock);
  if (!z.is_zero()) {
    const Fr z_over_n = z * ntt::field_from_u64<Fr>(size).inverse();
    hipLaunchKernelGGL(srs_scalars_kernel<Fr>, dim3(grid), dim3(kBlock), 0, stream_, tau, omega, z_over_n, n, d_s,
                       d_l);
  } else {
    // tau = w^j: L_j(tau) = 1, every other coefficient 0 (univariate_evaluation_domain.h:309-323)
    hipLaunchKernelGGL(srs_scalars_kernel<Fr>, dim3(grid), dim3(kBlock), 0, stream_, tau, omega, Fr::zero(), n, d_s,
                       static_cast<Fr*>(nullptr));
    std::vector<Fr> l(size, Fr::zero());
    Fr w = Fr::one();
    for (size_t j = 0; j < size; ++j, w = w * omega)
      if (w == tau) {
        l[j] = Fr::one();
        break;
      }
    TA_HIP(hipMemcpyAsync(d_l, l.data(), size * sizeof(Fr), hipMemcpyHostToDevice, stream_));
    TA_HIP(hipStreamSynchronize(stream_));
  }
  TA_HIP(hipGetLastError());
  const Aff g{from_words<F>(Generator<Curve>::x), from_words<F>(Generator<Curve>::y)};
  Aff* d_p = static_cast<Aff*>(powers_.ensure(size * sizeof(Aff)));
  Aff* d_lg = static_cast<Aff*>(lagrange_.ensure(size * sizeof(Aff)));
  hipLaunchKernelGGL(fixed_base_kernel<Curve>, dim3(grid), dim3(kBlock), 0, stream_, g, d_s, n, d_p);
  hipLaunchKernelGGL(fixed_base_kernel<Curve>, dim3(grid), dim3(kBlock), 0, stream_, g, d_l, n, d_lg);
  TA_HIP(hipGetLastError());
  TA_HIP(hipStreamSynchronize(stream_));
  n_ = size;
}

template <class Curve>
bool Kzg<Curve>::downsize(size_t n) {
  if (n >= n_) return false;
  n_ = n;  // the device arrays keep their capacity; only the prefix is used
  return true;
}

template <class Curve>
bool Kzg<Curve>::commit(const Fr* scalars, size_t len, bool lagrange, Aff* out) {
  if (len > n_) return false;
  *out = msm_->run(d_srs(lagrange), scalars, len).to_affine();
  return true;
}

// XYZZ -> affine for a whole batch with one inversion: x = X / ZZ = X (ZZZ^-1 ZZ)^2,
// y = Y / ZZZ (point_xyzz.h:199-212), the ZZZ inverted together by
// Montgomery's trick (prefix products, one inverse, backward pass); identity
// points (zz = 0) stay (0, 0).
template <class F>
void batch_to_affine(const std::vector<XYZZ<F>>& pts, Affine<F>* out) {
  const size_t m = pts.size();
  std::vector<F> prefix(m);
  F acc = F::one();
  for (size_t i = 0; i < m; ++i) {
    if (!pts[i].is_zero()) acc = acc * pts[i].zzz;
    prefix[i] = acc;
  }
  F inv = acc.inverse();  // product of the non-identity ZZZ: invertible
  for (size_t i = m; i-- > 0;) {
    if (pts[i].is_zero()) {
      out[i] = Affine<F>::zero();
      continue;
    }
    const F zinv3 = i > 0 ? inv * prefix[i - 1] : inv;  // 1 / ZZZ_i
    inv = inv * pts[i].zzz;
    const F zinv2 = (zinv3 * pts[i].zz).sqr();
    out[i] = Affine<F>{pts[i].x * zinv2, pts[i].y * zinv3}.canonical();
  }
}

template <class Curve>
bool Kzg<Curve>::commit_batch(const Fr* const* scalars, const size_t* lens, size_t count, bool lagrange, Aff* out) {
  for (size_t i = 0; i < count; ++i)
    if (lens[i] > n_) return false;
  // Polynomials of similar length go into one batched MSM (MsmGpu::run_batch:
  // a block of windows per polynomial, one recode / sort / accumulation /
  // reduction) over the SRS prefix of the group's longest one, the others
  // zero-padded.  Groups are taken longest first and closed when padding
  // would more than double the group's work (count x L > 2 x sum of lens),
  // at run_batch's limits (max_batch_count) or at kGroupScalars padded
  // scalars (the batch's sort buffers grow ~16 B per scalar-window); a
  // group of one is a plain MSM.  So a ragged batch costs about its real
  // work, and a halo2-sized batch (thousands of columns of 2^20) runs as
  // several batched MSMs instead of one refused one.
  constexpr size_t kGroupScalars = size_t(1) << 26;
  std::vector<size_t> order;
  for (size_t i = 0; i < count; ++i)
    if (lens[i]) order.push_back(i);
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return lens[a] > lens[b]; });
  std::vector<XYZZ<F>> pts(count, XYZZ<F>::zero());
  const Aff* srs = d_srs(lagrange);
  for (size_t i = 0; i < order.size();) {
    const size_t L = lens[order[i]];
    const size_t cap = std::min(msm_->max_batch_count(L), std::max<size_t>(1, kGroupScalars / L));
    size_t j = i + 1, sum = L;
    while (j < order.size() && j - i < cap && (j - i + 1) * L <= 2 * (sum + lens[order[j]])) sum += lens[order[j++]];
    const size_t g = j - i;
    if (g == 1) {
      pts[order[i]] = msm_->run(srs, scalars[order[i]], L);
    } else {
      Fr* padded = static_cast<Fr*>(batch_.ensure(g * L * sizeof(Fr)));
      TA_HIP(hipMemsetAsync(padded, 0, g * L * sizeof(Fr), msm_->stream()));
      for (size_t k = 0; k < g; ++k)  // host or device polynomials
        TA_HIP(hipMemcpyAsync(padded + k * L, scalars[order[i + k]], lens[order[i + k]] * sizeof(Fr),
                              hipMemcpyDefault, msm_->stream()));
      const auto res = msm_->run_batch(srs, padded, L, g);
      for (size_t k = 0; k < g; ++k) pts[order[i + k]] = res[k];
    }
    i = j;
  }
  batch_to_affine(pts, out);
  return true;
}

template <class Curve>
void Kzg<Curve>::copy_srs(bool lagrange, Aff* host_out) const {
  TA_HIP(hipMemcpy(host_out, d_srs(lagrange), n_ * sizeof(Aff), hipMemcpyDeviceToHost));
}

template class Kzg<Bn254G1>;
template class Kzg<Bls381G1>;

}  // namespace tachyon_amd::kzg
