// Groth16 prover on MI355X: circom zkey/wtns readers, the witness-map
// kernels and the proof assembly.  See groth16.h for the reference mapping.
#include "groth16.h"

#include <algorithm>
#include <chrono>
#include <exception>
#include <thread>

namespace tachyon_amd {
namespace circom {

namespace {

void check_magic(ByteReader& rd, const char* magic, uint32_t want_version, const char* what) {
  const uint8_t* m = rd.ptr(4);
  if (memcmp(m, magic, 4) != 0) throw std::runtime_error(std::string("circom: not a ") + what + " file (bad magic)");
  uint32_t version = rd.read<uint32_t>();
  if (version != want_version)
    throw std::runtime_error(std::string("circom: unsupported ") + what + " version " + std::to_string(version));
}

const std::pair<size_t, size_t>& section(const std::map<uint32_t, std::pair<size_t, size_t>>& secs, uint32_t id) {
  auto it = secs.find(id);
  if (it == secs.end()) throw std::runtime_error("circom: missing section " + std::to_string(id));
  return it->second;
}

template <class T>
void read_array(ByteReader& rd, std::vector<T>* out, size_t count) {
  out->resize(count);
  if (count) rd.take(out->data(), count * sizeof(T));
}

template <class F>
struct BaseCfgOf {
  using type = typename F::Config;
};
template <class B>
struct BaseCfgOf<Fp2<B>> {
  using type = typename B::Config;
};

}  // namespace

CurveId zkey_curve(const uint8_t* data, size_t len) {
  ByteReader rd(data, len);
  check_magic(rd, "zkey", 1, "zkey");
  auto secs = read_sections(rd);
  auto [off, size] = section(secs, 2);
  ByteReader g(data + off, size);
  uint32_t n8q = g.read<uint32_t>();
  const uint8_t* q = g.ptr(n8q);
  if (modulus_matches<consts::bn254_fq>(q, n8q)) return CurveId::kBn254;
  if (modulus_matches<consts::bls12_381_fq>(q, n8q)) return CurveId::kBls12_381;
  throw std::runtime_error("circom: zkey base field is neither BN254 nor BLS12-381");
}

template <class G1, class G2>
ZKey<G1, G2> parse_zkey(const uint8_t* data, size_t len) {
  using Z = ZKey<G1, G2>;
  using Fr = typename Z::Fr;
  Z z;
  ByteReader rd(data, len);
  check_magic(rd, "zkey", 1, "zkey");
  auto secs = read_sections(rd);
  {
    auto [off, size] = section(secs, 1);  // header: prover type 1 = Groth16
    ByteReader h(data + off, size);
    if (h.read<uint32_t>() != 1) throw std::runtime_error("circom: zkey prover type is not Groth16");
  }
  {
    auto [off, size] = section(secs, 2);
    ByteReader g(data + off, size);
    uint32_t n8q = g.read<uint32_t>();
    if (!modulus_matches<typename BaseCfgOf<typename G1::F>::type>(g.ptr(n8q), n8q))
      throw std::runtime_error("circom: zkey base field does not match the curve");
    uint32_t n8r = g.read<uint32_t>();
    if (!modulus_matches<typename Fr::Config>(g.ptr(n8r), n8r))
      throw std::runtime_error("circom: zkey scalar field does not match the curve");
    z.num_vars = g.read<uint32_t>();
    z.num_public = g.read<uint32_t>();
    z.domain_size = g.read<uint32_t>();
    if (z.num_vars < z.num_public + 1) throw std::runtime_error("circom: zkey has fewer variables than inputs");
    if (z.domain_size == 0 || (z.domain_size & (z.domain_size - 1)))
      throw std::runtime_error("circom: zkey domain size is not a power of two");
    z.alpha_g1 = g.read<typename Z::A1>();
    z.beta_g1 = g.read<typename Z::A1>();
    z.beta_g2 = g.read<typename Z::A2>();
    z.gamma_g2 = g.read<typename Z::A2>();
    z.delta_g1 = g.read<typename Z::A1>();
    z.delta_g2 = g.read<typename Z::A2>();
  }
  auto points = [&](uint32_t id, auto* out, size_t count) {
    auto [off, size] = section(secs, id);
    ByteReader p(data + off, size);
    read_array(p, out, count);
  };
  points(3, &z.ic, z.num_public + 1);
  {
    auto [off, size] = section(secs, 4);
    ByteReader c(data + off, size);
    uint32_t count = c.read<uint32_t>();
    z.coefficients.resize(count);
    for (uint32_t i = 0; i < count; ++i) {
      auto& e = z.coefficients[i];
      e.matrix = c.read<uint32_t>();
      e.constraint = c.read<uint32_t>();
      e.signal = c.read<uint32_t>();
      Fr raw;
      c.take(&raw, sizeof(Fr));
      // zkey.h:219-220: value = F::FromMontgomery(value.ToBigInt()), i.e. the
      // stored word times R^-1 becomes the Montgomery representation
      e.value = raw.from_mont();
    }
  }
  points(5, &z.a1, z.num_vars);
  points(6, &z.b1, z.num_vars);
  points(7, &z.b2, z.num_vars);
  points(8, &z.c1, z.num_witness());
  points(9, &z.h1, z.domain_size);
  return z;
}

template <class Fr>
std::vector<Fr> parse_wtns(const uint8_t* data, size_t len) {
  ByteReader rd(data, len);
  check_magic(rd, "wtns", 2, "wtns");
  auto secs = read_sections(rd);
  uint32_t count;
  {
    auto [off, size] = section(secs, 1);
    ByteReader h(data + off, size);
    uint32_t n8 = h.read<uint32_t>();
    if (!modulus_matches<typename Fr::Config>(h.ptr(n8), n8))
      throw std::runtime_error("circom: wtns field does not match the curve's scalar field");
    count = h.read<uint32_t>();
  }
  auto [off, size] = section(secs, 2);
  ByteReader d(data + off, size);
  std::vector<Fr> out(count);
  for (uint32_t i = 0; i < count; ++i) {
    Fr raw;
    d.take(&raw, sizeof(Fr));
    out[i] = raw.to_mont();  // wtns.h:116: F(witnesses[i].value()) -- canonical in, Montgomery out
  }
  return out;
}

template ZKey<Bn254G1, Bn254G2> parse_zkey<Bn254G1, Bn254G2>(const uint8_t*, size_t);
template ZKey<Bls381G1, Bls381G2> parse_zkey<Bls381G1, Bls381G2>(const uint8_t*, size_t);
template std::vector<Bn254Fr> parse_wtns<Bn254Fr>(const uint8_t*, size_t);
template std::vector<Bls381Fr> parse_wtns<Bls381Fr>(const uint8_t*, size_t);

}  // namespace circom

namespace groth16 {

namespace {

constexpr unsigned kBlock = 256;

// a_i = sum_A val * w[signal], b_i likewise, c_i = a_i * b_i
// (quadratic_arithmetic_program.h:38-72; the OpenMP-locked scatter becomes a
// gather over the constraint's CSR row -- field addition is exact, so the
// order of the terms does not change the values)
template <class Fr>
__global__ __launch_bounds__(kBlock) void qap_abc_kernel(const uint32_t* __restrict__ row_a,
                                                         const uint32_t* __restrict__ row_b,
                                                         const uint32_t* __restrict__ col,
                                                         const Fr* __restrict__ val, const Fr* __restrict__ w,
                                                         uint32_t n, Fr* __restrict__ abc) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Fr a = Fr::zero(), b = Fr::zero();
  for (uint32_t k = row_a[i], e = row_a[i + 1]; k < e; ++k) a = a + val[k] * w[col[k]];
  for (uint32_t k = row_b[i], e = row_b[i + 1]; k < e; ++k) b = b + val[k] * w[col[k]];
  abc[i] = a.canonical();
  abc[(size_t)n + i] = b.canonical();
  abc[2 * (size_t)n + i] = (a * b).canonical();
}

// h_i = a_i * b_i - c_i on the coset (quadratic_arithmetic_program.h:102-108), in place over a
template <class Fr>
__global__ __launch_bounds__(kBlock) void qap_h_kernel(Fr* __restrict__ abc, uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  abc[i] = (abc[i] * abc[(size_t)n + i] - abc[2 * (size_t)n + i]).canonical();
}

// k * P on the host, k a Montgomery-form scalar (double-and-add, high bit first)
template <class F, class Fr>
XYZZ<F> mul_scalar(const XYZZ<F>& P, const Fr& k) {
  Fr c = k.from_mont().canonical();
  XYZZ<F> r = XYZZ<F>::zero();
  for (int i = Fr::N * 32 - 1; i >= 0; --i) {
    r = r.dbl();
    if ((c.v[i / 32] >> (i % 32)) & 1) r = r + P;
  }
  return r;
}

template <class T>
T* upload(DeviceBuffer& buf, const std::vector<T>& v, size_t from = 0) {
  size_t count = v.size() > from ? v.size() - from : 0;
  T* d = static_cast<T*>(buf.ensure(std::max<size_t>(1, count) * sizeof(T)));
  if (count) TA_HIP(hipMemcpy(d, v.data() + from, count * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

using Clock = std::chrono::steady_clock;
inline float ms_since(Clock::time_point t0) {
  return std::chrono::duration<float, std::milli>(Clock::now() - t0).count();
}

}  // namespace

// the stream, the two domains and the two MSM contexts, on the current device
template <class G1, class G2>
void Groth16Prover<G1, G2>::init_device_state() {
  require_gpu();
  if (!stream_) {
    TA_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    own_stream_ = true;
  }
  n_ = key_.domain_size;
  uint32_t log_n = 0;
  while ((size_t(1) << log_n) < n_) ++log_n;
  dom_ = std::make_unique<ntt::NttDomain<Fr>>(n_, stream_);
  coset_ = std::make_unique<ntt::NttDomain<Fr>>(n_, stream_);
  // DistributePowers(poly, w_2n) then FFT == the FFT on the coset w_2n * <w_n>
  coset_->set_offset(ntt::root_of_unity<Fr>(log_n + 1));
  msm1_ = std::make_unique<msm::MsmGpu<G1>>(stream_);
  msm2_ = std::make_unique<msm::MsmGpu<G2>>(nullptr);  // own stream: runs beside the G1 MSMs
}

// A copy of `src` (on device src_device) on the current device: the device-
// resident proving key (query points, the merged C1 | H1 array, the CSR
// matrices) is copied peer to peer (xGMI between MI355X), the trimmed host key
// shared; the one-process multi-device prover builds one per device.
template <class G1, class G2>
Groth16Prover<G1, G2>::Groth16Prover(const Groth16Prover& src, int src_device, hipStream_t stream)
    : key_(src.key_), stream_(stream) {
  profile_ = src.profile_;
  c_a_ = src.c_a_;
  c_lh_ = src.c_lh_;
  c_b2_ = src.c_b2_;
  init_device_state();
  int dev = 0;
  TA_HIP(hipGetDevice(&dev));
  const std::pair<DeviceBuffer*, const DeviceBuffer*> bufs[] = {
      {&a1_, &src.a1_}, {&b1_, &src.b1_}, {&lh1_, &src.lh1_}, {&b2_, &src.b2_},
      {&row_a_, &src.row_a_}, {&row_b_, &src.row_b_}, {&col_, &src.col_}, {&val_, &src.val_}};
  for (const auto& [dst, from] : bufs) {
    void* d = dst->ensure(from->capacity());
    TA_HIP(hipMemcpyPeer(d, dev, from->template as<void>(), src_device, from->capacity()));
  }
  lh_.ensure(src.lh_.capacity());
  abc_.ensure(src.abc_.capacity());
  full_.ensure(src.full_.capacity());
  variant_ = src.variant_;
  // (no grouped-MSM layout: device copies only run the multi-rank split, world >= 2)
}

template <class G1, class G2>
Groth16Prover<G1, G2>::Groth16Prover(const Key& key, hipStream_t stream) : key_(key), stream_(stream) {
  init_device_state();

  upload(a1_, key_.a1);
  upload(b1_, key_.b1);
  upload(b2_, key_.b2);
  // C1 (witness query) and H1 back to back: their MSMs are only ever added
  // (C = ... + sum l_i C1_i + sum h_k H1_k, prove.h:146-160), so one MSM over
  // the concatenation (scalars: witness values | h) replaces two
  {
    const size_t nw = key_.c1.size(), nh = key_.h1.size();
    auto* d = static_cast<Affine<F1>*>(lh1_.ensure(std::max<size_t>(1, nw + nh) * sizeof(Affine<F1>)));
    if (nw) TA_HIP(hipMemcpy(d, key_.c1.data(), nw * sizeof(Affine<F1>), hipMemcpyHostToDevice));
    if (nh) TA_HIP(hipMemcpy(d + nw, key_.h1.data(), nh * sizeof(Affine<F1>), hipMemcpyHostToDevice));
    lh_.ensure(std::max<size_t>(1, nw + nh) * sizeof(Fr));
  }

  // CSR by constraint: A rows first, then B rows, in one col/val array
  const size_t n = n_;
  std::vector<uint32_t> cnt(2 * n + 1, 0);
  for (const auto& e : key_.coefficients) {
    if (e.constraint >= n) throw std::runtime_error("circom: coefficient constraint index outside the domain");
    if (e.signal >= key_.num_vars) throw std::runtime_error("circom: coefficient signal index out of range");
    cnt[(e.matrix ? n : 0) + e.constraint + 1]++;
  }
  for (size_t i = 1; i <= 2 * n; ++i) cnt[i] += cnt[i - 1];
  std::vector<uint32_t> col(key_.coefficients.size());
  std::vector<Fr> val(key_.coefficients.size());
  std::vector<uint32_t> fill(cnt.begin(), cnt.end() - 1);
  for (const auto& e : key_.coefficients) {
    uint32_t at = fill[(e.matrix ? n : 0) + e.constraint]++;
    col[at] = e.signal;
    val[at] = e.value;
  }
  std::vector<uint32_t> row_a(cnt.begin(), cnt.begin() + n + 1);
  std::vector<uint32_t> row_b(cnt.begin() + n, cnt.end());
  upload(row_a_, row_a);
  upload(row_b_, row_b);
  upload(col_, col);
  upload(val_, val);
  abc_.ensure(3 * n * sizeof(Fr));
  full_.ensure(std::max<size_t>(1, key_.num_vars) * sizeof(Fr));
  // the big host arrays are on the device now; keep the counts and the
  // query heads that the proof assembly reads on the host
  auto head = [](auto& v) { v.resize(std::min<size_t>(1, v.size())); v.shrink_to_fit(); };
  head(key_.a1);
  head(key_.b1);
  head(key_.b2);
  key_.c1.clear();
  key_.c1.shrink_to_fit();
  key_.h1.clear();
  key_.h1.shrink_to_fit();
  key_.coefficients.clear();
  key_.coefficients.shrink_to_fit();
  build_groups();
}

// A (queries 1..m-1 of a1) and the merged witness + h MSM (C1 | H1, nw + n
// points) as three groups of glen points with their own bases for
// MsmGpu::run_groups: [a1[1..m) | pad], [lh1[0, glen)], [lh1[glen, nw + n) |
// pad], identity bases and zero scalars as padding (they add nothing).  One
// recode / sort / accumulation / reduction for both MSMs: the smaller one's
// latency-bound reduction runs inside the larger one's launches.
template <class G1, class G2>
void Groth16Prover<G1, G2>::build_groups() {
  const size_t m = key_.num_vars, nlh = key_.num_witness() + n_;
  const size_t qa = m > 1 ? m - 1 : 0;
  glen_ = std::max(qa, (nlh + 1) / 2);
  if (glen_ == 0 || msm1_->max_batch_count(glen_) < 3) {
    glen_ = 0;
    return;
  }
  auto* gb = static_cast<Affine<F1>*>(gbases_.ensure(3 * glen_ * sizeof(Affine<F1>)));
  auto* gs = static_cast<Fr*>(gscalars_.ensure(3 * glen_ * sizeof(Fr)));
  TA_HIP(hipMemsetAsync(gb, 0, 3 * glen_ * sizeof(Affine<F1>), stream_));
  TA_HIP(hipMemsetAsync(gs, 0, 3 * glen_ * sizeof(Fr), stream_));
  if (qa) TA_HIP(hipMemcpyAsync(gb, a1_.as<Affine<F1>>() + 1, qa * sizeof(Affine<F1>), hipMemcpyDeviceToDevice, stream_));
  if (nlh) TA_HIP(hipMemcpyAsync(gb + glen_, lh1_.as<Affine<F1>>(), nlh * sizeof(Affine<F1>), hipMemcpyDeviceToDevice, stream_));
  TA_HIP(hipStreamSynchronize(stream_));
}

template <class G1, class G2>
Groth16Prover<G1, G2>::~Groth16Prover() {
  msm1_.reset();
  msm2_.reset();
  dom_.reset();
  coset_.reset();
  if (own_stream_) (void)hipStreamDestroy(stream_);
}

template <class G1, class G2>
void Groth16Prover<G1, G2>::witness_map(const Fr* d_full, Fr* d_h) {
  const uint32_t n = (uint32_t)n_;
  Fr* abc = abc_.as<Fr>();
  const unsigned grid = ceil_div(n, kBlock);
  hipLaunchKernelGGL(qap_abc_kernel<Fr>, dim3(grid), dim3(kBlock), 0, stream_, row_a_.as<uint32_t>(),
                     row_b_.as<uint32_t>(), col_.as<uint32_t>(), val_.as<Fr>(), d_full, n, abc);
  TA_HIP(hipGetLastError());
  dom_->inverse_device(abc, 3);    // a, b, c evaluations -> coefficients
  coset_->forward_device(abc, 3);  // -> evaluations on the coset w_2n <w_n>
  hipLaunchKernelGGL(qap_h_kernel<Fr>, dim3(grid), dim3(kBlock), 0, stream_, abc, n);
  TA_HIP(hipGetLastError());
  if (d_h != abc) TA_HIP(hipMemcpyAsync(d_h, abc, n_ * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
}

// The fold table of fixed proving-key bases (the caller set the window bits
// c on `msm`): the largest power of two up to `fold` dividing the plan's W
// whose table fits the device beside the MSM's working set
// (MsmGpu::fit_fold), built once and kept while the bases, length, window
// bits and requested fold stay.  Fold 1: no table (the plain MSM, which
// splits itself into point chunks when even that does not fit).
template <class G1, class G2>
template <class G>
unsigned Groth16Prover<G1, G2>::ensure_table(msm::MsmGpu<G>& msm, FoldTable& tab, const Affine<typename G::F>* bases,
                                             size_t len, unsigned fold, unsigned c) {
  if (len == 0) return 1;
  if (tab.fold != 0 && tab.want == fold && tab.c == c && tab.src == bases && tab.len == len) return tab.fold;
  const size_t old = tab.buf.capacity();
  const unsigned f = msm.fit_fold(len, msm.plan_windows(len), fold, msm.run_bytes(len), old);
  tab.fold = 0;
  if (f > 1) {
    if (old < msm::MsmGpu<G>::fold_table_bytes(len, f)) tab.buf.release();  // (free it before the larger one)
    msm.fold_bases(bases, len, f, tab.buf.ensure(msm::MsmGpu<G>::fold_table_bytes(len, f)));
  } else {
    tab.buf.release();
  }
  tab.fold = f;
  tab.want = fold;
  tab.c = c;
  tab.src = bases;
  tab.len = len;
  return f;
}

// An MSM over fixed proving-key bases: over their fold table (ensure_table),
// or plain when none fits
template <class G1, class G2>
template <class G>
XYZZ<typename G::F> Groth16Prover<G1, G2>::fixed_msm(msm::MsmGpu<G>& msm, FoldTable& tab,
                                                     const Affine<typename G::F>* bases, const Fr* scalars,
                                                     size_t len, unsigned fold, unsigned c) {
  if (len == 0) return XYZZ<typename G::F>::zero();
  const unsigned f = ensure_table(msm, tab, bases, len, fold, c);
  if (f <= 1) return msm.run(bases, scalars, len);
  return msm.run_folded(tab.buf.template as<void>(), scalars, len, f);
}

// The grouped A + witness/h MSM (run_groups over 3 x glen_ points): whether
// its working set fits the device at all, and its fold table if one fits
template <class G1, class G2>
bool Groth16Prover<G1, G2>::ensure_group_table(unsigned* fold_out) {
  *fold_out = 1;
  msm1_->set_force_window_bits(c_a_);
  const unsigned want = g1_fold();
  FoldTable& tab = g1_tab_;
  if (tab.fold != 0 && tab.want == want && tab.c == c_a_ && tab.len == glen_) {
    *fold_out = tab.fold;
    return group_fits_;
  }
  const size_t run_b = msm1_->batch_run_bytes(glen_, 3);
  const size_t old = tab.buf.capacity();
  group_fits_ = run_b <= msm1_->device_budget() + old;
  unsigned f = 1;
  if (group_fits_) f = msm1_->fit_fold(3 * glen_, msm1_->batch_windows(glen_), want, run_b, old);
  tab.fold = 0;
  if (f > 1) {
    const size_t bytes = msm::MsmGpu<G1>::fold_table_bytes(3 * glen_, f);
    if (old < bytes) tab.buf.release();
    msm1_->fold_bases_groups(gbases_.as<Affine<F1>>(), glen_, 3, f, tab.buf.ensure(bytes));
  } else {
    tab.buf.release();
  }
  tab.fold = f;
  tab.want = want;
  tab.c = c_a_;
  tab.src = gbases_.as<void>();
  tab.len = glen_;
  *fold_out = f;
  return group_fits_;
}

template <class G1, class G2>
typename Groth16Prover<G1, G2>::ShardPlan Groth16Prover<G1, G2>::shard_plan(uint32_t rank, uint32_t world) const {
  // this rank's chunk [lo, lo + len) of an MSM over `total` points
  auto shard = [&](size_t total, size_t* lo) {
    const size_t chunk = (total + world - 1) / world;
    *lo = std::min<size_t>((size_t)rank * chunk, total);
    return std::min(chunk, total - *lo);
  };
  ShardPlan p;
  const size_t m = key_.num_vars;
  p.q_len = m > 1 ? shard(m - 1, &p.q_lo) : 0;
  p.lh_len = shard(key_.num_witness() + n_, &p.lh_lo);
  // one process, one device: A and the witness + h MSM as ONE grouped MSM
  // (run_groups over the padded group layout of build_groups)
  p.grouped = world == 1 && glen_ > 0 && !(variant_ & 1);
  return p;
}

template <class G1, class G2>
size_t Groth16Prover<G1, G2>::prepare(uint32_t rank, uint32_t world, bool with_b1) {
  if (world == 0 || rank >= world) throw std::runtime_error("tachyon_mi355x: Groth16 shard rank >= world");
  ShardPlan sp = shard_plan(rank, world);
  const Affine<F1>* a1 = a1_.as<Affine<F1>>();
  const Affine<F1>* b1 = b1_.as<Affine<F1>>();
  const Affine<F2>* b2 = b2_.as<Affine<F2>>();
  msm2_->set_force_window_bits(c_b2_);
  folds_[0] = ensure_table(*msm2_, b2_tab_, b2 + 1 + sp.q_lo, sp.q_len, b2_fold(), c_b2_);
  folds_[1] = 0;
  if (sp.grouped) {
    unsigned f = 1;
    if (ensure_group_table(&f)) folds_[1] = f;
    else sp.grouped = false;
  }
  msm1_->set_force_window_bits(c_a_);
  folds_[2] = sp.grouped ? 0 : ensure_table(*msm1_, a_tab_, a1 + 1 + sp.q_lo, sp.q_len, g1_fold(), c_a_);
  folds_[3] = with_b1 ? ensure_table(*msm1_, b1_tab_, b1 + 1 + sp.q_lo, sp.q_len, g1_fold(), c_a_) : 0;
  folds_[4] = 0;
  if (!sp.grouped) {
    msm1_->set_force_window_bits(c_lh_);
    folds_[4] = ensure_table(*msm1_, lh_tab_, lh1_.as<Affine<F1>>() + sp.lh_lo, sp.lh_len, g1_fold(), c_lh_);
  }
  return fold_table_bytes();
}

template <class G1, class G2>
size_t Groth16Prover<G1, G2>::fold_table_bytes() const {
  return b2_tab_.buf.capacity() + a_tab_.buf.capacity() + b1_tab_.buf.capacity() + lh_tab_.buf.capacity() +
         g1_tab_.buf.capacity();
}

template <class G1, class G2>
void Groth16Prover<G1, G2>::last_folds(unsigned out[5]) const {
  for (int i = 0; i < 5; ++i) out[i] = folds_[i];
}

template <class G1, class G2>
ProofPartials<G1, G2> Groth16Prover<G1, G2>::partials(const Fr* full, size_t count, bool with_b1, uint32_t rank,
                                                      uint32_t world) {
  using P1 = XYZZ<F1>;
  using P2 = XYZZ<F2>;
  const size_t m = key_.num_vars;
  if (count != m)
    throw std::runtime_error("tachyon_mi355x: Groth16 assignment count " + std::to_string(count) +
                             " != num_vars " + std::to_string(m));
  if (world == 0 || rank >= world) throw std::runtime_error("tachyon_mi355x: Groth16 shard rank >= world");
  auto t0 = Clock::now();
  const Fr* d_full = full;
  int cur_device = 0;
  TA_HIP(hipGetDevice(&cur_device));
  const int src_device = pointer_device(full);
  if (src_device < 0) {
    d_full = full_.as<Fr>();
    TA_HIP(hipMemcpyAsync(const_cast<Fr*>(d_full), full, m * sizeof(Fr), hipMemcpyHostToDevice, stream_));
  } else if (src_device != cur_device) {
    // an assignment in another GPU's HBM (the one-process multi-device prover
    // hands every device the caller's pointer): a peer copy into this
    // device's buffer, never a direct cross-device read by the kernels
    d_full = full_.as<Fr>();
    TA_HIP(hipMemcpyPeerAsync(const_cast<Fr*>(d_full), cur_device, full, src_device, m * sizeof(Fr), stream_));
  }
  if (profile_) {
    TA_HIP(hipStreamSynchronize(stream_));
    timings_.upload = ms_since(t0);
  }
  ProofPartials<G1, G2> out;
  out.with_b1 = with_b1 ? 1u : 0u;
  out.rank = rank;
  out.world = world;
  // the fold tables of this shard (a no-op after prepare() for it)
  prepare(rank, world, with_b1);
  const ShardPlan sp = shard_plan(rank, world);

  // MSMs over device-resident bases and scalars (prove.h:95-146)
  const Affine<F1>* a1 = a1_.as<Affine<F1>>();
  const Affine<F1>* b1 = b1_.as<Affine<F1>>();
  const Affine<F2>* b2 = b2_.as<Affine<F2>>();
  const size_t q_lo = sp.q_lo;  // queries 1 .. m-1 (index 0 is added on the host)
  const size_t q_len = sp.q_len;
  // The G2 MSM (about 3x the work of a G1 one) needs only the witness: it
  // starts on its own stream from a second host thread as soon as the
  // witness is on the device, beside the witness map and the G1 MSMs here;
  // each MSM is synchronous on its host thread (its read-back of the chain
  // lengths).
  TA_HIP(hipStreamSynchronize(stream_));
  P2 acc_b2 = P2::zero();
  std::exception_ptr g2_error;
  int device = 0;
  TA_HIP(hipGetDevice(&device));  // a new host thread starts on device 0, not this rank's GPU
  std::thread g2_thread([&] {
    try {
      TA_HIP(hipSetDevice(device));
      auto tb = Clock::now();
      msm2_->set_force_window_bits(c_b2_);
      // the B2 query is fixed: a fold table (built once per shard / window
      // bits, the first proof's cost) shrinks the G2 window sums and their
      // host Horner on the proof's critical path
      acc_b2 = fixed_msm(*msm2_, b2_tab_, b2 + 1 + q_lo, d_full + 1 + q_lo, q_len, b2_fold(), c_b2_);
      timings_.msm_b2 = ms_since(tb);
    } catch (...) {
      g2_error = std::current_exception();
    }
  });
  struct Joiner {
    std::thread& t;
    ~Joiner() { if (t.joinable()) t.join(); }
  } joiner{g2_thread};

  auto t1 = Clock::now();
  // scalars of the merged witness + h MSM: [witness values | h]
  const size_t nw = key_.num_witness();
  // one process, one device: A and the witness + h MSM as ONE grouped MSM
  // (run_groups over the padded group layout of build_groups), when its
  // working set fits the device (prepare decided it: folds_[1] != 0)
  const bool grouped = sp.grouped && folds_[1] != 0;
  Fr* d_lh = grouped ? gscalars_.as<Fr>() + glen_ : lh_.as<Fr>();
  if (grouped && q_len)
    TA_HIP(hipMemcpyAsync(gscalars_.as<Fr>(), d_full + 1, q_len * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
  if (nw)
    TA_HIP(hipMemcpyAsync(d_lh, d_full + key_.num_instance(), nw * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
  witness_map(d_full, d_lh + nw);
  if (profile_) {
    TA_HIP(hipStreamSynchronize(stream_));
    timings_.qap = ms_since(t1);
  }
  // (Measured and dropped: the l + h MSM on a third stream and host thread
  // beside the A MSM, 12.23-12.37 vs 11.95-12.20 ms per 2^20 proof, and the A
  // MSM after B2 on the G2 stream, 12.34-13.13 vs 11.81-12.09 -- the GPU is
  // already full with the G2 MSM beside the G1 ones.)
  auto t2 = Clock::now();
  msm1_->set_force_window_bits(c_a_);
  if (grouped) {
    // groups: [A | pad], [witness + h, first glen], [the rest | pad]
    // the group bases are fixed too: their fold table (prepare)
    const unsigned f1 = folds_[1];
    std::vector<P1> r;
    if (f1 > 1) {
      r = msm1_->run_groups_folded(g1_tab_.buf.template as<Affine<F1>>(), gscalars_.as<Fr>(), glen_, 3, f1);
    } else {
      r = msm1_->run_groups(gbases_.as<Affine<F1>>(), gscalars_.as<Fr>(), glen_, 3);
    }
    out.a = r[0];
    out.lh = r[1] + r[2];
  } else {  // (the multi-rank shards, and variant bit 0: fold tables per MSM)
    out.a = fixed_msm(*msm1_, a_tab_, a1 + 1 + q_lo, d_full + 1 + q_lo, q_len, g1_fold(), c_a_);
  }
  timings_.msm_a = ms_since(t2);
  t2 = Clock::now();
  out.b1 = with_b1 ? fixed_msm(*msm1_, b1_tab_, b1 + 1 + q_lo, d_full + 1 + q_lo, q_len, g1_fold(), c_a_)
                   : P1::zero();
  timings_.msm_b1 = ms_since(t2);
  t2 = Clock::now();
  // witness (l) and h MSMs merged; h_coefficients.size() == h_g1_query.size()
  // == domain size: the else branch of prove.h:103-112
  if (!grouped) {
    const size_t lh_lo = sp.lh_lo, lh_len = sp.lh_len;
    msm1_->set_force_window_bits(c_lh_);
    out.lh = fixed_msm(*msm1_, lh_tab_, lh1_.as<Affine<F1>>() + lh_lo, d_lh + lh_lo, lh_len, g1_fold(), c_lh_);
  }
  timings_.msm_l = grouped ? 0.f : ms_since(t2);
  timings_.msm_h = 0;
  g2_thread.join();
  if (g2_error) std::rethrow_exception(g2_error);
  out.b2 = acc_b2;
  timings_.total = ms_since(t0);
  return out;
}

template <class G1, class G2>
Proof<G1, G2> Groth16Prover<G1, G2>::assemble(const ProofPartials<G1, G2>* parts, size_t world, const Fr* r_ptr,
                                              const Fr* s_ptr) const {
  using P1 = XYZZ<F1>;
  using P2 = XYZZ<F2>;
  const Fr r = r_ptr ? *r_ptr : Fr::zero();
  const Fr s = s_ptr ? *s_ptr : Fr::zero();
  if (world == 0) throw std::runtime_error("tachyon_mi355x: Groth16 assemble needs at least one partial");
  P1 acc_a = P1::zero(), acc_b1 = P1::zero(), acc_lh = P1::zero();
  P2 acc_b2 = P2::zero();
  std::vector<bool> seen(world, false);
  for (size_t k = 0; k < world; ++k) {
    const auto& p = parts[k];
    if (p.magic != ProofPartials<G1, G2>().magic || p.bytes != sizeof(ProofPartials<G1, G2>))
      throw std::runtime_error("tachyon_mi355x: Groth16 partials blob has another layout (library version mismatch)");
    if (p.world != world || p.rank >= world || seen[p.rank])
      throw std::runtime_error("tachyon_mi355x: Groth16 partials are not one rank each of the same world");
    if (!r.is_zero() && !p.with_b1)
      throw std::runtime_error("tachyon_mi355x: Groth16 partials lack the B1 MSM that r != 0 needs");
    seen[p.rank] = true;
    acc_a = acc_a + p.a;
    acc_b1 = acc_b1 + p.b1;
    acc_lh = acc_lh + p.lh;
    acc_b2 = acc_b2 + p.b2;
  }

  // assembly on the host (a handful of point operations)
  auto aff1 = [](const Affine<F1>& a) { return P1::from_affine(a); };
  auto aff2 = [](const Affine<F2>& a) { return P2::from_affine(a); };
  const P1 delta1 = aff1(key_.delta_g1);
  // [A]_1 = alpha + a_0 + sum x_i a_i + r delta   (CalculateCoeff, prove.h:33-49)
  const P1 r_delta1 = mul_scalar(delta1, r);
  const P1 A = r_delta1 + aff1(key_.a1[0]) + acc_a + aff1(key_.alpha_g1);
  // [B]_2 = beta + b_0 + sum x_i b_i + s delta
  const P2 B2 = mul_scalar(aff2(key_.delta_g2), s) + aff2(key_.b2[0]) + acc_b2 + aff2(key_.beta_g2);
  // [C]_1 = s A + r B_1 - s r delta + sum_witness l_i + h
  P1 C = mul_scalar(A, s);
  if (!r.is_zero()) {
    const P1 B1 = mul_scalar(delta1, s) + aff1(key_.b1[0]) + acc_b1 + aff1(key_.beta_g1);
    C = C + mul_scalar(B1, r);
    C = C + mul_scalar(r_delta1, s).neg();
  }
  C = C + acc_lh;  // sum_witness l_i + h
  return Proof<G1, G2>{A.to_affine(), B2.to_affine(), C.to_affine()};
}

template <class G1, class G2>
Proof<G1, G2> Groth16Prover<G1, G2>::prove(const Fr* full, size_t count, const Fr* r, const Fr* s) {
  auto t0 = Clock::now();
  const bool with_b1 = r && !r->is_zero();
  const ProofPartials<G1, G2> part = partials(full, count, with_b1, 0, 1);
  Proof<G1, G2> proof = assemble(&part, 1, r, s);
  timings_.total = ms_since(t0);
  return proof;
}

template class Groth16Prover<Bn254G1, Bn254G2>;
template class Groth16Prover<Bls381G1, Bls381G2>;

}  // namespace groth16
}  // namespace tachyon_amd
