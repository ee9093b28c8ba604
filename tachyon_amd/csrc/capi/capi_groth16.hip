// C-ABI of the Groth16 prover (include/tachyon_mi355x.h, "Groth16 prover").
// Reference driver restated: vendors/circom/prover_main.cc:82-160 (parse zkey
// and wtns, build the domain, WitnessMapFromMatrices, CreateProofWithAssignment
// (NoZK)); errors abort like the reference's CHECKs.
#include "../../../include/tachyon_mi355x.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <thread>
#include <type_traits>
#include <vector>

#include "../dist/comm.h"
#include "../groth16/groth16.h"

using namespace tachyon_amd;

namespace {

[[noreturn]] void die(const char* fn, const char* what) {
  fprintf(stderr, "[tachyon_mi355x] %s failed: %s\n", fn, what);
  fflush(stderr);
  abort();
}

#define GUARD_BEGIN try {
#define GUARD_END                                                \
  }                                                              \
  catch (const std::exception& e) { die(__func__, e.what()); }   \
  catch (...) { die(__func__, "unknown exception"); }

using BnProver = groth16::Groth16Prover<Bn254G1, Bn254G2>;
using BlsProver = groth16::Groth16Prover<Bls381G1, Bls381G2>;

template <class P>
void prove_into(P* p, const void* full, size_t count, const void* r, const void* s, void* a, void* b, void* c) {
  using Fr = typename P::Fr;
  auto proof = p->prove(static_cast<const Fr*>(full), count, static_cast<const Fr*>(r), static_cast<const Fr*>(s));
  memcpy(a, &proof.a, sizeof(proof.a));
  memcpy(b, &proof.b, sizeof(proof.b));
  memcpy(c, &proof.c, sizeof(proof.c));
}

template <class P>
using PartialsOf = groth16::ProofPartials<typename std::remove_pointer_t<P>::G1Type,
                                          typename std::remove_pointer_t<P>::G2Type>;

template <class P>
void partials_into(P* p, const void* full, size_t count, int with_b1, uint32_t rank, uint32_t world, void* out) {
  using Fr = typename P::Fr;
  static_assert(std::is_trivially_copyable_v<PartialsOf<P>>);
  auto part = p->partials(static_cast<const Fr*>(full), count, with_b1 != 0, rank, world);
  memcpy(out, &part, sizeof(part));
}

template <class P>
void assemble_into(P* p, const void* parts, size_t world, const void* r, const void* s, void* a, void* b, void* c) {
  using Fr = typename P::Fr;
  std::vector<PartialsOf<P>> v(world);
  if (world) memcpy(v.data(), parts, world * sizeof(PartialsOf<P>));
  auto proof = p->assemble(v.data(), world, static_cast<const Fr*>(r), static_cast<const Fr*>(s));
  memcpy(a, &proof.a, sizeof(proof.a));
  memcpy(b, &proof.b, sizeof(proof.b));
  memcpy(c, &proof.c, sizeof(proof.c));
}

template <class P>
void witness_map_into(P* p, const void* full, size_t count, void* out_h) {
  using Fr = typename P::Fr;
  const auto& k = p->key();
  if (count != k.num_vars) throw std::runtime_error("assignment count != num_vars");
  DeviceBuffer d_full, d_h;
  Fr* df = static_cast<Fr*>(d_full.ensure(count * sizeof(Fr)));
  Fr* dh = static_cast<Fr*>(d_h.ensure((size_t)k.domain_size * sizeof(Fr)));
  TA_HIP(hipMemcpyAsync(df, full, count * sizeof(Fr), hipMemcpyDefault, p->stream()));
  p->witness_map(df, dh);
  TA_HIP(hipMemcpyAsync(out_h, dh, (size_t)k.domain_size * sizeof(Fr), hipMemcpyDeviceToHost, p->stream()));
  TA_HIP(hipStreamSynchronize(p->stream()));
}

// One-process multi-device proof: the multi-rank split of prove() (every
// device runs the witness map and its contiguous 1/N chunk of every MSM,
// Groth16Prover::partials) with one host thread per device instead of one
// process per GPU, and the partials added on the host by assemble() -- so a
// single-process caller (the reference's circom prover_main.cc:116-128 and
// prove.h:64-147 run in one process) uses several MI355X.  Ids may repeat
// (logical devices: provers sharing one GPU on separate streams).
template <class P>
void multi_prove_into(P* primary, std::vector<std::unique_ptr<P>>& provs, const std::vector<int>& devices,
                      const void* full, size_t count, const void* r, const void* s, void* a, void* b, void* c) {
  using Fr = typename P::Fr;
  const size_t N = provs.size();
  std::vector<PartialsOf<P*>> parts(N);
  std::vector<std::exception_ptr> err(N);
  std::vector<std::thread> th;
  for (size_t k = 0; k < N; ++k) {
    th.emplace_back([&, k] {
      try {
        TA_HIP(hipSetDevice(devices[k]));
        parts[k] = provs[k]->partials(static_cast<const Fr*>(full), count, r != nullptr, (uint32_t)k, (uint32_t)N);
      } catch (...) {
        err[k] = std::current_exception();
      }
    });
  }
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
  auto proof = primary->assemble(parts.data(), N, static_cast<const Fr*>(r), static_cast<const Fr*>(s));
  memcpy(a, &proof.a, sizeof(proof.a));
  memcpy(b, &proof.b, sizeof(proof.b));
  memcpy(c, &proof.c, sizeof(proof.c));
}

// One rank's share of a proof over a communicator: the witness map and this
// rank's chunk of every MSM (partials), one all-gather of the fixed-size
// partials blobs, and the same assembly on every rank -- the multi-process
// form of multi_prove_into with the exchange inside the library
// (Groth16Prover.prove_sharded in tachyon_amd/groth16.py is the torch.distributed form)
template <class P>
void sharded_prove_into(P* p, dist::Comm* comm, const void* full, size_t count, const void* r, const void* s, void* a,
                        void* b, void* c) {
  using Fr = typename P::Fr;
  using Parts = PartialsOf<P*>;
  const uint32_t world = (uint32_t)comm->world(), rank = (uint32_t)comm->rank();
  // (a rank whose partials fail still enters the exchange: dist::gather_checked)
  const std::vector<Parts> all = dist::gather_checked<Parts>(
      comm, [&] { return p->partials(static_cast<const Fr*>(full), count, r != nullptr, rank, world); });
  auto proof = p->assemble(all.data(), world, static_cast<const Fr*>(r), static_cast<const Fr*>(s));
  memcpy(a, &proof.a, sizeof(proof.a));
  memcpy(b, &proof.b, sizeof(proof.b));
  memcpy(c, &proof.c, sizeof(proof.c));
}

template <class P>
void make_device_provers(const P* primary, const std::vector<int>& devices, std::vector<std::unique_ptr<P>>& out) {
  int prev = 0;
  TA_HIP(hipGetDevice(&prev));
  const int src_device = prev;  // the primary prover's device (created on the current one)
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  out.clear();
  for (int d : devices) {
    TA_HIP(hipSetDevice(d));
    out.push_back(std::make_unique<P>(*primary, src_device));  // the key's points and matrices, peer copies
  }
}

template <class P>
void free_device_provers(const std::vector<int>& devices, std::vector<std::unique_ptr<P>>& provs) {
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) prev = 0;
  for (size_t k = 0; k < provs.size(); ++k) {
    (void)hipSetDevice(devices[k]);
    provs[k].reset();
  }
  provs.clear();
  (void)hipSetDevice(prev);
}

}  // namespace

struct tachyon_mi355x_groth16_prover {
  circom::CurveId curve;
  std::unique_ptr<BnProver> bn;
  std::unique_ptr<BlsProver> bls;
  // tachyon_mi355x_groth16_set_devices: one prover per device entry (empty = bn / bls alone)
  std::vector<int> devices;
  std::vector<std::unique_ptr<BnProver>> bn_dev;
  std::vector<std::unique_ptr<BlsProver>> bls_dev;
  ~tachyon_mi355x_groth16_prover() {
    free_device_provers(devices, bn_dev);
    free_device_provers(devices, bls_dev);
  }
};

#define PROVER_DISPATCH(p, ...)                         \
  do {                                                  \
    if ((p)->curve == circom::CurveId::kBn254) {        \
      auto* impl = (p)->bn.get();                       \
      __VA_ARGS__;                                      \
    } else {                                            \
      auto* impl = (p)->bls.get();                      \
      __VA_ARGS__;                                      \
    }                                                   \
  } while (0)

extern "C" {

int tachyon_mi355x_zkey_curve(const uint8_t* zkey, size_t len) {
  GUARD_BEGIN return (int)circom::zkey_curve(zkey, len); GUARD_END
}

tachyon_mi355x_groth16_prover* tachyon_mi355x_groth16_prover_create(const uint8_t* zkey, size_t len) {
  GUARD_BEGIN
  auto* p = new tachyon_mi355x_groth16_prover();
  p->curve = circom::zkey_curve(zkey, len);
  if (p->curve == circom::CurveId::kBn254)
    p->bn = std::make_unique<BnProver>(circom::parse_zkey<Bn254G1, Bn254G2>(zkey, len));
  else
    p->bls = std::make_unique<BlsProver>(circom::parse_zkey<Bls381G1, Bls381G2>(zkey, len));
  return p;
  GUARD_END
}

void tachyon_mi355x_groth16_prover_destroy(tachyon_mi355x_groth16_prover* prover) { delete prover; }

void tachyon_mi355x_groth16_prover_info(const tachyon_mi355x_groth16_prover* prover, uint32_t* out4) {
  GUARD_BEGIN
  PROVER_DISPATCH(prover, {
    const auto& k = impl->key();
    out4[0] = (uint32_t)prover->curve;
    out4[1] = k.num_vars;
    out4[2] = k.num_public;
    out4[3] = k.domain_size;
  });
  GUARD_END
}

void tachyon_mi355x_groth16_prove(tachyon_mi355x_groth16_prover* prover, const void* full, size_t count,
                                  const void* r, const void* s, void* out_a, void* out_b, void* out_c) {
  GUARD_BEGIN
  if (!prover->devices.empty()) {
    if (prover->curve == circom::CurveId::kBn254)
      multi_prove_into(prover->bn.get(), prover->bn_dev, prover->devices, full, count, r, s, out_a, out_b, out_c);
    else
      multi_prove_into(prover->bls.get(), prover->bls_dev, prover->devices, full, count, r, s, out_a, out_b, out_c);
    return;
  }
  PROVER_DISPATCH(prover, prove_into(impl, full, count, r, s, out_a, out_b, out_c));
  GUARD_END
}

void tachyon_mi355x_groth16_prove_sharded(tachyon_mi355x_groth16_prover* prover, tachyon_mi355x_comm* comm,
                                          const void* full, size_t count, const void* r, const void* s, void* out_a,
                                          void* out_b, void* out_c) {
  GUARD_BEGIN
  if (!comm || !comm->impl) throw std::runtime_error("null communicator");
  PROVER_DISPATCH(prover, sharded_prove_into(impl, comm->impl.get(), full, count, r, s, out_a, out_b, out_c));
  GUARD_END
}

int tachyon_mi355x_groth16_set_devices(tachyon_mi355x_groth16_prover* prover, const int* device_ids, size_t count) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  for (size_t i = 0; i < count; ++i)
    if (device_ids[i] < 0 || device_ids[i] >= n) return 0;  // refused, nothing changed
  GUARD_BEGIN
  free_device_provers(prover->devices, prover->bn_dev);
  free_device_provers(prover->devices, prover->bls_dev);
  prover->devices.clear();
  if (count > 1) {
    prover->devices.assign(device_ids, device_ids + count);
    if (prover->curve == circom::CurveId::kBn254) make_device_provers(prover->bn.get(), prover->devices, prover->bn_dev);
    else make_device_provers(prover->bls.get(), prover->devices, prover->bls_dev);
  }
  return 1;
  GUARD_END
  return 0;
}

size_t tachyon_mi355x_groth16_partials_size(const tachyon_mi355x_groth16_prover* prover) {
  GUARD_BEGIN
  PROVER_DISPATCH(prover, return sizeof(PartialsOf<decltype(impl)>));
  GUARD_END
}

void tachyon_mi355x_groth16_prove_partials(tachyon_mi355x_groth16_prover* prover, const void* full, size_t count,
                                           int with_b1, uint32_t rank, uint32_t world, void* out) {
  GUARD_BEGIN PROVER_DISPATCH(prover, partials_into(impl, full, count, with_b1, rank, world, out)); GUARD_END
}

void tachyon_mi355x_groth16_assemble(tachyon_mi355x_groth16_prover* prover, const void* parts, size_t world,
                                     const void* r, const void* s, void* out_a, void* out_b, void* out_c) {
  GUARD_BEGIN PROVER_DISPATCH(prover, assemble_into(impl, parts, world, r, s, out_a, out_b, out_c)); GUARD_END
}

void tachyon_mi355x_groth16_witness_map(tachyon_mi355x_groth16_prover* prover, const void* full, size_t count,
                                        void* out_h) {
  GUARD_BEGIN PROVER_DISPATCH(prover, witness_map_into(impl, full, count, out_h)); GUARD_END
}

size_t tachyon_mi355x_groth16_prepare(tachyon_mi355x_groth16_prover* prover, uint32_t rank, uint32_t world,
                                      int with_b1) {
  GUARD_BEGIN
  if (!prover->devices.empty()) {  // every device prover for its entry of the one-process split
    const size_t N = prover->devices.size();
    int prev = 0;
    TA_HIP(hipGetDevice(&prev));
    size_t bytes = 0;
    for (size_t k = 0; k < N; ++k) {
      TA_HIP(hipSetDevice(prover->devices[k]));
      if (prover->curve == circom::CurveId::kBn254)
        bytes += prover->bn_dev[k]->prepare((uint32_t)k, (uint32_t)N, with_b1 != 0);
      else
        bytes += prover->bls_dev[k]->prepare((uint32_t)k, (uint32_t)N, with_b1 != 0);
    }
    TA_HIP(hipSetDevice(prev));
    return bytes;
  }
  PROVER_DISPATCH(prover, return impl->prepare(rank, world, with_b1 != 0));
  GUARD_END
}

void tachyon_mi355x_groth16_prover_folds(const tachyon_mi355x_groth16_prover* prover, uint32_t* out5) {
  GUARD_BEGIN
  PROVER_DISPATCH(prover, {
    unsigned f[5];
    if (!prover->bn_dev.empty()) prover->bn_dev[0]->last_folds(f);
    else if (!prover->bls_dev.empty()) prover->bls_dev[0]->last_folds(f);
    else impl->last_folds(f);
    for (int i = 0; i < 5; ++i) out5[i] = f[i];
  });
  GUARD_END
}

void tachyon_mi355x_groth16_set_profile(tachyon_mi355x_groth16_prover* prover, int on) {
  GUARD_BEGIN
  PROVER_DISPATCH(prover, impl->set_profile(on != 0));
  for (auto& p : prover->bn_dev) p->set_profile(on != 0);
  for (auto& p : prover->bls_dev) p->set_profile(on != 0);
  GUARD_END
}

int tachyon_mi355x_groth16_set_variant(tachyon_mi355x_groth16_prover* prover, int variant) {
  if (!BnProver::valid_variant(variant)) return 0;
  GUARD_BEGIN
  PROVER_DISPATCH(prover, impl->set_variant(variant));
  for (auto& p : prover->bn_dev) p->set_variant(variant);
  for (auto& p : prover->bls_dev) p->set_variant(variant);
  GUARD_END
  return 1;
}

void tachyon_mi355x_groth16_set_msm_window_bits(tachyon_mi355x_groth16_prover* prover, unsigned c_a, unsigned c_lh,
                                               unsigned c_b2) {
  GUARD_BEGIN
  PROVER_DISPATCH(prover, impl->set_msm_window_bits(c_a, c_lh, c_b2));
  for (auto& p : prover->bn_dev) p->set_msm_window_bits(c_a, c_lh, c_b2);
  for (auto& p : prover->bls_dev) p->set_msm_window_bits(c_a, c_lh, c_b2);
  GUARD_END
}

// After set_devices the proof runs on the per-device provers: report the lead
// device's (rank 0's) phases, as the MSM C-API reports multi->lead()
void tachyon_mi355x_groth16_last_timings(const tachyon_mi355x_groth16_prover* prover, float* out8) {
  GUARD_BEGIN
  PROVER_DISPATCH(prover, {
    const auto& t = !prover->bn_dev.empty() ? prover->bn_dev[0]->timings()
                    : !prover->bls_dev.empty() ? prover->bls_dev[0]->timings() : impl->timings();
    const float v[8] = {t.upload, t.qap, t.msm_a, t.msm_b2, t.msm_b1, t.msm_l, t.msm_h, t.total};
    memcpy(out8, v, sizeof(v));
  });
  GUARD_END
}

size_t tachyon_mi355x_wtns_parse(int curve, const uint8_t* wtns, size_t len, void* out, size_t cap) {
  GUARD_BEGIN
  auto emit = [&](const auto& v) {
    if (out) memcpy(out, v.data(), std::min(cap, v.size()) * sizeof(v[0]));
    return v.size();
  };
  if (curve == 0) return emit(circom::parse_wtns<Bn254Fr>(wtns, len));
  if (curve == 1) return emit(circom::parse_wtns<Bls381Fr>(wtns, len));
  throw std::runtime_error("curve must be 0 (bn254) or 1 (bls12_381)");
  GUARD_END
}

}  // extern "C"
