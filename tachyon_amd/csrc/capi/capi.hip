// C-ABI of the MI355X backend (include/tachyon_mi355x.h).
//
// Reference entry points restated here:
//   tachyon/c/math/elliptic_curves/generator/msm.cc.tpl, msm_gpu.cc.tpl
//   tachyon/c/math/elliptic_curves/msm/msm.h:13-48 (MSMApi / DoMSM)
//   tachyon/c/math/elliptic_curves/msm/msm_gpu.h:23-122 (MSMGpuApi / DoMSMGpu,
//     TACHYON_MSM_GPU_INPUT_DIR / TACHYON_LOG_MSM hooks)
//   tachyon/c/math/polynomials/univariate/bn254_univariate_evaluation_domain.cc:22-85
//   tachyon/c/math/polynomials/univariate/bn254_univariate_evaluations.cc
//   tachyon/c/math/polynomials/univariate/bn254_univariate_dense_polynomial.cc
#include "../../../include/tachyon_mi355x.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "../dist/comm.h"
#include "../msm/msm.h"
#include "../msm/msm_multi.h"
#include "../ntt/ntt.h"
#include "../util/device_ops.h"

using namespace tachyon_amd;

namespace {

[[noreturn]] void die(const char* fn, const char* what) {
  fprintf(stderr, "[tachyon_mi355x] %s failed: %s\n", fn, what);
  fflush(stderr);
  abort();  // the reference CHECK-aborts (msm.h:42-43, msm_gpu.h:79-80)
}

#define GUARD_BEGIN try {
#define GUARD_END                                   \
  }                                                 \
  catch (const std::exception& e) { die(__func__, e.what()); } \
  catch (...) { die(__func__, "unknown exception"); }

template <class Curve>
struct MsmCtx {
  msm::MsmGpu<Curve> impl;
  // several devices (tachyon_mi355x_msm_gpu_set_devices or TACHYON_MSM_GPU_DEVICES): one point
  // shard per device, results added on the host (msm/msm_multi.h); null = impl on the current device
  std::unique_ptr<msm::MsmMultiDevice<Curve>> multi;
  std::string input_dir;  // TACHYON_MSM_GPU_INPUT_DIR
  bool log = false;       // TACHYON_LOG_MSM=1
  size_t idx = 0;
  explicit MsmCtx(hipStream_t stream = nullptr) : impl(stream) {
    if (const char* d = getenv("TACHYON_MSM_GPU_INPUT_DIR")) input_dir = d;
    if (const char* l = getenv("TACHYON_LOG_MSM")) log = (std::string(l) == "1");
    if (const char* e = getenv("TACHYON_MSM_GPU_DEVICES")) {
      const std::vector<int> ids = msm::parse_device_list(e);
      if (ids.empty()) throw std::runtime_error(std::string("TACHYON_MSM_GPU_DEVICES: malformed device list '") + e + "'");
      if (ids.size() > 1) multi = std::make_unique<msm::MsmMultiDevice<Curve>>(ids);
    }
  }
  XYZZ<typename Curve::F> run(const void* bases, const void* scalars, size_t n) {
    return multi ? multi->run(bases, scalars, n) : impl.run(bases, scalars, n);
  }
};

template <class F>
void write_canonical(FILE* f, const F& x);

template <class C>
void write_canonical(FILE* f, const Fp<C>& x) {
  Fp<C> c = x.from_mont();
  fwrite(c.v, sizeof(c.v), 1, f);
}
template <class B>
void write_canonical(FILE* f, const Fp2<B>& x) {
  write_canonical(f, x.c0);
  write_canonical(f, x.c1);
}

// Replay dump (msm_gpu.h:99-119): u64 count, then canonical LE limbs
// (Buffer serialisation with s_is_in_montgomery = false, copyable.h:137-155).
template <class Curve>
void dump_inputs(const std::string& dir, size_t idx, const void* bases, const void* scalars, size_t n) {
  using F = typename Curve::F;
  using Fr = typename Curve::Fr;
  std::vector<Affine<F>> hb(n);
  std::vector<Fr> hs(n);
  TA_HIP(hipMemcpy(hb.data(), bases, n * sizeof(Affine<F>), hipMemcpyDefault));
  TA_HIP(hipMemcpy(hs.data(), scalars, n * sizeof(Fr), hipMemcpyDefault));
  std::string pb = dir + "/bases" + std::to_string(idx) + ".txt";
  std::string ps = dir + "/scalars" + std::to_string(idx) + ".txt";
  FILE* f = fopen(pb.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open " + pb);
  uint64_t cnt = n;
  fwrite(&cnt, 8, 1, f);
  for (auto& p : hb) {
    write_canonical(f, p.x);
    write_canonical(f, p.y);
  }
  fclose(f);
  f = fopen(ps.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open " + ps);
  fwrite(&cnt, 8, 1, f);
  for (auto& s : hs) write_canonical(f, s);
  fclose(f);
}

// canonical value in hex, "0x" + lowercase digits without leading zeros
// (BigInt::ToHexString, big_int.cc:55-58; fields print their canonical value)
template <class C>
void print_hex(const Fp<C>& x) {
  const Fp<C> c = x.from_mont();
  const uint32_t* l = c.v;
  int i = Fp<C>::N - 1;
  while (i > 0 && l[i] == 0) --i;
  printf("0x%x", l[i]);
  while (--i >= 0) printf("%08x", l[i]);
}
template <class B>
void print_hex(const Fp2<B>& x) {
  printf("(");
  print_hex(x.c0);
  printf(", ");
  print_hex(x.c1);
  printf(")");
}

// DoMSMGpu: run, normalise, return a new Jacobian (z = 1, or the (1,1,0) zero).
template <class Curve, class CJac>
CJac* do_msm(MsmCtx<Curve>* ctx, const void* bases, const void* scalars, size_t n) {
  using F = typename Curve::F;
  XYZZ<F> r = ctx->run(bases, scalars, n);
  Affine<F> a = r.to_affine();
  Jacobian<F> j = a.is_zero() ? Jacobian<F>::zero() : Jacobian<F>{a.x, a.y, F::one()};
  static_assert(sizeof(CJac) == sizeof(Jacobian<F>), "layout");
  CJac* out = new CJac();
  memcpy(out, &j, sizeof(j));
  if (ctx->log) {
    printf("DoMSMGpu()%zu\n(", ctx->idx);
    print_hex(a.x);
    printf(", ");
    print_hex(a.y);
    printf(")\n");
  }
  ctx->idx++;
  if (!ctx->input_dir.empty()) dump_inputs<Curve>(ctx->input_dir, ctx->idx - 1, bases, scalars, n);
  return out;
}

template <class Curve>
void msm_affine_out(void* ctx, const void* bases, const void* scalars, size_t n, void* out) {
  using F = typename Curve::F;
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  Affine<F> a = c->run(bases, scalars, n).to_affine();
  memcpy(out, &a, sizeof(a));
}

template <class Curve>
void msm_window_range_out(void* ctx, const void* bases, const void* scalars, size_t n, unsigned w_begin,
                          unsigned w_end, void* out) {
  using F = typename Curve::F;
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  Affine<F> a = c->impl.run_window_range(bases, scalars, n, w_begin, w_end).to_affine();
  memcpy(out, &a, sizeof(a));
}

template <class Curve>
void msm_folded_out(void* ctx, const void* folded_bases, const void* scalars, size_t n, unsigned fold, void* out) {
  using F = typename Curve::F;
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  Affine<F> a = c->impl.run_folded(folded_bases, scalars, n, fold).to_affine();
  memcpy(out, &a, sizeof(a));
}

// `count` MSMs over the same device-resident bases in one launch sequence
// (MsmGpu::run_batch): count affine results ((0, 0) = identity)
template <class Curve>
void msm_batch_out(void* ctx, const void* bases, size_t len, const void* scalars, size_t count, void* out) {
  using F = typename Curve::F;
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  const auto pts = c->impl.run_batch(bases, scalars, len, count);
  auto* o = static_cast<Affine<F>*>(out);
  for (size_t g = 0; g < count; ++g) o[g] = pts[g].to_affine();
}

// The MSM in the point form a C++ caller asks for (include/tachyon_mi355x_msm.h):
// 0 affine {x, y} ((0, 0) = identity); 1 projective / 2 Jacobian {x, y, z}
// (identity (1, 1, 0), projective_point.h:34-36, jacobian_point.h; otherwise
// z = 1); 3 XYZZ {x, y, zz, zzz} (identity (1, 1, 0, 0), point_xyzz.h:37-39) --
// the Bucket of VariableBaseMSM<AffinePoint> (pippenger_base.h:24-28).
template <class Curve>
void msm_form_out(void* ctx, const void* bases, const void* scalars, size_t n, int form, void* out) {
  using F = typename Curve::F;
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  const Affine<F> a = c->run(bases, scalars, n).to_affine();
  switch (form) {
    case 0:
      memcpy(out, &a, sizeof(a));
      break;
    case 1:
    case 2: {
      const Jacobian<F> j = a.is_zero() ? Jacobian<F>::zero() : Jacobian<F>{a.x, a.y, F::one()};
      memcpy(out, &j, sizeof(j));
      break;
    }
    case 3: {
      const XYZZ<F> p = XYZZ<F>::from_affine(a);
      memcpy(out, &p, sizeof(p));
      break;
    }
    default:
      throw std::runtime_error("point form must be 0 (affine), 1 (projective), 2 (jacobian) or 3 (xyzz)");
  }
}

// Non-affine bases (VariableBaseMSM<ProjectivePoint / JacobianPoint /
// PointXYZZ>): normalised to affine on the device, then the MSM above
template <class Curve>
void msm_points_form_out(void* ctx, const void* bases, int base_form, const void* scalars, size_t n, int form,
                         void* out) {
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  const void* aff = c->impl.affine_bases(bases, n, base_form);
  msm_form_out<Curve>(ctx, aff, scalars, n, form, out);
}

// One rank's shard of an MSM over a communicator: the local XYZZ partial,
// one all-gather of every rank's partial, the group sum in rank order (the
// same point on every rank) -- the kParallelTerm chunk-and-sum
// (pippenger_adapter.h:82-113) across processes, with the exchange inside
// the library (tachyon_amd.dist.sharded_msm is the torch.distributed form)
template <class Curve>
void msm_sharded_out(void* ctx, dist::Comm* comm, const void* bases, const void* scalars, size_t n, void* out) {
  using F = typename Curve::F;
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  // (a rank whose local MSM fails still enters the exchange: dist::gather_checked)
  const std::vector<XYZZ<F>> all = dist::gather_checked<XYZZ<F>>(comm, [&] {
    if (!c) throw std::runtime_error("null MSM context");
    return c->run(bases, scalars, n);
  });
  XYZZ<F> acc = XYZZ<F>::zero();
  for (const auto& p : all) acc = acc + p;
  const Affine<F> a = acc.to_affine();
  memcpy(out, &a, sizeof(a));
}

// One rank's part of a tachyon_mi355x_msm_shard plan: its point group over
// its window range (the hybrid partition; a point shard when window_groups
// is 1), the all-gather of the XYZZ partials and their sum in rank order.
// The window-range partials sum_{w in range} 2^(c w) S_w of the Q ranges of
// one point group add up to that group's MSM, the groups' to the whole MSM.
template <class Curve>
void msm_sharded_plan_out(void* ctx, dist::Comm* comm, const tachyon_mi355x_msm_shard& p, const void* bases,
                          const void* scalars, void* out) {
  using F = typename Curve::F;
  auto* c = static_cast<MsmCtx<Curve>*>(ctx);
  const std::vector<XYZZ<F>> all = dist::gather_checked<XYZZ<F>>(comm, [&]() -> XYZZ<F> {
    if (!c) throw std::runtime_error("null MSM context");
    if (p.window_groups <= 1) return c->run(bases, scalars, p.count);
    struct Restore {
      msm::MsmGpu<Curve>& m;
      unsigned c;
      ~Restore() { m.set_force_window_bits(c); }
    } restore{c->impl, c->impl.force_window_bits()};
    c->impl.set_force_window_bits(p.window_bits);
    return c->impl.run_window_range(bases, scalars, p.count, p.w_begin, p.w_end);
  });
  XYZZ<F> acc = XYZZ<F>::zero();
  for (const auto& q : all) acc = acc + q;
  const Affine<F> a = acc.to_affine();
  memcpy(out, &a, sizeof(a));
}

// The hybrid point x window partitions (curve id, world) -> (window groups Q,
// window bits c) that beat point shards on one MI355X (the slowest rank of
// each partition timed with the real kernels: BN254 G1 2^26 at 8 ranks 11.45
// vs 12.11 ms, profiles/r05c; BLS12-381 G2 2^24 at 4 / 8 ranks 31.16 / 17.21
// vs 32.19 / 17.81 ms, profiles/r05m); point shards everywhere else.
struct HybridPlan {
  int curve, world;
  unsigned q, c;
};
constexpr HybridPlan kHybridPlans[] = {{0, 8, 2, 19}, {3, 4, 2, 19}, {3, 8, 4, 16}};

template <class Curve>
void affine_sum(const void* pts, size_t count, void* out) {
  using F = typename Curve::F;
  const Affine<F>* p = static_cast<const Affine<F>*>(pts);
  XYZZ<F> acc = XYZZ<F>::zero();
  for (size_t i = 0; i < count; ++i) acc = acc.madd(p[i]);
  Affine<F> a = acc.to_affine();
  memcpy(out, &a, sizeof(a));
}

template <class Curve>
void jac_to_affine(const void* jac, void* out) {
  using F = typename Curve::F;
  Jacobian<F> j;
  memcpy(&j, jac, sizeof(j));
  Affine<F> a = XYZZ<F>::from_jacobian(j).to_affine();
  memcpy(out, &a, sizeof(a));
}

}  // namespace

namespace tachyon_amd::capi_detail {
// univariate containers hold std::vector<bn254::Fr>, like the reference
using FrC = tachyon_bn254_fr;
struct Vec {
  std::vector<FrC> v;
};
struct Domain {
  std::unique_ptr<ntt::NttDomain<Bn254Fr>> impl;
  int device = 0;  // the device the domain was created on (the multi-device primary)
  // set_devices: the four-step over several devices for the plain domain
  // (declared after impl: destroyed first, while impl's stream still exists)
  std::unique_ptr<ntt::NttMultiDevice<Bn254Fr>> multi;
  ntt::NttMultiDevice<Bn254Fr>* multi_for_plain() const {
    return multi && impl->offset().is_one() ? multi.get() : nullptr;
  }
};
// UnivariateEvaluations<RationalField<bn254::Fr>>: {numerator, denominator}
// pairs; Zero() = 0 / 1 (math/base/rational_field.h:33,199-200)
struct RationalVec {
  std::vector<FrC> num, den;
};
}  // namespace tachyon_amd::capi_detail
using tachyon_amd::capi_detail::RationalVec;
using tachyon_amd::capi_detail::Domain;
using tachyon_amd::capi_detail::FrC;
using tachyon_amd::capi_detail::Vec;

struct tachyon_bn254_univariate_evaluations : Vec {};
struct tachyon_bn254_univariate_dense_polynomial : Vec {};
struct tachyon_bn254_univariate_evaluation_domain : Domain {};
struct tachyon_bn254_univariate_rational_evaluations : RationalVec {};

struct tachyon_bn254_g1_msm : MsmCtx<Bn254G1> {};
struct tachyon_bn254_g1_msm_gpu : MsmCtx<Bn254G1> {};
struct tachyon_bls12_381_g1_msm : MsmCtx<Bls381G1> {};
struct tachyon_bls12_381_g1_msm_gpu : MsmCtx<Bls381G1> {};
struct tachyon_bn254_g2_msm_gpu : MsmCtx<Bn254G2> {};
struct tachyon_bls12_381_g2_msm_gpu : MsmCtx<Bls381G2> {};

extern "C" {

void tachyon_bn254_g1_init(void) {}
void tachyon_bls12_381_g1_init(void) {}
void tachyon_bn254_g2_init(void) {}
void tachyon_bls12_381_g2_init(void) {}

// ---- BN254 G1 ----
tachyon_bn254_g1_msm_ptr tachyon_bn254_g1_create_msm(uint8_t degree) {
  (void)degree;  // unused, as in msm.h:23
  GUARD_BEGIN return new tachyon_bn254_g1_msm(); GUARD_END
}
void tachyon_bn254_g1_destroy_msm(tachyon_bn254_g1_msm_ptr ptr) { delete ptr; }
tachyon_bn254_g1_jacobian* tachyon_bn254_g1_point2_msm(tachyon_bn254_g1_msm_ptr ptr,
                                                       const tachyon_bn254_g1_point2* bases,
                                                       const tachyon_bn254_fr* scalars, size_t size) {
  GUARD_BEGIN return do_msm<Bn254G1, tachyon_bn254_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}
tachyon_bn254_g1_jacobian* tachyon_bn254_g1_affine_msm(tachyon_bn254_g1_msm_ptr ptr,
                                                       const tachyon_bn254_g1_affine* bases,
                                                       const tachyon_bn254_fr* scalars, size_t size) {
  GUARD_BEGIN return do_msm<Bn254G1, tachyon_bn254_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}
tachyon_bn254_g1_msm_gpu_ptr tachyon_bn254_g1_create_msm_gpu(uint8_t degree) {
  (void)degree;
  GUARD_BEGIN return new tachyon_bn254_g1_msm_gpu(); GUARD_END
}
void tachyon_bn254_g1_destroy_msm_gpu(tachyon_bn254_g1_msm_gpu_ptr ptr) { delete ptr; }
tachyon_bn254_g1_jacobian* tachyon_bn254_g1_point2_msm_gpu(tachyon_bn254_g1_msm_gpu_ptr ptr,
                                                           const tachyon_bn254_g1_point2* bases,
                                                           const tachyon_bn254_fr* scalars, size_t size) {
  GUARD_BEGIN return do_msm<Bn254G1, tachyon_bn254_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}
tachyon_bn254_g1_jacobian* tachyon_bn254_g1_affine_msm_gpu(tachyon_bn254_g1_msm_gpu_ptr ptr,
                                                           const tachyon_bn254_g1_affine* bases,
                                                           const tachyon_bn254_fr* scalars, size_t size) {
  GUARD_BEGIN return do_msm<Bn254G1, tachyon_bn254_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}

// ---- BLS12-381 G1 ----
tachyon_bls12_381_g1_msm_ptr tachyon_bls12_381_g1_create_msm(uint8_t degree) {
  (void)degree;
  GUARD_BEGIN return new tachyon_bls12_381_g1_msm(); GUARD_END
}
void tachyon_bls12_381_g1_destroy_msm(tachyon_bls12_381_g1_msm_ptr ptr) { delete ptr; }
tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_point2_msm(tachyon_bls12_381_g1_msm_ptr ptr,
                                                               const tachyon_bls12_381_g1_point2* bases,
                                                               const tachyon_bls12_381_fr* scalars, size_t size) {
  GUARD_BEGIN return do_msm<Bls381G1, tachyon_bls12_381_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}
tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_affine_msm(tachyon_bls12_381_g1_msm_ptr ptr,
                                                               const tachyon_bls12_381_g1_affine* bases,
                                                               const tachyon_bls12_381_fr* scalars, size_t size) {
  GUARD_BEGIN return do_msm<Bls381G1, tachyon_bls12_381_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}
tachyon_bls12_381_g1_msm_gpu_ptr tachyon_bls12_381_g1_create_msm_gpu(uint8_t degree) {
  (void)degree;
  GUARD_BEGIN return new tachyon_bls12_381_g1_msm_gpu(); GUARD_END
}
void tachyon_bls12_381_g1_destroy_msm_gpu(tachyon_bls12_381_g1_msm_gpu_ptr ptr) { delete ptr; }
tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_point2_msm_gpu(tachyon_bls12_381_g1_msm_gpu_ptr ptr,
                                                                   const tachyon_bls12_381_g1_point2* bases,
                                                                   const tachyon_bls12_381_fr* scalars,
                                                                   size_t size) {
  GUARD_BEGIN return do_msm<Bls381G1, tachyon_bls12_381_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}
tachyon_bls12_381_g1_jacobian* tachyon_bls12_381_g1_affine_msm_gpu(tachyon_bls12_381_g1_msm_gpu_ptr ptr,
                                                                   const tachyon_bls12_381_g1_affine* bases,
                                                                   const tachyon_bls12_381_fr* scalars,
                                                                   size_t size) {
  GUARD_BEGIN return do_msm<Bls381G1, tachyon_bls12_381_g1_jacobian>(ptr, bases, scalars, size); GUARD_END
}

// ---- G2 (extension) ----
tachyon_bn254_g2_msm_gpu_ptr tachyon_bn254_g2_create_msm_gpu(uint8_t degree) {
  (void)degree;
  GUARD_BEGIN return new tachyon_bn254_g2_msm_gpu(); GUARD_END
}
void tachyon_bn254_g2_destroy_msm_gpu(tachyon_bn254_g2_msm_gpu_ptr ptr) { delete ptr; }
tachyon_bn254_g2_jacobian* tachyon_bn254_g2_affine_msm_gpu(tachyon_bn254_g2_msm_gpu_ptr ptr,
                                                           const tachyon_bn254_g2_affine* bases,
                                                           const tachyon_bn254_fr* scalars, size_t size) {
  GUARD_BEGIN return do_msm<Bn254G2, tachyon_bn254_g2_jacobian>(ptr, bases, scalars, size); GUARD_END
}
tachyon_bls12_381_g2_msm_gpu_ptr tachyon_bls12_381_g2_create_msm_gpu(uint8_t degree) {
  (void)degree;
  GUARD_BEGIN return new tachyon_bls12_381_g2_msm_gpu(); GUARD_END
}
void tachyon_bls12_381_g2_destroy_msm_gpu(tachyon_bls12_381_g2_msm_gpu_ptr ptr) { delete ptr; }
tachyon_bls12_381_g2_jacobian* tachyon_bls12_381_g2_affine_msm_gpu(tachyon_bls12_381_g2_msm_gpu_ptr ptr,
                                                                   const tachyon_bls12_381_g2_affine* bases,
                                                                   const tachyon_bls12_381_fr* scalars,
                                                                   size_t size) {
  GUARD_BEGIN return do_msm<Bls381G2, tachyon_bls12_381_g2_jacobian>(ptr, bases, scalars, size); GUARD_END
}

// ---- curve-generic extensions ----
#define CURVE_DISPATCH(curve, CALL)                               \
  switch (curve) {                                                \
    case 0: { using C = Bn254G1; CALL; } break;                   \
    case 1: { using C = Bn254G2; CALL; } break;                   \
    case 2: { using C = Bls381G1; CALL; } break;                  \
    case 3: { using C = Bls381G2; CALL; } break;                  \
    default: throw std::runtime_error("unknown curve id");        \
  }

void tachyon_mi355x_msm_gpu_affine(int curve, void* ctx, const void* bases, const void* scalars, size_t size,
                                   void* out_affine) {
  GUARD_BEGIN CURVE_DISPATCH(curve, msm_affine_out<C>(ctx, bases, scalars, size, out_affine)) GUARD_END
}
void tachyon_mi355x_msm_gpu_window_range_affine(int curve, void* ctx, const void* bases, const void* scalars,
                                                size_t size, unsigned w_begin, unsigned w_end, void* out_affine) {
  GUARD_BEGIN CURVE_DISPATCH(curve, msm_window_range_out<C>(ctx, bases, scalars, size, w_begin, w_end, out_affine))
  GUARD_END
}
int tachyon_mi355x_msm_gpu_batch_affine(int curve, void* ctx, const void* bases, size_t len, const void* scalars,
                                        size_t count, void* out_affine) {
  if (!is_device_pointer(bases)) return 0;
  GUARD_BEGIN CURVE_DISPATCH(curve, msm_batch_out<C>(ctx, bases, len, scalars, count, out_affine)) GUARD_END
  return 1;
}
unsigned tachyon_mi355x_msm_gpu_plan_windows(int curve, const void* ctx, size_t size) {
  GUARD_BEGIN CURVE_DISPATCH(curve, return static_cast<const MsmCtx<C>*>(ctx)->impl.plan_windows(size)) GUARD_END
  return 0;
}
int tachyon_mi355x_msm_gpu_fold_bases(int curve, void* ctx, const void* bases, size_t size, unsigned fold,
                                      void* out_bases) {
  if (fold == 0 || !is_device_pointer(bases) || !is_device_pointer(out_bases)) return 0;
  if (tachyon_mi355x_msm_gpu_plan_windows(curve, ctx, size) % fold != 0) return 0;  // refused, nothing written
  GUARD_BEGIN CURVE_DISPATCH(curve, static_cast<MsmCtx<C>*>(ctx)->impl.fold_bases(bases, size, fold, out_bases))
  GUARD_END
  return 1;
}
int tachyon_mi355x_msm_gpu_folded_affine(int curve, void* ctx, const void* folded_bases, const void* scalars,
                                         size_t size, unsigned fold, void* out_affine) {
  if (fold == 0 || !is_device_pointer(folded_bases) || !is_device_pointer(scalars)) return 0;
  if (fold > 1 && tachyon_mi355x_msm_gpu_plan_windows(curve, ctx, size) % fold != 0) return 0;
  GUARD_BEGIN CURVE_DISPATCH(curve, msm_folded_out<C>(ctx, folded_bases, scalars, size, fold, out_affine)) GUARD_END
  return 1;
}
void* tachyon_mi355x_msm_gpu_create(int curve, void* stream) {
  GUARD_BEGIN CURVE_DISPATCH(curve, return new MsmCtx<C>(static_cast<hipStream_t>(stream))) GUARD_END
  return nullptr;
}
void tachyon_mi355x_msm_gpu_destroy(int curve, void* ctx) {
  if (!ctx) return;
  GUARD_BEGIN CURVE_DISPATCH(curve, delete static_cast<MsmCtx<C>*>(ctx)) GUARD_END
}
int tachyon_mi355x_msm_gpu_run(int curve, void* ctx, const void* bases, size_t bases_size, const void* scalars,
                               size_t scalars_size, int form, void* out) {
  if (bases_size != scalars_size) return 0;  // IcicleMSM::Run / PippengerAdapter: sizes must match
  GUARD_BEGIN CURVE_DISPATCH(curve, msm_form_out<C>(ctx, bases, scalars, scalars_size, form, out)) GUARD_END
  return 1;
}
void tachyon_mi355x_msm_gpu_sharded_affine(int curve, void* ctx, tachyon_mi355x_comm* comm, const void* bases,
                                           const void* scalars, size_t size, void* out_affine) {
  GUARD_BEGIN
  if (!comm || !comm->impl) throw std::runtime_error("null communicator");
  CURVE_DISPATCH(curve, msm_sharded_out<C>(ctx, comm->impl.get(), bases, scalars, size, out_affine))
  GUARD_END
}
int tachyon_mi355x_msm_shard_plan(int curve, size_t n_total, int world, int rank, tachyon_mi355x_msm_shard* out) {
  if (!out || curve < 0 || curve > 3 || world < 1 || rank < 0 || rank >= world) return 0;
  unsigned q = 1, c = 0;
  for (const HybridPlan& h : kHybridPlans)
    if (h.curve == curve && h.world == world) {
      q = h.q;
      c = h.c;
    }
  const unsigned p = (unsigned)world / q;
  // point group rank / q: the ceil split of base::ParallelizeMap (dist.shard_range)
  const size_t chunk = (n_total + p - 1) / p;
  const size_t start = std::min<size_t>((size_t)(rank / q) * chunk, n_total);
  tachyon_mi355x_msm_shard s{};
  s.start = start;
  s.count = std::min(chunk, n_total - start);
  s.point_groups = p;
  s.window_groups = q;
  if (q > 1) {
    const unsigned bits = curve < 2 ? Bn254Fr::Config::kModulusBits : Bls381Fr::Config::kModulusBits;
    const unsigned W = (bits + 1 + c - 1) / c;
    const unsigned base = W / q, extra = W % q, j = (unsigned)rank % q;  // contiguous ranges (dist.window_range)
    s.window_bits = c;
    s.w_begin = j * base + std::min(j, extra);
    s.w_end = s.w_begin + base + (j < extra ? 1 : 0);
  }
  *out = s;
  return 1;
}
int tachyon_mi355x_msm_gpu_sharded_plan_affine(int curve, void* ctx, tachyon_mi355x_comm* comm,
                                               const tachyon_mi355x_msm_shard* plan, const void* bases,
                                               const void* scalars, void* out_affine) {
  // (no abort: a failure of any rank's local part reaches every rank through
  // the exchange, and every rank returns 0 with the message on stderr)
  try {
    if (!comm || !comm->impl) throw std::runtime_error("null communicator");
    if (!plan) throw std::runtime_error("null shard plan");
    CURVE_DISPATCH(curve, msm_sharded_plan_out<C>(ctx, comm->impl.get(), *plan, bases, scalars, out_affine))
    return 1;
  } catch (const std::exception& e) {
    fprintf(stderr, "[tachyon_mi355x] %s failed: %s\n", __func__, e.what());
    fflush(stderr);
  } catch (...) {
    fprintf(stderr, "[tachyon_mi355x] %s failed: unknown exception\n", __func__);
    fflush(stderr);
  }
  return 0;
}
int tachyon_mi355x_msm_gpu_run_points(int curve, void* ctx, const void* bases, size_t bases_size, int base_form,
                                      const void* scalars, size_t scalars_size, int form, void* out) {
  if (bases_size != scalars_size) return 0;
  GUARD_BEGIN CURVE_DISPATCH(curve, msm_points_form_out<C>(ctx, bases, base_form, scalars, scalars_size, form, out))
  GUARD_END
  return 1;
}
void tachyon_mi355x_msm_gpu_set_window_bits(int curve, void* ctx, unsigned c) {
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    auto* m = static_cast<MsmCtx<C>*>(ctx);
    m->impl.set_force_window_bits(c);
    if (m->multi) m->multi->set_force_window_bits(c);
  }) GUARD_END
}
int tachyon_mi355x_msm_gpu_set_devices(int curve, void* ctx, const int* device_ids, size_t count) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  for (size_t i = 0; i < count; ++i)
    if (device_ids[i] < 0 || device_ids[i] >= n) return 0;  // refused, nothing changed
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    auto* m = static_cast<MsmCtx<C>*>(ctx);
    m->multi.reset();
    if (count > 1) {
      m->multi = std::make_unique<msm::MsmMultiDevice<C>>(std::vector<int>(device_ids, device_ids + count));
      m->multi->copy_settings(m->impl);  // window bits, variant and profiling forced before set_devices
    }
  }) GUARD_END
  return 1;
}
size_t tachyon_mi355x_msm_gpu_last_shards(int curve, const void* ctx, float* shard_ms, size_t* shard_points,
                                          int* shard_devices, size_t cap) {
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    auto* m = static_cast<const MsmCtx<C>*>(ctx);
    if (!m->multi) return 0;
    const auto& ms = m->multi->last_shard_ms();
    const auto& np = m->multi->last_shard_points();
    const auto ids = m->multi->device_ids();
    for (size_t i = 0; i < ids.size() && i < cap; ++i) {
      if (shard_ms) shard_ms[i] = i < ms.size() ? ms[i] : 0.f;
      if (shard_points) shard_points[i] = i < np.size() ? np[i] : 0;
      if (shard_devices) shard_devices[i] = ids[i];
    }
    return ids.size();
  }) GUARD_END
  return 0;
}
void tachyon_mi355x_msm_gpu_set_profile(int curve, void* ctx, int on) {
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    auto* m = static_cast<MsmCtx<C>*>(ctx);
    m->impl.set_profile(on != 0);
    if (m->multi) m->multi->set_profile(on != 0);
  }) GUARD_END
}
int tachyon_mi355x_msm_gpu_set_variant(int curve, void* ctx, int variant) {
  if (variant < 0 || (variant & ~msm::kMsmVariantMask)) return 0;  // unknown bits: refused, nothing changed
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    auto* m = static_cast<MsmCtx<C>*>(ctx);
    m->impl.set_variant(variant);
    if (m->multi) m->multi->set_variant(variant);
  }) GUARD_END
  return 1;
}
void tachyon_mi355x_msm_gpu_last_timings(int curve, const void* ctx, float* out8) {
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    // multi-device: the timings of the shard that ran the most points
    auto* m = static_cast<const MsmCtx<C>*>(ctx);
    const msm::MsmTimings& t = m->multi ? m->multi->lead().timings() : m->impl.timings();
    out8[0] = t.h2d; out8[1] = t.recode; out8[2] = t.sort; out8[3] = t.prep; out8[4] = t.acc; out8[5] = t.reduce;
    out8[6] = t.total; out8[7] = t.acc_launches;
  }) GUARD_END
}
unsigned tachyon_mi355x_msm_gpu_last_schedule(int curve, const void* ctx) {
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    auto* m = static_cast<const MsmCtx<C>*>(ctx);
    return m->multi ? m->multi->lead().last_schedule() : m->impl.last_schedule();
  }) GUARD_END
  return 0;
}
double tachyon_mi355x_msm_madd_ceiling(int curve, int field_bits) {
  GUARD_BEGIN CURVE_DISPATCH(curve, return msm::MsmGpu<C>::madd_ceiling(field_bits)) GUARD_END
  return 0.0;
}
size_t tachyon_mi355x_msm_gpu_last_divisions(int curve, const void* ctx) {
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    auto* m = static_cast<const MsmCtx<C>*>(ctx);
    return m->multi ? m->multi->last_divisions() : m->impl.last_divisions();
  }) GUARD_END
  return 0;
}
void tachyon_mi355x_msm_plan(int curve, size_t size, unsigned* c, unsigned* windows) {
  GUARD_BEGIN CURVE_DISPATCH(curve, {
    msm::MsmPlan p = msm::MsmPlan::make(size, C::Fr::Config::kModulusBits);
    *c = p.c;
    *windows = p.windows;
  }) GUARD_END
}
void tachyon_mi355x_affine_sum(int curve, const void* points, size_t count, void* out_affine) {
  GUARD_BEGIN CURVE_DISPATCH(curve, affine_sum<C>(points, count, out_affine)) GUARD_END
}
void tachyon_mi355x_jacobian_to_affine(int curve, const void* jacobian, void* out_affine) {
  GUARD_BEGIN CURVE_DISPATCH(curve, jac_to_affine<C>(jacobian, out_affine)) GUARD_END
}

void tachyon_mi355x_gen_scalars(int field, uint64_t seed, size_t start, size_t n, void* d_out, void* stream) {
  GUARD_BEGIN util::gen_scalars(field, seed, start, n, d_out, static_cast<hipStream_t>(stream)); GUARD_END
}
void tachyon_mi355x_gen_bases(int curve, uint64_t seed, size_t n, size_t chunk, void* d_out, void* stream) {
  GUARD_BEGIN util::gen_bases(curve, seed, 0, n, chunk, d_out, static_cast<hipStream_t>(stream)); GUARD_END
}
void tachyon_mi355x_gen_bases_at(int curve, uint64_t seed, size_t start, size_t n, size_t chunk, void* d_out,
                                 void* stream) {
  GUARD_BEGIN util::gen_bases(curve, seed, start, n, chunk, d_out, static_cast<hipStream_t>(stream)); GUARD_END
}
void tachyon_mi355x_field_op(int field, int op, const void* a, const void* b, void* out, size_t count) {
  GUARD_BEGIN util::field_op(field, op, a, b, out, count); GUARD_END
}
void tachyon_mi355x_ec_op(int curve, int op, const void* a, const void* b, void* out, size_t count) {
  GUARD_BEGIN util::ec_op(curve, op, a, b, out, count); GUARD_END
}

void tachyon_mi355x_jacobian_destroy(int curve, void* jac) {
  switch (curve) {
    case 0: delete static_cast<tachyon_bn254_g1_jacobian*>(jac); break;
    case 1: delete static_cast<tachyon_bn254_g2_jacobian*>(jac); break;
    case 2: delete static_cast<tachyon_bls12_381_g1_jacobian*>(jac); break;
    case 3: delete static_cast<tachyon_bls12_381_g2_jacobian*>(jac); break;
  }
}

const char* tachyon_mi355x_version(void) { return "tachyon_mi355x 0.1 (gfx950)"; }
int tachyon_mi355x_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ---- univariate evaluation domain over BN254 Fr ----
tachyon_bn254_univariate_evaluation_domain* tachyon_bn254_univariate_evaluation_domain_create(size_t num_coeffs) {
  GUARD_BEGIN
  auto* d = new tachyon_bn254_univariate_evaluation_domain();
  d->impl.reset(new ntt::NttDomain<Bn254Fr>(num_coeffs));
  TA_HIP(hipGetDevice(&d->device));
  return d;
  GUARD_END
}
void tachyon_bn254_univariate_evaluation_domain_destroy(tachyon_bn254_univariate_evaluation_domain* domain) {
  delete domain;
}
// Domain::Zero<Evals>() = size() zeros (univariate_evaluations.h:251-255)
tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluation_domain_empty_evals(
    const tachyon_bn254_univariate_evaluation_domain* domain) {
  GUARD_BEGIN
  auto* e = new tachyon_bn254_univariate_evaluations();
  e->v.assign(domain->impl->size(), FrC{});
  return e;
  GUARD_END
}
tachyon_bn254_univariate_rational_evaluations* tachyon_bn254_univariate_evaluation_domain_empty_rational_evals(
    const tachyon_bn254_univariate_evaluation_domain* domain) {
  GUARD_BEGIN
  auto* e = new tachyon_bn254_univariate_rational_evaluations();
  const Bn254Fr one = Bn254Fr::one();
  FrC one_c;
  memcpy(&one_c, &one, sizeof(one_c));
  e->num.assign(domain->impl->size(), FrC{});
  e->den.assign(domain->impl->size(), one_c);
  return e;
  GUARD_END
}

// ---- bn254_univariate_rational_evaluations.h (reference .cc:18-88) ----
tachyon_bn254_univariate_rational_evaluations* tachyon_bn254_univariate_rational_evaluations_create(void) {
  GUARD_BEGIN return new tachyon_bn254_univariate_rational_evaluations(); GUARD_END
}
tachyon_bn254_univariate_rational_evaluations* tachyon_bn254_univariate_rational_evaluations_clone(
    const tachyon_bn254_univariate_rational_evaluations* evals) {
  GUARD_BEGIN return new tachyon_bn254_univariate_rational_evaluations(*evals); GUARD_END
}
void tachyon_bn254_univariate_rational_evaluations_destroy(tachyon_bn254_univariate_rational_evaluations* evals) {
  delete evals;
}
size_t tachyon_bn254_univariate_rational_evaluations_len(const tachyon_bn254_univariate_rational_evaluations* evals) {
  return evals->num.size();
}
// boundary checks are the caller's, as in the reference (.cc:42)
void tachyon_bn254_univariate_rational_evaluations_set_zero(tachyon_bn254_univariate_rational_evaluations* evals,
                                                            size_t i) {
  const Bn254Fr one = Bn254Fr::one();
  evals->num[i] = FrC{};
  memcpy(&evals->den[i], &one, sizeof(FrC));
}
void tachyon_bn254_univariate_rational_evaluations_set_trivial(tachyon_bn254_univariate_rational_evaluations* evals,
                                                               size_t i, const tachyon_bn254_fr* numerator) {
  const Bn254Fr one = Bn254Fr::one();
  evals->num[i] = *numerator;
  memcpy(&evals->den[i], &one, sizeof(FrC));
}
void tachyon_bn254_univariate_rational_evaluations_set_rational(tachyon_bn254_univariate_rational_evaluations* evals,
                                                                size_t i, const tachyon_bn254_fr* numerator,
                                                                const tachyon_bn254_fr* denominator) {
  evals->num[i] = *numerator;
  evals->den[i] = *denominator;
}
// RationalField::Evaluate (rational_field.h:115): numerator / denominator;
// a zero denominator fails like the reference's unwrap (abort)
void tachyon_bn254_univariate_rational_evaluations_evaluate(
    const tachyon_bn254_univariate_rational_evaluations* evals, size_t i, tachyon_bn254_fr* value) {
  GUARD_BEGIN
  Bn254Fr d;
  memcpy(&d, &evals->den[i], sizeof(d));
  if (d.is_zero()) throw std::runtime_error("RationalField::Evaluate: zero denominator");
  util::batch_evaluate_bn254_fr(&evals->num[i], &evals->den[i], value, 1);
  GUARD_END
}
tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_rational_evaluations_batch_evaluate(
    const tachyon_bn254_univariate_rational_evaluations* evals) {
  GUARD_BEGIN
  auto* out = new tachyon_bn254_univariate_evaluations();
  out->v.resize(evals->num.size());
  util::batch_evaluate_bn254_fr(evals->num.data(), evals->den.data(), out->v.data(), out->v.size());
  return out;
  GUARD_END
}
void tachyon_mi355x_bn254_univariate_rational_evaluations_resize(tachyon_bn254_univariate_rational_evaluations* evals,
                                                                 size_t len) {
  GUARD_BEGIN
  const Bn254Fr one = Bn254Fr::one();
  FrC one_c;
  memcpy(&one_c, &one, sizeof(one_c));
  evals->num.resize(len, FrC{});
  evals->den.resize(len, one_c);
  GUARD_END
}
void tachyon_mi355x_bn254_univariate_rational_evaluations_get(
    const tachyon_bn254_univariate_rational_evaluations* evals, size_t i, tachyon_bn254_fr* numerator,
    tachyon_bn254_fr* denominator) {
  *numerator = evals->num[i];
  *denominator = evals->den[i];
}

tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_evaluation_domain_empty_poly(
    const tachyon_bn254_univariate_evaluation_domain* domain) {
  GUARD_BEGIN
  auto* p = new tachyon_bn254_univariate_dense_polynomial();
  p->v.assign(domain->impl->size(), FrC{});
  return p;
  GUARD_END
}

}  // extern "C"

namespace {
// UnivariateEvaluationDomain::FFT (univariate_evaluation_domain.h:141-182):
// empty poly -> empty evals; otherwise n evaluations.  The transform runs in
// place on the vector it returns: the in-place entry points hand over the
// caller's vector (no second host allocation -- first-touch page faults of a
// fresh 512 MiB vector cost more than the transform), the copying ones copy
// the input once.
std::vector<FrC> do_fft(const Domain* d, std::vector<FrC>&& v) {
  if (v.empty()) return std::move(v);
  const size_t len = v.size(), n = d->impl->size();
  if (len < n) v.resize(n);  // zero padding
  if (auto* m = d->multi_for_plain())
    m->forward_host(reinterpret_cast<const Bn254Fr*>(v.data()), len, reinterpret_cast<Bn254Fr*>(v.data()));
  else
    d->impl->forward_host(reinterpret_cast<const Bn254Fr*>(v.data()), len, reinterpret_cast<Bn254Fr*>(v.data()));
  return std::move(v);
}
// IFFT + RemoveHighDegreeZeros (radix2_evaluation_domain.h:218-223)
std::vector<FrC> do_ifft(const Domain* d, std::vector<FrC>&& v) {
  if (v.empty()) return std::move(v);
  const size_t len = v.size(), n = d->impl->size();
  if (len < n) v.resize(n);
  if (auto* m = d->multi_for_plain())
    m->inverse_host(reinterpret_cast<const Bn254Fr*>(v.data()), len, reinterpret_cast<Bn254Fr*>(v.data()));
  else
    d->impl->inverse_host(reinterpret_cast<const Bn254Fr*>(v.data()), len, reinterpret_cast<Bn254Fr*>(v.data()));
  size_t keep = v.size();
  while (keep > 0) {
    const FrC& x = v[keep - 1];
    if (x.limbs[0] | x.limbs[1] | x.limbs[2] | x.limbs[3]) break;
    --keep;
  }
  v.resize(keep);
  return std::move(v);
}
}  // namespace

extern "C" {

tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluation_domain_fft(
    const tachyon_bn254_univariate_evaluation_domain* domain, const tachyon_bn254_univariate_dense_polynomial* poly) {
  GUARD_BEGIN
  auto* e = new tachyon_bn254_univariate_evaluations();
  e->v = do_fft(domain, std::vector<FrC>(poly->v));
  return e;
  GUARD_END
}
tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluation_domain_fft_inplace(
    const tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_univariate_dense_polynomial* poly) {
  GUARD_BEGIN
  auto* e = new tachyon_bn254_univariate_evaluations();
  std::vector<FrC> in = std::move(poly->v);  // moved-from, as FFT(DensePoly&&)
  poly->v.clear();
  e->v = do_fft(domain, std::move(in));
  return e;
  GUARD_END
}
tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_evaluation_domain_ifft(
    const tachyon_bn254_univariate_evaluation_domain* domain, const tachyon_bn254_univariate_evaluations* evals) {
  GUARD_BEGIN
  auto* p = new tachyon_bn254_univariate_dense_polynomial();
  p->v = do_ifft(domain, std::vector<FrC>(evals->v));
  return p;
  GUARD_END
}
tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_evaluation_domain_ifft_inplace(
    const tachyon_bn254_univariate_evaluation_domain* domain, tachyon_bn254_univariate_evaluations* evals) {
  GUARD_BEGIN
  auto* p = new tachyon_bn254_univariate_dense_polynomial();
  std::vector<FrC> in = std::move(evals->v);
  evals->v.clear();
  p->v = do_ifft(domain, std::move(in));
  return p;
  GUARD_END
}

tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluations_create(void) {
  return new tachyon_bn254_univariate_evaluations();
}
tachyon_bn254_univariate_evaluations* tachyon_bn254_univariate_evaluations_clone(
    const tachyon_bn254_univariate_evaluations* evals) {
  auto* e = new tachyon_bn254_univariate_evaluations();
  e->v = evals->v;
  return e;
}
void tachyon_bn254_univariate_evaluations_destroy(tachyon_bn254_univariate_evaluations* evals) { delete evals; }
size_t tachyon_bn254_univariate_evaluations_len(const tachyon_bn254_univariate_evaluations* evals) {
  return evals->v.size();
}
void tachyon_bn254_univariate_evaluations_set_value(tachyon_bn254_univariate_evaluations* evals, size_t i,
                                                    const tachyon_bn254_fr* value) {
  GUARD_BEGIN evals->v.at(i) = *value; GUARD_END  // .at() as in the reference: OOB aborts
}
tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_dense_polynomial_create(void) {
  return new tachyon_bn254_univariate_dense_polynomial();
}
tachyon_bn254_univariate_dense_polynomial* tachyon_bn254_univariate_dense_polynomial_clone(
    const tachyon_bn254_univariate_dense_polynomial* poly) {
  auto* p = new tachyon_bn254_univariate_dense_polynomial();
  p->v = poly->v;
  return p;
}
void tachyon_bn254_univariate_dense_polynomial_destroy(tachyon_bn254_univariate_dense_polynomial* poly) {
  delete poly;
}

void tachyon_mi355x_bn254_univariate_evaluations_get_value(const tachyon_bn254_univariate_evaluations* evals,
                                                           size_t i, tachyon_bn254_fr* value) {
  GUARD_BEGIN *value = evals->v.at(i); GUARD_END
}
tachyon_bn254_fr* tachyon_mi355x_bn254_univariate_evaluations_data(tachyon_bn254_univariate_evaluations* evals) {
  return evals->v.data();
}
void tachyon_mi355x_bn254_univariate_evaluations_resize(tachyon_bn254_univariate_evaluations* evals, size_t len) {
  GUARD_BEGIN evals->v.resize(len, FrC{}); GUARD_END
}
size_t tachyon_mi355x_bn254_univariate_dense_polynomial_len(const tachyon_bn254_univariate_dense_polynomial* poly) {
  return poly->v.size();
}
void tachyon_mi355x_bn254_univariate_dense_polynomial_resize(tachyon_bn254_univariate_dense_polynomial* poly,
                                                             size_t len) {
  GUARD_BEGIN poly->v.resize(len, FrC{}); GUARD_END
}
void tachyon_mi355x_bn254_univariate_dense_polynomial_set_value(tachyon_bn254_univariate_dense_polynomial* poly,
                                                                size_t i, const tachyon_bn254_fr* value) {
  GUARD_BEGIN poly->v.at(i) = *value; GUARD_END
}
void tachyon_mi355x_bn254_univariate_dense_polynomial_get_value(
    const tachyon_bn254_univariate_dense_polynomial* poly, size_t i, tachyon_bn254_fr* value) {
  GUARD_BEGIN *value = poly->v.at(i); GUARD_END
}
tachyon_bn254_fr* tachyon_mi355x_bn254_univariate_dense_polynomial_data(tachyon_bn254_univariate_dense_polynomial* poly) {
  return poly->v.data();
}

void tachyon_mi355x_bn254_halo2_override_subgroup_generator(void) { ntt::set_bn254_fr_halo2_generator(true); }
void tachyon_mi355x_bn254_halo2_restore_subgroup_generator(void) { ntt::set_bn254_fr_halo2_generator(false); }
int tachyon_mi355x_bn254_halo2_subgroup_generator_active(void) { return ntt::bn254_fr_halo2_generator() ? 1 : 0; }

size_t tachyon_mi355x_bn254_univariate_evaluation_domain_size(const tachyon_bn254_univariate_evaluation_domain* d) {
  return d->impl->size();
}
void tachyon_mi355x_bn254_univariate_evaluation_domain_group_gen(const tachyon_bn254_univariate_evaluation_domain* d,
                                                                 tachyon_bn254_fr* out) {
  memcpy(out, &d->impl->group_gen(), sizeof(*out));
}
void tachyon_mi355x_bn254_univariate_evaluation_domain_set_offset(tachyon_bn254_univariate_evaluation_domain* d,
                                                                  const tachyon_bn254_fr* offset) {
  GUARD_BEGIN
  Bn254Fr h;
  memcpy(&h, offset, sizeof(h));
  d->impl->set_offset(h);
  GUARD_END
}
void tachyon_mi355x_bn254_univariate_evaluation_domain_transform_device(tachyon_bn254_univariate_evaluation_domain* d,
                                                                        tachyon_bn254_fr* d_data, int inverse) {
  GUARD_BEGIN
  auto* x = reinterpret_cast<Bn254Fr*>(d_data);
  if (auto* m = d->multi_for_plain()) {
    if (inverse) m->inverse_device(x, x);
    else m->forward_device(x, x);
  } else if (inverse) {
    d->impl->inverse_device(x);
  } else {
    d->impl->forward_device(x);
  }
  GUARD_END
}
void tachyon_mi355x_bn254_univariate_evaluation_domain_transform_host(tachyon_bn254_univariate_evaluation_domain* d,
                                                                      tachyon_bn254_fr* inout, size_t len,
                                                                      int inverse) {
  GUARD_BEGIN
  if (len != d->impl->size())
    throw std::runtime_error("transform_host: the vector must hold exactly size() elements (" + std::to_string(len) +
                             " != " + std::to_string(d->impl->size()) + ")");
  auto* v = reinterpret_cast<Bn254Fr*>(inout);
  if (auto* m = d->multi_for_plain()) {
    if (inverse) m->inverse_host(v, len, v);
    else m->forward_host(v, len, v);
  } else if (inverse) {
    d->impl->inverse_host(v, len, v);
  } else {
    d->impl->forward_host(v, len, v);
  }
  GUARD_END
}
void tachyon_mi355x_bn254_univariate_evaluation_domain_transform_batch_device(
    tachyon_bn254_univariate_evaluation_domain* d, tachyon_bn254_fr* d_data, size_t batch, int inverse) {
  GUARD_BEGIN
  if (inverse) d->impl->inverse_device(reinterpret_cast<Bn254Fr*>(d_data), batch);
  else d->impl->forward_device(reinterpret_cast<Bn254Fr*>(d_data), batch);
  GUARD_END
}
void* tachyon_mi355x_bn254_univariate_evaluation_domain_stream(tachyon_bn254_univariate_evaluation_domain* d) {
  return d->impl->stream();
}
void tachyon_mi355x_bn254_univariate_evaluation_domain_set_profile(tachyon_bn254_univariate_evaluation_domain* d,
                                                                   int on) {
  d->impl->set_profile(on != 0);
}
int tachyon_mi355x_bn254_univariate_evaluation_domain_set_variant(tachyon_bn254_univariate_evaluation_domain* d,
                                                                  int variant) {
  GUARD_BEGIN return d->impl->set_variant(variant) ? 1 : 0; GUARD_END
  return 0;
}
int tachyon_mi355x_bn254_univariate_evaluation_domain_set_devices(tachyon_bn254_univariate_evaluation_domain* d,
                                                                   const int* ids, size_t count) {
  GUARD_BEGIN
  if (count <= 1) {
    d->multi.reset();
    return 1;
  }
  const size_t n = d->impl->size();
  if (n < 4) return 0;
  int avail = 0;
  TA_HIP(hipGetDeviceCount(&avail));
  for (size_t i = 0; i < count; ++i)
    if (ids[i] < 0 || ids[i] >= avail) return 0;
  // the four-step splits R and C by a power of two: the first 2^k of the ids,
  // 2^k <= count and <= R = 2^floor(log n / 2) (devices() reports them)
  size_t use = 1;
  while (use * 2 <= count && use * 2 <= (size_t(1) << (d->impl->log_size() / 2))) use *= 2;
  if (use < 2) return 0;
  if (use == 2) {  // two parts: the one-link all-to-all costs more than the transform (see the header)
    d->multi.reset();
    return 1;
  }
  const std::vector<int> dev(ids, ids + use);
  std::unique_ptr<ntt::NttMultiDevice<Bn254Fr>> m;
  try {
    m = std::make_unique<ntt::NttMultiDevice<Bn254Fr>>(d->impl->log_size(), dev, d->device, d->impl->stream());
  } catch (const std::exception&) {  // not a power of two, too many for the size, or a bad id
    return 0;
  }
  if (!(m->root() == d->impl->group_gen())) return 0;  // another generator set was active at create
  d->multi = std::move(m);
  return 1;
  GUARD_END
  return 0;
}
size_t tachyon_mi355x_bn254_univariate_evaluation_domain_devices(const tachyon_bn254_univariate_evaluation_domain* d,
                                                                 int* ids, size_t cap) {
  if (!d->multi) return 0;
  const auto& v = d->multi->device_ids();
  for (size_t i = 0; i < v.size() && i < cap; ++i) ids[i] = v[i];
  return v.size();
}
int tachyon_mi355x_bn254_univariate_evaluation_domain_last_timings(const tachyon_bn254_univariate_evaluation_domain* d,
                                                                   float* total_ms, float* pass_ms, int max_passes) {
  const auto& t = d->impl->timings();
  if (total_ms) *total_ms = t.total;
  int np = (int)t.passes.size();
  for (int i = 0; i < np && i < max_passes; ++i) pass_ms[i] = t.passes[i];
  return np;
}

struct tachyon_mi355x_bn254_ntt4 {
  ntt::Ntt4Step<Bn254Fr>* impl;
  DeviceBuffer send, recv;  // tachyon_mi355x_bn254_ntt4_run's exchange buffers
};
tachyon_mi355x_bn254_ntt4* tachyon_mi355x_bn254_ntt4_create(uint32_t log_n, uint32_t log_world, uint32_t rank,
                                                           void* stream) {
  GUARD_BEGIN
  return new tachyon_mi355x_bn254_ntt4{
      new ntt::Ntt4Step<Bn254Fr>(log_n, log_world, rank, static_cast<hipStream_t>(stream))};
  GUARD_END
}
tachyon_mi355x_bn254_ntt4* tachyon_mi355x_bn254_ntt4_create_split(uint32_t log_n, uint32_t log_r, uint32_t log_world,
                                                                 uint32_t rank, void* stream) {
  GUARD_BEGIN
  if (log_r == 0 || log_r >= log_n) throw std::runtime_error("tachyon_mi355x: ntt4 split needs 1 <= log_r < log_n");
  return new tachyon_mi355x_bn254_ntt4{
      new ntt::Ntt4Step<Bn254Fr>(log_n, log_world, rank, static_cast<hipStream_t>(stream), log_r)};
  GUARD_END
}
uint32_t tachyon_mi355x_bn254_ntt4_log_rows(const tachyon_mi355x_bn254_ntt4* plan) { return plan->impl->log_rows(); }
uint32_t tachyon_mi355x_ntt4_split_log_r(uint32_t log_n, uint32_t log_world) {
  return ntt::ntt4_split_log_r(log_n, log_world);
}
void tachyon_mi355x_bn254_ntt4_destroy(tachyon_mi355x_bn254_ntt4* plan) {
  if (!plan) return;
  delete plan->impl;
  delete plan;
}
size_t tachyon_mi355x_bn254_ntt4_local_size(const tachyon_mi355x_bn254_ntt4* plan) { return plan->impl->local_size(); }
void tachyon_mi355x_bn254_ntt4_stage(tachyon_mi355x_bn254_ntt4* plan, int stage, int inverse,
                                     const tachyon_bn254_fr* d_in, tachyon_bn254_fr* d_out) {
  GUARD_BEGIN
  const Bn254Fr* in = reinterpret_cast<const Bn254Fr*>(d_in);
  Bn254Fr* out = reinterpret_cast<Bn254Fr*>(d_out);
  if (stage != 1 && stage != 2) throw std::runtime_error("tachyon_mi355x: ntt4 stage is 1 or 2");
  if (!inverse) (stage == 1) ? plan->impl->forward_stage1(in, out) : plan->impl->forward_stage2(in, out);
  else (stage == 1) ? plan->impl->inverse_stage1(in, out) : plan->impl->inverse_stage2(in, out);
  GUARD_END
}
// Both stages and the all-to-all between them, on the plan's stream (RCCL:
// no host synchronisation; the host-staged communicator synchronises it)
void tachyon_mi355x_bn254_ntt4_run(tachyon_mi355x_bn254_ntt4* plan, tachyon_mi355x_comm* comm, int inverse,
                                   const tachyon_bn254_fr* d_in, tachyon_bn254_fr* d_out) {
  GUARD_BEGIN
  if (!comm || !comm->impl) throw std::runtime_error("null communicator");
  auto& p = *plan->impl;
  if ((uint32_t)comm->impl->world() != p.world() || (uint32_t)comm->impl->rank() != p.rank())
    throw std::runtime_error("tachyon_mi355x: ntt4 plan world/rank differ from the communicator's");
  const size_t bytes = p.local_size() * sizeof(Bn254Fr);
  Bn254Fr* send = static_cast<Bn254Fr*>(plan->send.ensure(bytes));
  Bn254Fr* recv = static_cast<Bn254Fr*>(plan->recv.ensure(bytes));
  const Bn254Fr* in = reinterpret_cast<const Bn254Fr*>(d_in);
  Bn254Fr* out = reinterpret_cast<Bn254Fr*>(d_out);
  if (!inverse) p.forward_stage1(in, send);
  else p.inverse_stage1(in, send);
  comm->impl->all_to_all_device(send, recv, bytes / p.world(), p.stream());
  if (!inverse) p.forward_stage2(recv, out);
  else p.inverse_stage2(recv, out);
  GUARD_END
}

// ---- communicators (dist/comm.h) ----
int tachyon_mi355x_comm_unique_id(void* out, size_t cap) {
  if (cap < sizeof(ncclUniqueId)) return 0;
  GUARD_BEGIN
  const ncclUniqueId id = dist::rccl_unique_id();
  memcpy(out, &id, sizeof(id));
  return (int)sizeof(id);
  GUARD_END
  return 0;
}
tachyon_mi355x_comm* tachyon_mi355x_comm_init_rccl(const void* unique_id, int world, int rank) {
  GUARD_BEGIN
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  auto* c = new tachyon_mi355x_comm();
  c->impl = std::make_unique<dist::RcclComm>(id, world, rank);
  return c;
  GUARD_END
  return nullptr;
}
tachyon_mi355x_comm* tachyon_mi355x_comm_from_rccl(void* nccl_comm) {
  GUARD_BEGIN
  auto* c = new tachyon_mi355x_comm();
  c->impl = std::make_unique<dist::RcclComm>(static_cast<ncclComm_t>(nccl_comm));
  return c;
  GUARD_END
  return nullptr;
}
tachyon_mi355x_comm* tachyon_mi355x_comm_create_host(int world, int rank, tachyon_mi355x_all_gather_fn all_gather,
                                                     tachyon_mi355x_all_to_all_fn all_to_all, void* user) {
  GUARD_BEGIN
  auto* c = new tachyon_mi355x_comm();
  c->impl = std::make_unique<dist::HostComm>(world, rank, all_gather, all_to_all, user);
  return c;
  GUARD_END
  return nullptr;
}
void tachyon_mi355x_comm_destroy(tachyon_mi355x_comm* comm) { delete comm; }
void tachyon_mi355x_comm_all_gather(tachyon_mi355x_comm* comm, const void* send, void* recv, size_t bytes) {
  GUARD_BEGIN comm->impl->all_gather_host(send, recv, bytes); GUARD_END
}
int tachyon_mi355x_comm_world(const tachyon_mi355x_comm* comm) { return comm->impl->world(); }
int tachyon_mi355x_comm_rank(const tachyon_mi355x_comm* comm) { return comm->impl->rank(); }
const char* tachyon_mi355x_comm_backend(const tachyon_mi355x_comm* comm) { return comm->impl->backend(); }

int tachyon_mi355x_bn254_ntt4_set_variant(tachyon_mi355x_bn254_ntt4* plan, int variant) {
  if (variant < 0 || variant > 15) return 0;
  GUARD_BEGIN plan->impl->set_variant(variant); GUARD_END
  return 1;
}
void* tachyon_mi355x_bn254_ntt4_stream(const tachyon_mi355x_bn254_ntt4* plan) {
  return static_cast<void*>(plan->impl->stream());
}
void tachyon_mi355x_bn254_ntt4_synchronize(tachyon_mi355x_bn254_ntt4* plan) {
  GUARD_BEGIN
  TA_HIP(hipStreamSynchronize(plan->impl->stream()));
  GUARD_END
}

}  // extern "C"

// ---- field-generic NTT domains (include/tachyon_mi355x.h) ----
// Radix2EvaluationDomain<F> on the GPU for bn254 Fr (field 1) and bls12_381
// Fr (field 3): the engine of the IcicleNTT<F> holder
// (icicle_ntt_bls12_381.cc:31-115 for BLS12-381).
struct tachyon_mi355x_ntt_domain {
  int field = 0;
  std::unique_ptr<ntt::NttDomain<Bn254Fr>> bn;
  std::unique_ptr<ntt::NttDomain<Bls381Fr>> bls;
};

namespace {
template <class Fn>
void ntt_dispatch(const tachyon_mi355x_ntt_domain* d, Fn&& fn) {
  if (d->bn) fn(*d->bn);
  else fn(*d->bls);
}
}  // namespace

extern "C" {

tachyon_mi355x_ntt_domain* tachyon_mi355x_ntt_domain_create(int field, size_t num_coeffs) {
  if (field != 1 && field != 3) return nullptr;
  GUARD_BEGIN
  auto d = std::make_unique<tachyon_mi355x_ntt_domain>();
  d->field = field;
  if (field == 1) d->bn = std::make_unique<ntt::NttDomain<Bn254Fr>>(num_coeffs);
  else d->bls = std::make_unique<ntt::NttDomain<Bls381Fr>>(num_coeffs);
  return d.release();
  GUARD_END
  return nullptr;
}
void tachyon_mi355x_ntt_domain_destroy(tachyon_mi355x_ntt_domain* d) { delete d; }
size_t tachyon_mi355x_ntt_domain_size(const tachyon_mi355x_ntt_domain* d) {
  size_t n = 0;
  ntt_dispatch(d, [&](auto& dom) { n = dom.size(); });
  return n;
}
int tachyon_mi355x_ntt_domain_field(const tachyon_mi355x_ntt_domain* d) { return d->field; }
void tachyon_mi355x_ntt_domain_group_gen(const tachyon_mi355x_ntt_domain* d, void* out) {
  ntt_dispatch(d, [&](auto& dom) { memcpy(out, &dom.group_gen(), sizeof(dom.group_gen())); });
}
void tachyon_mi355x_ntt_domain_set_offset(tachyon_mi355x_ntt_domain* d, const void* offset) {
  GUARD_BEGIN
  ntt_dispatch(d, [&](auto& dom) {
    using Fr = std::decay_t<decltype(dom.group_gen())>;
    Fr h = Fr::one();
    if (offset) memcpy(&h, offset, sizeof(h));
    dom.set_offset(h);
  });
  GUARD_END
}
void tachyon_mi355x_ntt_domain_transform_host(tachyon_mi355x_ntt_domain* d, void* inout, size_t len, int inverse) {
  GUARD_BEGIN
  ntt_dispatch(d, [&](auto& dom) {
    using Fr = std::decay_t<decltype(dom.group_gen())>;
    if (len != dom.size())
      throw std::runtime_error("transform_host: the vector must hold exactly size() elements (" +
                               std::to_string(len) + " != " + std::to_string(dom.size()) + ")");
    auto* v = static_cast<Fr*>(inout);
    if (inverse) dom.inverse_host(v, len, v);
    else dom.forward_host(v, len, v);
  });
  GUARD_END
}
void tachyon_mi355x_ntt_domain_transform_device(tachyon_mi355x_ntt_domain* d, void* d_data, size_t batch,
                                                int inverse) {
  GUARD_BEGIN
  ntt_dispatch(d, [&](auto& dom) {
    using Fr = std::decay_t<decltype(dom.group_gen())>;
    auto* x = static_cast<Fr*>(d_data);
    if (inverse) dom.inverse_device(x, batch);
    else dom.forward_device(x, batch);
  });
  GUARD_END
}
void* tachyon_mi355x_ntt_domain_stream(tachyon_mi355x_ntt_domain* d) {
  void* s = nullptr;
  ntt_dispatch(d, [&](auto& dom) { s = static_cast<void*>(dom.stream()); });
  return s;
}

}  // extern "C"
