// C-ABI of the KZG commitment scheme (include/tachyon_mi355x.h, "KZG").
// Reference: tachyon/crypto/commitments/kzg/kzg.h (UnsafeSetup :173-207,
// Downsize :210-215, Commit/CommitLagrange :217-258, device SRS :90-114);
// errors abort like the reference's CHECKs.
#include "../../../include/tachyon_mi355x.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>

#include "../kzg/kzg.h"

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

}  // namespace

struct tachyon_mi355x_kzg {
  int curve;  // 0 bn254_g1, 2 bls12_381_g1
  std::unique_ptr<kzg::Kzg<Bn254G1>> bn;
  std::unique_ptr<kzg::Kzg<Bls381G1>> bls;
};

#define KZG_DISPATCH(p, ...)          \
  do {                                \
    if ((p)->curve == 0) {            \
      auto* impl = (p)->bn.get();     \
      __VA_ARGS__;                    \
    } else {                          \
      auto* impl = (p)->bls.get();    \
      __VA_ARGS__;                    \
    }                                 \
  } while (0)

extern "C" {

tachyon_mi355x_kzg* tachyon_mi355x_kzg_create(int curve) {
  GUARD_BEGIN
  if (curve != 0 && curve != 2) throw std::runtime_error("KZG curve must be 0 (bn254_g1) or 2 (bls12_381_g1)");
  auto* p = new tachyon_mi355x_kzg();
  p->curve = curve;
  if (curve == 0) p->bn = std::make_unique<kzg::Kzg<Bn254G1>>();
  else p->bls = std::make_unique<kzg::Kzg<Bls381G1>>();
  return p;
  GUARD_END
}

void tachyon_mi355x_kzg_destroy(tachyon_mi355x_kzg* p) { delete p; }

void tachyon_mi355x_kzg_unsafe_setup(tachyon_mi355x_kzg* p, size_t size, const void* tau) {
  GUARD_BEGIN
  KZG_DISPATCH(p, impl->unsafe_setup(size, *static_cast<const typename std::remove_pointer_t<decltype(impl)>::Fr*>(tau)));
  GUARD_END
}

size_t tachyon_mi355x_kzg_n(const tachyon_mi355x_kzg* p) {
  GUARD_BEGIN KZG_DISPATCH(p, return impl->n()); GUARD_END
}

int tachyon_mi355x_kzg_downsize(tachyon_mi355x_kzg* p, size_t n) {
  GUARD_BEGIN KZG_DISPATCH(p, return impl->downsize(n) ? 1 : 0); GUARD_END
}

void tachyon_mi355x_kzg_get_srs(const tachyon_mi355x_kzg* p, int lagrange, void* out) {
  GUARD_BEGIN
  KZG_DISPATCH(p, impl->copy_srs(lagrange != 0, static_cast<typename std::remove_pointer_t<decltype(impl)>::Aff*>(out)));
  GUARD_END
}

int tachyon_mi355x_kzg_commit(tachyon_mi355x_kzg* p, int lagrange, const void* scalars, size_t len,
                              void* out_affine) {
  GUARD_BEGIN
  KZG_DISPATCH(p, {
    using K = std::remove_pointer_t<decltype(impl)>;
    typename K::Aff a;
    if (!impl->commit(static_cast<const typename K::Fr*>(scalars), len, lagrange != 0, &a)) return 0;
    memcpy(out_affine, &a, sizeof(a));
    return 1;
  });
  GUARD_END
}

int tachyon_mi355x_kzg_commit_batch(tachyon_mi355x_kzg* p, int lagrange, const void* const* scalars,
                                    const size_t* lens, size_t count, void* out_affine) {
  GUARD_BEGIN
  KZG_DISPATCH(p, {
    using K = std::remove_pointer_t<decltype(impl)>;
    return impl->commit_batch(reinterpret_cast<const typename K::Fr* const*>(scalars), lens, count, lagrange != 0,
                              static_cast<typename K::Aff*>(out_affine))
               ? 1
               : 0;
  });
  GUARD_END
}

}  // extern "C"
