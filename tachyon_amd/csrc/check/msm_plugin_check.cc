// Exercise include/tachyon_mi355x_msm.h the way Tachyon's callers use
// VariableBaseMSMGpu<Point> (prove.h:64-147: host std::vector inputs, a
// ProjectivePoint result; kzg.h:90-114: device-resident bases) and
// VariableBaseMSM<Point> (containers and iterators, PointXYZZ bucket), for the
// four groups the reference instantiates (icicle_msm.h:78-100).
//
//   msm_plugin_check <log_n> <seed>
//
// Inputs are the seeded synthetic bases / scalars of tachyon_mi355x_gen_*
// (the oracle's gen_bases / gen_scalars produce the same values), so the test
// (tests/test_gpu_harness.py) recomputes the expected point with the CPU
// oracle.  Prints one JSON line: per group the projective and XYZZ results
// (hex of the Montgomery bytes) and the self-checks below; exit 0 = ok.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <string>
#include <type_traits>
#include <vector>

#include "../../../include/tachyon_mi355x_msm.h"

namespace {

constexpr size_t kChunk = 16;  // base-chain length of the synthetic generator

template <typename T>
std::string hex(const T& v) {
  static const char* d = "0123456789abcdef";
  const unsigned char* p = reinterpret_cast<const unsigned char*>(&v);
  std::string s;
  for (size_t i = 0; i < sizeof(T); ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

template <typename T>
struct DeviceSpan {  // absl::Span-like view of device memory
  const T* ptr;
  size_t len;
  const T* data() const { return ptr; }
  size_t size() const { return len; }
};

// Base-field products on the device (tachyon_mi355x_field_op op 2) of
// `count` elements of `fq` bytes each; field 0 = BN254 Fq, 2 = BLS12-381 Fq.
std::vector<unsigned char> fq_mul(int field, size_t fq, const std::vector<unsigned char>& a,
                                  const std::vector<unsigned char>& b) {
  std::vector<unsigned char> out(a.size());
  tachyon_mi355x_field_op(field, 2, a.data(), b.data(), out.data(), a.size() / fq);
  return out;
}

// VariableBaseMSM<Point> over projective, Jacobian and XYZZ bases
// (variable_base_msm_unittest.cc:30-33): the affine bases re-expressed with a
// per-point z in Fq (Fq2 groups: z = (z, 0), so coordinates scale componentwise)
// taken from the scalar bytes, and every 37th point (i % 37 == 3) the identity
// (z = 0).  Bucket = the base's own form.  All three results must equal the
// affine-input MSM over the same bases with those points zeroed; that bucket's
// bytes are printed for the oracle check.
template <typename Point, typename Scalar, int kGroup>
bool check_non_affine(const std::vector<Point>& bases, const std::vector<Scalar>& scalars, std::string* json) {
  constexpr size_t kC = tachyon_mi355x::kCoordBytes[kGroup];
  constexpr bool kG2 = kGroup == tachyon_mi355x::kBn254G2 || kGroup == tachyon_mi355x::kBls12_381G2;
  constexpr size_t kFq = kG2 ? kC / 2 : kC;
  constexpr int kFqField = (kGroup == tachyon_mi355x::kBn254G1 || kGroup == tachyon_mi355x::kBn254G2) ? 0 : 2;
  const size_t n = bases.size();
  const size_t comps = kG2 ? 2 : 1;
  // z per point (one Fq), and its square and cube
  std::vector<unsigned char> z(n * kFq, 0);
  for (size_t i = 0; i < n; ++i)
    if (i % 37 != 3) std::memcpy(&z[i * kFq], &scalars[i], 32);  // < r < q: a valid Montgomery Fq
  const std::vector<unsigned char> z2 = fq_mul(kFqField, kFq, z, z), z3 = fq_mul(kFqField, kFq, z2, z);
  // coordinate c (0 = x, 1 = y) of every base as n x comps Fq elements, times a per-point factor
  auto scaled = [&](int c, const std::vector<unsigned char>& f) {
    std::vector<unsigned char> a(n * comps * kFq), b(n * comps * kFq);
    for (size_t i = 0; i < n; ++i)
      for (size_t k = 0; k < comps; ++k) {
        std::memcpy(&a[(i * comps + k) * kFq], reinterpret_cast<const unsigned char*>(&bases[i]) + c * kC + k * kFq, kFq);
        std::memcpy(&b[(i * comps + k) * kFq], &f[i * kFq], kFq);
      }
    return fq_mul(kFqField, kFq, a, b);
  };
  // a coordinate equal to z^e in Fq, embedded as (z^e, 0) for Fq2
  auto embed = [&](const std::vector<unsigned char>& f) {
    std::vector<unsigned char> v(n * kC, 0);
    for (size_t i = 0; i < n; ++i) std::memcpy(&v[i * kC], &f[i * kFq], kFq);
    return v;
  };
  auto pack = [&](std::initializer_list<const std::vector<unsigned char>*> coords) {
    std::vector<unsigned char> v(n * coords.size() * kC);
    for (size_t i = 0; i < n; ++i) {
      size_t j = 0;
      for (const auto* c : coords) std::memcpy(&v[(i * coords.size() + j++) * kC], &(*c)[i * kC], kC);
    }
    return v;
  };
  const auto xz = scaled(0, z), yz = scaled(1, z), xz2 = scaled(0, z2), yz3 = scaled(1, z3);
  const auto ez = embed(z), ez2 = embed(z2), ez3 = embed(z3);
  struct P3 { unsigned char b[3 * kC]; };
  struct P4 { unsigned char b[4 * kC]; };
  using CProj = std::conditional_t<kGroup == tachyon_mi355x::kBn254G1, tachyon_bn254_g1_projective,
                std::conditional_t<kGroup == tachyon_mi355x::kBn254G2, tachyon_bn254_g2_projective,
                std::conditional_t<kGroup == tachyon_mi355x::kBls12_381G1, tachyon_bls12_381_g1_projective,
                                   tachyon_bls12_381_g2_projective>>>;
  using CJac = std::conditional_t<kGroup == tachyon_mi355x::kBn254G1, tachyon_bn254_g1_jacobian,
               std::conditional_t<kGroup == tachyon_mi355x::kBn254G2, tachyon_bn254_g2_jacobian,
               std::conditional_t<kGroup == tachyon_mi355x::kBls12_381G1, tachyon_bls12_381_g1_jacobian,
                                  tachyon_bls12_381_g2_jacobian>>>;
  using CXyzz = std::conditional_t<kGroup == tachyon_mi355x::kBn254G1, tachyon_bn254_g1_xyzz,
                std::conditional_t<kGroup == tachyon_mi355x::kBn254G2, tachyon_bn254_g2_xyzz,
                std::conditional_t<kGroup == tachyon_mi355x::kBls12_381G1, tachyon_bls12_381_g1_xyzz,
                                   tachyon_bls12_381_g2_xyzz>>>;
  auto as_points = [&](const std::vector<unsigned char>& raw, auto tag) {
    using T = decltype(tag);
    std::vector<T> v(n);
    std::memcpy(v.data(), raw.data(), raw.size());
    return v;
  };
  const auto proj = as_points(pack({&xz, &yz, &ez}), CProj{});
  const auto jac = as_points(pack({&xz2, &yz3, &ez}), CJac{});
  const auto xyzz = as_points(pack({&xz2, &yz3, &ez2, &ez3}), CXyzz{});
  std::vector<Point> zeroed = bases;
  for (size_t i = 3; i < n; i += 37) std::memset(&zeroed[i], 0, sizeof(Point));

  tachyon_mi355x::VariableBaseMSM<Point> m_aff;
  tachyon_mi355x::VariableBaseMSM<CProj> m_proj;
  tachyon_mi355x::VariableBaseMSM<CJac> m_jac;
  tachyon_mi355x::VariableBaseMSM<CXyzz> m_xyzz;
  P4 want{}, got_x{};
  P3 got_p{}, got_j{};
  bool ok = m_aff.Run(zeroed, scalars, &want) && m_proj.Run(proj, scalars, &got_p) && m_jac.Run(jac, scalars, &got_j) &&
            m_xyzz.Run(xyzz.begin(), xyzz.end(), scalars.begin(), scalars.end(), &got_x);
  // normalised results: x, y equal across forms; z = zz = zzz = the affine bucket's zz
  ok = ok && std::memcmp(&got_x, &want, sizeof(want)) == 0 && std::memcmp(&got_p, &want, 3 * kC) == 0 &&
       std::memcmp(&got_j, &want, 3 * kC) == 0;
  // a size mismatch stays false for the non-affine path too
  P3 untouched{};
  std::vector<CProj> shorter(proj.begin(), proj.end() - 1);
  ok = ok && !m_proj.Run(shorter, scalars, &untouched);
  *json += ", \"non_affine_ok\": " + std::string(ok ? "true" : "false") + ", \"zeroed_xyzz\": \"" + hex(want) + "\"";
  return ok;
}

template <typename Point, typename Scalar, int kField, int kGroup>
bool check_group(size_t n, uint64_t seed, hipStream_t stream, std::string* json) {
  constexpr size_t kC = tachyon_mi355x::kCoordBytes[kGroup];
  struct Proj { unsigned char b[3 * kC]; };
  struct Xyzz { unsigned char b[4 * kC]; };

  Point* d_bases = nullptr;
  Scalar* d_scalars = nullptr;
  if (hipMalloc(&d_bases, n * sizeof(Point)) != hipSuccess) return false;
  if (hipMalloc(&d_scalars, n * sizeof(Scalar)) != hipSuccess) return false;
  tachyon_mi355x_gen_bases(kGroup, seed, n, kChunk, d_bases, stream);
  tachyon_mi355x_gen_scalars(kField, seed, 0, n, d_scalars, stream);
  if (hipStreamSynchronize(stream) != hipSuccess) return false;
  std::vector<Point> bases(n);
  std::vector<Scalar> scalars(n);
  if (hipMemcpy(bases.data(), d_bases, n * sizeof(Point), hipMemcpyDeviceToHost) != hipSuccess) return false;
  if (hipMemcpy(scalars.data(), d_scalars, n * sizeof(Scalar), hipMemcpyDeviceToHost) != hipSuccess) return false;

  // VariableBaseMSMGpu: host vectors, then device-resident bases (KZG's SRS)
  tachyon_mi355x::VariableBaseMSMGpu<Point> gpu(nullptr, stream);
  Proj proj{}, proj_dev{};
  const bool ok_host = gpu.Run(bases, scalars, &proj);
  const bool ok_dev = gpu.Run(DeviceSpan<Point>{d_bases, n}, scalars, &proj_dev);
  // |bases| != |scalars|: false, result untouched (icicle_msm_bn254_g1.cc:30-33)
  Proj untouched{};
  std::memset(&untouched, 0x5a, sizeof(untouched));
  Proj before = untouched;
  std::vector<Point> shorter(bases.begin(), bases.end() - 1);
  const bool mismatch_false = !gpu.Run(shorter, scalars, &untouched) &&
                              std::memcmp(&before, &untouched, sizeof(before)) == 0;

  // VariableBaseMSM: containers and contiguous iterators, XYZZ bucket
  tachyon_mi355x::VariableBaseMSM<Point> cpu_api;
  Xyzz bucket{}, bucket_it{};
  const bool ok_c = cpu_api.Run(bases, scalars, &bucket);
  const bool ok_i = cpu_api.Run(bases.begin(), bases.end(), scalars.begin(), scalars.end(), &bucket_it);
  Xyzz empty{};
  const bool ok_e = cpu_api.Run(std::vector<Point>{}, std::vector<Scalar>{}, &empty);

  (void)hipFree(d_bases);
  (void)hipFree(d_scalars);
  const bool ok = ok_host && ok_dev && ok_c && ok_i && ok_e && mismatch_false &&
                  std::memcmp(&proj, &proj_dev, sizeof(proj)) == 0 &&
                  std::memcmp(&bucket, &bucket_it, sizeof(bucket)) == 0;
  char head[128];
  snprintf(head, sizeof(head), "\"%d\": {\"ok\": %s, \"mismatch_false\": %s, ", kGroup, ok ? "true" : "false",
           mismatch_false ? "true" : "false");
  *json += head;
  *json += "\"projective\": \"" + hex(proj) + "\", \"xyzz\": \"" + hex(bucket) + "\", \"empty_xyzz\": \"" +
           hex(empty) + "\"";
  const bool ok_na = check_non_affine<Point, Scalar, kGroup>(bases, scalars, json);
  *json += "}";
  return ok && ok_na;
}

}  // namespace

int main(int argc, char** argv) {
  const unsigned log_n = argc > 1 ? (unsigned)atoi(argv[1]) : 10;
  const uint64_t seed = argc > 2 ? strtoull(argv[2], nullptr, 0) : 0x7AC40001ULL;
  const size_t n = size_t(1) << log_n;
  hipStream_t stream = nullptr;
  if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return 2;
  tachyon_bn254_g1_init();
  tachyon_bls12_381_g1_init();
  std::string json = "{\"n\": " + std::to_string(n) + ", \"seed\": " + std::to_string(seed) + ", \"groups\": {";
  bool ok = check_group<tachyon_bn254_g1_affine, tachyon_bn254_fr, 1, tachyon_mi355x::kBn254G1>(n, seed, stream, &json);
  json += ", ";
  ok &= check_group<tachyon_bn254_g2_affine, tachyon_bn254_fr, 1, tachyon_mi355x::kBn254G2>(n, seed, stream, &json);
  json += ", ";
  ok &= check_group<tachyon_bls12_381_g1_affine, tachyon_bls12_381_fr, 3, tachyon_mi355x::kBls12_381G1>(n, seed, stream,
                                                                                                      &json);
  json += ", ";
  ok &= check_group<tachyon_bls12_381_g2_affine, tachyon_bls12_381_fr, 3, tachyon_mi355x::kBls12_381G2>(n, seed, stream,
                                                                                                      &json);
  json += "}}";
  printf("%s\n", json.c_str());
  (void)hipStreamDestroy(stream);
  return ok ? 0 : 1;
}
