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
#include <string>
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
           hex(empty) + "\"}";
  return ok;
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
