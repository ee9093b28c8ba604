// msm_benchmark_gpu: the reference's benchmark/msm/msm_benchmark_gpu.cc harness
// on the MI355X backend, written against the public C-ABI only.
//
//   msm_benchmark_gpu -k 16 -k 20 ... [--test_set random|non_uniform]
//                     [--check_results] [--device_resident] [--curve bn254|bls12_381]
//                     [--expect FILE]
//
// Kept from the reference (msm_benchmark_gpu.cc:20-75, msm_config.cc:39-82,
// msm_runner.h:45-61): sizes 2^k sorted ascending, one timed call per size
// through tachyon_<curve>_g1_affine_msm_gpu on host-resident bases/scalars
// (the wall clock includes the host-to-device copies), a table of seconds per
// size; "non_uniform" = NonUniform(n, 1), every scalar identical
// (variable_base_msm_test_set.h:43-53).  Inputs are seeded doubling-chain
// bases and random scalars generated on the device (tachyon_mi355x_gen_*) and
// copied to pageable host vectors, like the reference's std::vector test set.
//
// Stated differences: one untimed warm-up call at the largest size precedes
// the sweep (module load, buffer growth); --device_resident times the same
// entry point on HBM inputs (the reference's device-pointer path,
// icicle_msm_bn254_g1.cc:37-45).  --check_results: the reference compares the
// GPU point with its CPU MSM of the same inputs (msm_benchmark_gpu.cc:57-70).
// The product links no CPU MSM, so the CPU results come in through --expect
// FILE: per size (ascending) the affine CPU result of the first 2^k inputs
// (tests/test_gpu_harness.py writes it with the CPU oracle, which it also
// times).  Without --expect, --check_results checks the chunk-sum invariance
// of pippenger_adapter_unittest.cc: MSM(first half) + MSM(second half) ==
// MSM(all).  Inputs: seed 0x7AC40001, base chains of 2^10 (gen_bases).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/tachyon_mi355x.h"

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    exit(1);
  }
}

int usage() {
  std::cerr << "usage: msm_benchmark_gpu -k K [-k K ...] [--test_set random|non_uniform] [--check_results]\n"
               "                         [--device_resident] [--curve bn254|bls12_381] [--expect FILE]\n";
  return 1;
}

// the reference entry point: a new-allocated Jacobian, freed by the caller
void* reference_msm(bool bls, void* msm, const void* bases, const void* scalars, size_t n) {
  if (bls)
    return tachyon_bls12_381_g1_affine_msm_gpu(static_cast<tachyon_bls12_381_g1_msm_gpu_ptr>(msm),
                                               static_cast<const tachyon_bls12_381_g1_affine*>(bases),
                                               static_cast<const tachyon_bls12_381_fr*>(scalars), n);
  return tachyon_bn254_g1_affine_msm_gpu(static_cast<tachyon_bn254_g1_msm_gpu_ptr>(msm),
                                         static_cast<const tachyon_bn254_g1_affine*>(bases),
                                         static_cast<const tachyon_bn254_fr*>(scalars), n);
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<unsigned> ks;
  bool non_uniform = false, check = false, device_resident = false;
  std::string curve = "bn254", expect_path;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "-k" && i + 1 < argc) ks.push_back((unsigned)std::stoul(argv[++i]));
    else if (a == "--test_set" && i + 1 < argc) {
      std::string t = argv[++i];
      if (t == "non_uniform") non_uniform = true;
      else if (t != "random") return usage();
    } else if (a == "--check_results") check = true;
    else if (a == "--device_resident") device_resident = true;
    else if (a == "--curve" && i + 1 < argc) curve = argv[++i];
    else if (a == "--expect" && i + 1 < argc) expect_path = argv[++i];
    else return usage();
  }
  if (ks.empty() || (curve != "bn254" && curve != "bls12_381")) return usage();
  std::sort(ks.begin(), ks.end());
  const bool bls = curve == "bls12_381";
  const int curve_id = bls ? 2 : 0, field_id = bls ? 3 : 1;
  const size_t pb = bls ? 96 : 64, sb = 32;
  const size_t n_max = size_t(1) << ks.back();
  std::vector<uint8_t> expect;
  if (!expect_path.empty()) {
    FILE* f = fopen(expect_path.c_str(), "rb");
    if (!f) return usage();
    expect.resize(ks.size() * pb);
    const size_t got = fread(expect.data(), 1, expect.size(), f);
    fclose(f);
    if (got != expect.size()) {
      std::cerr << "--expect file must hold " << ks.size() << " affine points" << std::endl;
      return 1;
    }
  }

  std::cout << "Generating random points..." << std::endl;
  void *d_bases = nullptr, *d_scalars = nullptr;
  hip_check(hipMalloc(&d_bases, n_max * pb), "hipMalloc");
  hip_check(hipMalloc(&d_scalars, n_max * sb), "hipMalloc");
  tachyon_mi355x_gen_bases(curve_id, 0x7AC40001ULL, n_max, 1 << 10, d_bases, nullptr);
  tachyon_mi355x_gen_scalars(field_id, 0x7AC40001ULL, 0, non_uniform ? 1 : n_max, d_scalars, nullptr);
  hip_check(hipDeviceSynchronize(), "sync");
  if (non_uniform) {  // NonUniform(n, 1): replicate the one scalar
    std::vector<uint8_t> all(n_max * sb);
    hip_check(hipMemcpy(all.data(), d_scalars, sb, hipMemcpyDeviceToHost), "copy");
    for (size_t i = 1; i < n_max; ++i) memcpy(all.data() + i * sb, all.data(), sb);
    hip_check(hipMemcpy(d_scalars, all.data(), all.size(), hipMemcpyHostToDevice), "copy");
  }
  std::vector<uint8_t> h_bases, h_scalars;
  if (!device_resident) {
    h_bases.resize(n_max * pb);
    h_scalars.resize(n_max * sb);
    hip_check(hipMemcpy(h_bases.data(), d_bases, h_bases.size(), hipMemcpyDeviceToHost), "copy");
    hip_check(hipMemcpy(h_scalars.data(), d_scalars, h_scalars.size(), hipMemcpyDeviceToHost), "copy");
  }
  std::cout << "Generation completed" << std::endl;
  const uint8_t* bases = static_cast<const uint8_t*>(device_resident ? d_bases : (void*)h_bases.data());
  const uint8_t* scalars = static_cast<const uint8_t*>(device_resident ? d_scalars : (void*)h_scalars.data());

  void* msm = bls ? (void*)tachyon_bls12_381_g1_create_msm_gpu((uint8_t)ks.back())
                  : (void*)tachyon_bn254_g1_create_msm_gpu((uint8_t)ks.back());
  std::vector<uint8_t> res(pb), half(2 * pb), sum(pb);
  tachyon_mi355x_msm_gpu_affine(curve_id, msm, bases, scalars, n_max, res.data());  // warm-up

  std::vector<double> secs;
  bool ok = true;
  for (size_t ki = 0; ki < ks.size(); ++ki) {
    const unsigned k = ks[ki];
    const size_t n = size_t(1) << k;
    auto t0 = std::chrono::steady_clock::now();
    void* r = reference_msm(bls, msm, bases, scalars, n);
    secs.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    tachyon_mi355x_jacobian_to_affine(curve_id, r, res.data());
    tachyon_mi355x_jacobian_destroy(curve_id, r);
    if (check && !expect.empty()) {  // CHECK_EQ(cpu result, gpu result)
      if (memcmp(res.data(), expect.data() + ki * pb, pb) != 0) {
        std::cerr << "Results not matched at 2^" << k << std::endl;
        ok = false;
      }
    } else if (check) {
      const size_t h = n / 2;
      tachyon_mi355x_msm_gpu_affine(curve_id, msm, bases, scalars, h, half.data());
      tachyon_mi355x_msm_gpu_affine(curve_id, msm, bases + h * pb, scalars + h * sb, n - h, half.data() + pb);
      tachyon_mi355x_affine_sum(curve_id, half.data(), 2, sum.data());
      if (sum != res) {
        std::cerr << "Result not matched at 2^" << k << std::endl;
        ok = false;
      }
    }
  }

  printf("MSM Benchmark (%s G1, %s, %s)\n", curve.c_str(), non_uniform ? "non_uniform" : "random",
         device_resident ? "device-resident inputs" : "host-resident inputs, H2D included");
  printf("%-22s", "Degree (2^x)");
  for (unsigned k : ks) printf("%14u", k);
  printf("\n%-22s", "tachyon_mi355x (s)");
  for (double s : secs) printf("%14.6f", s);
  printf("\n%-22s", "scalars/s");
  for (size_t i = 0; i < ks.size(); ++i) printf("%14.4g", (double)(size_t(1) << ks[i]) / secs[i]);
  printf("\n{\"benchmark\": \"msm\", \"curve\": \"%s_g1\", \"test_set\": \"%s\", \"device_resident\": %s, "
         "\"check_results\": %s, \"checked_against\": \"%s\", \"results\": [",
         curve.c_str(), non_uniform ? "non_uniform" : "random", device_resident ? "true" : "false",
         check ? (ok ? "\"pass\"" : "\"FAIL\"") : "null", expect.empty() ? "chunk_sum" : "expect_file");
  for (size_t i = 0; i < ks.size(); ++i) printf("%s{\"k\": %u, \"seconds\": %.6f}", i ? ", " : "", ks[i], secs[i]);
  printf("]}\n");

  if (bls) tachyon_bls12_381_g1_destroy_msm_gpu(static_cast<tachyon_bls12_381_g1_msm_gpu_ptr>(msm));
  else tachyon_bn254_g1_destroy_msm_gpu(static_cast<tachyon_bn254_g1_msm_gpu_ptr>(msm));
  hip_check(hipFree(d_bases), "hipFree");
  hip_check(hipFree(d_scalars), "hipFree");
  return ok ? 0 : 1;
}
