// fft_benchmark_gpu: the reference's benchmark/fft/fft_benchmark_gpu.cc harness
// on the MI355X backend, written against the public C-ABI only.
//
//   fft_benchmark_gpu -k 20 -k 24 ... [--run_ifft] [--check_results] [--device_resident]
//                     [--expect FILE]
//
// Kept from the reference (fft_benchmark_gpu.cc:25-87, fft_config.cc:13-56,
// fft_runner.h:49-61): for each k a random input of 2^k elements (degree
// 2^k - 1), a domain Create(degree + 1), and one timed call of
// tachyon_bn254_univariate_evaluation_domain_fft_inplace (or _ifft_inplace
// with --run_ifft) on host-resident containers (H2D + transform + D2H, as the
// reference's icicle path).  Stated differences: the input comes from the
// device generator (seeded, canonical Montgomery values); one untimed warm-up
// call per size; --device_resident times the in-HBM transform
// (tachyon_mi355x_..._transform_device) instead.  --check_results: the
// reference compares the timed GPU output with its CPU transform of the same
// input (fft_benchmark_gpu.cc:81-83); the product has no CPU transform, so the
// CPU outputs come in through --expect FILE (per size, ascending, 2^k
// Montgomery elements; tests/test_gpu_harness.py writes it with the CPU
// oracle from the same seeded input, seed 0x7AC40001 + k).  Without --expect it
// checks the round trip IFFT(FFT(x)) == x.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
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
  std::cerr << "usage: fft_benchmark_gpu -k K [-k K ...] [--run_ifft] [--check_results] [--device_resident]\n"
               "                         [--expect FILE]\n";
  return 1;
}

using Clock = std::chrono::steady_clock;

}  // namespace

int main(int argc, char** argv) {
  std::vector<unsigned> ks;
  bool ifft = false, check = false, device_resident = false;
  std::string expect_path;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "-k" && i + 1 < argc) ks.push_back((unsigned)std::stoul(argv[++i]));
    else if (a == "--run_ifft") ifft = true;
    else if (a == "--check_results") check = true;
    else if (a == "--device_resident") device_resident = true;
    else if (a == "--expect" && i + 1 < argc) expect_path = argv[++i];
    else return usage();
  }
  if (ks.empty()) return usage();
  std::sort(ks.begin(), ks.end());
  FILE* expect_file = nullptr;
  if (!expect_path.empty() && !(expect_file = fopen(expect_path.c_str(), "rb"))) return usage();
  std::vector<double> secs;
  bool ok = true;
  for (unsigned k : ks) {
    const size_t n = size_t(1) << k;
    void* d_in = nullptr;
    hip_check(hipMalloc(&d_in, n * sizeof(tachyon_bn254_fr)), "hipMalloc");
    tachyon_mi355x_gen_scalars(1, 0x7AC40001ULL + k, 0, n, d_in, nullptr);
    hip_check(hipDeviceSynchronize(), "sync");
    std::vector<tachyon_bn254_fr> input(n);
    hip_check(hipMemcpy(input.data(), d_in, n * sizeof(tachyon_bn254_fr), hipMemcpyDeviceToHost), "copy");
    tachyon_bn254_univariate_evaluation_domain* dom = tachyon_bn254_univariate_evaluation_domain_create(n);
    double dt = 0;
    std::vector<tachyon_bn254_fr> result(n, tachyon_bn254_fr{});  // the timed call's output
    if (device_resident) {
      void* d_work = nullptr;
      hip_check(hipMalloc(&d_work, n * sizeof(tachyon_bn254_fr)), "hipMalloc");
      auto* stream = static_cast<hipStream_t>(tachyon_mi355x_bn254_univariate_evaluation_domain_stream(dom));
      for (int rep = 0; rep < 2; ++rep) {  // rep 0 = warm-up
        hip_check(hipMemcpy(d_work, d_in, n * sizeof(tachyon_bn254_fr), hipMemcpyDeviceToDevice), "copy");
        auto t0 = Clock::now();
        tachyon_mi355x_bn254_univariate_evaluation_domain_transform_device(
            dom, static_cast<tachyon_bn254_fr*>(d_work), ifft ? 1 : 0);
        hip_check(hipStreamSynchronize(stream), "sync");
        dt = std::chrono::duration<double>(Clock::now() - t0).count();
      }
      hip_check(hipMemcpy(result.data(), d_work, n * sizeof(tachyon_bn254_fr), hipMemcpyDeviceToHost), "copy");
      hip_check(hipFree(d_work), "hipFree");
    } else {
      for (int rep = 0; rep < 2; ++rep) {  // rep 0 = warm-up
        // fresh container per call: the in-place entry points take it over
        if (ifft) {
          tachyon_bn254_univariate_evaluations* e = tachyon_bn254_univariate_evaluations_create();
          tachyon_mi355x_bn254_univariate_evaluations_resize(e, n);
          memcpy(tachyon_mi355x_bn254_univariate_evaluations_data(e), input.data(), n * sizeof(tachyon_bn254_fr));
          auto t0 = Clock::now();
          tachyon_bn254_univariate_dense_polynomial* p =
              tachyon_bn254_univariate_evaluation_domain_ifft_inplace(dom, e);
          dt = std::chrono::duration<double>(Clock::now() - t0).count();
          const size_t len = tachyon_mi355x_bn254_univariate_dense_polynomial_len(p);  // trimmed
          memcpy(result.data(), tachyon_mi355x_bn254_univariate_dense_polynomial_data(p),
                 len * sizeof(tachyon_bn254_fr));
          tachyon_bn254_univariate_dense_polynomial_destroy(p);
          tachyon_bn254_univariate_evaluations_destroy(e);
        } else {
          tachyon_bn254_univariate_dense_polynomial* p = tachyon_bn254_univariate_dense_polynomial_create();
          tachyon_mi355x_bn254_univariate_dense_polynomial_resize(p, n);
          memcpy(tachyon_mi355x_bn254_univariate_dense_polynomial_data(p), input.data(),
                 n * sizeof(tachyon_bn254_fr));
          auto t0 = Clock::now();
          tachyon_bn254_univariate_evaluations* e = tachyon_bn254_univariate_evaluation_domain_fft_inplace(dom, p);
          dt = std::chrono::duration<double>(Clock::now() - t0).count();
          memcpy(result.data(), tachyon_mi355x_bn254_univariate_evaluations_data(e), n * sizeof(tachyon_bn254_fr));
          tachyon_bn254_univariate_evaluations_destroy(e);
          tachyon_bn254_univariate_dense_polynomial_destroy(p);
        }
      }
    }
    secs.push_back(dt);
    if (check && expect_file) {  // CHECK_EQ(cpu result, gpu result)
      std::vector<tachyon_bn254_fr> want(n);
      if (fread(want.data(), sizeof(tachyon_bn254_fr), n, expect_file) != n ||
          memcmp(want.data(), result.data(), n * sizeof(tachyon_bn254_fr)) != 0) {
        std::cerr << "Results not matched at 2^" << k << std::endl;
        ok = false;
      }
    } else if (check) {  // IFFT(FFT(x)) == x through the reference entry points
      tachyon_bn254_univariate_dense_polynomial* p = tachyon_bn254_univariate_dense_polynomial_create();
      tachyon_mi355x_bn254_univariate_dense_polynomial_resize(p, n);
      memcpy(tachyon_mi355x_bn254_univariate_dense_polynomial_data(p), input.data(), n * sizeof(tachyon_bn254_fr));
      tachyon_bn254_univariate_evaluations* e = tachyon_bn254_univariate_evaluation_domain_fft(dom, p);
      tachyon_bn254_univariate_dense_polynomial* back = tachyon_bn254_univariate_evaluation_domain_ifft(dom, e);
      const size_t len = tachyon_mi355x_bn254_univariate_dense_polynomial_len(back);
      const tachyon_bn254_fr* bd = tachyon_mi355x_bn254_univariate_dense_polynomial_data(back);
      // the IFFT drops trailing zero coefficients (RemoveHighDegreeZeros)
      bool same = len <= n && memcmp(bd, input.data(), len * sizeof(tachyon_bn254_fr)) == 0;
      for (size_t i = len; same && i < n; ++i)
        for (int l = 0; l < 4; ++l) same = same && input[i].limbs[l] == 0;
      if (!same) {
        std::cerr << "Results not matched at 2^" << k << std::endl;
        ok = false;
      }
      tachyon_bn254_univariate_dense_polynomial_destroy(back);
      tachyon_bn254_univariate_evaluations_destroy(e);
      tachyon_bn254_univariate_dense_polynomial_destroy(p);
    }
    tachyon_bn254_univariate_evaluation_domain_destroy(dom);
    hip_check(hipFree(d_in), "hipFree");
  }
  printf("%s Benchmark GPU (%s)\n", ifft ? "IFFT" : "FFT",
         device_resident ? "device-resident data" : "host-resident containers, H2D + D2H included");
  printf("%-22s", "Degree (2^x)");
  for (unsigned k : ks) printf("%14u", k);
  printf("\n%-22s", "tachyon_mi355x (s)");
  for (double s : secs) printf("%14.6f", s);
  printf("\n%-22s", "elems/s");
  for (size_t i = 0; i < ks.size(); ++i) printf("%14.4g", (double)(size_t(1) << ks[i]) / secs[i]);
  printf("\n{\"benchmark\": \"%s\", \"device_resident\": %s, \"check_results\": %s, \"checked_against\": \"%s\", "
         "\"results\": [",
         ifft ? "ifft" : "fft", device_resident ? "true" : "false", check ? (ok ? "\"pass\"" : "\"FAIL\"") : "null",
         expect_file ? "expect_file" : "round_trip");
  if (expect_file) fclose(expect_file);
  for (size_t i = 0; i < ks.size(); ++i) printf("%s{\"k\": %u, \"seconds\": %.6f}", i ? ", " : "", ks[i], secs[i]);
  printf("]}\n");
  return ok ? 0 : 1;
}
