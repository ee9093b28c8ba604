// Exercise include/tachyon_mi355x_ntt_holder.h the way a Tachyon build would
// use IcicleNTTHolder (univariate_evaluation_domain.h:141-232): in-place FFT /
// IFFT on host vectors, plain and on the coset 5*<w>
// (univariate_evaluation_domain_gpu_unittest.cc:51-66).  Checks: FFT equals the
// C-ABI domain's _fft, IFFT(FFT(v)) == v, coset IFFT(coset FFT(v)) == v, and
// the coset FFT differs from the plain one.  Prints one JSON line; exit 0 = ok.
//   ntt_holder_check [log_n] [--dump file]  (dump: input | fft | coset fft)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/tachyon_mi355x_ntt_holder.h"

namespace {

bool same(const std::vector<tachyon_bn254_fr>& a, const std::vector<tachyon_bn254_fr>& b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(a[0])) == 0;
}

}  // namespace

int main(int argc, char** argv) {
  unsigned log_n = 12;
  const char* dump = nullptr;
  for (int i = 1; i < argc; ++i) {
    if (std::string(argv[i]) == "--dump" && i + 1 < argc) dump = argv[++i];
    else log_n = (unsigned)atoi(argv[i]);
  }
  const size_t n = size_t(1) << log_n;
  tachyon_bn254_fr* d = nullptr;
  if (hipMalloc(&d, n * sizeof(tachyon_bn254_fr)) != hipSuccess) return 2;
  tachyon_mi355x_gen_scalars(1, 0x7AC40001ULL, 0, n, d, nullptr);
  std::vector<tachyon_bn254_fr> input(n);
  if (hipMemcpy(input.data(), d, n * sizeof(tachyon_bn254_fr), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  (void)hipFree(d);

  auto holder = tachyon_mi355x::NTTHolder::Create(n);
  // the C-ABI domain path for comparison
  tachyon_bn254_univariate_dense_polynomial* p = tachyon_bn254_univariate_dense_polynomial_create();
  tachyon_mi355x_bn254_univariate_dense_polynomial_resize(p, n);
  std::memcpy(tachyon_mi355x_bn254_univariate_dense_polynomial_data(p), input.data(), n * sizeof(input[0]));
  tachyon_bn254_univariate_evaluation_domain* dom = tachyon_bn254_univariate_evaluation_domain_create(n);
  tachyon_bn254_univariate_evaluations* e = tachyon_bn254_univariate_evaluation_domain_fft(dom, p);
  std::vector<tachyon_bn254_fr> via_capi(n);
  for (size_t i = 0; i < n; ++i) tachyon_mi355x_bn254_univariate_evaluations_get_value(e, i, &via_capi[i]);

  std::vector<tachyon_bn254_fr> v = input;
  holder->FFT(v);
  const bool fft_ok = same(v, via_capi);
  const std::vector<tachyon_bn254_fr> plain = v;
  holder->IFFT(v);
  const bool round_ok = same(v, input);

  // coset offset 5 (Montgomery form of 5 = 5 R mod r)
  tachyon_bn254_fr five = {{0x1b0d0ef99fffffe6ULL, 0xeaba68a3a32a913fULL, 0x47d8eb76d8dd0689ULL,
                            0x15d0085520f5bbc3ULL}};
  holder->FFT(v, &five);
  const std::vector<tachyon_bn254_fr> coset = v;
  const bool coset_differs = !same(coset, plain);
  holder->IFFT(v, &five);
  const bool coset_round_ok = same(v, input);
  if (dump) {
    FILE* f = fopen(dump, "wb");
    if (!f) return 2;
    fwrite(input.data(), sizeof(input[0]), n, f);
    fwrite(plain.data(), sizeof(plain[0]), n, f);
    fwrite(coset.data(), sizeof(coset[0]), n, f);
    fclose(f);
  }
  tachyon_bn254_univariate_evaluations_destroy(e);
  tachyon_bn254_univariate_dense_polynomial_destroy(p);
  tachyon_bn254_univariate_evaluation_domain_destroy(dom);
  const bool ok = fft_ok && round_ok && coset_differs && coset_round_ok;
  printf("{\"log_n\": %u, \"fft_matches_capi\": %s, \"round_trip\": %s, \"coset_differs\": %s, "
         "\"coset_round_trip\": %s}\n",
         log_n, fft_ok ? "true" : "false", round_ok ? "true" : "false", coset_differs ? "true" : "false",
         coset_round_ok ? "true" : "false");
  return ok ? 0 : 1;
}
