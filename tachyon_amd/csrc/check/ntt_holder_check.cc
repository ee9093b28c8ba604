// Exercise include/tachyon_mi355x_ntt_holder.h the way a Tachyon build would
// use IcicleNTTHolder (univariate_evaluation_domain.h:141-232): in-place FFT /
// IFFT on host vectors, plain and on a coset
// (univariate_evaluation_domain_gpu_unittest.cc:51-66).
//   bn254 (default): NTTHolder over the reference's C-ABI domain, coset 5<w>;
//     checks FFT == the C-ABI domain's _fft.
//   --field bls12_381: FieldNTTHolder<kBls12_381Fr> (IcicleNTT<bls12_381::Fr>,
//     icicle_ntt_bls12_381.cc:31-115), coset 7<w> (the BUILD subgroup
//     generator); checks FFT == the field-generic domain's device transform.
// Both: IFFT(FFT(v)) == v, coset IFFT(coset FFT(v)) == v, coset FFT != plain.
// Prints one JSON line; exit 0 = ok.
//   ntt_holder_check [log_n] [--field bn254|bls12_381] [--dump file]
//   (dump: input | fft | coset fft, 32-byte Montgomery elements)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/tachyon_mi355x_ntt_holder.h"

namespace {

struct Fr4 {
  uint64_t limbs[4];
};

bool same(const std::vector<Fr4>& a, const std::vector<Fr4>& b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(a[0])) == 0;
}

// the reference path each holder replaces, for the plain FFT
std::vector<Fr4> reference_fft(bool bls, const std::vector<Fr4>& input) {
  const size_t n = input.size();
  std::vector<Fr4> out(n);
  if (!bls) {  // tachyon_bn254_univariate_evaluation_domain_fft (the reference C-ABI)
    tachyon_bn254_univariate_dense_polynomial* p = tachyon_bn254_univariate_dense_polynomial_create();
    tachyon_mi355x_bn254_univariate_dense_polynomial_resize(p, n);
    std::memcpy(tachyon_mi355x_bn254_univariate_dense_polynomial_data(p), input.data(), n * sizeof(Fr4));
    tachyon_bn254_univariate_evaluation_domain* dom = tachyon_bn254_univariate_evaluation_domain_create(n);
    tachyon_bn254_univariate_evaluations* e = tachyon_bn254_univariate_evaluation_domain_fft(dom, p);
    for (size_t i = 0; i < n; ++i)
      tachyon_mi355x_bn254_univariate_evaluations_get_value(e, i, reinterpret_cast<tachyon_bn254_fr*>(&out[i]));
    tachyon_bn254_univariate_evaluations_destroy(e);
    tachyon_bn254_univariate_dense_polynomial_destroy(p);
    tachyon_bn254_univariate_evaluation_domain_destroy(dom);
    return out;
  }
  // the field-generic domain's device-resident transform
  tachyon_mi355x_ntt_domain* dom = tachyon_mi355x_ntt_domain_create(3, n);
  void* d = nullptr;
  if (hipMalloc(&d, n * sizeof(Fr4)) != hipSuccess) exit(2);
  if (hipMemcpy(d, input.data(), n * sizeof(Fr4), hipMemcpyHostToDevice) != hipSuccess) exit(2);
  tachyon_mi355x_ntt_domain_transform_device(dom, d, 1, 0);
  if (hipStreamSynchronize(static_cast<hipStream_t>(tachyon_mi355x_ntt_domain_stream(dom))) != hipSuccess) exit(2);
  if (hipMemcpy(out.data(), d, n * sizeof(Fr4), hipMemcpyDeviceToHost) != hipSuccess) exit(2);
  (void)hipFree(d);
  tachyon_mi355x_ntt_domain_destroy(dom);
  return out;
}

template <class Holder>
int run(Holder& holder, bool bls, unsigned log_n, const Fr4& offset, const char* dump) {
  const size_t n = size_t(1) << log_n;
  Fr4* d = nullptr;
  if (hipMalloc(&d, n * sizeof(Fr4)) != hipSuccess) return 2;
  tachyon_mi355x_gen_scalars(bls ? 3 : 1, 0x7AC40001ULL, 0, n, d, nullptr);
  std::vector<Fr4> input(n);
  if (hipMemcpy(input.data(), d, n * sizeof(Fr4), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  (void)hipFree(d);
  const std::vector<Fr4> want = reference_fft(bls, input);

  std::vector<Fr4> v = input;
  holder->FFT(v);
  const bool fft_ok = same(v, want);
  const std::vector<Fr4> plain = v;
  holder->IFFT(v);
  const bool round_ok = same(v, input);
  holder->FFT(v, &offset);
  const std::vector<Fr4> coset = v;
  const bool coset_differs = !same(coset, plain);
  holder->IFFT(v, &offset);
  const bool coset_round_ok = same(v, input);
  if (dump) {
    FILE* f = fopen(dump, "wb");
    if (!f) return 2;
    fwrite(input.data(), sizeof(Fr4), n, f);
    fwrite(plain.data(), sizeof(Fr4), n, f);
    fwrite(coset.data(), sizeof(Fr4), n, f);
    fclose(f);
  }
  const bool ok = fft_ok && round_ok && coset_differs && coset_round_ok;
  printf("{\"field\": \"%s\", \"log_n\": %u, \"fft_matches_capi\": %s, \"round_trip\": %s, \"coset_differs\": %s, "
         "\"coset_round_trip\": %s}\n",
         bls ? "bls12_381_fr" : "bn254_fr", log_n, fft_ok ? "true" : "false", round_ok ? "true" : "false",
         coset_differs ? "true" : "false", coset_round_ok ? "true" : "false");
  return ok ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
  unsigned log_n = 12;
  const char* dump = nullptr;
  bool bls = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--dump" && i + 1 < argc) dump = argv[++i];
    else if (a == "--field" && i + 1 < argc) bls = std::string(argv[++i]) == "bls12_381";
    else log_n = (unsigned)atoi(argv[i]);
  }
  const size_t n = size_t(1) << log_n;
  if (bls) {
    // 7 in Montgomery form (7 R mod r, BLS12-381 Fr)
    const Fr4 seven = {{0x0000000efffffff1ULL, 0x17e363d300189c0fULL, 0xff9c57876f8457b0ULL, 0x351332208fc5a8c4ULL}};
    auto holder = tachyon_mi355x::FieldNTTHolder<tachyon_mi355x::kBls12_381Fr>::Create(n);
    return run(holder, true, log_n, seven, dump);
  }
  // 5 in Montgomery form (5 R mod r, BN254 Fr)
  const Fr4 five = {{0x1b0d0ef99fffffe6ULL, 0xeaba68a3a32a913fULL, 0x47d8eb76d8dd0689ULL, 0x15d0085520f5bbc3ULL}};
  auto holder = tachyon_mi355x::NTTHolder::Create(n);
  return run(holder, false, log_n, five, dump);
}
