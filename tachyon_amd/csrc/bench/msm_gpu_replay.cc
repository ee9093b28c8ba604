// msm_gpu_replay: the reference's tachyon/c/math/elliptic_curves/msm/msm_gpu_replay.cc
// on the MI355X backend (C-ABI only).  Replays MSM inputs dumped by any
// process that ran tachyon_bn254_g1_*_msm_gpu with TACHYON_MSM_GPU_INPUT_DIR
// set (msm_gpu.h:99-119: bases<idx>.txt / scalars<idx>.txt, each a u64 count
// followed by canonical little-endian limbs -- base::Buffer serialisation with
// s_is_in_montgomery = false), so production inputs (e.g. from the halo2 Rust
// bridge) can be re-run against this backend.
//
//   msm_gpu_replay --input_dir DIR --degree D --idx 0 [--idx 1 ...]
//
// Prints, per index, the wall time of tachyon_bn254_g1_affine_msm_gpu and the
// affine result as (0x<x>, 0x<y>) canonical hex (ToAffine().ToHexString()).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "../../../include/tachyon_mi355x.h"

namespace {

std::vector<uint64_t> read_words(const std::string& path, size_t words_per_item, size_t* count) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    std::cerr << "cannot open " << path << std::endl;
    exit(1);
  }
  uint64_t n = 0;
  f.read(reinterpret_cast<char*>(&n), 8);
  std::vector<uint64_t> v(n * words_per_item);
  f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(v.size() * 8));
  if (!f || f.peek() != EOF) {  // buffer.Done(): the whole file is consumed
    std::cerr << "malformed dump " << path << std::endl;
    exit(1);
  }
  *count = n;
  return v;
}

std::string hex(const uint64_t* l, int n) {
  int i = n - 1;
  while (i > 0 && l[i] == 0) --i;
  char buf[32];
  snprintf(buf, sizeof buf, "0x%llx", (unsigned long long)l[i]);
  std::string s = buf;
  while (--i >= 0) {
    snprintf(buf, sizeof buf, "%016llx", (unsigned long long)l[i]);
    s += buf;
  }
  return s;
}

}  // namespace

int main(int argc, char** argv) {
  if (getenv("TACHYON_MSM_GPU_INPUT_DIR")) {  // msm_gpu_replay.cc:41-44
    std::cerr << "If this is set, the log is overwritten" << std::endl;
    return 1;
  }
  std::vector<int> idxes;
  int degree = -1;
  std::string dir;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--idx" && i + 1 < argc) idxes.push_back(std::atoi(argv[++i]));
    else if (a == "--degree" && i + 1 < argc) degree = std::atoi(argv[++i]);
    else if (a == "--input_dir" && i + 1 < argc) dir = argv[++i];
    else {
      std::cerr << "usage: msm_gpu_replay --input_dir DIR --degree D --idx I [--idx I ...]" << std::endl;
      return 1;
    }
  }
  if (idxes.empty() || degree < 0 || dir.empty()) {
    std::cerr << "--idx, --degree and --input_dir are required" << std::endl;
    return 1;
  }
  tachyon_bn254_g1_init();
  tachyon_bn254_g1_msm_gpu_ptr msm = tachyon_bn254_g1_create_msm_gpu((uint8_t)degree);
  for (int idx : idxes) {
    size_t nb = 0, ns = 0;
    std::vector<uint64_t> bases = read_words(dir + "/bases" + std::to_string(idx) + ".txt", 8, &nb);
    std::vector<uint64_t> scalars = read_words(dir + "/scalars" + std::to_string(idx) + ".txt", 4, &ns);
    if (nb != ns) {
      std::cerr << "bases and scalars differ in length" << std::endl;
      return 1;
    }
    // canonical -> Montgomery (the reader's FromBigInt), on the device
    std::vector<uint64_t> bm(bases.size()), sm(scalars.size());
    if (nb) {
      tachyon_mi355x_field_op(0, 6, bases.data(), bases.data(), bm.data(), 2 * nb);
      tachyon_mi355x_field_op(1, 6, scalars.data(), scalars.data(), sm.data(), ns);
    }
    auto t0 = std::chrono::steady_clock::now();
    tachyon_bn254_g1_jacobian* r = tachyon_bn254_g1_affine_msm_gpu(
        msm, reinterpret_cast<const tachyon_bn254_g1_affine*>(bm.data()),
        reinterpret_cast<const tachyon_bn254_fr*>(sm.data()), ns);
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t aff[8], canon[8];
    tachyon_mi355x_jacobian_to_affine(0, r, aff);
    tachyon_mi355x_jacobian_destroy(0, r);
    tachyon_mi355x_field_op(0, 7, aff, aff, canon, 2);  // Montgomery -> canonical
    std::cout << dt << " s" << std::endl;
    std::cout << "(" << hex(canon, 4) << ", " << hex(canon + 4, 4) << ")" << std::endl;
  }
  tachyon_bn254_g1_destroy_msm_gpu(msm);
  return 0;
}
