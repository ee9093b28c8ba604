// circom_prover: the reference's vendors/circom/prover_main.cc on the MI355X
// backend, written against the public C-ABI only (include/tachyon_mi355x.h).
//
//   circom_prover --zkey circuit.zkey --wtns witness.wtns --proof proof.json \
//                 --public public.json [--curve bn254|bls12_381] [--no_zk] [-n N] [--devices 0,1,..]
//
// Same flags, outputs and JSON layout as the reference (prover_main.cc:188-283;
// proof JSON: circomlib/json/groth16_proof.h + points.h -- decimal canonical
// coordinates, projective "1" / ["1","0"] third coordinate, "protocol":
// "groth16", "curve": "bn128" | "bls12381"; public JSON: prime_field.h -- an
// array of decimal strings).  --verify is rejected: this backend has no
// pairing (the test-suite's oracle checks proofs with one).  --no_use_mmap is
// accepted and ignored (the files are read once into memory).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <fstream>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/tachyon_mi355x.h"

namespace {

// moduli (little-endian 64-bit limbs): scalar field r and base field q
const uint64_t kBn254Fr[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                              0x30644e72e131a029ULL};
const uint64_t kBn254Fq[4] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL,
                              0x30644e72e131a029ULL};
const uint64_t kBls381Fr[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                               0x73eda753299d7d48ULL};
const uint64_t kBls381Fq[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                               0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};

using Limbs = std::vector<uint64_t>;

// a * b mod m for little-endian limb vectors (schoolbook + shift-subtract;
// only used for a handful of values per proof)
bool geq(const Limbs& a, const Limbs& b) {
  for (size_t i = a.size(); i-- > 0;)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}
void sub_in(Limbs& a, const Limbs& b) {
  unsigned __int128 borrow = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    unsigned __int128 d = (unsigned __int128)a[i] - b[i] - borrow;
    a[i] = (uint64_t)d;
    borrow = (d >> 64) ? 1 : 0;
  }
}
// x * 2 mod m (x < m)
void dbl_mod(Limbs& x, const Limbs& m) {
  uint64_t carry = 0;
  for (auto& v : x) {
    uint64_t nc = v >> 63;
    v = (v << 1) | carry;
    carry = nc;
  }
  if (carry || geq(x, m)) sub_in(x, m);
}
void add_mod(Limbs& x, const Limbs& y, const Limbs& m) {
  unsigned __int128 c = 0;
  for (size_t i = 0; i < x.size(); ++i) {
    c += (unsigned __int128)x[i] + y[i];
    x[i] = (uint64_t)c;
    c >>= 64;
  }
  if (c || geq(x, m)) sub_in(x, m);
}
// canonical value of a Montgomery word: x * R^-1 mod m, R = 2^(64 N) -- via
// x * 2^-1 repeated 64 N times
Limbs from_mont(const uint64_t* w, const Limbs& m) {
  Limbs x(w, w + m.size());
  for (size_t k = 0; k < 64 * m.size(); ++k) {
    if (x[0] & 1) {  // (x + m) / 2
      unsigned __int128 c = 0;
      for (size_t i = 0; i < x.size(); ++i) {
        c += (unsigned __int128)x[i] + m[i];
        x[i] = (uint64_t)c;
        c >>= 64;
      }
      for (size_t i = 0; i < x.size(); ++i) x[i] = (x[i] >> 1) | (i + 1 < x.size() ? x[i + 1] << 63 : (uint64_t)c << 63);
    } else {
      for (size_t i = 0; i < x.size(); ++i) x[i] = (x[i] >> 1) | (i + 1 < x.size() ? x[i + 1] << 63 : 0);
    }
  }
  return x;
}
// canonical value -> Montgomery word: v * 2^(64 N) mod m
Limbs to_mont(Limbs v, const Limbs& m) {
  while (geq(v, m)) sub_in(v, m);
  for (size_t k = 0; k < 64 * m.size(); ++k) dbl_mod(v, m);
  return v;
}
std::string decimal(Limbs v) {
  std::string out;
  bool zero = true;
  for (auto x : v) zero = zero && x == 0;
  if (zero) return "0";
  while (true) {
    bool nz = false;
    unsigned __int128 rem = 0;
    for (size_t i = v.size(); i-- > 0;) {
      unsigned __int128 cur = (rem << 64) | v[i];
      v[i] = (uint64_t)(cur / 10);
      rem = cur % 10;
      nz = nz || v[i];
    }
    out.push_back(char('0' + (int)rem));
    if (!nz) break;
  }
  return std::string(out.rbegin(), out.rend());
}

std::vector<uint8_t> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct CurveInfo {
  int id;
  const char* json_name;
  Limbs q, r;
  size_t fq_bytes() const { return q.size() * 8; }
};

std::string coord(const uint8_t* w, const Limbs& q) { return decimal(from_mont(reinterpret_cast<const uint64_t*>(w), q)); }

std::string g1_json(const uint8_t* p, const CurveInfo& c) {
  const size_t f = c.fq_bytes();
  return "[\"" + coord(p, c.q) + "\",\"" + coord(p + f, c.q) + "\",\"1\"]";
}
std::string g2_json(const uint8_t* p, const CurveInfo& c) {
  const size_t f = c.fq_bytes();
  return "[[\"" + coord(p, c.q) + "\",\"" + coord(p + f, c.q) + "\"],[\"" + coord(p + 2 * f, c.q) + "\",\"" +
         coord(p + 3 * f, c.q) + "\"],[\"1\",\"0\"]]";
}

int usage() {
  std::cerr << "usage: circom_prover --zkey F --wtns F --proof F --public F [--curve bn254|bls12_381] [--no_zk]\n"
               "                     [-n|--num_runs N] [--no_use_mmap] [--devices 0,1,...]\n";
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  std::string zkey_path, wtns_path, proof_path, public_path, curve_name = "bn254";
  bool no_zk = false;
  size_t num_runs = 1;
  std::vector<int> devices;  // --devices 0,1,...: one-process multi-device proofs
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
      return argv[++i];
    };
    if (a == "--zkey" || a == "zkey") zkey_path = next();
    else if (a == "--wtns" || a == "wtns") wtns_path = next();
    else if (a == "--proof" || a == "proof") proof_path = next();
    else if (a == "--public" || a == "public") public_path = next();
    else if (a == "--curve") curve_name = next();
    else if (a == "--no_zk") no_zk = true;
    else if (a == "--no_use_mmap") {}
    else if (a == "-n" || a == "--num_runs") num_runs = std::stoul(next());
    else if (a == "--verify") { std::cerr << "--verify is not supported by this backend\n"; return 1; }
    else if (a == "--trace_path") next();
    else if (a == "--devices") {
      // comma-separated non-negative ids; empty fields are skipped, anything
      // else that is not a number is a usage error (not an uncaught throw)
      std::string list = next();
      size_t pos = 0;
      while (pos <= list.size()) {
        size_t comma = list.find(',', pos);
        if (comma == std::string::npos) comma = list.size();
        const std::string field = list.substr(pos, comma - pos);
        pos = comma + 1;
        if (field.empty()) continue;
        if (field.find_first_not_of("0123456789") != std::string::npos || field.size() > 6) return usage();
        devices.push_back(std::stoi(field));
      }
      if (devices.empty()) return usage();
    }
    else return usage();
  }
  if (zkey_path.empty() || wtns_path.empty() || proof_path.empty() || public_path.empty() || num_runs == 0)
    return usage();
  CurveInfo c;
  if (curve_name == "bn254") c = {0, "bn128", Limbs(kBn254Fq, kBn254Fq + 4), Limbs(kBn254Fr, kBn254Fr + 4)};
  else if (curve_name == "bls12_381") c = {1, "bls12381", Limbs(kBls381Fq, kBls381Fq + 6), Limbs(kBls381Fr, kBls381Fr + 4)};
  else return usage();

  using Clock = std::chrono::steady_clock;
  auto start = Clock::now();
  std::cout << "Start parsing zkey" << std::endl;
  std::vector<uint8_t> zkey = read_file(zkey_path);
  if (tachyon_mi355x_zkey_curve(zkey.data(), zkey.size()) != c.id) {
    std::cerr << "zkey curve does not match --curve " << curve_name << std::endl;
    return 1;
  }
  tachyon_mi355x_groth16_prover* prover = tachyon_mi355x_groth16_prover_create(zkey.data(), zkey.size());
  zkey.clear();
  zkey.shrink_to_fit();
  uint32_t info[4];
  tachyon_mi355x_groth16_prover_info(prover, info);
  if (devices.size() > 1 && !tachyon_mi355x_groth16_set_devices(prover, devices.data(), devices.size())) {
    std::cerr << "--devices: a device id is out of range" << std::endl;
    return 1;
  }
  auto now = Clock::now();
  std::cout << "Time taken for parsing zkey (and uploading the proving key): "
            << std::chrono::duration<double>(now - start).count() << " s" << std::endl;
  start = now;

  std::cout << "Start parsing witness" << std::endl;
  std::vector<uint8_t> wtns = read_file(wtns_path);
  size_t count = tachyon_mi355x_wtns_parse(c.id, wtns.data(), wtns.size(), nullptr, 0);
  std::vector<uint8_t> full(count * 32);
  tachyon_mi355x_wtns_parse(c.id, wtns.data(), wtns.size(), full.data(), count);
  now = Clock::now();
  std::cout << "Time taken for parsing witness: " << std::chrono::duration<double>(now - start).count() << " s"
            << std::endl;
  start = now;

  const size_t g1b = 2 * c.fq_bytes(), g2b = 4 * c.fq_bytes();
  std::vector<uint8_t> a(g1b), b(g2b), cc(g1b);
  std::random_device rd;
  std::mt19937_64 rng(((uint64_t)rd() << 32) ^ rd());
  double total = 0, worst = 0;
  std::cout << "Start proving" << std::endl;
  for (size_t run = 0; run < num_runs; ++run) {
    if (no_zk) {
      tachyon_mi355x_groth16_prove(prover, full.data(), count, nullptr, nullptr, a.data(), b.data(), cc.data());
    } else {
      // F::Random() blinding (prove.h:170-176): uniform below r, Montgomery form
      Limbs rs[2];
      for (auto& v : rs) {
        v.assign(4, 0);
        do {
          for (auto& x : v) x = rng();
          v[3] &= (1ULL << 63) - 1;
        } while (geq(v, c.r));
        v = to_mont(v, c.r);
      }
      tachyon_mi355x_groth16_prove(prover, full.data(), count, rs[0].data(), rs[1].data(), a.data(), b.data(),
                                   cc.data());
    }
    now = Clock::now();
    double dt = std::chrono::duration<double>(now - start).count();
    std::cout << "Time taken for proving #" << run << ": " << dt << " s" << std::endl;
    total += dt;
    worst = std::max(worst, dt);
    start = now;
  }
  std::cout << "Avg time taken for proving: " << total / num_runs << " s" << std::endl;
  std::cout << "Max time taken for proving: " << worst << " s" << std::endl;

  std::ofstream pf(proof_path);
  pf << "{\"pi_a\":" << g1_json(a.data(), c) << ",\"pi_b\":" << g2_json(b.data(), c)
     << ",\"pi_c\":" << g1_json(cc.data(), c) << ",\"protocol\":\"groth16\",\"curve\":\"" << c.json_name << "\"}";
  pf.close();
  std::cout << "Proof is saved to \"" << proof_path << "\"" << std::endl;
  std::ofstream pub(public_path);
  pub << "[";
  for (uint32_t i = 1; i <= info[2]; ++i) {
    if (i > 1) pub << ",";
    pub << "\"" << decimal(from_mont(reinterpret_cast<const uint64_t*>(full.data() + 32 * i), c.r)) << "\"";
  }
  pub << "]";
  pub.close();
  std::cout << "Public input is saved to \"" << public_path << "\"" << std::endl;
  tachyon_mi355x_groth16_prover_destroy(prover);
  return 0;
}
