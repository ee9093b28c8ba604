// Circom binary formats on the host: zkey v1 (Groth16 proving key) and
// wtns v2 (witness).  Host-only C++; the parsed arrays are handed to the GPU
// prover (groth16.h) which uploads them once.
//
// Reference readers restated here:
//   vendors/circom/circomlib/zkey/zkey.h:64-84 (magic/version), :89-100
//     (section ids), :114-123 (header, prover_type 1), :147-153 (Groth header:
//     q, r, num_vars, num_public_inputs, domain_size, verifying key),
//     :176-190 (point sections), :211-223 (coefficients, value re-read with
//     FromMontgomery), :255-296 (section order and element counts)
//   vendors/circom/circomlib/zkey/verifying_key.h (alpha_g1, beta_g1,
//     beta_g2, gamma_g2, delta_g1, delta_g2 -- in that order on disk)
//   vendors/circom/circomlib/wtns/wtns.h:75-117 (header: modulus, count;
//     data: canonical LE values converted to Montgomery)
//   vendors/circom/circomlib/base/sections.h (u32 count, then {u32 type,
//     u64 size, bytes} records)
// Points are stored as Montgomery-form LE coordinates, (0, 0) = identity --
// the in-memory layout of the reference's AffinePoint, so they are copied
// bit for bit.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../ec/point.h"

namespace tachyon_amd::circom {

enum class CurveId : uint32_t { kBn254 = 0, kBls12_381 = 1 };

// Little-endian cursor over a byte range; every read is bounds-checked.
class ByteReader {
 public:
  ByteReader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  template <class T>
  T read() {
    T v;
    take(&v, sizeof(T));
    return v;
  }
  void take(void* dst, size_t bytes) {
    need(bytes);
    memcpy(dst, p_ + off_, bytes);
    off_ += bytes;
  }
  const uint8_t* ptr(size_t bytes) {
    need(bytes);
    const uint8_t* r = p_ + off_;
    off_ += bytes;
    return r;
  }
  size_t offset() const { return off_; }
  void seek(size_t off) {
    if (off > n_) throw std::runtime_error("circom: seek past end of file");
    off_ = off;
  }

 private:
  void need(size_t bytes) const {
    if (bytes > n_ - off_) throw std::runtime_error("circom: truncated file");
  }
  const uint8_t* p_;
  size_t n_;
  size_t off_ = 0;
};

// sections.h: u32 count, then {u32 type, u64 size, payload}.  Returns
// type -> (offset, size); a repeated type keeps the first (as MoveTo does).
inline std::map<uint32_t, std::pair<size_t, size_t>> read_sections(ByteReader& rd) {
  std::map<uint32_t, std::pair<size_t, size_t>> out;
  uint32_t count = rd.read<uint32_t>();
  for (uint32_t i = 0; i < count; ++i) {
    uint32_t type = rd.read<uint32_t>();
    uint64_t size = rd.read<uint64_t>();
    size_t off = rd.offset();
    rd.ptr(size);
    out.emplace(type, std::make_pair(off, (size_t)size));
  }
  return out;
}

// Which pairing curve a modulus belongs to (n8 = 32: BN254, 48: BLS12-381);
// the bytes must equal that curve's base/scalar modulus exactly.
template <class Cfg>
inline bool modulus_matches(const uint8_t* bytes, uint32_t n8) {
  return n8 == Cfg::N64 * 8 && memcmp(bytes, Cfg::kP64, n8) == 0;
}

template <class G1, class G2>
struct ZKey {
  using Fr = typename G1::Fr;
  using A1 = Affine<typename G1::F>;
  using A2 = Affine<typename G2::F>;
  struct Coefficient {  // coefficient.h: matrix (0 = A, else B), constraint, signal, value
    uint32_t matrix, constraint, signal;
    Fr value;             // Montgomery form, as the reference holds it after FromMontgomery
  };
  uint32_t num_vars = 0, num_public = 0, domain_size = 0;
  A1 alpha_g1, beta_g1, delta_g1;
  A2 beta_g2, gamma_g2, delta_g2;
  std::vector<A1> ic, a1, b1, c1, h1;
  std::vector<A2> b2;
  std::vector<Coefficient> coefficients;

  size_t num_instance() const { return (size_t)num_public + 1; }
  size_t num_witness() const { return (size_t)num_vars - num_public - 1; }
};

// Peek the curve of a zkey (from the Groth header's base-field modulus).
CurveId zkey_curve(const uint8_t* data, size_t len);

template <class G1, class G2>
ZKey<G1, G2> parse_zkey(const uint8_t* data, size_t len);

// wtns v2 -> Montgomery-form witnesses of field Fr.
template <class Fr>
std::vector<Fr> parse_wtns(const uint8_t* data, size_t len);

}  // namespace tachyon_amd::circom
