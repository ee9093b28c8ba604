// Device helpers around the hot path:
//  * synthetic MSM inputs generated on the GPU (the bench needs 2^26 points in
//    HBM; the scheme mirrors test/random.h:12-28 and big_int.h:107-115, and is
//    bit-identical to the oracle's generator so tests can cross-check it);
//  * elementwise field / point parity kernels (the reference's
//    prime_field_correctness_gpu_test.cc and *_point_correctness_gpu_test.cc).
#include "device_ops.h"

#include "../common/hip_util.h"
#include "../field/curve_constants.h"

namespace tachyon_amd::util {

namespace {

constexpr unsigned kBlock = 256;
constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kBaseSeedXor = 0xBA5E5EEDBA5E5EEDull;

__device__ __forceinline__ uint64_t sm_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t rand_u64(uint64_t seed, uint64_t ctr) { return sm_mix(seed + (ctr + 1) * kGamma); }

// canonical 4-limb scalar below the modulus of Fr (BigInt<4>::Random semantics)
template <class Fr>
__device__ void rand_scalar(uint64_t seed, uint64_t i, uint64_t out[4]) {
  for (int k = 0; k < 4; ++k) out[k] = rand_u64(seed, i * 4 + k);
  const uint64_t* m = Fr::Config::kP64;
  for (;;) {
    bool ge = true;
    for (int k = 3; k >= 0; --k) {
      if (out[k] != m[k]) { ge = out[k] > m[k]; break; }
    }
    if (!ge) break;
    for (int k = 0; k < 3; ++k) out[k] = (out[k] >> 1) | (out[k + 1] << 63);
    out[3] >>= 1;
  }
}

template <class Fr>
__device__ Fr limbs_to_fr(const uint64_t c[4]) {
  Fr x;
  for (int k = 0; k < 4; ++k) {
    x.v[2 * k] = (uint32_t)c[k];
    x.v[2 * k + 1] = (uint32_t)(c[k] >> 32);
  }
  return x;
}

template <class Fr>
__global__ __launch_bounds__(kBlock) void gen_scalars_kernel(uint64_t seed, uint64_t start, uint64_t n, Fr* out) {
  uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint64_t c[4];
  rand_scalar<Fr>(seed, start + i, c);
  out[i] = limbs_to_fr<Fr>(c).to_mont().canonical();
}

template <class F>
__host__ __device__ F load_generator_coord(const uint64_t* src) {
  F r;
  uint32_t* dst = reinterpret_cast<uint32_t*>(&r);
  for (size_t i = 0; i < sizeof(F) / 4; ++i) dst[i] = (uint32_t)(src[i / 2] >> (32 * (i & 1)));
  return r;
}

template <class Curve>
struct Gen;
template <>
struct Gen<Bn254G1> {
  static constexpr const uint64_t* x() { return consts::bn254_g1::kXMont64; }
  static constexpr const uint64_t* y() { return consts::bn254_g1::kYMont64; }
};
template <>
struct Gen<Bn254G2> {
  static constexpr const uint64_t* x() { return consts::bn254_g2::kXMont64; }
  static constexpr const uint64_t* y() { return consts::bn254_g2::kYMont64; }
};
template <>
struct Gen<Bls381G1> {
  static constexpr const uint64_t* x() { return consts::bls12_381_g1::kXMont64; }
  static constexpr const uint64_t* y() { return consts::bls12_381_g1::kYMont64; }
};
template <>
struct Gen<Bls381G2> {
  static constexpr const uint64_t* x() { return consts::bls12_381_g2::kXMont64; }
  static constexpr const uint64_t* y() { return consts::bls12_381_g2::kYMont64; }
};

// One thread per chunk: k_j * G by double-and-add, then a doubling chain,
// each point normalised to affine (per-point inversion; a one-off setup cost).
// The call writes the global points [start, start + n): chunk j of the call is
// global chunk chunk0 + j, and the first one skips the (start - chunk0 * chunk)
// points before `start` with doublings, so any start gives the same sequence.
template <class Curve>
__global__ __launch_bounds__(kBlock) void gen_bases_kernel(uint64_t seed, uint64_t start, uint64_t n, uint64_t chunk,
                                                           uint64_t chunk0, Affine<typename Curve::F>* out) {
  using F = typename Curve::F;
  using Fr = typename Curve::Fr;
  uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t gbeg = (chunk0 + j) * chunk;  // global index of this chunk's first point
  const uint64_t lo = max(gbeg, start), hi = min(gbeg + chunk, start + n);
  if (lo >= hi) return;
  Affine<F> G{load_generator_coord<F>(Gen<Curve>::x()), load_generator_coord<F>(Gen<Curve>::y())};
  uint64_t k[4];
  rand_scalar<Fr>(seed ^ kBaseSeedXor, chunk0 + j, k);
  XYZZ<F> r = XYZZ<F>::zero();
  for (int limb = 3; limb >= 0; --limb)
    for (int bit = 63; bit >= 0; --bit) {
      r = r.dbl();
      if ((k[limb] >> bit) & 1) r = r.madd(G);
    }
  for (uint64_t i = gbeg; i < lo; ++i) r = r.dbl();
  for (uint64_t i = lo; i < hi; ++i) {
    out[i - start] = r.to_affine();
    r = r.dbl();
  }
}

template <class F>
__global__ __launch_bounds__(kBlock) void field_op_kernel(int op, const F* a, const F* b, F* out, size_t count) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= count) return;
  F x = a[i], y = b[i], r;
  switch (op) {
    case 0: r = x + y; break;
    case 1: r = x - y; break;
    case 2: r = x * y; break;
    case 3: r = x.sqr(); break;
    case 4: r = -x; break;
    case 5: r = x.inverse(); break;
    case 6: r = x.to_mont(); break;
    case 7: r = x.from_mont(); break;
    case 8: r = x.dbl(); break;
    case 9:  // x (any value < 2^(32N)) times the plain canonical constant y
      if constexpr (F::N == 8 && F::kLazyCapable) r = x.mul_shoup(y, F::shoup_quotient(y));
      else r = x * y.to_mont();
      break;
    // x y - y x (zero) and x y - x^2 through the fused a b - c d, in the hot
    // kernels' inline view (12-limb fields fuse only there)
    case 10: r = HotFp<F>(x).mul_sub(HotFp<F>(y), HotFp<F>(y), HotFp<F>(x)); break;
    case 11: r = HotFp<F>(x).mul_sub(HotFp<F>(y), HotFp<F>(x), HotFp<F>(x)); break;
    default: r = F::zero();
  }
  out[i] = r.canonical();
}

template <class F>
__global__ __launch_bounds__(kBlock) void ec_op_kernel(int op, const Affine<F>* a, const Affine<F>* b, Affine<F>* out,
                                                       size_t count) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= count) return;
  XYZZ<F> p = XYZZ<F>::from_affine(a[i]);
  XYZZ<F> r;
  switch (op) {
    case 0: r = p + XYZZ<F>::from_affine(b[i]); break;
    case 1: r = p.dbl(); break;
    case 2: r = p.madd(b[i]); break;
    default: r = XYZZ<F>::zero();
  }
  out[i] = r.to_affine();
}

template <class F>
void run_field_op(int op, const void* a, const void* b, void* out, size_t count) {
  if (count == 0) return;
  DeviceBuffer da, db, dout;
  size_t bytes = count * sizeof(F);
  TA_HIP(hipMemcpy(da.ensure(bytes), a, bytes, hipMemcpyHostToDevice));
  TA_HIP(hipMemcpy(db.ensure(bytes), b, bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(field_op_kernel<F>, dim3(ceil_div(count, kBlock)), dim3(kBlock), 0, 0, op, da.as<F>(),
                     db.as<F>(), static_cast<F*>(dout.ensure(bytes)), count);
  TA_HIP(hipGetLastError());
  TA_HIP(hipMemcpy(out, dout.as<F>(), bytes, hipMemcpyDeviceToHost));
}

// RationalField<F>::BatchEvaluate (math/base/rational_field.h:51-76):
// out[i] = num[i] / den[i], with MultiplicativeGroup::DoBatchInverse's rule for
// a zero denominator (groups.h:124-180: its inverse is 0, so out[i] = 0).
// Montgomery's trick per thread over `chunk` consecutive elements: prefix
// products of the non-zero denominators go to `prefix`, one Fermat inverse
// per chunk, then the backward pass.  Results are canonical, so any chunking
// gives the reference's bytes.
template <class F>
__global__ __launch_bounds__(kBlock) void batch_evaluate_kernel(const F* __restrict__ num, const F* __restrict__ den,
                                                                F* __restrict__ out, F* __restrict__ prefix, size_t n,
                                                                uint32_t chunk) {
  const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t s = t * chunk;
  if (s >= n) return;
  const size_t e = s + chunk < n ? s + chunk : n;
  F prod = F::one();
  for (size_t i = s; i < e; ++i) {
    const F d = den[i];
    if (!d.is_zero()) prod = prod * d;
    prefix[i] = prod;
  }
  F inv = prod.inverse();  // product of non-zero values: invertible
  for (size_t i = e; i-- > s;) {
    const F d = den[i];
    if (d.is_zero()) {
      out[i] = F::zero();
      continue;
    }
    const F before = i > s ? prefix[i - 1] : F::one();  // product of the non-zero den[s..i)
    out[i] = (num[i] * (inv * before)).canonical();
    inv = inv * d;
  }
}

template <class F>
void run_ec_op(int op, const void* a, const void* b, void* out, size_t count) {
  if (count == 0) return;
  DeviceBuffer da, db, dout;
  size_t bytes = count * sizeof(Affine<F>);
  TA_HIP(hipMemcpy(da.ensure(bytes), a, bytes, hipMemcpyHostToDevice));
  TA_HIP(hipMemcpy(db.ensure(bytes), b, bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ec_op_kernel<F>, dim3(ceil_div(count, kBlock)), dim3(kBlock), 0, 0, op, da.as<Affine<F>>(),
                     db.as<Affine<F>>(), static_cast<Affine<F>*>(dout.ensure(bytes)), count);
  TA_HIP(hipGetLastError());
  TA_HIP(hipMemcpy(out, dout.as<Affine<F>>(), bytes, hipMemcpyDeviceToHost));
}

}  // namespace

void batch_evaluate_bn254_fr(const void* num, const void* den, void* out, size_t n) {
  if (n == 0) return;
  using F = Bn254Fr;
  constexpr uint32_t kChunk = 32;
  DeviceBuffer dn, dd, dout, dpre;
  const size_t bytes = n * sizeof(F);
  TA_HIP(hipMemcpy(dn.ensure(bytes), num, bytes, hipMemcpyHostToDevice));
  TA_HIP(hipMemcpy(dd.ensure(bytes), den, bytes, hipMemcpyHostToDevice));
  const size_t threads = (n + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(batch_evaluate_kernel<F>, dim3(ceil_div(threads, kBlock)), dim3(kBlock), 0, 0, dn.as<F>(),
                     dd.as<F>(), static_cast<F*>(dout.ensure(bytes)), static_cast<F*>(dpre.ensure(bytes)), n, kChunk);
  TA_HIP(hipGetLastError());
  TA_HIP(hipMemcpy(out, dout.as<F>(), bytes, hipMemcpyDeviceToHost));
}

void gen_scalars(int field, uint64_t seed, size_t start, size_t n, void* d_out, hipStream_t stream) {
  if (n == 0) return;
  if (field == 1)
    hipLaunchKernelGGL(gen_scalars_kernel<Bn254Fr>, dim3(ceil_div(n, kBlock)), dim3(kBlock), 0, stream, seed, start,
                       n, static_cast<Bn254Fr*>(d_out));
  else if (field == 3)
    hipLaunchKernelGGL(gen_scalars_kernel<Bls381Fr>, dim3(ceil_div(n, kBlock)), dim3(kBlock), 0, stream, seed,
                       start, n, static_cast<Bls381Fr*>(d_out));
  else
    throw std::runtime_error("tachyon_mi355x_gen_scalars: unknown scalar field");
  TA_HIP(hipGetLastError());
}

void gen_bases(int curve, uint64_t seed, size_t start, size_t n, size_t chunk, void* d_out, hipStream_t stream) {
  if (n == 0) return;
  if (chunk == 0) throw std::runtime_error("tachyon_mi355x_gen_bases: chunk must be > 0");
  const uint64_t chunk0 = start / chunk;
  const size_t chunks = (start - chunk0 * chunk + n + chunk - 1) / chunk;
  dim3 g(ceil_div(chunks, kBlock)), b(kBlock);
  switch (curve) {
    case 0: hipLaunchKernelGGL(gen_bases_kernel<Bn254G1>, g, b, 0, stream, seed, start, n, chunk, chunk0,
                               static_cast<Affine<Bn254Fq>*>(d_out)); break;
    case 1: hipLaunchKernelGGL(gen_bases_kernel<Bn254G2>, g, b, 0, stream, seed, start, n, chunk, chunk0,
                               static_cast<Affine<Bn254Fq2>*>(d_out)); break;
    case 2: hipLaunchKernelGGL(gen_bases_kernel<Bls381G1>, g, b, 0, stream, seed, start, n, chunk, chunk0,
                               static_cast<Affine<Bls381Fq>*>(d_out)); break;
    case 3: hipLaunchKernelGGL(gen_bases_kernel<Bls381G2>, g, b, 0, stream, seed, start, n, chunk, chunk0,
                               static_cast<Affine<Bls381Fq2>*>(d_out)); break;
    default: throw std::runtime_error("tachyon_mi355x_gen_bases: unknown curve");
  }
  TA_HIP(hipGetLastError());
}

void field_op(int field, int op, const void* a, const void* b, void* out, size_t count) {
  switch (field) {
    case 0: run_field_op<Bn254Fq>(op, a, b, out, count); break;
    case 1: run_field_op<Bn254Fr>(op, a, b, out, count); break;
    case 2: run_field_op<Bls381Fq>(op, a, b, out, count); break;
    case 3: run_field_op<Bls381Fr>(op, a, b, out, count); break;
    default: throw std::runtime_error("tachyon_mi355x_field_op: unknown field");
  }
}

void ec_op(int curve, int op, const void* a, const void* b, void* out, size_t count) {
  switch (curve) {
    case 0: run_ec_op<Bn254Fq>(op, a, b, out, count); break;
    case 1: run_ec_op<Bn254Fq2>(op, a, b, out, count); break;
    case 2: run_ec_op<Bls381Fq>(op, a, b, out, count); break;
    case 3: run_ec_op<Bls381Fq2>(op, a, b, out, count); break;
    default: throw std::runtime_error("tachyon_mi355x_ec_op: unknown curve");
  }
}

}  // namespace tachyon_amd::util
