// Batch-affine bucket additions against the accumulation's XYZZ madd, both in
// registers over the same 29-bit BN254 Fq code (field/f29.h) -- the A/B of
// VERDICT r04 item 3 as an upper bound: no gathers from HBM, no bucket runs,
// no exceptional cases, so a real batch-affine accumulation can only be slower
// than the batch rows here.
//
//   batch_affine_probe [rounds]
//
// Rows (one JSON line each, G additions per lane per round):
//   madd_reg    the accumulation's madd-2008-s with the base in registers
//               (madd_ceiling29_kernel of msm_impl.h, 3 waves per SIMD)
//   madd_tab    the same with both coordinates read from a 64-point LDS table
//               per addition (the batch rows read their points the same way)
//   batch G     Montgomery's trick over G independent affine additions per
//               lane: forward prefix products d_0 d_1 ... (d_i = x2 - x1, the
//               prefixes in VGPRs), ONE inversion of the last prefix per lane,
//               backward: inv_i = inv * prefix_{i-1}, inv *= d_i,
//               lambda = (y2 - y1) inv_i, x3 = lambda^2 - x1 - x2,
//               y3 = lambda (x1 - x3) - y1: 6 products per addition + the
//               inversion / G.  inv = fermat: a^(p-2), 253 squarings + 109
//               products; inv = free: one product in its place (the bound for
//               any inverter, safegcd included).
// Each row reports additions/s over the whole chip, best of 3 launches
// (HIP events), and the ratio to madd_reg measured in the same process.  The
// fermat rows check inv * prefix = 1 in every lane (mismatches counted).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>

#include "../msm/acc29.h"

namespace {

using namespace tachyon_amd::f29;
namespace ac = tachyon_amd::msm::acc29_core;

constexpr int kBlock = 256;
constexpr int kTab = 64;  // points in the LDS table

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// p - 2 of BN254 Fq, little-endian words (bit 253 the top)
__constant__ uint32_t kExp[8] = {0xd87cfd45u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                 0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};

__device__ F29 fermat_inverse(const F29& a) {
  F29 r = a;
#pragma unroll 1
  for (int b = 252; b >= 0; --b) {
    r = sqr(r);
    if ((kExp[b >> 5] >> (b & 31)) & 1) r = mul(r, a);  // uniform branch: one exponent for every lane
  }
  return r;
}

// K - a - b limb-wise (K = 8p with low limbs raised by 2^31: above two N-form limbs)
__device__ __forceinline__ F29 ksub_ab(const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = kK8[i] - a.l[i] - b.l[i];
  return r;
}

__device__ __forceinline__ void sink(F29& s, const F29& v) {
#pragma unroll
  for (int i = 0; i < 9; ++i) s.l[i] ^= v.l[i];
}

// the 64-point table in LDS, coordinates in R' form (< 3p), plane-major
struct Tab {
  uint32_t x[9][kTab], y[9][kTab];
};
__device__ __forceinline__ void load_tab(Tab& t, const uint32_t* __restrict__ src) {
  for (int k = threadIdx.x; k < kTab; k += blockDim.x) {
    uint32_t w[8];
    for (int j = 0; j < 8; ++j) w[j] = src[k * 16 + j];
    const F29 x = from32(w);
    for (int j = 0; j < 8; ++j) w[j] = src[k * 16 + 8 + j];
    const F29 y = from32(w);
    for (int i = 0; i < 9; ++i) {
      t.x[i][k] = x.l[i];
      t.y[i][k] = y.l[i];
    }
  }
  __syncthreads();
}
__device__ __forceinline__ F29 tx(const Tab& t, int k) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = t.x[i][k];
  return r;
}
__device__ __forceinline__ F29 ty(const Tab& t, int k) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = t.y[i][k];
  return r;
}

__global__ __launch_bounds__(kBlock, 3) void madd_reg_kernel(const uint32_t* __restrict__ pts, uint32_t* __restrict__ out,
                                                             int iters) {
  __shared__ Tab tab;
  load_tab(tab, pts);
  const int t = blockIdx.x * kBlock + threadIdx.x;
  const F29 x2 = tx(tab, (t + 5) & (kTab - 1)), y2 = ty(tab, (t + 5) & (kTab - 1));
  ac::Acc acc{tx(tab, t & (kTab - 1)), ty(tab, t & (kTab - 1)), konst(kOne29), konst(kOne29)};
  int special = 0;
  for (int i = 0; i < iters; ++i) acc = ac::madd(acc, x2, y2, &special);
  F29 s = acc.x;
  sink(s, acc.y);
  sink(s, acc.zz);
  sink(s, acc.zzz);
  out[t] = s.l[0] ^ s.l[8] ^ (uint32_t)special;
}

__global__ __launch_bounds__(kBlock, 3) void madd_tab_kernel(const uint32_t* __restrict__ pts, uint32_t* __restrict__ out,
                                                             int iters) {
  __shared__ Tab tab;
  load_tab(tab, pts);
  const int t = blockIdx.x * kBlock + threadIdx.x;
  ac::Acc acc{tx(tab, t & (kTab - 1)), ty(tab, t & (kTab - 1)), konst(kOne29), konst(kOne29)};
  int special = 0;
  for (int i = 0; i < iters; ++i) {
    const int k = (t + 7 * i + 1) & (kTab - 1);
    acc = ac::madd(acc, tx(tab, k), ty(tab, k), &special);
  }
  F29 s = acc.x;
  sink(s, acc.y);
  sink(s, acc.zz);
  sink(s, acc.zzz);
  out[t] = s.l[0] ^ s.l[8] ^ (uint32_t)special;
}

template <int G>
struct BatchWaves {
  static constexpr int value = G <= 4 ? 3 : G <= 8 ? 2 : 1;
};

// kFermat: the inversion by a^(p-2) (and the check inv * prefix = 1), else one product
template <int G, bool kFermat>
__global__ __launch_bounds__(kBlock, BatchWaves<G>::value) void batch_affine_kernel(const uint32_t* __restrict__ pts,
                                                                                     uint32_t* __restrict__ out,
                                                                                     int rounds) {
  __shared__ Tab tab;
  load_tab(tab, pts);
  const int t = blockIdx.x * kBlock + threadIdx.x;
  F29 s{};
  uint32_t bad = 0;
  for (int r = 0; r < rounds; ++r) {
    F29 pre[G];
    // forward: prefix products of d_i = x2 - x1 (the pair i: table points
    // a_i != b_i); every index a compile-time constant so pre[] stays in VGPRs
    auto fwd = [&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const int a = (t + 7 * i + 3 * r) & (kTab - 1), b = (a + 1 + i) & (kTab - 1);
      const F29 d = add_ksub(tx(tab, b), kK4, tx(tab, a));
      if constexpr (i == 0) pre[0] = d;
      else pre[i] = mul(pre[i - 1], d);
    };
    [&]<int... I>(std::integer_sequence<int, I...>) __attribute__((always_inline)) { (fwd(std::integral_constant<int, I>{}), ...); }(
        std::make_integer_sequence<int, G>{});
    F29 inv;
    if constexpr (kFermat) {
      inv = fermat_inverse(pre[G - 1]);
      const F29 one = mul(inv, pre[G - 1]);
      bad |= is_zero_mod_p(normalize(add_ksub(one, kK4, konst(kOne29)))) ? 0u : 1u;  // limbs carried first
    } else {
      inv = mul(pre[G - 1], pre[G - 1]);
    }
    // backward (i = G - 1 .. 0): each addition's inverse, then the affine sum
    auto bwd = [&](auto ic) __attribute__((always_inline)) {
      constexpr int i = G - 1 - decltype(ic)::value;
      const int a = (t + 7 * i + 3 * r) & (kTab - 1), b = (a + 1 + i) & (kTab - 1);
      const F29 x1 = tx(tab, a), x2 = tx(tab, b);
      F29 inv_i = inv;
      if constexpr (i > 0) {
        inv_i = mul(inv, pre[i - 1]);
        inv = mul(inv, add_ksub(x2, kK4, x1));
      }
      const F29 y1 = ty(tab, a);
      const F29 lam = mul(add_ksub(ty(tab, b), kK4, y1), inv_i);
      const F29 x3 = sqr_add(lam, ksub_ab(x1, x2));
      const F29 y3 = mul_add(lam, add_ksub(x1, kK16, x3), ksub(kK4, y1));
      sink(s, x3);
      sink(s, y3);
    };
    [&]<int... I>(std::integer_sequence<int, I...>) __attribute__((always_inline)) { (bwd(std::integral_constant<int, I>{}), ...); }(
        std::make_integer_sequence<int, G>{});
  }
  out[t] = (s.l[0] ^ s.l[8]) & ~1u;
  if (kFermat) out[t] |= bad;
}

// the same with the prefixes in LDS (plane-major per thread: what a real
// accumulation would do -- G prefixes in VGPRs cost 9 G registers on top of
// the products' ~100, the G = 8 register kernel already spills at 2 waves per
// SIMD).  LDS: sizeof(Tab) + G x 36 B per thread; G = 16 fills a CU's 160 KiB
// with one 256-thread block, G = 32 with one 128-thread block.
template <int G, bool kFermat, int kThreads>
__global__ __launch_bounds__(kThreads) void batch_affine_lds_kernel(const uint32_t* __restrict__ pts,
                                                                    uint32_t* __restrict__ out, int rounds) {
  extern __shared__ uint32_t dyn[];
  Tab& tab = *reinterpret_cast<Tab*>(dyn);
  uint32_t* pl = dyn + sizeof(Tab) / 4;
  load_tab(tab, pts);
  const int t = blockIdx.x * kThreads + threadIdx.x;
  auto put = [&](int i, const F29& v) {
#pragma unroll
    for (int l = 0; l < 9; ++l) pl[(i * 9 + l) * kThreads + threadIdx.x] = v.l[l];
  };
  auto get = [&](int i) {
    F29 v;
#pragma unroll
    for (int l = 0; l < 9; ++l) v.l[l] = pl[(i * 9 + l) * kThreads + threadIdx.x];
    return v;
  };
  F29 s{};
  uint32_t bad = 0;
  for (int r = 0; r < rounds; ++r) {
    F29 pre;
#pragma unroll 1
    for (int i = 0; i < G; ++i) {
      const int a = (t + 7 * i + 3 * r) & (kTab - 1), b = (a + 1 + i) & (kTab - 1);
      const F29 d = add_ksub(tx(tab, b), kK4, tx(tab, a));
      pre = i == 0 ? d : mul(pre, d);
      if (i + 1 < G) put(i, pre);
    }
    F29 inv;
    if constexpr (kFermat) {
      inv = fermat_inverse(pre);
      const F29 one = mul(inv, pre);
      bad |= is_zero_mod_p(normalize(add_ksub(one, kK4, konst(kOne29)))) ? 0u : 1u;  // limbs carried first
    } else {
      inv = mul(pre, pre);
    }
#pragma unroll 1
    for (int i = G - 1; i >= 0; --i) {
      const int a = (t + 7 * i + 3 * r) & (kTab - 1), b = (a + 1 + i) & (kTab - 1);
      const F29 x1 = tx(tab, a), x2 = tx(tab, b);
      F29 inv_i = inv;
      if (i > 0) {
        inv_i = mul(inv, get(i - 1));
        inv = mul(inv, add_ksub(x2, kK4, x1));
      }
      const F29 y1 = ty(tab, a);
      const F29 lam = mul(add_ksub(ty(tab, b), kK4, y1), inv_i);
      const F29 x3 = sqr_add(lam, ksub_ab(x1, x2));
      const F29 y3 = mul_add(lam, add_ksub(x1, kK16, x3), ksub(kK4, y1));
      sink(s, x3);
      sink(s, y3);
    }
  }
  out[t] = (s.l[0] ^ s.l[8]) & ~1u;
  if (kFermat) out[t] |= bad;
}

struct Row {
  const char* name;
  int g;  // additions per lane per round (madd: per iteration, 1)
  const char* inv;
  int waves;
};

template <class K>
double time_kernel(K kern, int blocks, const uint32_t* pts, uint32_t* out, int iters, float* best_ms,
                   int threads = kBlock, size_t lds = 0) {
  if (lds > 65536) CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, 0, pts, out, 1);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, 0, pts, out, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  CHECK(hipGetLastError());
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *best_ms = best;
  return best;
}

}  // namespace

int main(int argc, char** argv) {
  const int base_rounds = argc > 1 ? std::max(1, atoi(argv[1])) : 4;
  // the table: 64 (x, y) pairs of field values below p in R form (not curve
  // points: the formulas' cost does not depend on it)
  std::vector<uint32_t> h(kTab * 16);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < h.size(); ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h[i] = (i % 8) == 7 ? (uint32_t)(s >> 32) & 0x0fffffffu : (uint32_t)(s >> 32);
  }
  constexpr int kBlocks = 256 * 12;
  uint32_t *pts = nullptr, *out = nullptr;
  CHECK(hipMalloc(&pts, h.size() * 4));
  CHECK(hipMalloc(&out, (size_t)kBlocks * kBlock * 4));
  CHECK(hipMemcpy(pts, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const double lanes = (double)kBlocks * kBlock;
  std::vector<uint32_t> ho((size_t)kBlocks * kBlock);

  double ref = 0;
  auto report = [&](const char* name, int g, const char* inv, int waves, double adds, float ms, bool check) {
    const double rate = adds / (ms * 1e-3) / 1e9;
    if (ref == 0) ref = rate;
    long bad = -1;
    if (check) {
      CHECK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
      bad = 0;
      for (uint32_t v : ho) bad += v & 1u;
    }
    printf("{\"row\": \"%s\", \"g\": %d, \"inv\": \"%s\", \"waves_per_simd\": %d, \"additions\": %.0f, \"ms\": %.3f, "
           "\"g_additions_per_s\": %.3f, \"vs_madd_reg\": %.3f, \"inverse_check_failures\": %ld}\n",
           name, g, inv, waves, adds, ms, rate, rate / ref, bad);
    fflush(stdout);
  };
  float ms = 0;
  const int madd_iters = 100 * base_rounds;
  time_kernel(&madd_reg_kernel, kBlocks, pts, out, madd_iters, &ms);
  report("madd_reg", 1, "-", 3, lanes * madd_iters, ms, false);
  time_kernel(&madd_tab_kernel, kBlocks, pts, out, madd_iters, &ms);
  report("madd_tab", 1, "-", 3, lanes * madd_iters, ms, false);
  // prefixes in VGPRs (G = 4: 168 VGPRs, 3 waves per SIMD)
  {
    const int rounds = 25 * base_rounds;
    time_kernel(&batch_affine_kernel<4, false>, kBlocks, pts, out, rounds, &ms);
    report("batch_vgpr", 4, "free", 3, lanes * rounds * 4, ms, false);
    const int frounds = std::max(1, rounds / 4);
    time_kernel(&batch_affine_kernel<4, true>, kBlocks, pts, out, frounds, &ms);
    report("batch_vgpr", 4, "fermat", 3, lanes * frounds * 4, ms, true);
  }
  // prefixes in LDS
#define LDS_ROW(G, T, W)                                                                                      \
  {                                                                                                           \
    const int blocks = kBlocks * kBlock / T;                                                                  \
    const size_t lds = sizeof(Tab) + (size_t)G * 36 * T;                                                      \
    const int rounds = std::max(1, 100 * base_rounds / G);                                                    \
    time_kernel(&batch_affine_lds_kernel<G, false, T>, blocks, pts, out, rounds, &ms, T, lds);                \
    report("batch_lds", G, "free", W, lanes * rounds * G, ms, false);                                         \
    const int frounds = std::max(1, rounds / 4);                                                              \
    time_kernel(&batch_affine_lds_kernel<G, true, T>, blocks, pts, out, frounds, &ms, T, lds);                \
    report("batch_lds", G, "fermat", W, lanes * frounds * G, ms, true);                                       \
  }
  LDS_ROW(4, 256, 3)
  LDS_ROW(8, 256, 2)
  LDS_ROW(16, 256, 1)
  LDS_ROW(32, 128, 1)
#undef LDS_ROW
  CHECK(hipFree(pts));
  CHECK(hipFree(out));
  return 0;
}
