// A/B evidence for VERDICT r02 item 3 (batch-affine bucket accumulation):
// the MEMORY SKELETON of a per-thread batch-affine accumulation of the 2^26
// BN254 G1 MSM, with no field arithmetic -- if its loads and stores alone take
// longer than the whole XYZZ accumulation kernel (seg_acc_kernel, 66.5 ms at
// 2^26 in BENCH_r03), the batch-affine variant cannot win on this chip.
//
// The variant it models (the only form whose inversion cost is small enough,
// DESIGN.md section 4): every thread owns K consecutive sorted entries and
// sums them as a pairwise tree of AFFINE additions, one Montgomery batch
// inversion per tree level over all of the level's pairs in the thread
// (K/2 + K/4 + ... pairs, log2 K inversions of ~258 products each: ~0.8
// products per addition at K = 4096 + 5 products + 1 square per addition =
// ~6.6 product equivalents vs XYZZ's 9.06).  Its per-lane batch (prefix
// products and the level's points) cannot live in registers or LDS
// (K/2 x 96 B per lane), so it streams through HBM, laid out [i][thread] so a
// wave's accesses coalesce:
//   forward  : gather both points of pair i (level 0: 2 x 64 B bases at random
//              indices; later levels: the previous level's outputs), write the
//              32 B prefix product;
//   backward : read the prefix back, re-gather both points (x1, y1, x2, y2 are
//              all needed for lambda, x3, y3), write the 64 B sum.
// Per addition: 128 + 32 + 32 + 128 + 64 = 384 B (level 0's gathers random).
// The skeleton performs exactly those accesses (XOR-folding the loaded words
// so nothing is dead) for W * n entries, and times them with HIP events.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                    \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

struct P64 { uint4 a, b, c, d; };  // one affine BN254 G1 point (64 B)
struct W32 { uint4 a, b; };        // one field element (32 B)

__device__ __forceinline__ uint32_t fold(const P64& p) {
  return p.a.x ^ p.b.y ^ p.c.z ^ p.d.w ^ p.a.w ^ p.d.x;
}

// level 0: pairs of gathered bases -> level-1 points (out), prefixes in pre
__global__ __launch_bounds__(256) void level0(const P64* __restrict__ bases, const uint64_t* __restrict__ ents,
                                              uint64_t T, uint32_t K, W32* __restrict__ pre, P64* __restrict__ out,
                                              uint32_t* __restrict__ sink) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  const uint32_t pairs = K / 2;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < pairs; ++i) {  // forward
    const uint64_t e0 = ents[t * K + 2 * i], e1 = ents[t * K + 2 * i + 1];
    const P64 p = bases[(uint32_t)e0 & 0x3FFFFFF], q = bases[(uint32_t)e1 & 0x3FFFFFF];
    acc ^= fold(p) + fold(q);
    pre[(uint64_t)i * T + t] = W32{make_uint4(acc, 0, 0, 0), make_uint4(0, 0, 0, acc)};
  }
  for (uint32_t i = pairs; i-- > 0;) {  // backward
    const W32 w = pre[(uint64_t)i * T + t];
    const uint64_t e0 = ents[t * K + 2 * i], e1 = ents[t * K + 2 * i + 1];
    const P64 p = bases[(uint32_t)e0 & 0x3FFFFFF], q = bases[(uint32_t)e1 & 0x3FFFFFF];
    acc ^= w.a.x + fold(p) + fold(q);
    out[(uint64_t)i * T + t] = P64{make_uint4(acc, 1, 2, 3), p.b, q.c, make_uint4(acc, 4, 5, 6)};
  }
  sink[t] = acc;
}

// level >= 1: pairs of the previous level's points (coalesced [i][thread])
__global__ __launch_bounds__(256) void level_up(const P64* __restrict__ in, uint64_t T, uint32_t pairs,
                                                W32* __restrict__ pre, P64* __restrict__ out,
                                                uint32_t* __restrict__ sink) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  uint32_t acc = sink[t];
  for (uint32_t i = 0; i < pairs; ++i) {
    const P64 p = in[(uint64_t)(2 * i) * T + t], q = in[(uint64_t)(2 * i + 1) * T + t];
    acc ^= fold(p) + fold(q);
    pre[(uint64_t)i * T + t] = W32{make_uint4(acc, 0, 0, 0), make_uint4(0, 0, 0, acc)};
  }
  for (uint32_t i = pairs; i-- > 0;) {
    const W32 w = pre[(uint64_t)i * T + t];
    const P64 p = in[(uint64_t)(2 * i) * T + t], q = in[(uint64_t)(2 * i + 1) * T + t];
    acc ^= w.a.x + fold(p) + fold(q);
    out[(uint64_t)i * T + t] = P64{make_uint4(acc, 1, 2, 3), p.b, q.c, make_uint4(acc, 4, 5, 6)};
  }
  sink[t] = acc;
}

__global__ void fill_entries(uint64_t* ents, uint64_t m, uint32_t n, uint64_t seed) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;  // splitmix64: random base index per entry
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  ents[i] = (z % n) | ((i / (m / 13)) << 40);
}

int main(int argc, char** argv) {
  const uint32_t logn = argc > 1 ? atoi(argv[1]) : 26;
  const uint32_t n = 1u << logn, W = 13;
  const uint64_t m = (uint64_t)W * n;
  P64* bases;
  uint64_t* ents;
  CHECK(hipMalloc(&bases, (size_t)n * sizeof(P64)));
  CHECK(hipMalloc(&ents, m * 8));
  CHECK(hipMemset(bases, 0x5a, (size_t)n * sizeof(P64)));
  hipLaunchKernelGGL(fill_entries, dim3((m + 255) / 256), dim3(256), 0, 0, ents, m, n, 0x7AC40001ull);
  CHECK(hipDeviceSynchronize());
  printf("{\"log_n\": %u, \"entries\": %llu, \"note\": \"memory skeleton of a per-thread batch-affine "
         "accumulation (384 B per addition), no field arithmetic\"}\n",
         logn, (unsigned long long)m);
  for (uint32_t K : {1024u, 4096u}) {
    const uint64_t T = m / K;
    W32* pre;
    P64 *buf_a, *buf_b;
    uint32_t* sink;
    CHECK(hipMalloc(&pre, (size_t)(K / 2) * T * sizeof(W32)));
    CHECK(hipMalloc(&buf_a, (size_t)(K / 2) * T * sizeof(P64)));
    CHECK(hipMalloc(&buf_b, (size_t)(K / 4) * T * sizeof(P64)));
    CHECK(hipMalloc(&sink, T * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipEventRecord(e0));
      const unsigned grid = (unsigned)((T + 255) / 256);
      hipLaunchKernelGGL(level0, dim3(grid), dim3(256), 0, 0, bases, ents, T, K, pre, buf_a, sink);
      P64* cur = buf_a;
      P64* nxt = buf_b;
      for (uint32_t pairs = K / 4; pairs >= 1; pairs /= 2) {
        hipLaunchKernelGGL(level_up, dim3(grid), dim3(256), 0, 0, cur, T, pairs, pre, nxt, sink);
        std::swap(cur, nxt);
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double additions = (double)T * (K - 1);
    printf("{\"K\": %u, \"threads\": %llu, \"additions\": %.0f, \"bytes\": %.3e, \"ms\": %.2f, \"GBps\": %.0f, "
           "\"scratch_GB\": %.1f}\n",
           K, (unsigned long long)T, additions, additions * 384.0, best, additions * 384.0 / (best * 1e6),
           ((double)(K / 2) * T * (sizeof(W32) + sizeof(P64)) + (double)(K / 4) * T * sizeof(P64)) / 1e9);
    CHECK(hipFree(pre));
    CHECK(hipFree(buf_a));
    CHECK(hipFree(buf_b));
    CHECK(hipFree(sink));
  }
  return 0;
}
