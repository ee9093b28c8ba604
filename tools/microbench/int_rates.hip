// Microbenchmark: per-instruction throughput of the integer/fp64 ops that a
// 256-bit Montgomery multiply is built from, on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 8;  // independent chains per lane

__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint64_t acc[CH];
  uint32_t a = threadIdx.x * 2654435761u + seed, b = blockIdx.x + 12345u;
  for (int c = 0; c < CH; ++c) acc[c] = c + seed;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = (uint64_t)(a + c) * b + acc[c];
    b ^= (uint32_t)acc[0];
  }
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH];
  uint32_t b = blockIdx.x + 12345u;
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = acc[c] * b + 1u;  // v_mad_u32_u24? no: v_mul_lo_u32 + add
  }
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t acc[CH];
  uint32_t b = blockIdx.x + 0x9e3779b9u;
  for (int c = 0; c < CH; ++c) acc[c] = c + seed + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __umulhi(acc[c], b) ^ acc[c];
  }
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add64(uint64_t* out, uint32_t seed) {
  uint64_t acc[CH];
  uint64_t b = ((uint64_t)blockIdx.x << 32) | (threadIdx.x + seed);
  for (int c = 0; c < CH; ++c) acc[c] = c + seed;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = acc[c] + (b ^ (uint64_t)c);
  }
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(double* out, uint32_t seed) {
  double acc[CH];
  double a = 1.0000001 + threadIdx.x * 1e-9, b = 0.9999999 + seed * 1e-12;
  for (int c = 0; c < CH; ++c) acc[c] = c + seed;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __fma_rn(acc[c], a, b);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename T, typename K>
int run(const char* name, K kern, double ops_per_iter_lane) {
  const int blocks = 256 * 16, threads = 256;
  T* d;
  CHECK(hipMalloc(&d, sizeof(T) * blocks * threads));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, 2u + r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  double ops = 5.0 * blocks * threads * (double)ITERS * CH * ops_per_iter_lane;
  printf("%-8s %8.3f ms  %8.2f Gop/s (lane-ops)\n", name, ms, ops / (ms * 1e6));
  CHECK(hipFree(d));
  return 0;
}

int main() {
  run<uint64_t>("mad64", k_mad64, 1.0);
  run<uint32_t>("mullo", k_mullo, 1.0);
  run<uint32_t>("mulhi", k_mulhi, 1.0);
  run<uint64_t>("add64", k_add64, 1.0);
  run<double>("fma64", k_fma64, 1.0);
  return 0;
}
