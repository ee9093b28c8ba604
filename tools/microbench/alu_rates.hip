// Issue-rate probe for the instructions a field multiplication can be built
// from on gfx950: v_mad_u64_u32, v_fma_f64, v_mul_lo/hi_u32, f64 and i8 MFMA.
// Each kernel runs 8 independent dependency chains per lane so latency hides
// behind throughput; prints G instr/s (per lane) for the whole chip.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

constexpr int kIters = 4096;

__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint64_t acc[8];
  uint32_t a = seed + threadIdx.x, b = seed ^ blockIdx.x;
  for (int j = 0; j < 8; ++j) acc[j] = j + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t r;
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(acc[j]) : "vcc");
      acc[j] = r;
    }
  }
  uint64_t s = 0;
  for (int j = 0; j < 8; ++j) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint64_t* out, uint32_t seed) {
  uint32_t acc[8];
  uint32_t b = seed ^ blockIdx.x;
  for (int j = 0; j < 8; ++j) acc[j] = j + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t r;
      asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(acc[j]), "v"(b));
      acc[j] = r;
    }
  }
  uint64_t s = 0;
  for (int j = 0; j < 8; ++j) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(uint64_t* out, uint32_t seed) {
  double acc[8];
  double a = 1.0000001 + seed * 1e-12, b = 0.9999999;
  for (int j = 0; j < 8; ++j) acc[j] = j + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      double r;
      asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(acc[j]), "v"(a), "v"(b));
      acc[j] = r;
    }
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_add32(uint64_t* out, uint32_t seed) {
  uint32_t acc[8];
  uint32_t b = seed ^ blockIdx.x;
  for (int j = 0; j < 8; ++j) acc[j] = j + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t r;
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(acc[j]), "v"(b));
      acc[j] = r;
    }
  }
  uint64_t s = 0;
  for (int j = 0; j < 8; ++j) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k_mfma_f64(uint64_t* out, uint32_t seed) {
  d4 acc[4];
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - seed * 1e-12;
  for (int j = 0; j < 4; ++j) acc[j] = d4{0, 0, 0, (double)j};
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  double s = 0;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

typedef int i4 __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));
__global__ void k_mfma_i8(uint64_t* out, uint32_t seed) {
  i4 acc[4];
  i4v a = {(int)(seed + threadIdx.x), 3, 5, 7};
  i4v b = {11, 13, (int)seed, 17};
  for (int j = 0; j < 4; ++j) acc[j] = i4{0, 0, 0, j};
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[j], 0, 0, 0);
  }
  int s = 0;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

template <class K>
static int run(const char* name, K kern, double ops_per_lane_iter, double lanes_per_op, uint64_t* d) {
  const int blocks = 256 * 8, threads = 256;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, 2u);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  double lanes = (double)blocks * threads;
  double instr = lanes * kIters * ops_per_lane_iter / lanes_per_op;  // wave-lane instructions
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"G_lane_instr_per_s\": %.1f}\n", name, ms, instr / (ms * 1e6));
  return 0;
}

int main() {
  uint64_t* d;
  CK(hipMalloc(&d, 256 * 8 * 256 * sizeof(uint64_t)));
  if (run("v_add_u32", k_add32, 8, 1, d)) return 1;
  if (run("v_mul_lo_u32", k_mullo, 8, 1, d)) return 1;
  if (run("v_mad_u64_u32", k_mad64, 8, 1, d)) return 1;
  if (run("v_fma_f64", k_fma64, 8, 1, d)) return 1;
  // MFMA lines report lane-instructions too (1 MFMA per wave counted as 64 lane-instr);
  // FLOP: f64 16x16x4 = 2*16*16*4 per wave, i8 16x16x64 = 2*16*16*64 per wave
  if (run("mfma_f64_16x16x4", k_mfma_f64, 4, 1, d)) return 1;
  if (run("mfma_i32_16x16x64_i8", k_mfma_i8, 4, 1, d)) return 1;
  CK(hipFree(d));
  return 0;
}
