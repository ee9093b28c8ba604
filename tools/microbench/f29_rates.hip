#include <hip/hip_runtime.h>
#include <cstdio>
#include "f29_proto.h"
#include "../../tachyon_amd/csrc/field/ff.h"
using namespace tachyon_amd;
using F = Bn254Fq;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int CH, int MINW>
__global__ __launch_bounds__(256, MINW) void k29(F29* out, const F29* in, int iters) {
  int t = blockIdx.x * 256 + threadIdx.x;
  F29 x[CH];
  F29 y = in[(t + 7) & 1023];
  for (int c = 0; c < CH; ++c) x[c] = in[(t + c) & 1023];
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = mul29(x[c], y);
  }
  F29 s = x[0];
  for (int c = 1; c < CH; ++c) s = add29(s, x[c]);
  out[t] = s;
}
template <int CH, int MINW>
__global__ __launch_bounds__(256, MINW) void k29s(F29* out, const F29* in, int iters) {
  int t = blockIdx.x * 256 + threadIdx.x;
  F29 x[CH];
  for (int c = 0; c < CH; ++c) x[c] = in[(t + c) & 1023];
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = sqr29(x[c]);
  }
  F29 s = x[0];
  for (int c = 1; c < CH; ++c) s = add29(s, x[c]);
  out[t] = s;
}
template <int CH, int MINW>
__global__ __launch_bounds__(256, MINW) void kff(F* out, const F* in, int iters) {
  int t = blockIdx.x * 256 + threadIdx.x;
  F x[CH];
  F y = in[(t + 7) & 1023];
  for (int c = 0; c < CH; ++c) x[c] = in[(t + c) & 1023];
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = x[c] * y;
  }
  F s = x[0];
  for (int c = 1; c < CH; ++c) s = s + x[c];
  out[t] = s;
}

template <class K, class T>
int run(const char* name, K kern, T* d_out, T* d_in, int blocks, int iters, int ch) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_out, d_in, iters);
  CHECK(hipDeviceSynchronize());
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_out, d_in, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  double mm = (double)blocks * 256 * iters * ch;
  printf("%-34s %8.3f ms  %7.1f G mulmod/s\n", name, best, mm / (best * 1e6));
  return 0;
}

int main() {
  const int blocks = 256 * 8, iters = 2000;
  F29 *a29, *o29; F *aff, *off;
  CHECK(hipMalloc(&a29, 1024 * sizeof(F29))); CHECK(hipMalloc(&o29, (size_t)blocks * 256 * sizeof(F29)));
  CHECK(hipMalloc(&aff, 1024 * sizeof(F))); CHECK(hipMalloc(&off, (size_t)blocks * 256 * sizeof(F)));
  static F29 h29[1024]; static F hf[1024];
  for (int i = 0; i < 1024; ++i) {
    for (int j = 0; j < 9; ++j) h29[i].l[j] = (0x9e3779b9u * (i + j + 1)) & kM29;
    h29[i].l[8] &= 0x3fffff;
    for (int j = 0; j < 8; ++j) hf[i].v[j] = (j == 7) ? (uint32_t)(i * 77 + 5) & 0x0fffffff : 0x9e3779b9u * (i + j + 1);
  }
  CHECK(hipMemcpy(a29, h29, sizeof h29, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(aff, hf, sizeof hf, hipMemcpyHostToDevice));
  // correctness: one chain on GPU vs host
  {
    hipLaunchKernelGGL((k29<1, 1>), dim3(1), dim3(256), 0, 0, o29, a29, 3);
    static F29 g[256]; CHECK(hipMemcpy(g, o29, sizeof g, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int t = 0; t < 256; ++t) { F29 x = h29[t & 1023], y = h29[(t + 7) & 1023]; for (int i = 0; i < 3; ++i) x = mul29(x, y);
      for (int j = 0; j < 9; ++j) bad += x.l[j] != g[t].l[j]; }
    printf("mul29 gpu==host mismatches: %d\n", bad);
  }
  run("ff 1 chain minw1", kff<1, 1>, off, aff, blocks, iters, 1);
  run("ff 2 chains minw1", kff<2, 1>, off, aff, blocks, iters, 2);
  run("ff 1 chain minw4", kff<1, 4>, off, aff, blocks, iters, 1);
  run("f29 mul 1 chain minw1", k29<1, 1>, o29, a29, blocks, iters, 1);
  run("f29 mul 2 chains minw1", k29<2, 1>, o29, a29, blocks, iters, 2);
  run("f29 mul 4 chains minw1", k29<4, 1>, o29, a29, blocks, iters, 4);
  run("f29 mul 1 chain minw4", k29<1, 4>, o29, a29, blocks, iters, 1);
  run("f29 mul 2 chains minw4", k29<2, 4>, o29, a29, blocks, iters, 2);
  run("f29 mul 1 chain minw8", k29<1, 8>, o29, a29, blocks, iters, 1);
  run("f29 sqr 1 chain minw1", k29s<1, 1>, o29, a29, blocks, iters, 1);
  run("f29 sqr 2 chains minw1", k29s<2, 1>, o29, a29, blocks, iters, 2);
  run("f29 sqr 1 chain minw4", k29s<1, 4>, o29, a29, blocks, iters, 1);
  return 0;
}
