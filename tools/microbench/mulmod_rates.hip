// Microbenchmark: BN254 Fq Montgomery-multiply throughput on gfx950 for the
// field code the kernels use (tachyon_amd/csrc/field/ff.h), one vs several
// independent chains per thread, at different occupancies.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../tachyon_amd/csrc/field/ff.h"

using namespace tachyon_amd;
using F = Bn254Fq;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int CH, int MINW>
__global__ __launch_bounds__(256, MINW) void k_chain(F* out, const F* in, int iters) {
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

template <int CH, int MINW>
int run(const char* name, F* d_out, F* d_in, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_chain<CH, MINW>), dim3(blocks), dim3(256), 0, 0, d_out, d_in, iters);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_chain<CH, MINW>), dim3(blocks), dim3(256), 0, 0, d_out, d_in, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  double mm = (double)blocks * 256 * iters * CH;
  printf("%-28s %8.3f ms  %7.1f G mulmod/s\n", name, ms, mm / (ms * 1e6));
  return 0;
}

int main() {
  F* d_in;
  F* d_out;
  const int blocks = 256 * 8;
  CHECK(hipMalloc(&d_in, 1024 * sizeof(F)));
  CHECK(hipMalloc(&d_out, (size_t)blocks * 256 * sizeof(F)));
  F h[1024];
  for (int i = 0; i < 1024; ++i)
    for (int j = 0; j < 8; ++j) h[i].v[j] = (j == 7) ? (uint32_t)(i * 77 + 5) & 0x0fffffff : 0x9e3779b9u * (i + j + 1);
  CHECK(hipMemcpy(d_in, h, sizeof h, hipMemcpyHostToDevice));
  const int iters = 2000;
  run<1, 1>("1 chain, minw1", d_out, d_in, blocks, iters);
  run<2, 1>("2 chains, minw1", d_out, d_in, blocks, iters);
  run<4, 1>("4 chains, minw1", d_out, d_in, blocks, iters);
  run<1, 4>("1 chain, minw4", d_out, d_in, blocks, iters);
  run<2, 4>("2 chains, minw4", d_out, d_in, blocks, iters);
  run<1, 8>("1 chain, minw8", d_out, d_in, blocks, iters);
  run<2, 8>("2 chains, minw8", d_out, d_in, blocks, iters);
  return 0;
}
