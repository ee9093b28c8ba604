// Microbenchmark: issue cost of the VALU instructions a FIPS Montgomery
// multiply / carry-chain add is made of, on gfx950, at a given occupancy.
//   hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates && ./valu_rates
// Prints, per instruction form, SIMD-cycles per wave-instruction (assuming the
// measured shader clock from s_memtime) and lane-ops/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 32768;

#define R8(X) X X X X X X X X

// each kernel: ITERS x 8 x (instructions per body) wave-instructions
template <int KIND>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t seed, unsigned long long* cyc) {
  uint64_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15;
  uint32_t x = threadIdx.x * 2654435761u, y = seed ^ blockIdx.x, c = 0;
  uint32_t v0 = x, v1 = x + 1, v2 = x + 2, v3 = x + 3, v4 = x + 4, v5 = x + 5, v6 = x + 6, v7 = x + 7;
  uint64_t sc;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (KIND == 0) {  // v_mad_u64_u32, 8 independent accumulators
      asm volatile(
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %1, %[s], %[x], %[y], %1\n\t"
          "v_mad_u64_u32 %2, %[s], %[x], %[y], %2\n\tv_mad_u64_u32 %3, %[s], %[x], %[y], %3\n\t"
          "v_mad_u64_u32 %4, %[s], %[x], %[y], %4\n\tv_mad_u64_u32 %5, %[s], %[x], %[y], %5\n\t"
          "v_mad_u64_u32 %6, %[s], %[x], %[y], %6\n\tv_mad_u64_u32 %7, %[s], %[x], %[y], %7"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), [s] "=&s"(sc)
          : [x] "v"(x), [y] "v"(y));
    } else if constexpr (KIND == 1) {  // one dependent accumulator (FIPS column)
      asm volatile(
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\t"
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\t"
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\t"
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %0, %[s], %[x], %[y], %0"
          : "+v"(a0), [s] "=&s"(sc) : [x] "v"(x), [y] "v"(y));
    } else if constexpr (KIND == 2) {  // v_addc_co_u32 (vcc chain, e32)
      asm volatile(
          "v_addc_co_u32 %0, vcc, %0, %8, vcc\n\tv_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
          "v_addc_co_u32 %2, vcc, %2, %8, vcc\n\tv_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
          "v_addc_co_u32 %4, vcc, %4, %8, vcc\n\tv_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
          "v_addc_co_u32 %6, vcc, %6, %8, vcc\n\tv_addc_co_u32 %7, vcc, %7, %8, vcc"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(y) : "vcc");
    } else if constexpr (KIND == 3) {  // v_add_u32 (no carry)
      asm volatile(
          "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
          "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(y));
    } else if constexpr (KIND == 4) {  // v_mul_lo_u32
      asm volatile(
          "v_mul_lo_u32 %0, %0, %8\n\tv_mul_lo_u32 %1, %1, %8\n\tv_mul_lo_u32 %2, %2, %8\n\tv_mul_lo_u32 %3, %3, %8\n\t"
          "v_mul_lo_u32 %4, %4, %8\n\tv_mul_lo_u32 %5, %5, %8\n\tv_mul_lo_u32 %6, %6, %8\n\tv_mul_lo_u32 %7, %7, %8"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(y));
    } else if constexpr (KIND == 5) {  // mad + addc pairs, carry via rotated SGPRs (the FIPS body)
      uint64_t s1, s2;
      asm volatile(
          "v_mad_u64_u32 %0, %[s0], %[x], %[y], %0\n\tv_mad_u64_u32 %0, %[s1], %[x], %[y], %0\n\t"
          "v_mad_u64_u32 %0, %[s2], %[x], %[y], %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s0]\n\t"
          "v_mad_u64_u32 %0, %[s0], %[x], %[y], %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s1]\n\t"
          "v_mad_u64_u32 %0, %[s1], %[x], %[y], %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s2]\n\t"
          "v_mad_u64_u32 %0, %[s2], %[x], %[y], %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s0]\n\t"
          "v_mad_u64_u32 %0, %[s0], %[x], %[y], %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s1]\n\t"
          "v_mad_u64_u32 %0, %[s1], %[x], %[y], %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s2]\n\t"
          "v_mad_u64_u32 %0, %[s2], %[x], %[y], %0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s0]\n\t"
          "s_nop 0\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s1]\n\tv_addc_co_u32 %1, vcc, 0, %1, %[s2]"
          : "+v"(a0), "+v"(c), [s0] "=&s"(sc), [s1] "=&s"(s1), [s2] "=&s"(s2) : [x] "v"(x), [y] "v"(y) : "vcc");
    } else if constexpr (KIND == 6) {  // v_mov_b32
      asm volatile(
          "v_mov_b32 %0, %8\n\tv_mov_b32 %1, %8\n\tv_mov_b32 %2, %8\n\tv_mov_b32 %3, %8\n\t"
          "v_mov_b32 %4, %8\n\tv_mov_b32 %5, %8\n\tv_mov_b32 %6, %8\n\tv_mov_b32 %7, %8"
          : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3), "=v"(v4), "=v"(v5), "=v"(v6), "=v"(v7) : "v"(y));
      y += v7;
    } else if constexpr (KIND == 7) {  // 2 independent mad chains interleaved (8 mads)
      asm volatile(
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %1, %[s], %[x], %[y], %1\n\t"
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %1, %[s], %[x], %[y], %1\n\t"
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %1, %[s], %[x], %[y], %1\n\t"
          "v_mad_u64_u32 %0, %[s], %[x], %[y], %0\n\tv_mad_u64_u32 %1, %[s], %[x], %[y], %1"
          : "+v"(a0), "+v"(a1), [s] "=&s"(sc) : [x] "v"(x), [y] "v"(y));
    } else if constexpr (KIND == 8) {  // v_lshrrev_b64
      asm volatile(
          "v_lshrrev_b64 %0, 29, %0\n\tv_lshrrev_b64 %1, 29, %1\n\tv_lshrrev_b64 %2, 29, %2\n\tv_lshrrev_b64 %3, 29, %3\n\t"
          "v_lshrrev_b64 %4, 29, %4\n\tv_lshrrev_b64 %5, 29, %5\n\tv_lshrrev_b64 %6, 29, %6\n\tv_lshrrev_b64 %7, 29, %7"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (KIND == 9) {  // v_lshl_add_u64
      asm volatile(
          "v_lshl_add_u64 %0, %0, 0, %1\n\tv_lshl_add_u64 %1, %1, 0, %2\n\tv_lshl_add_u64 %2, %2, 0, %3\n\tv_lshl_add_u64 %3, %3, 0, %4\n\t"
          "v_lshl_add_u64 %4, %4, 0, %5\n\tv_lshl_add_u64 %5, %5, 0, %6\n\tv_lshl_add_u64 %6, %6, 0, %7\n\tv_lshl_add_u64 %7, %7, 0, %0"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (KIND == 10) {  // v_alignbit_b32
      asm volatile(
          "v_alignbit_b32 %0, %0, %8, 7\n\tv_alignbit_b32 %1, %1, %8, 7\n\tv_alignbit_b32 %2, %2, %8, 7\n\tv_alignbit_b32 %3, %3, %8, 7\n\t"
          "v_alignbit_b32 %4, %4, %8, 7\n\tv_alignbit_b32 %5, %5, %8, 7\n\tv_alignbit_b32 %6, %6, %8, 7\n\tv_alignbit_b32 %7, %7, %8, 7"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(y));
    } else if constexpr (KIND == 11) {  // v_add3_u32
      asm volatile(
          "v_add3_u32 %0, %0, %8, %1\n\tv_add3_u32 %1, %1, %8, %2\n\tv_add3_u32 %2, %2, %8, %3\n\tv_add3_u32 %3, %3, %8, %4\n\t"
          "v_add3_u32 %4, %4, %8, %5\n\tv_add3_u32 %5, %5, %8, %6\n\tv_add3_u32 %6, %6, %8, %7\n\tv_add3_u32 %7, %7, %8, %0"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(y));
    } else if constexpr (KIND == 12) {  // v_and_b32
      asm volatile(
          "v_and_b32 %0, %0, %8\n\tv_and_b32 %1, %1, %8\n\tv_and_b32 %2, %2, %8\n\tv_and_b32 %3, %3, %8\n\t"
          "v_and_b32 %4, %4, %8\n\tv_and_b32 %5, %5, %8\n\tv_and_b32 %6, %6, %8\n\tv_and_b32 %7, %7, %8"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(y));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] =
      (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) ^ v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7 ^ c ^ (uint32_t)sc;
}

template <int KIND>
int run(const char* name, int instrs_per_iter, int waves_per_simd, uint32_t* out, unsigned long long* cyc) {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1u, cyc);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, out, 2u, cyc);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[1];
  CHECK(hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost));
  double wave_instr_per_simd = (double)ITERS * instrs_per_iter * waves_per_simd;
  double lane_ops = (double)blocks * 256 * ITERS * instrs_per_iter;
  // s_memtime counts at the shader clock: cycles per wave-instruction on one SIMD
  printf("%-34s waves/SIMD %2d  %8.3f ms  %7.2f cyc/wave-instr (memtime)  %9.1f G lane-ops/s  clk %.2f GHz\n", name,
         waves_per_simd, ms, (double)h[0] / wave_instr_per_simd, lane_ops / ms / 1e6,
         (double)h[0] / (ms * 1e6));
  return 0;
}

int main() {
  uint32_t* out;
  unsigned long long* cyc;
  CHECK(hipMalloc(&out, 256 * 256 * 32 * 4));
  CHECK(hipMalloc(&cyc, 256 * 32 * 8));
  for (int w : {3, 8}) {
    run<8>("v_lshrrev_b64", 8, w, out, cyc);
    run<9>("v_lshl_add_u64", 8, w, out, cyc);
    run<10>("v_alignbit_b32", 8, w, out, cyc);
    run<11>("v_add3_u32", 8, w, out, cyc);
    run<12>("v_and_b32", 8, w, out, cyc);
    run<0>("v_mad_u64_u32 x8 indep", 8, w, out, cyc);
    run<1>("v_mad_u64_u32 x8 dependent", 8, w, out, cyc);
    run<7>("v_mad_u64_u32 2 chains", 8, w, out, cyc);
    run<5>("mad+addc FIPS body (8+8, 1 nop)", 17, w, out, cyc);
    run<2>("v_addc_co_u32 vcc chain-indep", 8, w, out, cyc);
    run<3>("v_add_u32", 8, w, out, cyc);
    run<4>("v_mul_lo_u32", 8, w, out, cyc);
    run<6>("v_mov_b32", 8, w, out, cyc);
  }
  return 0;
}
