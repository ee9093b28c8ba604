// Microbenchmark: the cost of collecting v_mad_u64_u32 carry-outs on gfx950.
// The 8-limb FIPS product (mont_asm.h) issues one v_mad_u64_u32 + one
// v_addc_co_u32 (VOP3, carry-in from a rotating SGPR pair) per limb product;
// its measured rate (139 G products/s) is ~30 % below what 2-cycle carry adds
// would give.  This times, per thread and loop iteration, 16 products in the
// FIPS pattern with the carry collected by
//   A: v_addc_co_u32 (VOP3) from rotating SGPR pairs s[0:1], s[2:3], s[4:5]
//   B: v_addc_co_u32_e32 (VOP2) from VCC, the mad writing VCC
//   C: no carry collect (mads only), the floor
// and prints lane-ops/s of each, so that the cycles per carry add follow.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

// 16 mads into one 64-bit column accumulator, carries collected per variant
__global__ __launch_bounds__(256) void kA(const uint32_t* in, uint64_t* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t a = in[t & 1023], b = in[(t + 1) & 1023];
  uint64_t acc = a;
  uint32_t c2 = 0;
  for (int i = 0; i < iters; ++i) {
    asm volatile(
        "v_mad_u64_u32 %[acc], s[0:1], %[a], %[b], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[2:3], %[b], %[a], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[4:5], %[a], %[a], %[acc]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[0:1]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[b], %[b], %[acc]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[2:3]\n"
        "v_mad_u64_u32 %[acc], s[2:3], %[a], %[b], %[acc]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[4:5]\n"
        "v_mad_u64_u32 %[acc], s[4:5], %[b], %[a], %[acc]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[0:1]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[a], %[a], %[acc]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[2:3]\n"
        "v_mad_u64_u32 %[acc], s[2:3], %[b], %[b], %[acc]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[4:5]\n"
        "v_mad_u64_u32 %[acc], s[4:5], %[a], %[b], %[acc]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[0:1]\n"
        "s_nop 1\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[2:3]\n"
        "v_addc_co_u32 %[c2], vcc, 0, %[c2], s[4:5]\n"
        : [acc] "+v"(acc), [c2] "+v"(c2)
        : [a] "v"(a), [b] "v"(b)
        : "s0", "s1", "s2", "s3", "s4", "s5", "vcc");
    a += c2;
  }
  out[t] = acc + c2;
}

__global__ __launch_bounds__(256) void kB(const uint32_t* in, uint64_t* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t a = in[t & 1023], b = in[(t + 1) & 1023];
  uint64_t acc = a;
  uint32_t c2 = 0;
  for (int i = 0; i < iters; ++i) {
    asm volatile(
        "v_mad_u64_u32 %[acc], vcc, %[a], %[b], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[b], %[a], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[a], %[a], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[b], %[b], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[a], %[b], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[b], %[a], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[a], %[a], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[b], %[b], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        "v_mad_u64_u32 %[acc], vcc, %[a], %[b], %[acc]\n"
        "v_addc_co_u32_e32 %[c2], vcc, 0, %[c2], vcc\n"
        : [acc] "+v"(acc), [c2] "+v"(c2)
        : [a] "v"(a), [b] "v"(b)
        : "vcc");
    a += c2;
  }
  out[t] = acc + c2;
}

__global__ __launch_bounds__(256) void kC(const uint32_t* in, uint64_t* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t a = in[t & 1023], b = in[(t + 1) & 1023];
  uint64_t acc = a;
  for (int i = 0; i < iters; ++i) {
    asm volatile(
        "v_mad_u64_u32 %[acc], s[0:1], %[a], %[b], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[b], %[a], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[a], %[a], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[b], %[b], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[a], %[b], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[b], %[a], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[a], %[a], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[b], %[b], %[acc]\n"
        "v_mad_u64_u32 %[acc], s[0:1], %[a], %[b], %[acc]\n"
        : [acc] "+v"(acc)
        : [a] "v"(a), [b] "v"(b)
        : "s0", "s1");
    a += (uint32_t)acc;
  }
  out[t] = acc;
}

template <class K>
int run(const char* name, K kern, const uint32_t* in, uint64_t* out, int blocks, int iters, int mads) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, in, out, 10);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  printf("%-44s %8.3f ms  %7.2f T mad/s\n", name, best, (double)blocks * 256 * iters * mads / (best * 1e9));
  return 0;
}

int main() {
  const int blocks = 256 * 16, iters = 20000;
  uint32_t* in;
  uint64_t* out;
  CHECK(hipMalloc(&in, 1024 * 4));
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 8));
  CHECK(hipMemset(in, 0x5b, 1024 * 4));
  // same results with SGPR (A) and VCC (B) carries: no hazard corrupts B's chain
  static uint64_t ra[256 * 64], rb[256 * 64];
  uint32_t hin[1024];
  for (int i = 0; i < 1024; ++i) hin[i] = 0x9e3779b9u * (i + 1);
  CHECK(hipMemcpy(in, hin, sizeof hin, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(kA, dim3(64), dim3(256), 0, 0, in, out, 1000);
  CHECK(hipMemcpy(ra, out, sizeof ra, hipMemcpyDeviceToHost));
  hipLaunchKernelGGL(kB, dim3(64), dim3(256), 0, 0, in, out, 1000);
  CHECK(hipMemcpy(rb, out, sizeof rb, hipMemcpyDeviceToHost));
  int diff = 0;
  for (int i = 0; i < 256 * 64; ++i) diff += ra[i] != rb[i];
  printf("A vs B result mismatches: %d of %d\n", diff, 256 * 64);
  run("A: 9 mad + 9 addc VOP3 (SGPR carries)", kA, in, out, blocks, iters, 9);
  run("B: 9 mad + 9 addc_e32 (VCC carries)", kB, in, out, blocks, iters, 9);
  run("C: 9 mad, no carries", kC, in, out, blocks, iters, 9);
  return 0;
}
