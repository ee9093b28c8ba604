// Microbenchmark: mixed-addition (madd-2008-s, XYZZ += affine) throughput of
// the two BN254 G1 accumulation field paths, in registers (no gathers, no run
// logic): the 32-bit FIPS field (ff.h, XYZZ<HotFp<Bn254Fq>>::madd_nz as in
// seg_acc_kernel) and the 29-bit carry-free field (f29.h, acc29::madd as in
// seg_acc29_kernel).  The MSM accumulation of 2^26 points does 872 M of these;
// its measured rate (872 M / kernel time) against this ceiling is the
// kernel's non-arithmetic overhead.
//   ./madd_rates            (prints G madd/s per variant and occupancy bound)
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../tachyon_amd/csrc/ec/point.h"
#include "../../tachyon_amd/csrc/field/f29.h"

using namespace tachyon_amd;
using F = HotFp<Bn254Fq>;
using namespace tachyon_amd::f29;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

struct Acc {
  F29 x, y, zz, zzz;
};

__device__ __forceinline__ Acc madd29(const Acc& A, const F29& x2, const F29& y2) {
  const F29 P = mul_add(x2, A.zz, ksub(kK16, A.x));
  const F29 R = mul_add(y2, A.zzz, ksub(kK4, A.y));
  const F29 PP = sqr(P);
  const F29 PPP = mul(P, PP);
  const F29 Q = mul(A.x, PP);
  Acc C;
  C.x = sqr_add(R, ksub2(kK8, PPP, Q));
  const F29 T = add_ksub(Q, kK16, C.x);
  C.y = mul2_add(R, T, ksub(kK4, A.y), PPP);
  C.zz = mul(A.zz, PP);
  C.zzz = mul(A.zzz, PPP);
  return C;
}

// accumulate `iters` additions of a per-thread point chain into one accumulator
template <int MINW>
__global__ __launch_bounds__(256, MINW) void k32(const Affine<Bn254Fq>* pts, XYZZ<Bn254Fq>* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  Affine<F> p{pts[t & 1023].x, pts[t & 1023].y};
  const Affine<F> q{pts[(t + 5) & 1023].x, pts[(t + 5) & 1023].y};
  XYZZ<F> acc{p.x, p.y, F::one(), F::one()};
  bool z = false;
  for (int i = 0; i < iters; ++i) {
    acc = acc.madd_nz(q, &z);
    p.x = p.x + q.y;  // vary the operand a little so nothing is hoisted
    acc.x = acc.x + p.x;
  }
  out[t] = XYZZ<Bn254Fq>{acc.x, acc.y, acc.zz, acc.zzz};
}

template <int MINW>
__global__ __launch_bounds__(256, MINW) void k29(const Affine<Bn254Fq>* pts, XYZZ<Bn254Fq>* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const F29 x2 = shl5_repack(pts[(t + 5) & 1023].x.v), y2 = shl5_repack(pts[(t + 5) & 1023].y.v);
  Acc acc{from32(pts[t & 1023].x.v), from32(pts[t & 1023].y.v), konst(kOne29), konst(kOne29)};
  for (int i = 0; i < iters; ++i) acc = madd29(acc, x2, y2);
  XYZZ<Bn254Fq> r;
  to32(acc.x, r.x.v);
  to32(acc.y, r.y.v);
  to32(acc.zz, r.zz.v);
  to32(acc.zzz, r.zzz.v);
  out[t] = r;
}

template <class K>
int run(const char* name, K kern, const Affine<Bn254Fq>* pts, XYZZ<Bn254Fq>* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, pts, out, 4);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, pts, out, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  printf("%-30s %8.3f ms  %6.2f G madd/s\n", name, best, (double)blocks * 256 * iters / (best * 1e6));
  return 0;
}

int main() {
  const int blocks = 256 * 12, iters = 400;
  Affine<Bn254Fq>* pts;
  XYZZ<Bn254Fq>* out;
  CHECK(hipMalloc(&pts, 1024 * sizeof(Affine<Bn254Fq>)));
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(XYZZ<Bn254Fq>)));
  static Affine<Bn254Fq> h[1024];
  for (int i = 0; i < 1024; ++i)  // arbitrary canonical-looking limbs (field values, not curve points)
    for (int j = 0; j < 8; ++j) {
      h[i].x.v[j] = j == 7 ? (uint32_t)(i * 77 + 5) & 0x0fffffff : 0x9e3779b9u * (i + j + 1);
      h[i].y.v[j] = j == 7 ? (uint32_t)(i * 31 + 9) & 0x0fffffff : 0x85ebca6bu * (i + 2 * j + 3);
    }
  CHECK(hipMemcpy(pts, h, sizeof h, hipMemcpyHostToDevice));
  run("fips32 madd, minw1", k32<1>, pts, out, blocks, iters);
  run("fips32 madd, minw3", k32<3>, pts, out, blocks, iters);
  run("f29 madd, minw1", k29<1>, pts, out, blocks, iters);
  run("f29 madd, minw2", k29<2>, pts, out, blocks, iters);
  run("f29 madd, minw3", k29<3>, pts, out, blocks, iters);
  return 0;
}
