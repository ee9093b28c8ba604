// Variable-base MSM kernels for MI355X (gfx950) and their host driver
// (template definitions; one translation unit per curve instantiates them:
// msm_bn254_g1.hip, msm_bn254_g2.hip, msm_bls12_381_g1.hip, msm_bls12_381_g2.hip).
// See msm.h for the pipeline; reference semantics: pippenger.h:28-170,
// pippenger_base.h:36-77 (the answer is the same group element; the parity
// tests compare affine coordinates bytewise).
#pragma once
#include "msm.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>

namespace tachyon_amd::msm {

namespace detail {
namespace {  // internal linkage: every per-curve TU gets its own copy

constexpr unsigned kBlock = 256;
constexpr uint32_t kSignBit = 0x80000000u;

// ---------------------------------------------------------------------------
// recode: Montgomery scalar -> canonical -> signed base-2^c digits
// (FillDigits, pippenger.h:28-51: digits in [-2^(c-1), 2^(c-1)), carry into
// the top digit; W*c >= bits+1 keeps the top digit in [0, 2^(c-1)]).
// key = |digit| (0 = no contribution), val = point index | sign << 31.
template <class Fr>
__global__ __launch_bounds__(kBlock) void recode_kernel(const Fr* __restrict__ scalars, uint32_t n,
                                                        unsigned c, unsigned W,
                                                        uint32_t* __restrict__ keys,
                                                        uint32_t* __restrict__ vals) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  constexpr int N = Fr::N;
  Fr s = scalars[i].from_mont();
  uint32_t limbs[N];
#pragma unroll
  for (int k = 0; k < N; ++k) limbs[k] = s.v[k];
  const uint32_t mask = (1u << c) - 1;
  const uint32_t half = 1u << (c - 1);
  uint32_t carry = 0;
  for (unsigned w = 0; w < W; ++w) {
    uint32_t coeff = (limbs[0] & mask) + carry;
    // shift the scalar right by c (c < 32), constant-indexed limbs only
#pragma unroll
    for (int k = 0; k < N - 1; ++k) limbs[k] = (limbs[k] >> c) | (limbs[k + 1] << (32 - c));
    limbs[N - 1] >>= c;
    uint32_t key, sign;
    if (w + 1 < W) {
      carry = (coeff + half) >> c;
      int32_t d = (int32_t)coeff - (int32_t)(carry << c);
      sign = d < 0 ? kSignBit : 0u;
      key = (uint32_t)(d < 0 ? -d : d);
    } else {
      key = coeff;  // top digit, carry folded in, non-negative
      sign = 0;
    }
    size_t o = (size_t)w * n + i;
    keys[o] = key;
    vals[o] = i | sign;
  }
}

// bucket [start, end) per (window, |digit|) from the sorted keys
__global__ __launch_bounds__(kBlock) void bounds_kernel(const uint32_t* __restrict__ keys, uint32_t n,
                                                        unsigned W, unsigned B,
                                                        uint32_t* __restrict__ start,
                                                        uint32_t* __restrict__ end) {
  size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t total = (size_t)n * W;
  if (p >= total) return;
  uint32_t w = (uint32_t)(p / n);
  uint32_t q = (uint32_t)(p - (size_t)w * n);
  uint32_t k = keys[p];
  if (k == 0) return;
  size_t b = (size_t)w * B + (k - 1);
  // positions are stored window-relative offsets into the window's slice
  if (q == 0 || keys[p - 1] != k) start[b] = (uint32_t)q;
  if (q == n - 1 || keys[p + 1] != k) end[b] = (uint32_t)q + 1;
}

// number of accumulation chunks per bucket
__global__ __launch_bounds__(kBlock) void chunk_count_kernel(const uint32_t* __restrict__ start,
                                                             const uint32_t* __restrict__ end,
                                                             size_t nb, unsigned K,
                                                             uint32_t* __restrict__ cnt,
                                                             uint32_t* __restrict__ max_len) {
  size_t b = (size_t)blockIdx.x * kBlock + threadIdx.x;
  uint32_t len = 0;
  if (b < nb) {
    len = end[b] - start[b];
    cnt[b] = (len + K - 1) / K;
  } else if (b == nb) {
    cnt[b] = 0;
  }
  // largest bucket -> the host sizes the partial-reduction tree (one 4-byte
  // read-back instead of a worst-case tree for every input)
  __shared__ uint32_t red[kBlock / 64];
  for (int o = 32; o > 0; o >>= 1) len = max(len, (uint32_t)__shfl_xor(len, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = len;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t m = red[0];
    for (unsigned w = 1; w < kBlock / 64; ++w) m = max(m, red[w]);
    if (m) atomicMax(max_len, m);
  }
}

// chunk counts of the next reduction level from the current offsets
__global__ __launch_bounds__(kBlock) void level_count_kernel(const uint32_t* __restrict__ off, size_t nb,
                                                             unsigned K2, uint32_t* __restrict__ cnt) {
  size_t b = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (b > nb) return;
  if (b == nb) { cnt[b] = 0; return; }
  uint32_t len = off[b + 1] - off[b];
  cnt[b] = (len + K2 - 1) / K2;
}

// largest b in [0, nb) with off[b] <= t  (off is non-decreasing, off[nb] = total)
__device__ __forceinline__ uint32_t find_segment(const uint32_t* __restrict__ off, uint32_t nb, uint32_t t) {
  uint32_t lo = 0, hi = nb;  // invariant: off[lo] <= t < off[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

// Bucket accumulation: thread t owns chunk t of bucket b = find_segment(off, t)
// and sums up to K signed affine bases into an XYZZ partial with madd-2008-s.
template <class Curve, int kMinWaves>
__global__ __launch_bounds__(kBlock, kMinWaves) void acc_kernel(const Affine<typename Curve::F>* __restrict__ bases,
                                                     const uint32_t* __restrict__ vals, uint32_t n,
                                                     unsigned B, const uint32_t* __restrict__ start,
                                                     const uint32_t* __restrict__ end,
                                                     const uint32_t* __restrict__ off, uint32_t nb,
                                                     unsigned K, XYZZ<typename Curve::F>* __restrict__ out) {
  using F = typename Curve::F;
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  uint32_t total = off[nb];
  if (t >= total) return;
  uint32_t b = find_segment(off, nb, t);
  uint32_t q = t - off[b];
  uint32_t w = b / B;
  const uint32_t* wv = vals + (size_t)w * n;
  uint32_t e0 = start[b] + q * K;
  uint32_t e1 = min(end[b], e0 + K);
  XYZZ<F> acc = XYZZ<F>::zero();
  // Two-deep software pipeline: the point index for e+2 and the base for e+1
  // are in flight while the madd for e runs, so neither the (L2-served) index
  // load nor the (HBM) 64-byte base gather sits on the critical path.
  uint32_t v = wv[e0];
  uint32_t v1 = (e0 + 1 < e1) ? wv[e0 + 1] : v;
  Affine<F> P = bases[v & ~kSignBit];
  for (uint32_t e = e0; e < e1; ++e) {
    uint32_t v2 = (e + 2 < e1) ? wv[e + 2] : v1;
    Affine<F> Pn = bases[v1 & ~kSignBit];
    if ((v & kSignBit) && !P.is_zero()) P.y = -P.y;
    acc = acc.madd(P);
    v = v1;
    v1 = v2;
    P = Pn;
  }
  out[t] = acc;
}

// One K2-ary reduction level over per-bucket partial lists.
template <class Curve>
__global__ __launch_bounds__(kBlock) void reduce_level_kernel(const XYZZ<typename Curve::F>* __restrict__ in,
                                                              const uint32_t* __restrict__ in_off,
                                                              const uint32_t* __restrict__ out_off,
                                                              uint32_t nb, unsigned K2,
                                                              XYZZ<typename Curve::F>* __restrict__ out) {
  using F = typename Curve::F;
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  uint32_t total = out_off[nb];
  if (t >= total) return;
  uint32_t b = find_segment(out_off, nb, t);
  uint32_t q = t - out_off[b];
  uint32_t e0 = in_off[b] + q * K2;
  uint32_t e1 = min(in_off[b + 1], e0 + K2);
  XYZZ<F> acc = in[e0];
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = acc + in[e];
  out[t] = acc;
}

// m * P for a small non-negative integer m (double-and-add, high bit first)
template <class F>
__device__ XYZZ<F> small_mul(const XYZZ<F>& P, uint32_t m) {
  XYZZ<F> r = XYZZ<F>::zero();
  if (m == 0 || P.is_zero()) return r;
  int top = 31 - __builtin_clz(m);
  r = P;
  for (int bit = top - 1; bit >= 0; --bit) {
    r = r.dbl();
    if ((m >> bit) & 1) r = r + P;
  }
  return r;
}

// Window reduction, stage 1: segment j of window w covers buckets
// [j*L, (j+1)*L) (bucket b holds |digit| = b+1).  Running sums from the top
// give S = sum (b - jL + 1) B_b and R = sum B_b; the segment's share of
// sum_b (b+1) B_b is S + jL * R  (PippengerBase::AccumulateBuckets,
// pippenger_base.h:36-57, split across threads).
template <class Curve>
__global__ __launch_bounds__(kBlock) void window_segment_kernel(const XYZZ<typename Curve::F>* __restrict__ pts,
                                                                const uint32_t* __restrict__ off,
                                                                unsigned W, unsigned B, unsigned L,
                                                                XYZZ<typename Curve::F>* __restrict__ out) {
  using F = typename Curve::F;
  uint32_t S = B / L;
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S) return;
  uint32_t w = t / S, j = t - w * S;
  uint32_t base = w * B + j * L;
  XYZZ<F> R = XYZZ<F>::zero(), acc = XYZZ<F>::zero();
  for (int k = (int)L - 1; k >= 0; --k) {
    uint32_t b = base + k;
    uint32_t o0 = off[b], o1 = off[b + 1];
    if (o1 > o0) R = R + pts[o0];
    acc = acc + R;
  }
  acc = acc + small_mul(R, j * L);
  out[t] = acc;
}

// Window reduction, stage 2: sum K2 consecutive segment sums per window.
template <class Curve>
__global__ __launch_bounds__(kBlock) void reduce_uniform_kernel(const XYZZ<typename Curve::F>* __restrict__ in,
                                                                unsigned W, unsigned S_in, unsigned K2,
                                                                XYZZ<typename Curve::F>* __restrict__ out) {
  using F = typename Curve::F;
  uint32_t S_out = (S_in + K2 - 1) / K2;
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S_out) return;
  uint32_t w = t / S_out, q = t - w * S_out;
  uint32_t e0 = q * K2, e1 = min(S_in, e0 + K2);
  const XYZZ<F>* src = in + (size_t)w * S_in;
  XYZZ<F> acc = src[e0];
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = acc + src[e];
  out[t] = acc;
}

inline unsigned grid_for(size_t threads) { return (unsigned)std::max<size_t>(1, (threads + kBlock - 1) / kBlock); }

}  // namespace
}  // namespace detail
using namespace detail;

template <class Curve>
MsmGpu<Curve>::MsmGpu(hipStream_t stream) : stream_(stream) {
  require_gpu();
  if (!stream_) {
    TA_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    own_stream_ = true;
  }
  for (auto& e : ev_) TA_HIP(hipEventCreate(&e));
  TA_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_max_), 4, hipHostMallocDefault));
}

template <class Curve>
MsmGpu<Curve>::~MsmGpu() {
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
  if (h_max_) (void)hipHostFree(h_max_);
  if (own_stream_) (void)hipStreamDestroy(stream_);
}

template <class Curve>
void MsmGpu<Curve>::enqueue(const Aff* d_bases, const Fr* d_scalars, size_t n, const MsmPlan& plan,
                            Point* d_windows) {
  const unsigned W = plan.windows, B = plan.buckets, c = plan.c;
  const size_t entries = n * W;
  const size_t nb = (size_t)W * B;
  if (n >= (size_t(1) << 31)) throw std::runtime_error("tachyon_mi355x: MSM size must be < 2^31 per device");

  uint32_t* keys = static_cast<uint32_t*>(keys_.ensure(entries * 4));
  uint32_t* vals = static_cast<uint32_t*>(vals_.ensure(entries * 4));
  uint32_t* keys2 = static_cast<uint32_t*>(keys2_.ensure(entries * 4));
  uint32_t* vals2 = static_cast<uint32_t*>(vals2_.ensure(entries * 4));
  uint32_t* start = static_cast<uint32_t*>(start_.ensure(nb * 4));
  uint32_t* end = static_cast<uint32_t*>(end_.ensure(nb * 4));
  uint32_t* cnt = static_cast<uint32_t*>(cnt_.ensure((nb + 1) * 4));
  uint32_t* off_a = static_cast<uint32_t*>(off_a_.ensure((nb + 1) * 4));
  uint32_t* off_b = static_cast<uint32_t*>(off_b_.ensure((nb + 1) * 4));

  if (profile_) TA_HIP(hipEventRecord(ev_[1], stream_));
  hipLaunchKernelGGL(recode_kernel<Fr>, dim3(grid_for(n)), dim3(kBlock), 0, stream_, d_scalars, (uint32_t)n, c,
                     W, keys, vals);
  TA_HIP(hipGetLastError());
  if (profile_) TA_HIP(hipEventRecord(ev_[2], stream_));

  // ---- sort each window's (bucket, point) pairs ----
  size_t sort_bytes = 0;
  TA_HIP(rocprim::radix_sort_pairs(nullptr, sort_bytes, keys, keys2, vals, vals2, (uint32_t)n, 0, c, stream_));
  void* sort_tmp = sort_tmp_.ensure(sort_bytes);
  for (unsigned w = 0; w < W; ++w) {
    size_t o = (size_t)w * n;
    TA_HIP(rocprim::radix_sort_pairs(sort_tmp, sort_bytes, keys + o, keys2 + o, vals + o, vals2 + o, (uint32_t)n,
                                     0, c, stream_));
  }
  if (profile_) TA_HIP(hipEventRecord(ev_[3], stream_));

  // ---- bucket bounds and chunking ----
  TA_HIP(hipMemsetAsync(start, 0, nb * 4, stream_));
  TA_HIP(hipMemsetAsync(end, 0, nb * 4, stream_));
  uint32_t* d_max = static_cast<uint32_t*>(maxlen_.ensure(4));
  TA_HIP(hipMemsetAsync(d_max, 0, 4, stream_));
  hipLaunchKernelGGL(bounds_kernel, dim3(grid_for(entries)), dim3(kBlock), 0, stream_, keys2, (uint32_t)n, W, B,
                     start, end);
  hipLaunchKernelGGL(chunk_count_kernel, dim3(grid_for(nb + 1)), dim3(kBlock), 0, stream_, start, end, nb, plan.K,
                     cnt, d_max);
  TA_HIP(hipMemcpyAsync(h_max_, d_max, 4, hipMemcpyDeviceToHost, stream_));
  size_t scan_bytes = 0;
  TA_HIP(rocprim::exclusive_scan(nullptr, scan_bytes, cnt, off_a, 0u, nb + 1, rocprim::plus<uint32_t>(), stream_));
  void* scan_tmp = scan_tmp_.ensure(scan_bytes);
  TA_HIP(rocprim::exclusive_scan(scan_tmp, scan_bytes, cnt, off_a, 0u, nb + 1, rocprim::plus<uint32_t>(), stream_));

  // ---- accumulation ----
  if (profile_) TA_HIP(hipEventRecord(ev_[6], stream_));
  size_t max_chunks = entries / plan.K + nb + 1;
  // size both ping-pong buffers up front: nothing may be freed while queued
  // kernels still read it
  Point* part_a = static_cast<Point*>(part_a_.ensure(max_chunks * sizeof(Point)));
  Point* part_b = static_cast<Point*>(part_b_.ensure((max_chunks / plan.K2 + nb + 1) * sizeof(Point)));
  auto acc_fn = (variant_ & 1) ? acc_kernel<Curve, 4> : acc_kernel<Curve, 1>;
  hipLaunchKernelGGL(acc_fn, dim3(grid_for(max_chunks)), dim3(kBlock), 0, stream_, d_bases, vals2,
                     (uint32_t)n, B, start, end, off_a, (uint32_t)nb, plan.K, part_a);
  TA_HIP(hipGetLastError());
  if (profile_) TA_HIP(hipEventRecord(ev_[4], stream_));

  // ---- reduce chunk partials per bucket ----
  // levels needed for the largest bucket (the sync overlaps the acc kernel)
  TA_HIP(hipStreamSynchronize(stream_));
  unsigned levels = 0;
  for (size_t chunks = (*h_max_ + plan.K - 1) / plan.K; chunks > 1; chunks = (chunks + plan.K2 - 1) / plan.K2)
    ++levels;
  last_levels_ = levels;
  Point* cur = part_a;
  uint32_t* cur_off = off_a;
  size_t cur_max = max_chunks;
  for (unsigned l = 0; l < levels; ++l) {
    uint32_t* nxt_off = (cur_off == off_a) ? off_b : off_a;
    hipLaunchKernelGGL(level_count_kernel, dim3(grid_for(nb + 1)), dim3(kBlock), 0, stream_, cur_off, nb, plan.K2,
                       cnt);
    TA_HIP(rocprim::exclusive_scan(scan_tmp, scan_bytes, cnt, nxt_off, 0u, nb + 1, rocprim::plus<uint32_t>(),
                                   stream_));
    size_t nxt_max = cur_max / plan.K2 + nb + 1;
    Point* nxt = (cur == part_a) ? part_b : part_a;
    hipLaunchKernelGGL(reduce_level_kernel<Curve>, dim3(grid_for(nxt_max)), dim3(kBlock), 0, stream_, cur, cur_off,
                       nxt_off, (uint32_t)nb, plan.K2, nxt);
    TA_HIP(hipGetLastError());
    cur = nxt;
    cur_off = nxt_off;
    cur_max = nxt_max;
  }

  // ---- window sums ----
  unsigned S = B / plan.seg;
  Point* seg_a = static_cast<Point*>(seg_a_.ensure((size_t)W * S * sizeof(Point)));
  Point* seg_b = static_cast<Point*>(seg_b_.ensure((size_t)W * S * sizeof(Point)));
  hipLaunchKernelGGL(window_segment_kernel<Curve>, dim3(grid_for((size_t)W * S)), dim3(kBlock), 0, stream_, cur,
                     cur_off, W, B, plan.seg, seg_a);
  TA_HIP(hipGetLastError());
  Point* s_cur = seg_a;
  Point* s_nxt = seg_b;
  while (S > 1) {
    unsigned S_out = (S + plan.K2 - 1) / plan.K2;
    Point* dst = (S_out == 1) ? d_windows : s_nxt;
    hipLaunchKernelGGL(reduce_uniform_kernel<Curve>, dim3(grid_for((size_t)W * S_out)), dim3(kBlock), 0, stream_,
                       s_cur, W, S, plan.K2, dst);
    TA_HIP(hipGetLastError());
    std::swap(s_cur, s_nxt);
    S = S_out;
  }
  if (s_cur == seg_a && S == 1 && B / plan.seg == 1) {
    TA_HIP(hipMemcpyAsync(d_windows, seg_a, W * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
  }
  if (profile_) TA_HIP(hipEventRecord(ev_[5], stream_));
}

template <class Curve>
void MsmGpu<Curve>::run_windows(const void* bases, const void* scalars, size_t n, std::vector<Point>* out,
                                MsmPlan* plan_out) {
  MsmPlan plan = MsmPlan::make(n, Fr::Config::kModulusBits, force_c_);
  if (plan_out) *plan_out = plan;
  out->assign(plan.windows, Point::zero());
  if (n == 0) return;
  if (profile_) TA_HIP(hipEventRecord(ev_[0], stream_));
  const Aff* d_bases = static_cast<const Aff*>(bases);
  const Fr* d_scalars = static_cast<const Fr*>(scalars);
  if (!is_device_pointer(bases)) {
    void* p = bases_.ensure(n * sizeof(Aff));
    TA_HIP(hipMemcpyAsync(p, bases, n * sizeof(Aff), hipMemcpyHostToDevice, stream_));
    d_bases = static_cast<const Aff*>(p);
  }
  if (!is_device_pointer(scalars)) {
    void* p = scalars_.ensure(n * sizeof(Fr));
    TA_HIP(hipMemcpyAsync(p, scalars, n * sizeof(Fr), hipMemcpyHostToDevice, stream_));
    d_scalars = static_cast<const Fr*>(p);
  }
  Point* d_windows = static_cast<Point*>(windows_.ensure(plan.windows * sizeof(Point)));
  enqueue(d_bases, d_scalars, n, plan, d_windows);
  TA_HIP(hipMemcpyAsync(out->data(), d_windows, plan.windows * sizeof(Point), hipMemcpyDeviceToHost, stream_));
  TA_HIP(hipStreamSynchronize(stream_));
  if (profile_) {
    TA_HIP(hipEventElapsedTime(&timings_.h2d, ev_[0], ev_[1]));
    TA_HIP(hipEventElapsedTime(&timings_.recode, ev_[1], ev_[2]));
    TA_HIP(hipEventElapsedTime(&timings_.sort, ev_[2], ev_[3]));
    TA_HIP(hipEventElapsedTime(&timings_.prep, ev_[3], ev_[6]));
    TA_HIP(hipEventElapsedTime(&timings_.acc, ev_[6], ev_[4]));
    TA_HIP(hipEventElapsedTime(&timings_.reduce, ev_[4], ev_[5]));
    TA_HIP(hipEventElapsedTime(&timings_.total, ev_[0], ev_[5]));
  }
}

// Horner over windows, high to low, c doublings in between
// (PippengerBase::AccumulateWindowSums, pippenger_base.h:59-77).
template <class Curve>
typename MsmGpu<Curve>::Point MsmGpu<Curve>::combine_windows(const std::vector<Point>& ws, unsigned c) {
  Point total = Point::zero();
  for (size_t w = ws.size(); w-- > 0;) {
    if (w + 1 < ws.size())
      for (unsigned k = 0; k < c; ++k) total = total.dbl();
    total = total + ws[w];
  }
  return total;
}

template <class Curve>
typename MsmGpu<Curve>::Point MsmGpu<Curve>::run(const void* bases, const void* scalars, size_t n) {
  std::vector<Point> ws;
  MsmPlan plan;
  run_windows(bases, scalars, n, &ws, &plan);
  if (n == 0) return Point::zero();
  return combine_windows(ws, plan.c);
}


}  // namespace tachyon_amd::msm
