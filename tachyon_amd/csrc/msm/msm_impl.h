// Variable-base MSM kernels for MI355X (gfx950) and their host driver
// (template definitions; one translation unit per curve instantiates them:
// msm_bn254_g1.hip, msm_bn254_g2.hip, msm_bls12_381_g1.hip, msm_bls12_381_g2.hip).
// See msm.h for the pipeline; reference semantics: pippenger.h:28-170,
// pippenger_base.h:36-77 (the answer is the same group element; the parity
// tests compare affine coordinates bytewise).
#pragma once
#include "msm.h"
#include "../field/f29.h"
#include "acc29.h"
#include "acc28.h"
#include "acc_pair.h"
#include "pair28.h"
#include "pair29.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <thread>

namespace tachyon_amd::msm {

namespace detail {
namespace {  // internal linkage: every per-curve TU gets its own copy

constexpr unsigned kBlock = 256;
constexpr uint32_t kSignBit = 0x80000000u;
constexpr uint32_t kNoBucket = 0xFFFFFFFFu;
enum : uint32_t { kHead = 1, kTail = 2, kSingle = 4 };

// ---------------------------------------------------------------------------
// recode: Montgomery scalar -> canonical -> signed base-2^c digits
// (FillDigits, pippenger.h:28-51: digits in [-2^(c-1), 2^(c-1)), carry into
// the top digit; W*c >= bits+1 keeps the top digit in [0, 2^(c-1)]).
// key = window << c | |digit| (digit 0 = no contribution), so one radix sort
// over all windows orders the entries by (window, bucket) and every window
// keeps its slice [w*n, (w+1)*n); val = point index | sign << 31.
// An entry is one 64-bit word, key << 32 | val: the radix passes sort words
// on bits [32, 32 + key bits) (keys-only, one array) and the accumulation
// reads one 8-byte word per entry.
// Signed c-bit digits of one scalar, window by window: emit(w, key, val).
// Windows [w0, w0 + wr) of W are emitted, as local windows 0 .. wr-1 (the
// lower windows still run for their carries).
template <class Fr, class Emit>
// glen > 0 (a batch of MSMs, run_batch / run_groups): scalar i belongs to
// MSM g = i / glen, its windows are g * wr .. g * wr + wr - 1 of the key space
// and its base index is i - g * gstep (gstep = glen: the MSMs share one base
// array; gstep = 0: MSM g has its own bases at [g glen, (g+1) glen)).
// fold_w > 0 (run_folded: F = W / fold_w copies of the bases, copy k =
// 2^(k c fold_w) P): window w goes to key window w mod fold_w (of MSM g's
// block g fold_w in a batch) and to copy w / fold_w, base index
// vi + (w / fold_w) fold_n (fold_n = the length of one copy).
__device__ __forceinline__ void recode_scalar(const Fr& scalar, uint32_t i, unsigned c, unsigned W, unsigned w0,
                                              unsigned wr, Emit emit, uint32_t glen = 0, uint32_t gstep = 0,
                                              uint32_t fold_w = 0, uint32_t fold_n = 0) {
  constexpr int N = Fr::N;
  Fr s = scalar.from_mont();
  uint32_t limbs[N];
#pragma unroll
  for (int k = 0; k < N; ++k) limbs[k] = s.v[k];
  const uint32_t mask = (1u << c) - 1;
  const uint32_t half = 1u << (c - 1);
  uint32_t gw = 0, vi = i;
  if (glen) {
    const uint32_t g = i / glen;
    gw = g * (fold_w ? fold_w : wr);
    vi = i - g * gstep;
  }
  uint32_t carry = 0;
  for (unsigned w = 0; w < w0 + wr; ++w) {
    uint32_t coeff = (limbs[0] & mask) + carry;
    // shift the scalar right by c (c < 32), constant-indexed limbs only: one
    // funnel shift (v_alignbit_b32) per limb
#pragma unroll
    for (int k = 0; k < N - 1; ++k) limbs[k] = __builtin_amdgcn_alignbit(limbs[k + 1], limbs[k], c);
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
    if (fold_w) {
      const uint32_t part = w / fold_w;
      emit(w, ((gw + w - part * fold_w) << c) | key, (vi + part * fold_n) | sign);
    } else if (w >= w0) {
      emit(w - w0, ((gw + w - w0) << c) | key, vi | sign);
    }
  }
}

__device__ __forceinline__ uint64_t make_entry(uint32_t key, uint32_t val) { return (uint64_t)key << 32 | val; }
__device__ __forceinline__ uint32_t entry_key(uint64_t e) { return (uint32_t)(e >> 32); }
__device__ __forceinline__ uint32_t entry_val(uint64_t e) { return (uint32_t)e; }

template <class Fr>
__global__ __launch_bounds__(kBlock) void recode_kernel(const Fr* __restrict__ scalars, uint32_t n,
                                                        unsigned c, unsigned W, unsigned w0, unsigned wr,
                                                        uint64_t* __restrict__ ents, uint32_t glen, uint32_t gstep,
                                                        uint32_t fold_w, uint32_t fold_n) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  recode_scalar(
      scalars[i], i, c, W, w0, wr,
      [&](unsigned w, uint32_t key, uint32_t val) { ents[(size_t)w * n + i] = make_entry(key, val); }, glen, gstep,
      fold_w, fold_n);
}

// Recode fused with the first radix pass (key bits 0..7), in two launches:
// recode_hist_kernel counts, per block of spt x 256 scalars, the entries
// of each low-byte bin (LDS atomics) into the block's row hist[block * 256 +
// bin]; bin_chunk_sums / bin_chunk_scan / bin_offsets_kernel turn the rows
// into every (block, bin)'s global slot (bin-major order: all of bin 0's
// entries first, blocks in order within a bin), written as rows again, and
// recode_scatter_kernel recomputes the digits and
// writes every (key, val) to its bin's slot (the rank inside the block's run
// from LDS atomics).  This pass need not be stable -- the later stable passes
// over bits 8.. keep the bin grouping, and the order inside a bucket does not
// change the bucket's sum -- so it replaces the recode's 8-byte write plus one
// full onesweep pass (read + write + histogram read) with two reads of the
// 32-byte scalars and one write.
constexpr unsigned kRecodeSpt = 2;  // default scalars per thread of the fused recode

// LDS bin ranks with one atomic per wave when every active lane hits the
// same bin -- NonUniform(n, 1) scalars (variable_base_msm_test_set.h:43-53),
// small scalars' empty high windows -- instead of 64 serialised atomics on
// one address (2^26 NonUniform recode 12.8 -> see DESIGN.md); otherwise one
// atomic per lane.  The test is wave-uniform (ballots), so no divergence.
// (recode_hist_kernel makes the same test once per entry for its three bins.)
// A returning add of 1: this lane's slot in bin's run
__device__ __forceinline__ uint32_t lds_rank(uint32_t* cur, uint32_t bin) {
  const uint32_t b0 = __builtin_amdgcn_readfirstlane(bin);
  const uint64_t active = __ballot(1);
  if (__ballot(bin == b0) == active) {
    const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)active) - 1);
    const uint32_t below = (uint32_t)__popcll(active & ((1ull << __lane_id()) - 1));
    uint32_t base = 0;
    if (__lane_id() == leader) base = atomicAdd(&cur[b0], (uint32_t)__popcll(active));
    return __shfl(base, leader, 64) + below;
  }
  return atomicAdd(&cur[bin], 1u);
}

// Places > 0 (key bits 8..15, 16..23): with `places` > 0 the kernel also
// counts those digits per block, into later[((p - 1) * nblocks + block) * 256
// + bin], so the onesweep passes over those places need no histogram pass of
// their own over the W*n entries (digit_count_kernel + digit_scan_kernel turn
// the counts into rocPRIM's global digit offsets).
template <class Fr>
__global__ __launch_bounds__(kBlock) void recode_hist_kernel(const Fr* __restrict__ scalars, uint32_t n, unsigned c,
                                                             unsigned W, unsigned w0, unsigned wr,
                                                             uint32_t nblocks, uint32_t spt, uint32_t places,
                                                             uint32_t* __restrict__ hist,
                                                             uint32_t* __restrict__ later,
                                                             uint4* __restrict__ zero, size_t zero_n, uint32_t glen,
                                                             uint32_t gstep, uint32_t fold_w, uint32_t fold_n) {
  // cnt2: the third place's counts (key bits 16..23) in four copies, one per
  // lane & 3, 264 words apart: those bits are the window (the same in every
  // lane of a step) and the digit's top bits, a handful of values per wave --
  // one copy gave up to 8 lanes per address in a 32-lane atomic group (8-way
  // conflicts); with the copies on distinct banks a group spreads over 4x the
  // addresses.  A wave-uniform value takes one atomic (c <= 16: the bits are
  // the window alone).
  constexpr uint32_t kCopy = 264;
  __shared__ uint32_t cnt[2][256];
  __shared__ uint32_t cnt2[4 * kCopy];
  const uint32_t t = threadIdx.x;
  // the bucket sums start as the identity (all-zero words): cleared here, not by a memset launch
  for (size_t i = (size_t)blockIdx.x * kBlock + t; i < zero_n; i += (size_t)nblocks * kBlock) zero[i] = uint4{0, 0, 0, 0};
  cnt[0][t] = 0;
  cnt[1][t] = 0;
  for (uint32_t j = t; j < 4 * kCopy; j += kBlock) cnt2[j] = 0;
  __syncthreads();
  for (uint32_t k = 0; k < spt; ++k) {
    const uint32_t i = blockIdx.x * spt * kBlock + k * kBlock + t;
    if (i < n)
      recode_scalar(scalars[i], i, c, W, w0, wr, [&](unsigned, uint32_t key, uint32_t) {
        // one wave-uniformity test for the entry's three bins (equal keys
        // have equal bins): NonUniform inputs take one atomic per wave
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
        const uint64_t active = __ballot(1);
        const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)active) - 1);
        if (__ballot(key == k0) == active) {
          if (__lane_id() == leader) {
            const uint32_t m = (uint32_t)__popcll(active);
            atomicAdd(&cnt[0][k0 & 255], m);
            if (places > 0) atomicAdd(&cnt[1][(k0 >> 8) & 255], m);
            if (places > 1) atomicAdd(&cnt2[(k0 >> 16) & 255], m);
          }
        } else {
          atomicAdd(&cnt[0][key & 255], 1u);
          if (places > 0) atomicAdd(&cnt[1][(key >> 8) & 255], 1u);
          if (places > 1) {
            const uint32_t b2 = (key >> 16) & 255, v0 = __builtin_amdgcn_readfirstlane(b2);
            if (__ballot(b2 == v0) == active) {
              if (__lane_id() == leader) atomicAdd(&cnt2[v0], (uint32_t)__popcll(active));
            } else {
              atomicAdd(&cnt2[(__lane_id() & 3) * kCopy + b2], 1u);
            }
          }
        }
      }, glen, gstep, fold_w, fold_n);
  }
  __syncthreads();
  hist[(size_t)blockIdx.x * 256 + t] = cnt[0][t];  // one coalesced 1 KiB row per block
  if (places > 0) later[(size_t)blockIdx.x * 256 + t] = cnt[1][t];
  if (places > 1)
    later[((size_t)nblocks + blockIdx.x) * 256 + t] = cnt2[t] + cnt2[kCopy + t] + cnt2[2 * kCopy + t] + cnt2[3 * kCopy + t];
}

// counts[q * 256 + bin] += the later-place counts of a chunk of recode blocks
// (grid: chunks x places; one coalesced 1 KiB row per block)
__global__ __launch_bounds__(kBlock) void digit_count_kernel(const uint32_t* __restrict__ later, uint32_t nblocks,
                                                             uint32_t per_chunk, uint32_t* __restrict__ counts) {
  const uint32_t q = blockIdx.y, t = threadIdx.x;
  const uint32_t b0 = blockIdx.x * per_chunk, b1 = min(nblocks, b0 + per_chunk);
  const uint32_t* rows = later + (size_t)q * nblocks * 256;
  uint32_t acc = 0;
  for (uint32_t b = b0; b < b1; ++b) acc += rows[(size_t)b * 256 + t];
  if (acc) atomicAdd(&counts[q * 256 + t], acc);
}

// exclusive prefix sums of each place's 256 digit counts (one workgroup per
// place): rocPRIM's global digit offsets, place q at [q * 256, (q + 1) * 256)
__global__ __launch_bounds__(kBlock) void digit_scan_kernel(const uint32_t* __restrict__ counts,
                                                            uint32_t* __restrict__ offsets) {
  const uint32_t q = blockIdx.x, t = threadIdx.x;
  const uint32_t mine = counts[q * 256 + t];
  uint32_t v = mine;  // 4 waves x 64 lanes
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, 64);
    if ((t & 63) >= (uint32_t)d) v += u;
  }
  __shared__ uint32_t wave_tot[kBlock / 64];
  if ((t & 63) == 63) wave_tot[t >> 6] = v;
  __syncthreads();
  uint32_t add = 0;
  for (uint32_t w = 0; w < (t >> 6); ++w) add += wave_tot[w];
  offsets[q * 256 + t] = v - mine + add;
}

// The fused recode's slots from its per-block bin rows (hist[block][bin],
// 256 bins): slot(block, bin) = sum_{bin' < bin} total(bin') + sum_{block' <
// block} hist[block'][bin] -- the exclusive scan of the bin-major flattening,
// computed over coalesced 1 KiB rows (the bin-major array itself would be
// written and read one 4-byte word per 64-byte line by the recode kernels).
// Chunks of per_chunk consecutive blocks: csum[chunk][bin] = the chunk's sum.
__global__ __launch_bounds__(kBlock) void bin_chunk_sums_kernel(const uint32_t* __restrict__ rows, uint32_t nblocks,
                                                                uint32_t per_chunk, uint32_t* __restrict__ csum) {
  const uint32_t t = threadIdx.x, b0 = blockIdx.x * per_chunk, b1 = min(nblocks, b0 + per_chunk);
  uint32_t acc = 0;
  for (uint32_t b = b0; b < b1; ++b) acc += rows[(size_t)b * 256 + t];
  csum[(size_t)blockIdx.x * 256 + t] = acc;
}

// workgroup = one bin: cpre[chunk][bin] = exclusive prefix of csum[.][bin]
// over the chunks, total[bin] = the bin's count (a block scan per 256 chunks)
__global__ __launch_bounds__(kBlock) void bin_chunk_scan_kernel(const uint32_t* __restrict__ csum, uint32_t chunks,
                                                                uint32_t* __restrict__ cpre,
                                                                uint32_t* __restrict__ total) {
  const uint32_t bin = blockIdx.x, t = threadIdx.x;
  __shared__ uint32_t wave_tot[kBlock / 64];
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < chunks; c0 += kBlock) {
    const uint32_t ch = c0 + t;
    const uint32_t mine = ch < chunks ? csum[(size_t)ch * 256 + bin] : 0u;
    uint32_t v = mine;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t u = __shfl_up(v, d, 64);
      if ((t & 63) >= (uint32_t)d) v += u;
    }
    if ((t & 63) == 63) wave_tot[t >> 6] = v;
    __syncthreads();
    uint32_t add = carry, tile = 0;
    for (uint32_t w = 0; w < kBlock / 64; ++w) {
      if (w < (t >> 6)) add += wave_tot[w];
      tile += wave_tot[w];
    }
    if (ch < chunks) cpre[(size_t)ch * 256 + bin] = v - mine + add;
    carry += tile;
    __syncthreads();  // wave_tot is rewritten by the next tile
  }
  if (t == 0) total[bin] = carry;
}

// workgroup = one chunk, thread = one bin: the chunk's rows of slots
__global__ __launch_bounds__(kBlock) void bin_offsets_kernel(const uint32_t* __restrict__ rows, uint32_t nblocks,
                                                             uint32_t per_chunk, const uint32_t* __restrict__ cpre,
                                                             const uint32_t* __restrict__ total,
                                                             uint32_t* __restrict__ off) {
  const uint32_t t = threadIdx.x, b0 = blockIdx.x * per_chunk, b1 = min(nblocks, b0 + per_chunk);
  // exclusive scan of the 256 bin totals: this bin's base
  const uint32_t mine = total[t];
  uint32_t v = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, 64);
    if ((t & 63) >= (uint32_t)d) v += u;
  }
  __shared__ uint32_t wave_tot[kBlock / 64];
  if ((t & 63) == 63) wave_tot[t >> 6] = v;
  __syncthreads();
  uint32_t run = v - mine + cpre[(size_t)blockIdx.x * 256 + t];
  for (uint32_t w = 0; w < (t >> 6); ++w) run += wave_tot[w];
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t c = rows[(size_t)b * 256 + t];
    off[(size_t)b * 256 + t] = run;
    run += c;
  }
}

// kNarrow: keys of <= 24 bits are staged as 7 bytes (val, key >> 8, bin),
// 47 KiB instead of 53 KiB per block at 13 windows -- three workgroups per
// CU instead of two.
template <class Fr, bool kNarrow>
__global__ __launch_bounds__(kBlock) void recode_scatter_kernel(const Fr* __restrict__ scalars, uint32_t n,
                                                                unsigned c, unsigned W, unsigned w0, unsigned wr,
                                                                uint32_t nblocks, uint32_t spt,
                                                                const uint32_t* __restrict__ hist,
                                                                const uint32_t* __restrict__ off,
                                                                uint64_t* __restrict__ ents, uint32_t glen,
                                                                uint32_t gstep, uint32_t fold_w, uint32_t fold_n) {
  // the block's entries are binned in LDS first, then written out bin run by
  // bin run, so consecutive lanes store to consecutive addresses
  extern __shared__ uint64_t lds_u64[];
  uint64_t* lents = lds_u64;                      // spt * kBlock * wr (wide)
  uint32_t* lvals = reinterpret_cast<uint32_t*>(lds_u64);  // narrow: vals, then the 16-bit key tops
  uint16_t* lkeys = reinterpret_cast<uint16_t*>(lvals + (size_t)spt * kBlock * wr);
  uint8_t* lbins = reinterpret_cast<uint8_t*>(lkeys + (size_t)spt * kBlock * wr);
  __shared__ uint32_t base[256], loff[256], cur[256];
  const uint32_t t = threadIdx.x;
  base[t] = off[(size_t)blockIdx.x * 256 + t];
  const uint32_t mine = hist[(size_t)blockIdx.x * 256 + t];
  // exclusive scan of the block's 256 bin counts (4 waves x 64 lanes)
  uint32_t v = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, 64);
    if ((t & 63) >= (uint32_t)d) v += u;
  }
  __shared__ uint32_t wave_tot[kBlock / 64];
  if ((t & 63) == 63) wave_tot[t >> 6] = v;
  __syncthreads();
  uint32_t add = 0;
  for (uint32_t w = 0; w < (t >> 6); ++w) add += wave_tot[w];
  loff[t] = v - mine + add;
  cur[t] = 0;
  __syncthreads();
  for (uint32_t k = 0; k < spt; ++k) {
    const uint32_t i = blockIdx.x * spt * kBlock + k * kBlock + t;
    if (i < n)
      recode_scalar(scalars[i], i, c, W, w0, wr, [&](unsigned, uint32_t key, uint32_t val) {
        const uint32_t bin = key & 255;
        const uint32_t p = loff[bin] + lds_rank(cur, bin);
        if constexpr (kNarrow) {
          lvals[p] = val;
          lkeys[p] = (uint16_t)(key >> 8);
          lbins[p] = (uint8_t)bin;
        } else {
          lents[p] = make_entry(key, val);
        }
      }, glen, gstep, fold_w, fold_n);
  }
  __syncthreads();
  const uint32_t total = loff[255] + cur[255];
  if constexpr (kNarrow) {
    for (uint32_t p = t; p < total; p += kBlock) {
      const uint32_t bin = lbins[p];
      ents[base[bin] + (p - loff[bin])] = make_entry(((uint32_t)lkeys[p] << 8) | bin, lvals[p]);
    }
  } else {
    for (uint32_t p = t; p < total; p += kBlock) {
      const uint64_t e = lents[p];
      const uint32_t bin = entry_key(e) & 255;
      ents[base[bin] + (p - loff[bin])] = e;
    }
  }
}

// ---------------------------------------------------------------------------
// Non-affine bases -> affine (VariableBaseMSM<ProjectivePoint / JacobianPoint /
// PointXYZZ>, variable_base_msm_unittest.cc:30-33): Montgomery's trick per
// thread over `chunk` consecutive points -- the denominators' prefix products
// to `prefix`, one inversion, then the backward pass.  form 1 projective
// {X, Y, Z}: (X/Z, Y/Z); 2 Jacobian {X, Y, Z}: (X/Z^2, Y/Z^3); 3 XYZZ
// {X, Y, ZZ, ZZZ}: (X (ZZ/ZZZ)^2, Y/ZZZ) (point_xyzz.h:199-212, ZZ^3 = ZZZ^2).
// A zero denominator is the identity -> (0, 0).  Canonical outputs.
template <class F>
__global__ __launch_bounds__(kBlock) void points_to_affine_kernel(const F* __restrict__ in, int form,
                                                                  Affine<F>* __restrict__ out,
                                                                  F* __restrict__ prefix, size_t n, uint32_t chunk) {
  const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t s = t * chunk;
  if (s >= n) return;
  const size_t e = s + chunk < n ? s + chunk : n;
  const unsigned stride = form == 3 ? 4 : 3;  // coordinates per input point
  const unsigned den = form == 3 ? 3 : 2;     // the denominator's coordinate
  F prod = F::one();
  for (size_t i = s; i < e; ++i) {
    const F d = in[i * stride + den];
    if (!d.is_zero()) prod = prod * d;
    prefix[i] = prod;
  }
  F inv = prod.inverse();  // product of the non-zero denominators
  for (size_t i = e; i-- > s;) {
    const F* p = in + i * stride;
    const F d = p[den];
    if (d.is_zero()) {
      out[i] = Affine<F>::zero();
      continue;
    }
    const F dinv = i > s ? inv * prefix[i - 1] : inv;
    inv = inv * d;
    Affine<F> a;
    if (form == 1) {
      a = {p[0] * dinv, p[1] * dinv};
    } else if (form == 2) {
      const F d2 = dinv.sqr();
      a = {p[0] * d2, p[1] * (d2 * dinv)};
    } else {
      a = {p[0] * (p[2] * dinv).sqr(), p[1] * dinv};
    }
    out[i] = a.canonical();
  }
}

// Folded bases (MsmGpu::fold_bases): copy k of point i = 2^(k shift) P_i as
// XYZZ (x, y, zz, zzz words) at out[(k n + i) * 4], by k shift doublings of
// one thread; points_to_affine_kernel (form 3) then normalises them.  A
// one-time table build (a proving key's), not a per-MSM pass.
template <class F>
__global__ __launch_bounds__(kBlock) void fold_points_kernel(const Affine<F>* __restrict__ in, size_t n, unsigned fold,
                                                             unsigned shift, F* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  XYZZ<F> p = XYZZ<F>::from_affine(in[i]);
  for (unsigned k = 0; k < fold; ++k) {
    if (k > 0)
      for (unsigned d = 0; d < shift; ++d) p = p.dbl();
    F* o = out + ((size_t)k * n + i) * 4;
    o[0] = p.x;
    o[1] = p.y;
    o[2] = p.zz;
    o[3] = p.zzz;
  }
}

// ---------------------------------------------------------------------------
// Load-balanced bucket accumulation.
//
// The per-window sorted (bucket, point) lists are one array of W*n entries,
// ordered by (window, bucket).  Thread t owns entries [t*K, (t+1)*K) -- every
// lane runs exactly K mixed additions whatever the bucket sizes (a bucket per
// lane left lanes idle for the longest bucket of their wave).  A run of equal
// buckets inside the range is summed with madd-2008-s (XYZZ += +-affine):
//   * a run that starts and ends inside the range is that bucket's whole sum
//     -> stored straight to bucket_sum[b] (the only writer);
//   * the first run, if the bucket started in an earlier thread ("head"), and
//     the last run, if it continues into the next thread ("tail"), go to
//     pieces[2t] / pieces[2t+1] and are joined by the chain kernels below.
// Minimum waves per SIMD of the point-arithmetic kernels.  Left alone, the
// scheduler interleaves the three Karatsuba products of an Fq2 multiply and
// the G2 kernels land at 256+ VGPRs = one wave per SIMD; capping them at two
// waves (a little scratch) made the BN254 G2 2^24 accumulation 89 -> 61 ms
// and BLS12-381 G2 212 -> 174 ms.
template <class Curve>
struct AccWaves {
  static constexpr int value = 1;
};
// BLS12-381 G1: two waves per SIMD for the 28-bit reductions (the window
// segment kernel then spills 348 B per lane, but at one wave it ran 1664 waves
// of dependent products on 1024 SIMDs): 2^24 reduction 5.5 -> 5.0 ms
// (profiles/r06p/ab_bls_g1_reduction_waves.log)
#ifndef TACHYON_BLS_G1_RED_WAVES
#define TACHYON_BLS_G1_RED_WAVES 2
#endif
template <>
struct AccWaves<Bls381G1> {
  static constexpr int value = TACHYON_BLS_G1_RED_WAVES;
};
template <>
struct AccWaves<Bn254G2> {
  static constexpr int value = 2;
};
template <>
struct AccWaves<Bls381G2> {
  static constexpr int value = 2;
};
// The identity accumulator as a flag (see seg_acc_kernel): every curve but
// BN254 G2, whose inline Fq2 products leave no registers for the extra live
// state (2^20 accumulation 5.30 -> 5.59 ms with it; BLS12-381 G2, whose Fq
// products are calls, 23.4 -> 21.3 ms at 2^21).  The 2-wave cap above
// measured best for both G2 kernels against 1 and 3 waves.
template <class Curve>
struct AccFlag {
  static constexpr bool value = true;
};
template <>
struct AccFlag<Bn254G2> {
  static constexpr bool value = false;
};

template <class Curve>
__global__ __launch_bounds__(kBlock, AccWaves<Curve>::value) void seg_acc_kernel(const Affine<typename Curve::F>* __restrict__ bases,
                                                         const uint64_t* __restrict__ ents, uint32_t c,
                                                         uint64_t gbeg, uint64_t gend, uint64_t tbase,
                                                         uint32_t K, uint32_t idx_mask,
                                                         XYZZ<typename Curve::F>* __restrict__ bucket_sum,
                                                         XYZZ<typename Curve::F>* __restrict__ pieces,
                                                         uint32_t* __restrict__ tflags,
                                                         uint32_t* __restrict__ tlast) {
  using F = typename HotOf<typename Curve::F>::type;  // inline products in this kernel (same layout)
  const Affine<F>* __restrict__ hbases = reinterpret_cast<const Affine<F>*>(bases);
  XYZZ<F>* __restrict__ hsum = reinterpret_cast<XYZZ<F>*>(bucket_sum);
  XYZZ<F>* __restrict__ hpieces = reinterpret_cast<XYZZ<F>*>(pieces);
  const uint64_t tl = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t g0 = gbeg + tl * K;
  if (g0 >= gend) return;
  const uint64_t g1 = min(g0 + K, gend);
  const uint64_t t = tbase + tl;  // global thread slot (pieces/flags are in entry order)
  const uint32_t dmask = (1u << c) - 1;
  // bucket id (w * 2^(c-1) + |digit| - 1) of a combined key, or none for digit 0
  auto bucket_of_key = [&](uint32_t key) -> uint32_t {
    uint32_t d = key & dmask;
    return d ? ((key >> c) << (c - 1)) + (d - 1) : kNoBucket;
  };
  // neighbours outside this launch's entry range belong to other windows
  // (possibly not sorted yet): they never share a bucket
  const uint32_t prev_b = g0 > gbeg ? bucket_of_key(entry_key(ents[g0 - 1])) : kNoBucket;
  const uint32_t next_b = (g1 < gend) ? bucket_of_key(entry_key(ents[g1])) : kNoBucket;

  uint32_t flags = 0, runs = 0, cur = kNoBucket;
  XYZZ<F> acc = XYZZ<F>::zero();
  // The identity accumulator is a flag, not a test of zz: a run starts from
  // its first non-identity base (no madd), identity bases (0, 0) -- canonical
  // input, so a plain limb OR -- add nothing, and madd_nz reports the rare
  // cancellation P = -acc.  Signed digits negate y as p - y by limb selects.
  // (AccFlag: all curves but BN254 G2)
  constexpr bool kFlag = AccFlag<Curve>::value;
  bool acc_zero = true;
  // two-deep software pipeline: the entry of g+2 and the base of g+1 are in
  // flight while the madd for g runs (one-word and BLS12-381 Fq fields).  (A 3-deep pipeline and >= 4 waves per
  // SIMD at 128 VGPRs measured the same for BN254 G1 -- 72.4 / 72.2 vs 72.2
  // ms at 2^26 -- the kernel is issue-bound; the array-rotated 3-deep form
  // also cost the BLS12-381 G2 kernel 8 % in scratch traffic.)
  // Fq2 (G2) kernels load each base at its own iteration: the prefetched
  // next point (64 / 96 words) costs them spills at the 2-wave register cap
  // (BLS12-381 G2 2^21 accumulation 25.7 -> 23.6 ms, BN254 G2 2^20 5.55 ->
  // 5.42 without it; the second wave covers the gather latency)
  constexpr bool kPrefetchBase = sizeof(F) <= 48;
  uint64_t e0 = ents[g0];
  uint64_t e1 = (g0 + 1 < g1) ? ents[g0 + 1] : 0;
  Affine<F> P;
  if constexpr (kPrefetchBase) P = hbases[entry_val(e0) & idx_mask];
  for (uint64_t g = g0; g < g1; ++g) {
    const uint64_t e2 = (g + 2 < g1) ? ents[g + 2] : 0;
    Affine<F> Pn;
    if constexpr (kPrefetchBase) Pn = hbases[entry_val(e1) & idx_mask];
    else P = hbases[entry_val(e0) & idx_mask];
    const uint32_t k0 = entry_key(e0), v0 = entry_val(e0);
    const uint32_t b = bucket_of_key(k0);
    if (b != kNoBucket) {
      if (b != cur) {
        if (cur != kNoBucket) {  // close a run that is not the last one
          if constexpr (kFlag)
            if (acc_zero) acc = XYZZ<F>::zero();
          if (runs == 1 && cur == prev_b) { hpieces[2 * t] = acc; flags |= kHead; }
          else hsum[cur] = acc;
        }
        cur = b;
        ++runs;
        if constexpr (kFlag) acc_zero = true;
        else acc = XYZZ<F>::zero();
      }
      if constexpr (kFlag) {
        if (!P.is_zero_canonical()) {
          P.y = P.y.cond_neg_canonical(v0 & kSignBit);
          if (acc_zero) {
            acc = XYZZ<F>{P.x, P.y, F::one(), F::one()};
            acc_zero = false;
          } else {
            acc = acc.madd_nz(P, &acc_zero);
          }
        }
      } else {
        // BN254 G2: the generic identity-aware madd and no flag (AccFlag)
        if ((v0 & kSignBit) && !P.is_zero()) P.y = -P.y;
        acc = acc.madd(P);
      }
    }
    e0 = e1;
    e1 = e2;
    if constexpr (kPrefetchBase) P = Pn;
  }
  if constexpr (kFlag)
    if (acc_zero) acc = XYZZ<F>::zero();
  if (cur != kNoBucket) {  // the last run
    const bool head = runs == 1 && cur == prev_b;
    const bool tail = cur == next_b;
    if (head) { hpieces[2 * t] = acc; flags |= kHead; }
    if (tail) flags |= kTail;
    if (tail && !head) hpieces[2 * t + 1] = acc;
    if (!head && !tail) hsum[cur] = acc;
  }
  if (runs <= 1) flags |= kSingle;
  // absent pieces are the identity so every chain sums a contiguous range
  if (!(flags & kHead)) hpieces[2 * t] = XYZZ<F>::zero();
  const bool through = (flags & kHead) && (flags & kTail) && (flags & kSingle);
  if (!(flags & kTail) || through) hpieces[2 * t + 1] = XYZZ<F>::zero();
  tflags[t] = flags;
  tlast[t] = cur;
}

// ---------------------------------------------------------------------------
// BN254 G1 accumulation over the carry-free 29-bit-limb field (field/f29.h).
// The same load-balanced run logic as seg_acc_kernel; the accumulator lives
// in R' = 2^261 form (Raw stores) -- the point formulas and their value
// bounds are in msm/acc29.h.
namespace acc29 {
using namespace ::tachyon_amd::f29;
using namespace ::tachyon_amd::msm::acc29_core;  // Acc, from_shifted, madd, add, dbl (msm/acc29.h)
__device__ __forceinline__ XYZZ<Bn254Fq> to_xyzz(const Acc& a) {
  XYZZ<Bn254Fq> r;
  to32(a.x, r.x.v);
  to32(a.y, r.y.v);
  to32(a.zz, r.zz.v);
  to32(a.zzz, r.zzz.v);
  return r;
}
// P == acc: through the R-form doubling (rare).  Inline: an out-of-line call
// takes the accumulator's address and the compiler then keeps it in scratch
// for the whole loop (a 288-byte scratch round trip per madd: 2^26 82.7 ms)
__device__ __forceinline__ Acc dbl_slow(const Acc& a) {
  using HF = HotFp<Bn254Fq>;
  XYZZ<Bn254Fq> s = to_xyzz(a);
  XYZZ<HF> h{s.x, s.y, s.zz, s.zzz};
  h = h.dbl();
  return {from32(h.x.v), from32(h.y.v), from32(h.zz.v), from32(h.zzz.v)};
}



// A reduction operand with its identity flag, to and from the R-form arrays
struct Pt {
  Acc a;
  bool zero;
};
__device__ __forceinline__ Pt load_pt(const XYZZ<Bn254Fq>* __restrict__ p, size_t i) {
  const XYZZ<Bn254Fq> q = p[i];
  if (q.is_zero()) return {Acc{}, true};
  return {{from32(q.x.v), from32(q.y.v), from32(q.zz.v), from32(q.zzz.v)}, false};
}
__device__ __forceinline__ void store_pt(XYZZ<Bn254Fq>* __restrict__ p, size_t i, const Pt& v) {
  p[i] = v.zero ? XYZZ<Bn254Fq>::zero() : to_xyzz(v.a);
}
__device__ __forceinline__ Pt add(const Pt& a, const Pt& b) {
  if (a.zero) return b;
  if (b.zero) return a;
  int special = 0;
  const Acc s = add(a.a, b.a, &special);
  if (special == 1) return {Acc{}, true};
  return {special == 2 ? dbl(a.a) : s, false};
}
// A bucket or piece as the 29-bit accumulation leaves it (R' form, 4 x 9
// limbs, 144 B; all-zero limbs = the identity): the accumulation's run-end
// stores skip the four R-form conversions (they run in the loop's divergent
// branch whenever any lane of the wave changes bucket) and the 29-bit
// reductions read it without converting.
struct alignas(16) Raw {
  F29 x, y, zz, zzz;
};
// the identity is zz = 0 alone (load_raw tests zz; x, y, zzz are not read
// then): one 9-limb select instead of four in the run-end stores
__device__ __forceinline__ Raw raw_of(const Acc& a, bool zero) {
  Raw r{a.x, a.y, a.zz, a.zzz};
#pragma unroll
  for (int k = 0; k < 9; ++k) r.zz.l[k] = zero ? 0u : a.zz.l[k];
  return r;
}
__device__ __forceinline__ Pt load_raw(const void* __restrict__ p, size_t i) {
  const Raw r = static_cast<const Raw*>(p)[i];
  uint32_t nz = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) nz |= r.zz.l[k];
  return {{r.x, r.y, r.zz, r.zzz}, nz == 0};
}
__device__ __forceinline__ void store_raw(void* __restrict__ p, size_t i, const Pt& v) {
  static_cast<Raw*>(p)[i] = raw_of(v.a, v.zero);
}

// m P for a small m (double-and-add from the top bit)
__device__ __forceinline__ Pt small_mul(const Pt& P, uint32_t m) {
  if (m == 0 || P.zero) return {Acc{}, true};
  Pt r = P;
  for (int bit = 30 - __builtin_clz(m); bit >= 0; --bit) {
    r.a = dbl(r.a);  // (no point of this prime-order group doubles to the identity)
    if ((m >> bit) & 1) r = add(r, P);
  }
  return r;
}
}  // namespace acc29

// The field policies of seg_acc_limb_body: BN254 G1 over the 9 x 29-bit field
// (Raw 144-byte stores, the rare doubling through the R-form FIPS field) and
// BLS12-381 G1 over the 14 x 28-bit field (R-form stores for the FIPS
// reductions, the doubling in 28-bit limbs).
struct Pol29 {
  using Fq = Bn254Fq;
  using F = f29::F29;
  using Acc = acc29::Acc;
  using Raw = acc29::Raw;
  static __device__ __forceinline__ F shift_repack(const uint32_t* w) { return f29::shl5_repack(w); }
  // the base's y for a digit of sign `neg`: y~ << 5 (< 32p), negated in the
  // 29-bit limbs as 33p - y~ << 5 (kK33's raised limbs: no borrows; the value
  // stays < 33p, which madd's bounds allow) -- 9 subtractions and 9 selects
  // instead of a borrow chain over the canonical 32-bit words
  static __device__ __forceinline__ F repack_y(const Fq& y, uint32_t neg) {
    F r = f29::shl5_repack(y.v);
    const F m = f29::ksub(f29::kK33, r);
#pragma unroll
    for (int i = 0; i < 9; ++i) r.l[i] = neg ? m.l[i] : r.l[i];
    return r;
  }
  static __device__ __forceinline__ Acc from_shifted(const F& x, const F& y) { return acc29::from_shifted(x, y); }
  static __device__ __forceinline__ Acc madd(const Acc& a, const F& x, const F& y, int* sp) {
    return acc29::madd(a, x, y, sp);
  }
  static __device__ __forceinline__ Acc dbl_slow(const Acc& a) { return acc29::dbl_slow(a); }
  static __device__ __forceinline__ Raw raw_of(const Acc& a, bool zero) { return acc29::raw_of(a, zero); }
  static __device__ __forceinline__ XYZZ<Fq> to_xyzz(const Acc& a) { return acc29::to_xyzz(a); }
};
struct Pol28 {
  using Fq = Bls381Fq;
  using F = f28::F28;
  using Acc = acc28_core::Acc;
  // Raw: the accumulator as it is (14 x 28-bit limbs per coordinate, 224 B);
  // the identity is zz = 0 alone, as acc29::Raw
  using Raw = Acc;
  static __device__ __forceinline__ F shift_repack(const uint32_t* w) { return f28::shl8_repack(w); }
  // 257p with the low limbs raised by 2^28 (limbs < 2^29): 257p - y~ << 8 is a
  // borrow-free negation of the shifted canonical y~ (< 256p), < 257p -- inside
  // acc28's base bound of 512p (tests/test_f28_host.py)
  static constexpr uint32_t kK257[14] = {0x1faa55abu, 0x1feffffeu, 0x13ffb9b7u, 0x1feb0054u, 0x1a42caaau,
                                         0x197a7a70u, 0x16980372u, 0x17897d21u, 0x1bc2d077u, 0x1f8843bcu,
                                         0x135df98du, 0x180e566bu, 0x1c23b965u, 0x01a1b12eu};
  static __device__ __forceinline__ F repack_y(const Fq& y, uint32_t neg) {
    F r = f28::shl8_repack(y.v);
    const F m = f28::ksub(kK257, r);
#pragma unroll
    for (int i = 0; i < 14; ++i) r.l[i] = neg ? m.l[i] : r.l[i];
    return r;
  }
  static __device__ __forceinline__ Acc from_shifted(const F& x, const F& y) { return acc28_core::from_shifted(x, y); }
  static __device__ __forceinline__ Acc madd(const Acc& a, const F& x, const F& y, int* sp) {
    return acc28_core::madd(a, x, y, sp);
  }
  static __device__ __forceinline__ Acc dbl_slow(const Acc& a) { return acc28_core::dbl(a); }
  static __device__ __forceinline__ Raw raw_of(const Acc& a, bool zero) {
    Raw r = a;
#pragma unroll
    for (int k = 0; k < 14; ++k) r.zz.l[k] = zero ? 0u : a.zz.l[k];
    return r;
  }
  static __device__ __forceinline__ XYZZ<Fq> to_xyzz(const Acc& a) {
    XYZZ<Fq> r;
    f28::to32(a.x, r.x.v);
    f28::to32(a.y, r.y.v);
    f28::to32(a.zz, r.zz.v);
    f28::to32(a.zzz, r.zzz.v);
    return r;
  }
};

// kPrefetch: 0 = gather each base at its own iteration; 1 = the next base in
// registers (16 VGPRs: 186, two waves per SIMD); 2 = the next base through
// LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR destination, so the
// kernel keeps its 3-wave register budget with the gather one iteration ahead)
typedef __attribute__((address_space(3))) void lds_void_t;
#ifndef TACHYON_GATHER_NT
#define TACHYON_GATHER_NT 0  // 1: nontemporal base gathers (A/B build)
#endif
// kEnt: how a lane reads its K sorted entries.  A lane's entries sit K x 8
// bytes from its neighbours', so a wave's entry load touches 64 lines, and
// the bases' gathers (~3.5 TB/s of lines) evict them from the XCD's L2
// before the lane's next iteration: an 8-byte load per iteration fetched a
// line per entry (123 vs 72 algorithmic HBM bytes per entry, FETCH_SIZE).
//   0: one 8-byte load per iteration, two ahead (rounds 1-6a)
//   1: aligned 16-byte pairs (entries 2m, 2m + 1), the next pair an iteration
//      ahead -- a line per two entries (FETCH 93.7 B per entry; 2^26
//      accumulation 59.6 -> 58.9 ms, profiles/r06h/ab_ent_pairs.log)
//   2: 64-byte chunks (8 entries) through LDS by LDS-DMA, the next chunk
//      8 iterations ahead, double-buffered: 4 KiB per wave, no VGPRs; the
//      lane's first entry must be 16-byte aligned (g0 even: gbeg and K even)
//      and the entry array 64 bytes longer than gend (MsmGpu::enqueue's
//      slack).  FETCH 72.4 B per entry = the 64-byte base + 8; 2^26
//      accumulation 58.8 -> 57.0 ms, BLS12-381 G1 2^24 31.4 -> 30.8 ms
//      (profiles/r06i/ab_entries_staged.log).  The default where g0 is even.
template <class Pol, int kPrefetch, bool kRaw, int kEnt = 0>
__device__ __forceinline__ void seg_acc_limb_body(const Affine<typename Pol::Fq>* __restrict__ bases,
                                                  const uint64_t* __restrict__ ents, uint32_t c, uint64_t gbeg,
                                                  uint64_t gend, uint64_t tbase, uint32_t K, uint32_t idx_mask,
                                                  XYZZ<typename Pol::Fq>* __restrict__ bucket_sum,
                                                  XYZZ<typename Pol::Fq>* __restrict__ pieces,
                                                  uint32_t* __restrict__ tflags, uint32_t* __restrict__ tlast) {
  static_assert(kEnt != 2 || kPrefetch == 0, "LDS-staged entries only with the unprefetched base gather");
  using Fq = typename Pol::Fq;
  using F = typename Pol::F;
  using Acc = typename Pol::Acc;
  const uint64_t tl = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t g0 = gbeg + tl * K;
  if (g0 >= gend) return;
  const uint64_t g1 = min(g0 + K, gend);
  const uint64_t t = tbase + tl;
  const uint32_t dmask = (1u << c) - 1;
  auto bucket_of_key = [&](uint32_t key) -> uint32_t {
    uint32_t d = key & dmask;
    return d ? ((key >> c) << (c - 1)) + (d - 1) : kNoBucket;
  };
  const uint32_t prev_b = g0 > gbeg ? bucket_of_key(entry_key(ents[g0 - 1])) : kNoBucket;
  const uint32_t next_b = (g1 < gend) ? bucket_of_key(entry_key(ents[g1])) : kNoBucket;
  uint32_t flags = 0, runs = 0, cur = kNoBucket;
  Acc acc{};  // (any defined value: the stores mask it while acc_zero)
  bool acc_zero = true;
  // kRaw: the accumulator as it is (Raw); otherwise R form, the identity as
  // zz = zzz = 0 (x, y are not read)
  auto put = [&](XYZZ<Fq>* dst, size_t i) {
    if constexpr (kRaw) {
      reinterpret_cast<typename Pol::Raw*>(dst)[i] = Pol::raw_of(acc, acc_zero);
    } else {
      XYZZ<Fq> s = Pol::to_xyzz(acc);
      const uint32_t keep = acc_zero ? 0u : ~0u;
#pragma unroll
      for (int k = 0; k < Fq::N; ++k) {
        s.zz.v[k] &= keep;
        s.zzz.v[k] &= keep;
      }
      dst[i] = s;
    }
  };
  uint64_t e0 = 0, e1 = 0;
  uint64_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;  // kEnt 1: entries 2m .. 2m + 3, m = g / 2
  auto load_pair = [&](uint64_t i, uint64_t& a, uint64_t& b) {  // entries i, i + 1 (i even), zeros past gend
    if (i + 1 < gend) {
      const uint4 v = *reinterpret_cast<const uint4*>(ents + i);
      a = (uint64_t)v.y << 32 | v.x;
      b = (uint64_t)v.w << 32 | v.z;
    } else {
      a = i < gend ? ents[i] : 0;
      b = 0;
    }
  };
  // kEnt 2: [buffer][wave][16-byte piece][lane]; chunk j of a lane (entries
  // g0 + 8j ..) in buffer j & 1
  __shared__ uint4 estage[kEnt == 2 ? 2 : 1][kEnt == 2 ? kBlock / 64 : 1][4][kEnt == 2 ? 64 : 1];
  const uint32_t ewave = threadIdx.x >> 6, elane = threadIdx.x & 63;
  auto fetch_chunk = [&](uint64_t first, uint32_t buf) {
    const uint4* src = reinterpret_cast<const uint4*>(ents + first);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(src + q, (lds_void_t*)&estage[buf][ewave][q][0], 16, 0, 0);
  };
  if constexpr (kEnt == 1) {
    load_pair(g0 & ~uint64_t(1), q0, q1);
    load_pair((g0 & ~uint64_t(1)) + 2, q2, q3);
    e0 = (g0 & 1) ? q1 : q0;
    e1 = (g0 & 1) ? q2 : q1;
  } else if constexpr (kEnt == 2) {
    fetch_chunk(g0, 0);
  } else {
    e0 = ents[g0];
    e1 = (g0 + 1 < g1) ? ents[g0 + 1] : 0;
  }
  Affine<Fq> P;
  // LDS-DMA staging: [slot][wave][16-byte chunk][lane], 32 KiB per workgroup; a
  // wave-instruction writes its 64 lanes' chunks contiguously (base + 16 lane)
  __shared__ uint4 stage[kPrefetch == 2 ? 2 : 1][kPrefetch == 2 ? kBlock / 64 : 1][4][64];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto issue = [&](uint64_t e, uint32_t slot) {  // the base of entry e into stage[slot]
    const uint4* src = reinterpret_cast<const uint4*>(bases + (entry_val(e) & idx_mask));
#pragma unroll
    for (int ch = 0; ch < 4; ++ch)
      __builtin_amdgcn_global_load_lds(src + ch, (lds_void_t*)&stage[slot][wave][ch][0], 16, 0, TACHYON_GATHER_NT ? 2 : 0);
  };
  if constexpr (kPrefetch == 1) P = bases[entry_val(e0) & idx_mask];
  if constexpr (kPrefetch == 2) issue(e0, 0);
  uint32_t it = 0;  // iteration count: the same for every lane of the wave (K entries each)
  for (uint64_t g = g0; g < g1; ++g, ++it) {
    uint64_t e2 = 0;
    if constexpr (kEnt == 1) {
      // (g & 1 is the same for every lane of the wave when K and gbeg are even)
      if (g & 1) {  // entry g + 2 opens the next pair: shift, and load the one after
        e2 = q3;
        q0 = q2;
        q1 = q3;
        load_pair(g + 3, q2, q3);
      } else {
        e2 = q2;
      }
    } else if constexpr (kEnt == 2) {
      if ((it & 7) == 0) {  // a new chunk: it has landed (this wave's own LDS-DMA); fetch the next one
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (g + 8 < g1) fetch_chunk(g + 8, ((it >> 3) + 1) & 1);
      }
      const uint32_t sl = it & 7;
      const uint2 w = reinterpret_cast<const uint2*>(&estage[(it >> 3) & 1][ewave][sl >> 1][elane])[sl & 1];
      e0 = (uint64_t)w.y << 32 | w.x;
    } else {
      e2 = (g + 2 < g1) ? ents[g + 2] : 0;
    }
    Affine<Fq> Pn;
    if constexpr (kPrefetch == 1) {
      Pn = bases[entry_val(e1) & idx_mask];
    } else if constexpr (kPrefetch == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this iteration's base has landed
      const uint32_t slot = it & 1;
      uint4 ch[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) ch[q] = stage[slot][wave][q][lane];
      memcpy(&P, ch, sizeof(P));
      if (g + 1 < g1) issue(e1, slot ^ 1);  // the next base, under this iteration's madd
    } else if constexpr (TACHYON_GATHER_NT) {  // A/B: the base gather with the nontemporal policy
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4* src = reinterpret_cast<const u32x4*>(bases + (entry_val(e0) & idx_mask));
      constexpr int kChunks = sizeof(Affine<Fq>) / 16;
      u32x4 ch[kChunks];
#pragma unroll
      for (int q = 0; q < kChunks; ++q) ch[q] = __builtin_nontemporal_load(src + q);
      memcpy(&P, ch, sizeof(P));
    } else {
      P = bases[entry_val(e0) & idx_mask];
    }
    const uint32_t k0 = entry_key(e0), v0 = entry_val(e0);
    const uint32_t b = bucket_of_key(k0);
    if (b != kNoBucket) {
      if (b != cur) {
        if (cur != kNoBucket) {
          // one store for both destinations (a head piece or the bucket's
          // sum): a single conversion block when the wave's lanes differ
          const bool head = runs == 1 && cur == prev_b;
          if (head) flags |= kHead;
          put(head ? pieces : bucket_sum, head ? 2 * t : cur);
        }
        cur = b;
        ++runs;
        acc_zero = true;
      }
      if (!P.is_zero_canonical()) {
        const F x2 = Pol::shift_repack(P.x.v), y2 = Pol::repack_y(P.y, v0 & kSignBit);  // both paths
        if (acc_zero) {
          acc = Pol::from_shifted(x2, y2);
          acc_zero = false;
        } else {
          int special = 0;
          acc = Pol::madd(acc, x2, y2, &special);  // (unchanged when special)
          if (special == 1) acc_zero = true;
          else if (special == 2) acc = Pol::dbl_slow(acc);
        }
      }
    }
    e0 = e1;
    e1 = e2;
    if constexpr (kPrefetch == 1) P = Pn;
  }
  if (cur != kNoBucket) {
    const bool head = runs == 1 && cur == prev_b;
    const bool tail = cur == next_b;
    if (head) { put(pieces, 2 * t); flags |= kHead; }
    if (tail) flags |= kTail;
    if (tail && !head) put(pieces, 2 * t + 1);
    if (!head && !tail) put(bucket_sum, cur);
  }
  if (runs <= 1) flags |= kSingle;
  acc_zero = true;  // absent pieces are the identity
  if (!(flags & kHead)) put(pieces, 2 * t);
  const bool through = (flags & kHead) && (flags & kTail) && (flags & kSingle);
  if (!(flags & kTail) || through) put(pieces, 2 * t + 1);
  tflags[t] = flags;
  tlast[t] = cur;
}


// (4 waves per SIMD -- <= 128 VGPRs, 14 spilled -- measured slower at 2^26:
// 76.1-76.4 vs 75.0-75.5 ms, profiles/r04b/tune_sort_tiles_recode_spt_4waves_2_24_26.log)
template <int kPrefetch, bool kRaw, int kEnt>
__global__ __launch_bounds__(kBlock, kPrefetch == 1 ? 1 : 3) void seg_acc29_kernel(const Affine<Bn254Fq>* __restrict__ bases,
                                                           const uint64_t* __restrict__ ents, uint32_t c,
                                                           uint64_t gbeg, uint64_t gend, uint64_t tbase, uint32_t K,
                                                           uint32_t idx_mask, XYZZ<Bn254Fq>* __restrict__ bucket_sum,
                                                           XYZZ<Bn254Fq>* __restrict__ pieces,
                                                           uint32_t* __restrict__ tflags, uint32_t* __restrict__ tlast) {
  seg_acc_limb_body<Pol29, kPrefetch, kRaw, kEnt>(bases, ents, c, gbeg, gend, tbase, K, idx_mask, bucket_sum, pieces,
                                                  tflags, tlast);
}
// BLS12-381 G1 over the 14 x 28-bit field: R-form stores (the FIPS chain join
// and window reductions read them); 2 waves per SIMD (the 14-limb madd holds
// ~4 x 14 accumulator + 2 x 14 base words)
template <int kEnt, bool kRaw>
__global__ __launch_bounds__(kBlock, 2) void seg_acc28_kernel(const Affine<Bls381Fq>* __restrict__ bases,
                                                              const uint64_t* __restrict__ ents, uint32_t c,
                                                              uint64_t gbeg, uint64_t gend, uint64_t tbase, uint32_t K,
                                                              uint32_t idx_mask,
                                                              XYZZ<Bls381Fq>* __restrict__ bucket_sum,
                                                              XYZZ<Bls381Fq>* __restrict__ pieces,
                                                              uint32_t* __restrict__ tflags,
                                                              uint32_t* __restrict__ tlast) {
  seg_acc_limb_body<Pol28, 0, kRaw, kEnt>(bases, ents, c, gbeg, gend, tbase, K, idx_mask, bucket_sum, pieces, tflags,
                                          tlast);
}

// ---------------------------------------------------------------------------
// G2 (Fq2) accumulation with a lane pair per virtual thread (acc_pair.h): the
// run logic of seg_acc_kernel, lane h holding component h of every Fq2 value.
// Both lanes of a pair read the same entries and take the same branches.
template <class Curve, bool kCall>
__global__ __launch_bounds__(kBlock) void seg_acc_pair_kernel(const Affine<typename Curve::F>* __restrict__ bases,
                                                              const uint64_t* __restrict__ ents, uint32_t c,
                                                              uint64_t gbeg, uint64_t gend, uint64_t tbase, uint32_t K,
                                                              uint32_t idx_mask,
                                                              XYZZ<typename Curve::F>* __restrict__ bucket_sum,
                                                              XYZZ<typename Curve::F>* __restrict__ pieces,
                                                              uint32_t* __restrict__ tflags,
                                                              uint32_t* __restrict__ tlast) {
  using Fb = typename Curve::F::Base;  // Fq
  using F = HotFp<Fb>;
  using namespace pair;
  using H = Half<F, kCall>;
  const uint32_t h = threadIdx.x & 1u;
  const uint64_t tl = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 1;
  const uint64_t g0 = gbeg + tl * K;
  if (g0 >= gend) return;  // both lanes of the pair
  const uint64_t g1 = min(g0 + K, gend);
  const uint64_t t = tbase + tl;
  const uint32_t dmask = (1u << c) - 1;
  auto bucket_of_key = [&](uint32_t key) -> uint32_t {
    uint32_t d = key & dmask;
    return d ? ((key >> c) << (c - 1)) + (d - 1) : kNoBucket;
  };
  const uint32_t prev_b = g0 > gbeg ? bucket_of_key(entry_key(ents[g0 - 1])) : kNoBucket;
  const uint32_t next_b = (g1 < gend) ? bucket_of_key(entry_key(ents[g1])) : kNoBucket;
  // component views: a point is {x.c0, x.c1, y.c0, y.c1}, an XYZZ {x.c0, x.c1, ..., zzz.c1}
  const Fb* comp = reinterpret_cast<const Fb*>(bases);
  Fb* bsum = reinterpret_cast<Fb*>(bucket_sum);
  Fb* pcs = reinterpret_cast<Fb*>(pieces);
  const F one_h = h ? F::zero() : F::one();
  Acc<H> acc;
  bool acc_zero = true;
  auto store = [&](Fb* dst, uint64_t idx) {  // this lane's components of the run sum (identity if none)
    Fb* o = dst + 8 * idx;
    if (acc_zero) {
      o[h] = one_h;
      o[2 + h] = one_h;
      o[4 + h] = Fb::zero();
      o[6 + h] = Fb::zero();
    } else {
      o[h] = acc.x.v;
      o[2 + h] = acc.y.v;
      o[4 + h] = acc.zz.v;
      o[6 + h] = acc.zzz.v;
    }
  };
  uint32_t flags = 0, runs = 0, cur = kNoBucket;
  uint64_t e0 = ents[g0];
  for (uint64_t g = g0; g < g1; ++g) {
    const uint64_t e1 = (g + 1 < g1) ? ents[g + 1] : 0;
    const uint32_t k0 = entry_key(e0), v0 = entry_val(e0);
    const uint32_t b = bucket_of_key(k0);
    if (b != kNoBucket) {
      const Fb* pt = comp + 4 * (size_t)(v0 & idx_mask);
      H px{pt[h]}, py{pt[2 + h]};
      if (b != cur) {
        if (cur != kNoBucket) {
          if (runs == 1 && cur == prev_b) { store(pcs, 2 * t); flags |= kHead; }
          else store(bsum, cur);
        }
        cur = b;
        ++runs;
        acc_zero = true;
      }
      const uint32_t pz = (px.v.is_zero_canonical() && py.v.is_zero_canonical()) ? 1u : 0u;
      if (!(pz & dpp<kSwap>(pz))) {  // not the identity base (both components zero)
        py.v = py.v.cond_neg_canonical(v0 & kSignBit);
        if (acc_zero) {
          acc = Acc<H>{px, py, H{one_h}, H{one_h}};
          acc_zero = false;
        } else {
          int special = 0;
          acc = madd(acc, px, py, h != 0, &special);  // (unchanged when special)
          if (special == 1) acc_zero = true;
          else if (special == 2) acc = pair::dbl(acc, h != 0);
        }
      }
    }
    e0 = e1;
  }
  if (cur != kNoBucket) {
    const bool head = runs == 1 && cur == prev_b;
    const bool tail = cur == next_b;
    if (head) { store(pcs, 2 * t); flags |= kHead; }
    if (tail) flags |= kTail;
    if (tail && !head) store(pcs, 2 * t + 1);
    if (!head && !tail) store(bsum, cur);
  }
  if (runs <= 1) flags |= kSingle;
  acc_zero = true;  // absent pieces are the identity
  if (!(flags & kHead)) store(pcs, 2 * t);
  const bool through = (flags & kHead) && (flags & kTail) && (flags & kSingle);
  if (!(flags & kTail) || through) store(pcs, 2 * t + 1);
  if (h == 0) {
    tflags[t] = flags;
    tlast[t] = cur;
  }
}

// The limb-field lane pairs of G2 (field policies of seg_acc_pair_limb_kernel):
// BLS12-381 over the 14 x 28-bit Fq (msm/pair28.h), BN254 over the 9 x 29-bit
// Fq (msm/pair29.h).
struct PairPol28 {
  using Fb = Bls381Fq;
  using F2 = Bls381Fq2;
  using F = f28::F28;
  using Acc = pair28::Acc;
  static __device__ __forceinline__ F repack(const uint32_t* w) { return f28::shl8_repack(w); }
  static __device__ __forceinline__ Acc start(const F& x, const F& y, bool h) { return pair28::from_shifted(x, y, h); }
  static __device__ __forceinline__ Acc madd(const Acc& a, const F& x, const F& y, bool h, int* sp) {
    return pair28::madd(a, x, y, h, sp);
  }
  static __device__ __forceinline__ Acc dbl(const Acc& a, bool h) { return pair28::dbl(a, h); }
  static __device__ __forceinline__ Acc add(const Acc& a, const Acc& b, bool h, int* sp) {
    return pair28::add(a, b, h, sp);
  }
  static __device__ __forceinline__ void to32(const F& x, uint32_t* w) { f28::to32(x, w); }
  static __device__ __forceinline__ F from32(const uint32_t* w) { return f28::from32(w); }
};
struct PairPol29 {
  using Fb = Bn254Fq;
  using F2 = Bn254Fq2;
  using F = f29::F29;
  using Acc = pair29::Acc;
  static __device__ __forceinline__ F repack(const uint32_t* w) { return f29::shl5_repack(w); }
  static __device__ __forceinline__ Acc start(const F& x, const F& y, bool h) { return pair29::from_shifted(x, y, h); }
  static __device__ __forceinline__ Acc madd(const Acc& a, const F& x, const F& y, bool h, int* sp) {
    return pair29::madd(a, x, y, h, sp);
  }
  static __device__ __forceinline__ Acc dbl(const Acc& a, bool h) { return pair29::dbl(a, h); }
  static __device__ __forceinline__ Acc add(const Acc& a, const Acc& b, bool h, int* sp) {
    return pair29::add(a, b, h, sp);
  }
  static __device__ __forceinline__ void to32(const F& x, uint32_t* w) { f29::to32(x, w); }
  static __device__ __forceinline__ F from32(const uint32_t* w) { return f29::from32(w); }
};

// G2 with a lane pair per point over a limb field: seg_acc_pair_kernel's run
// logic; the stores convert this lane's components to the R form the
// lane-pair FIPS reductions read.  set_variant bit 20 restores the FIPS pair.
// kStaged: the entries in 64-byte chunks through LDS as seg_acc_limb_body's
// kEnt 2 (a pair's two lanes DMA the chunk's four 16-byte pieces, two each;
// g0 even and 64 bytes of slack after the entry array)
template <class Pol, bool kStaged, bool kRaw>
__global__ __launch_bounds__(kBlock) void seg_acc_pair_limb_kernel(const Affine<typename Pol::F2>* __restrict__ bases,
                                                                   const uint64_t* __restrict__ ents, uint32_t c,
                                                                   uint64_t gbeg, uint64_t gend, uint64_t tbase,
                                                                   uint32_t K, uint32_t idx_mask,
                                                                   XYZZ<typename Pol::F2>* __restrict__ bucket_sum,
                                                                   XYZZ<typename Pol::F2>* __restrict__ pieces,
                                                                   uint32_t* __restrict__ tflags,
                                                                   uint32_t* __restrict__ tlast) {
  using Fb = typename Pol::Fb;
  using F = typename Pol::F;
  using Acc = typename Pol::Acc;
  const uint32_t h = threadIdx.x & 1u;
  const uint64_t tl = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 1;
  const uint64_t g0 = gbeg + tl * K;
  if (g0 >= gend) return;  // both lanes of the pair
  const uint64_t g1 = min(g0 + K, gend);
  const uint64_t t = tbase + tl;
  const uint32_t dmask = (1u << c) - 1;
  auto bucket_of_key = [&](uint32_t key) -> uint32_t {
    uint32_t d = key & dmask;
    return d ? ((key >> c) << (c - 1)) + (d - 1) : kNoBucket;
  };
  const uint32_t prev_b = g0 > gbeg ? bucket_of_key(entry_key(ents[g0 - 1])) : kNoBucket;
  const uint32_t next_b = (g1 < gend) ? bucket_of_key(entry_key(ents[g1])) : kNoBucket;
  const Fb* comp = reinterpret_cast<const Fb*>(bases);
  Fb* bsum = reinterpret_cast<Fb*>(bucket_sum);
  Fb* pcs = reinterpret_cast<Fb*>(pieces);
  const Fb one_h = h ? Fb::zero() : Fb::one();
  Acc acc{};  // (any defined value: the raw stores mask it while acc_zero)
  bool acc_zero = true;
  auto store = [&](Fb* dst, uint64_t idx) {  // this lane's components of the run sum (identity if none)
    if constexpr (kRaw) {  // the limbs as they are (LimbPairArith<Pol, true>::load), identity = zz zero
      F* o = reinterpret_cast<F*>(dst) + 8 * idx;
      F zz = acc.zz;
#pragma unroll
      for (int k = 0; k < (int)(sizeof(F) / 4); ++k) zz.l[k] = acc_zero ? 0u : zz.l[k];
      o[h] = acc.x;
      o[2 + h] = acc.y;
      o[4 + h] = zz;
      o[6 + h] = acc.zzz;
      return;
    }
    Fb* o = dst + 8 * idx;
    if (acc_zero) {
      o[h] = one_h;
      o[2 + h] = one_h;
      o[4 + h] = Fb::zero();
      o[6 + h] = Fb::zero();
    } else {
      Fb v;
      Pol::to32(acc.x, v.v);
      o[h] = v;
      Pol::to32(acc.y, v.v);
      o[2 + h] = v;
      Pol::to32(acc.zz, v.v);
      o[4 + h] = v;
      Pol::to32(acc.zzz, v.v);
      o[6 + h] = v;
    }
  };
  uint32_t flags = 0, runs = 0, cur = kNoBucket;
  // [buffer][wave][piece pair q][lane]: lane 2 vt + h' holds piece 2q + h' of virtual thread vt's chunk
  __shared__ uint4 estage[kStaged ? 2 : 1][kStaged ? kBlock / 64 : 1][2][kStaged ? 64 : 1];
  const uint32_t ewave = threadIdx.x >> 6, elane = threadIdx.x & 63;
  auto fetch_chunk = [&](uint64_t first, uint32_t buf) {
    const uint4* src = reinterpret_cast<const uint4*>(ents + first) + h;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      __builtin_amdgcn_global_load_lds(src + 2 * q, (lds_void_t*)&estage[buf][ewave][q][0], 16, 0, 0);
  };
  uint64_t e0 = 0;
  if constexpr (kStaged) fetch_chunk(g0, 0);
  else e0 = ents[g0];
  uint32_t it = 0;  // (the same for both lanes of a pair and every pair of the wave)
  for (uint64_t g = g0; g < g1; ++g, ++it) {
    uint64_t e1 = 0;
    if constexpr (kStaged) {
      if ((it & 7) == 0) {  // a new chunk: landed (this wave's own LDS-DMA); fetch the next one
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (g + 8 < g1) fetch_chunk(g + 8, ((it >> 3) + 1) & 1);
      }
      const uint32_t sl = it & 7, piece = sl >> 1;
      const uint2 w = reinterpret_cast<const uint2*>(
          &estage[(it >> 3) & 1][ewave][piece >> 1][(elane & ~1u) | (piece & 1)])[sl & 1];
      e0 = (uint64_t)w.y << 32 | w.x;
    } else {
      e1 = (g + 1 < g1) ? ents[g + 1] : 0;
    }
    const uint32_t k0 = entry_key(e0), v0 = entry_val(e0);
    const uint32_t b = bucket_of_key(k0);
    if (b != kNoBucket) {
      const Fb* pt = comp + 4 * (size_t)(v0 & idx_mask);
      const Fb px = pt[h];
      Fb py = pt[2 + h];
      if (b != cur) {
        if (cur != kNoBucket) {  // (one store block for both destinations, as seg_acc_limb_body)
          const bool head = runs == 1 && cur == prev_b;
          if (head) flags |= kHead;
          store(head ? pcs : bsum, head ? 2 * t : cur);
        }
        cur = b;
        ++runs;
        acc_zero = true;
      }
      const uint32_t pz = (px.is_zero_canonical() && py.is_zero_canonical()) ? 1u : 0u;
      if (!(pz & pair::dpp<pair::kSwap>(pz))) {  // not the identity base (both components zero)
        py = py.cond_neg_canonical(v0 & kSignBit);
        const F x2 = Pol::repack(px.v), y2 = Pol::repack(py.v);
        if (acc_zero) {
          acc = Pol::start(x2, y2, h != 0);
          acc_zero = false;
        } else {
          int special = 0;
          acc = Pol::madd(acc, x2, y2, h != 0, &special);  // (unchanged when special)
          if (special == 1) acc_zero = true;
          else if (special == 2) acc = Pol::dbl(acc, h != 0);
        }
      }
    }
    if constexpr (!kStaged) e0 = e1;
  }
  if (cur != kNoBucket) {
    const bool head = runs == 1 && cur == prev_b;
    const bool tail = cur == next_b;
    if (head) { store(pcs, 2 * t); flags |= kHead; }
    if (tail) flags |= kTail;
    if (tail && !head) store(pcs, 2 * t + 1);
    if (!head && !tail) store(bsum, cur);
  }
  if (runs <= 1) flags |= kSingle;
  acc_zero = true;  // absent pieces are the identity
  if (!(flags & kHead)) store(pcs, 2 * t);
  const bool through = (flags & kHead) && (flags & kTail) && (flags & kSingle);
  if (!(flags & kTail) || through) store(pcs, 2 * t + 1);
  if (h == 0) {
    tflags[t] = flags;
    tlast[t] = cur;
  }
}

// A bucket that crosses thread boundaries forms a chain t0 < ... < t1: the
// tail of t0, the whole-range heads of the "through" threads in between and
// the head of t1 -- i.e. pieces[2*t0+1 .. 2*t1] (absent tails are identity).
__device__ __forceinline__ bool chain_start(uint32_t f) {
  const bool through = (f & kHead) && (f & kTail) && (f & kSingle);
  return (f & kTail) && !through;
}
__device__ __forceinline__ bool chain_end(uint32_t f) {
  const bool through = (f & kHead) && (f & kTail) && (f & kSingle);
  return (f & kHead) && !through;
}

// The accumulation's run flags (kHead / kTail / kSingle) and last bucket of
// every thread, from the sorted keys alone: the values seg_acc*_kernel writes
// (head = the first run continues the previous thread's last bucket, tail =
// the last run continues into the next thread, single = at most one run).  So
// the chain tables below can be built on a second stream WHILE the
// accumulation runs, and the host's read-back of the chain count and length
// hides behind it (small MSMs: the tables, the read-back and the join-level
// offsets were ~90 us on the critical path of a 0.7 ms 2^16 MSM).  Keys are
// sorted, so equal first and last buckets mean one run; the loop runs only
// when an end of the range holds digit-0 entries (no bucket).
// Debug check (set_variant bit 21): the run flags chain_flags_kernel derived
// from the sorted keys before the accumulation equal the ones the accumulation
// wrote (the small-MSM chain tables are built from the former).
__global__ __launch_bounds__(kBlock) void chain_flags_check_kernel(const uint32_t* __restrict__ tflags,
                                                                   const uint32_t* __restrict__ tlast,
                                                                   const uint32_t* __restrict__ cflags,
                                                                   const uint32_t* __restrict__ clast, uint32_t T,
                                                                   uint32_t* __restrict__ mismatches) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= T) return;
  if (tflags[t] != cflags[t] || tlast[t] != clast[t]) atomicAdd(mismatches, 1u);
}

__global__ __launch_bounds__(kBlock) void chain_flags_kernel(const uint64_t* __restrict__ ents, uint32_t c,
                                                             uint64_t gbeg, uint64_t gend, uint32_t K, uint32_t T,
                                                             uint32_t* __restrict__ tflags,
                                                             uint32_t* __restrict__ tlast) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= T) return;
  const uint64_t g0 = gbeg + (uint64_t)t * K, g1 = min(g0 + K, gend);
  const uint32_t dmask = (1u << c) - 1;
  auto bucket = [&](uint64_t g) -> uint32_t {
    const uint32_t key = entry_key(ents[g]), d = key & dmask;
    return d ? ((key >> c) << (c - 1)) + (d - 1) : kNoBucket;
  };
  const uint32_t prev_b = g0 > gbeg ? bucket(g0 - 1) : kNoBucket;
  const uint32_t next_b = g1 < gend ? bucket(g1) : kNoBucket;
  uint32_t first = bucket(g0), last = bucket(g1 - 1);
  bool single = first == last;
  if (first == kNoBucket || last == kNoBucket) {
    uint32_t runs = 0, cur = kNoBucket;
    first = kNoBucket;
    for (uint64_t g = g0; g < g1; ++g) {
      const uint32_t b = bucket(g);
      if (b != kNoBucket && b != cur) {
        if (runs == 0) first = b;
        cur = b;
        ++runs;
      }
    }
    last = cur;
    single = runs <= 1;
  }
  uint32_t flags = single ? kSingle : 0u;
  if (first != kNoBucket && first == prev_b) flags |= kHead;
  if (last != kNoBucket && last == next_b) flags |= kTail;
  tflags[t] = flags;
  tlast[t] = last;
}

__global__ __launch_bounds__(kBlock) void chain_mark_kernel(const uint32_t* __restrict__ tflags, uint32_t T,
                                                            uint32_t* __restrict__ is_start,
                                                            uint32_t* __restrict__ max_len) {
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t == 0) *max_len = 0;  // seg_count_kernel's atomicMax target (no memset launch)
  if (t > T) return;
  is_start[t] = (t < T && chain_start(tflags[t])) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void chain_build_kernel(const uint32_t* __restrict__ tflags,
                                                             const uint32_t* __restrict__ tlast,
                                                             const uint32_t* __restrict__ cid, uint32_t T,
                                                             uint32_t* __restrict__ cbeg, uint32_t* __restrict__ cend,
                                                             uint32_t* __restrict__ cbucket,
                                                             uint32_t* __restrict__ nchains) {
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= T) return;
  uint32_t f = tflags[t];
  if (chain_end(f)) cend[cid[t] - 1] = 2 * t + 1;  // the chain opened by the last start before t
  if (chain_start(f)) {
    cbeg[cid[t]] = 2 * t + 1;
    cbucket[cid[t]] = tlast[t];
  }
  if (t == T - 1) nchains[0] = cid[t] + (chain_start(f) ? 1u : 0u);
}

// per-chain piece count for the first reduction level, and the longest chain
__global__ __launch_bounds__(kBlock) void seg_count_kernel(const uint32_t* __restrict__ beg,
                                                           const uint32_t* __restrict__ end,
                                                           const uint32_t* __restrict__ nseg_ptr, uint32_t nseg_cap,
                                                           unsigned K2, uint32_t* __restrict__ cnt,
                                                           uint32_t* __restrict__ max_len) {
  uint32_t s = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t nseg = nseg_ptr ? *nseg_ptr : nseg_cap;
  uint32_t len = 0;
  if (s < nseg) {
    len = end[s] - beg[s];
    cnt[s] = (len + K2 - 1) / K2;
  } else if (s <= nseg_cap) {
    cnt[s] = 0;
  }
  if (max_len) {
    __shared__ uint32_t red[kBlock / 64];
    for (int o = 32; o > 0; o >>= 1) len = max(len, (uint32_t)__shfl_xor(len, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = len;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t m = red[0];
      for (unsigned i = 1; i < kBlock / 64; ++i) m = max(m, red[i]);
      if (m) atomicMax(max_len, m);
    }
  }
}

// A join level's output offsets in ONE workgroup when there are few chains:
// off[s] = sum over s' < s of ceil(len_s' / K2), len_s = end[s] - beg[s]
// (end = nullptr: end[s] = beg[s + 1]).  Replaces seg_count + rocPRIM's
// two-kernel scan (three launches of a few microseconds on a latency-bound
// level) for nseg <= kJoinSmallChains.
constexpr unsigned kJoinOffBlock = 1024, kJoinSmallChains = 64 * 1024;
enum ChainMode { kChainsInStream, kChainsBefore, kChainsAfter };  // see MsmGpu::enqueue
__device__ __forceinline__ void join_offsets_body(const uint32_t* __restrict__ beg, const uint32_t* __restrict__ end,
                                                  uint32_t nseg, unsigned K2, uint32_t* __restrict__ off,
                                                  uint32_t* part) {
  const uint32_t t = threadIdx.x, per = (nseg + kJoinOffBlock - 1) / kJoinOffBlock;
  const uint32_t s0 = min(nseg, t * per), s1 = min(nseg, s0 + per);
  auto count = [&](uint32_t s) {
    const uint32_t len = (end ? end[s] : beg[s + 1]) - beg[s];
    return (len + K2 - 1) / K2;
  };
  uint32_t sum = 0;
  for (uint32_t s = s0; s < s1; ++s) sum += count(s);
  part[t] = sum;
  __syncthreads();
  for (unsigned d = 1; d < kJoinOffBlock; d <<= 1) {  // inclusive scan of the per-thread sums
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;  // exclusive prefix of this thread's range
  for (uint32_t s = s0; s < s1; ++s) {
    off[s] = run;
    run += count(s);
  }
  if (t == kJoinOffBlock - 1) off[nseg] = part[t];
}
__global__ __launch_bounds__(kJoinOffBlock) void join_offsets_kernel(const uint32_t* __restrict__ beg,
                                                                     const uint32_t* __restrict__ end, uint32_t nseg,
                                                                     unsigned K2, uint32_t* __restrict__ off) {
  __shared__ uint32_t part[kJoinOffBlock];
  join_offsets_body(beg, end, nseg, K2, off, part);
}

// The join levels' count and fan-in from the longest chain (the host makes
// the same choice from the read-back): 4-ary levels when a chain is longer
// than K2 pieces and the accumulation ran fewer than 2^20 threads
constexpr unsigned kJoinFanLong = 4;  // chain-join fan-in for chains longer than MsmPlan::K2
__host__ __device__ __forceinline__ unsigned join_fan_in(uint32_t max_len, unsigned K2, size_t T) {
  return (max_len > K2 && T < (size_t(1) << 20)) ? kJoinFanLong : K2;
}
__host__ __device__ __forceinline__ unsigned join_levels(uint32_t max_len, unsigned K2) {
  unsigned levels = 0;
  for (uint32_t len = max_len; len > 1; len = (len + K2 - 1) / K2) ++levels;
  return levels;
}

// Every join level's output offsets in one workgroup, BEFORE the
// accumulation (small MSMs): the chain count and the longest chain come from
// the chain tables in device memory (dscal), so nothing waits for the host;
// level l's table at ltab + l * stride (stride = T + 2 >= chains + 2).
__global__ __launch_bounds__(kJoinOffBlock) void join_offsets_all_kernel(const uint32_t* __restrict__ beg,
                                                                         const uint32_t* __restrict__ end,
                                                                         const uint32_t* __restrict__ dscal,
                                                                         unsigned K2base, uint32_t T, unsigned lv_max,
                                                                         size_t stride, uint32_t* __restrict__ ltab) {
  __shared__ uint32_t part[kJoinOffBlock];
  const uint32_t nseg = dscal[0], max_len = dscal[1];
  if (nseg == 0) return;
  const unsigned K2 = join_fan_in(max_len, K2base, T);
  const unsigned levels = min(join_levels(max_len, K2), lv_max);
  for (unsigned l = 0; l < levels; ++l) {
    const uint32_t* pbeg = l == 0 ? beg : ltab + (l - 1) * stride;
    join_offsets_body(pbeg, l == 0 ? end : nullptr, nseg, K2, ltab + l * stride, part);
    __syncthreads();  // the next level reads this table
  }
}

// largest s in [0, nseg) with off[s] <= t  (off non-decreasing)
__device__ __forceinline__ uint32_t find_segment(const uint32_t* __restrict__ off, uint32_t nseg, uint32_t t) {
  uint32_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

// The arithmetic of the one-lane reductions: the FIPS field (XYZZ<HotFp>, the
// arrays as they are) or a limb field (BLS12-381 G1 over 14 x 28-bit limbs,
// msm/acc28.h) that converts the R-form arrays on load (from32, < 3p) and
// store (to32), identities as flags.
template <class Curve>
struct FipsArith {
  using F = typename HotOf<typename Curve::F>::type;  // inline products (same layout)
  using A = XYZZ<F>;
  static __device__ __forceinline__ A load(const XYZZ<typename Curve::F>* p, size_t i) {
    return reinterpret_cast<const XYZZ<F>*>(p)[i];
  }
  static __device__ __forceinline__ void store(XYZZ<typename Curve::F>* p, size_t i, const A& a) {
    reinterpret_cast<XYZZ<F>*>(p)[i] = a;
  }
  static __device__ __forceinline__ A add(const A& a, const A& b) { return a + b; }
  static __device__ __forceinline__ A zero() { return A::zero(); }
  static __device__ __forceinline__ A dbl(const A& a) { return a.dbl(); }
  static __device__ __forceinline__ bool is_zero(const A& a) { return a.is_zero(); }
};
// kRawIn / kRawOut: the arrays hold Pol28::Raw (224-byte accumulator limbs,
// the identity as zz = 0) instead of R-form XYZZ -- the accumulation's raw
// stores read by the chain join and the window segments without conversions
// (madd's and add's outputs, X < 9.02p, Y, ZZ, ZZZ < 1.05p, are inside add's
// input invariant, msm/acc28.h)
template <bool kRawIn, bool kRawOut>
struct Limb28ArithT {
  using Fq = Bls381Fq;
  struct A {
    acc28_core::Acc a;
    bool zero;
  };
  static __device__ __forceinline__ A load(const XYZZ<Fq>* p, size_t i) {
    if constexpr (kRawIn) {
      const acc28_core::Acc r = reinterpret_cast<const acc28_core::Acc*>(p)[i];
      uint32_t nz = 0;
#pragma unroll
      for (int k = 0; k < 14; ++k) nz |= r.zz.l[k];
      return {r, nz == 0};
    } else {
      const XYZZ<Fq> q = p[i];
      if (q.is_zero()) return {acc28_core::Acc{}, true};
      return {{f28::from32(q.x.v), f28::from32(q.y.v), f28::from32(q.zz.v), f28::from32(q.zzz.v)}, false};
    }
  }
  static __device__ __forceinline__ void store(XYZZ<Fq>* p, size_t i, const A& a) {
    if constexpr (kRawOut) {
      reinterpret_cast<acc28_core::Acc*>(p)[i] = Pol28::raw_of(a.a, a.zero);
      return;
    }
    if (a.zero) {
      p[i] = XYZZ<Fq>::zero();
      return;
    }
    XYZZ<Fq> r;
    f28::to32(a.a.x, r.x.v);
    f28::to32(a.a.y, r.y.v);
    f28::to32(a.a.zz, r.zz.v);
    f28::to32(a.a.zzz, r.zzz.v);
    p[i] = r;
  }
  static __device__ __forceinline__ A add(const A& a, const A& b) {
    if (a.zero) return b;
    if (b.zero) return a;
    int special = 0;
    const acc28_core::Acc s = acc28_core::add(a.a, b.a, &special);
    if (special == 1) return {a.a, true};
    return {special == 2 ? acc28_core::dbl(a.a) : s, false};
  }
  static __device__ __forceinline__ A zero() { return {acc28_core::Acc{}, true}; }
  static __device__ __forceinline__ A dbl(const A& a) {  // (no point of this prime-order group doubles to the identity)
    return a.zero ? a : A{acc28_core::dbl(a.a), false};
  }
  static __device__ __forceinline__ bool is_zero(const A& a) { return a.zero; }
};
using Limb28Arith = Limb28ArithT<false, false>;

// One K2-ary level of the segmented tree: output q of segment s is the sum of
// in[beg[s] + q*K2 .. min(end[s], +K2)).  On the last level every segment has
// one output, which goes to bucket_sum[bucket[s]].
template <class Curve, class Ar = FipsArith<Curve>>
__global__ __launch_bounds__(kBlock, AccWaves<Curve>::value) void seg_reduce_kernel(const XYZZ<typename Curve::F>* __restrict__ in,
                                                            const uint32_t* __restrict__ beg,
                                                            const uint32_t* __restrict__ end,
                                                            const uint32_t* __restrict__ out_off, uint32_t nseg,
                                                            unsigned K2, XYZZ<typename Curve::F>* __restrict__ out,
                                                            const uint32_t* __restrict__ bucket,
                                                            XYZZ<typename Curve::F>* __restrict__ bucket_sum) {
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= out_off[nseg]) return;
  uint32_t s = find_segment(out_off, nseg, t);
  uint32_t q = t - out_off[s];
  uint32_t e0 = beg[s] + q * K2;
  uint32_t e1 = min(end[s], e0 + K2);
  typename Ar::A acc = Ar::load(in, e0);
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = Ar::add(acc, Ar::load(in, e));
  if (bucket) Ar::store(bucket_sum, bucket[s], acc);
  else Ar::store(out, t, acc);
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
template <class Ar>
__device__ typename Ar::A small_mul_ar(const typename Ar::A& P, uint32_t m) {
  if (m == 0 || Ar::is_zero(P)) return Ar::zero();
  typename Ar::A r = P;
  for (int bit = 30 - __builtin_clz(m); bit >= 0; --bit) {
    r = Ar::dbl(r);
    if ((m >> bit) & 1) r = Ar::add(r, P);
  }
  return r;
}

// Window reduction, stage 1: segment j of window w covers buckets
// [j*L, (j+1)*L) (bucket b holds |digit| = b+1).  Running sums from the top
// give S = sum (b - jL + 1) B_b and R = sum B_b; the segment's share of
// sum_b (b+1) B_b is S + jL * R  (PippengerBase::AccumulateBuckets,
// pippenger_base.h:36-57, split across threads).
template <class Curve, class Ar = FipsArith<Curve>>
__global__ __launch_bounds__(kBlock, AccWaves<Curve>::value) void window_segment_kernel(const XYZZ<typename Curve::F>* __restrict__ bucket_sum,
                                                                unsigned W, unsigned B, unsigned L,
                                                                XYZZ<typename Curve::F>* __restrict__ out) {
  uint32_t S = B / L;
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S) return;
  uint32_t w = t / S, j = t - w * S;
  const size_t b0 = (size_t)w * B + (size_t)j * L;
  typename Ar::A R = Ar::zero(), acc = Ar::zero();
  for (int k = (int)L - 1; k >= 0; --k) {
    R = Ar::add(R, Ar::load(bucket_sum, b0 + k));
    acc = Ar::add(acc, R);
  }
  acc = Ar::add(acc, small_mul_ar<Ar>(R, j * L));
  Ar::store(out, t, acc);
}

// Two-level window sums with one lane per point (the pair kernels below
// explain the scheme): level 1 A_j, R_j per L1-bucket segment without fix-up,
// level 2 sum_j j R_j with 0-based weights, out = sum_j A_j + L1 sum_j j R_j.
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, AccWaves<Curve>::value) void window_seg1_kernel(
    const XYZZ<typename Curve::F>* __restrict__ bucket_sum, unsigned W, unsigned B, unsigned L,
    XYZZ<typename Curve::F>* __restrict__ out_a, XYZZ<typename Curve::F>* __restrict__ out_r) {
  const uint32_t S = B / L;
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S) return;
  const uint32_t w = t / S, j = t - w * S;
  const size_t b0 = (size_t)w * B + (size_t)j * L;
  typename Ar::A R = Ar::zero(), acc = Ar::zero();
  for (int k = (int)L - 1; k >= 0; --k) {
    R = Ar::add(R, Ar::load(bucket_sum, b0 + k));
    acc = Ar::add(acc, R);
  }
  Ar::store(out_a, t, acc);
  Ar::store(out_r, t, R);
}
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, AccWaves<Curve>::value) void window_seg2_kernel(
    const XYZZ<typename Curve::F>* __restrict__ in, unsigned W, unsigned S, unsigned L2,
    XYZZ<typename Curve::F>* __restrict__ out) {
  const uint32_t S2 = S / L2;
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S2) return;
  const uint32_t w = t / S2, q = t - w * S2;
  const size_t b0 = (size_t)w * S + (size_t)q * L2;
  typename Ar::A R = Ar::zero(), acc = Ar::zero();
  for (int k = (int)L2 - 1; k >= 0; --k) {  // acc before R: weights k, not k + 1
    acc = Ar::add(acc, R);
    R = Ar::add(R, Ar::load(in, b0 + k));
  }
  acc = Ar::add(acc, small_mul_ar<Ar>(R, q * L2));
  Ar::store(out, t, acc);
}
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, AccWaves<Curve>::value) void window_combine_kernel(
    const XYZZ<typename Curve::F>* __restrict__ a, const XYZZ<typename Curve::F>* __restrict__ b, unsigned W,
    unsigned m, XYZZ<typename Curve::F>* __restrict__ out) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W) return;
  Ar::store(out, t, Ar::add(Ar::load(a, t), small_mul_ar<Ar>(Ar::load(b, t), m)));
}

// The G2 reductions with a lane pair per point (acc_pair.h): the one-lane
// XYZZ<Fq2> additions hold two points and their temporaries (BLS12-381:
// 220-460 spilled VGPRs per kernel, 21 ms of a 2^24 MSM); split by component
// they stay in registers.  Same schedules as the one-lane kernels above.
// The arithmetic of the pair reductions: the FIPS lane pair (acc_pair.h) or a
// limb-field pair (msm/pair28.h, pair29.h) that converts the R-form arrays on
// load (from32, < 3p) and store (to32), keeping identities as flags.
template <class Curve>
struct FipsPairArith {
  using Fb = typename Curve::F::Base;
  using H = pair::Half<HotFp<Fb>, Fb::N == 12>;
  using A = pair::Acc<H>;
  static __device__ __forceinline__ A load(const Fb* p, size_t i, uint32_t h) { return pair::load<H>(p, i, h); }
  static __device__ __forceinline__ void store(Fb* p, size_t i, uint32_t h, const A& a) { pair::store(p, i, h, a); }
  static __device__ __forceinline__ A add(const A& a, const A& b, bool h) { return pair::add(a, b, h); }
  static __device__ __forceinline__ A zero(bool h) { return pair::zero<H>(h); }
  static __device__ __forceinline__ A small_mul(const A& P, uint32_t m, bool h) { return pair::small_mul(P, m, h); }
};
// kRawIn / kRawOut: the arrays hold the lane pair's limb-field components
// as they are (8 Pol::F per point: x, y, zz, zzz x 2 components; the identity
// = zz zero in both) instead of R-form Fq2 XYZZ: the raw accumulation stores,
// read by the chain join and the window segments (madd's and add's outputs
// keep add's input invariant X < 10p, Y < 6p, ZZ, ZZZ < 3p, msm/pair28.h,
// pair29.h)
template <class Pol, bool kRawIn = false, bool kRawOut = false>
struct LimbPairArith {
  using Fb = typename Pol::Fb;
  using F = typename Pol::F;
  struct A {
    typename Pol::Acc a;
    bool zero;
  };
  static __device__ __forceinline__ A load(const Fb* p, size_t i, uint32_t h) {
    if constexpr (kRawIn) {
      const F* o = reinterpret_cast<const F*>(p) + 8 * i;
      const F x = o[h], y = o[2 + h], zz = o[4 + h], zzz = o[6 + h];
      uint32_t nz = 0;
#pragma unroll
      for (int k = 0; k < (int)(sizeof(F) / 4); ++k) nz |= zz.l[k];
      nz |= pair::dpp<pair::kSwap>(nz);
      return {{x, y, zz, zzz}, nz == 0};
    }
    const Fb* o = p + 8 * i;
    const Fb x = o[h], y = o[2 + h], zz = o[4 + h], zzz = o[6 + h];
    uint32_t nz = 0;
#pragma unroll
    for (int k = 0; k < Fb::N; ++k) nz |= zz.v[k];
    nz |= pair::dpp<pair::kSwap>(nz);  // the identity: zz = 0 in both components
    return {{Pol::from32(x.v), Pol::from32(y.v), Pol::from32(zz.v), Pol::from32(zzz.v)}, nz == 0};
  }
  static __device__ __forceinline__ void store(Fb* p, size_t i, uint32_t h, const A& a) {
    if constexpr (kRawOut) {
      F* o = reinterpret_cast<F*>(p) + 8 * i;
      F zz = a.a.zz;
#pragma unroll
      for (int k = 0; k < (int)(sizeof(F) / 4); ++k) zz.l[k] = a.zero ? 0u : zz.l[k];
      o[h] = a.a.x;
      o[2 + h] = a.a.y;
      o[4 + h] = zz;
      o[6 + h] = a.a.zzz;
      return;
    }
    Fb* o = p + 8 * i;
    if (a.zero) {
      const Fb one_h = h ? Fb::zero() : Fb::one();
      o[h] = one_h;
      o[2 + h] = one_h;
      o[4 + h] = Fb::zero();
      o[6 + h] = Fb::zero();
      return;
    }
    Fb v;
    Pol::to32(a.a.x, v.v);
    o[h] = v;
    Pol::to32(a.a.y, v.v);
    o[2 + h] = v;
    Pol::to32(a.a.zz, v.v);
    o[4 + h] = v;
    Pol::to32(a.a.zzz, v.v);
    o[6 + h] = v;
  }
  static __device__ __forceinline__ A add(const A& a, const A& b, bool h) {
    if (a.zero) return b;
    if (b.zero) return a;
    int special = 0;
    const typename Pol::Acc s = Pol::add(a.a, b.a, h, &special);
    if (special == 1) return {a.a, true};
    return {special == 2 ? Pol::dbl(a.a, h) : s, false};
  }
  static __device__ __forceinline__ A zero(bool) { return {typename Pol::Acc{}, true}; }
  static __device__ __forceinline__ A small_mul(const A& P, uint32_t m, bool h) {
    if (m == 0 || P.zero) return zero(h);
    A r = P;
    for (int bit = 30 - __builtin_clz(m); bit >= 0; --bit) {
      r.a = Pol::dbl(r.a, h);  // (no point of this prime-order group doubles to the identity)
      if ((m >> bit) & 1) r = add(r, P, h);
    }
    return r;
  }
};

template <class Curve, class Ar = FipsPairArith<Curve>>
__global__ __launch_bounds__(kBlock, 2) void seg_reduce_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ in,
                                                                 const uint32_t* __restrict__ beg,
                                                                 const uint32_t* __restrict__ end,
                                                                 const uint32_t* __restrict__ out_off, uint32_t nseg,
                                                                 unsigned K2, XYZZ<typename Curve::F>* __restrict__ out,
                                                                 const uint32_t* __restrict__ bucket,
                                                                 XYZZ<typename Curve::F>* __restrict__ bucket_sum) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= out_off[nseg]) return;  // both lanes of the pair
  const uint32_t s = find_segment(out_off, nseg, t);
  const uint32_t e0 = beg[s] + (t - out_off[s]) * K2;
  const uint32_t e1 = min(end[s], e0 + K2);
  const Fb* src = reinterpret_cast<const Fb*>(in);
  typename Ar::A acc = Ar::load(src, e0, h);
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = Ar::add(acc, Ar::load(src, e, h), h != 0);
  if (bucket) Ar::store(reinterpret_cast<Fb*>(bucket_sum), bucket[s], h, acc);
  else Ar::store(reinterpret_cast<Fb*>(out), t, h, acc);
}

// (BLS12-381's limb pair spills here at the two-wave cap; one wave per SIMD
// without spills measured slower: reduction 14.1 -> 14.7 ms at 2^24,
// profiles/r04b/ab_window_segment_one_wave_rejected.log)
template <class Curve, class Ar = FipsPairArith<Curve>>
#ifndef TACHYON_SEG_PAIR_WAVES
#define TACHYON_SEG_PAIR_WAVES 2  // (A/B builds: 1 lifts the VGPR cap that makes the BLS12-381 G2 segment sums spill)
#endif
__global__ __launch_bounds__(kBlock, TACHYON_SEG_PAIR_WAVES) void window_segment_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ bucket_sum,
                                                                     unsigned W, unsigned B, unsigned L,
                                                                     XYZZ<typename Curve::F>* __restrict__ out) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t S = B / L;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W * S) return;
  const uint32_t w = t / S, j = t - w * S;
  const Fb* bs = reinterpret_cast<const Fb*>(bucket_sum);
  const size_t b0 = (size_t)w * B + (size_t)j * L;
  typename Ar::A R = Ar::zero(h != 0), acc = R;
  for (int k = (int)L - 1; k >= 0; --k) {
    R = Ar::add(R, Ar::load(bs, b0 + k, h), h != 0);
    acc = Ar::add(acc, R, h != 0);
  }
  acc = Ar::add(acc, Ar::small_mul(R, j * L, h != 0), h != 0);
  Ar::store(reinterpret_cast<Fb*>(out), t, h, acc);
}

// Two-level window sums (G2 lane pairs, round 5).  sum_b (b + 1) B_b over a
// window's B buckets in segments of L1: level 1 gives each segment j its local
// weighted sum A_j = sum_k (k + 1) B_{j L1 + k} and plain sum R_j with no
// (j L1) R_j fix-up; level 2 prices all fix-ups at once, sum_j j R_j, by the
// same running sums over the R_j (0-based weights, segments of L2 with the
// small fix-up of the one-level kernel); the window is sum_j A_j + L1 sum_j j
// R_j.  Per bucket ~2 + 3 / L1 additions instead of 2 + (the ~log2(B)
// doublings and adds of a fix-up) / L, and with L1 = 16 four times the threads
// of L = 64.  Measured slower (set_variant bit 23, see the window sums in
// enqueue): the trees over the partial sums add more than the fix-ups cost.
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, 2) void window_seg1_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ bucket_sum,
                                                                  unsigned W, unsigned B, unsigned L,
                                                                  XYZZ<typename Curve::F>* __restrict__ out_a,
                                                                  XYZZ<typename Curve::F>* __restrict__ out_r) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t S = B / L;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W * S) return;
  const uint32_t w = t / S, j = t - w * S;
  const Fb* bs = reinterpret_cast<const Fb*>(bucket_sum);
  const size_t b0 = (size_t)w * B + (size_t)j * L;
  typename Ar::A R = Ar::zero(h != 0), acc = R;
  for (int k = (int)L - 1; k >= 0; --k) {
    R = Ar::add(R, Ar::load(bs, b0 + k, h), h != 0);
    acc = Ar::add(acc, R, h != 0);
  }
  Ar::store(reinterpret_cast<Fb*>(out_a), t, h, acc);
  Ar::store(reinterpret_cast<Fb*>(out_r), t, h, R);
}
// level 2: out[w S2 + q] = sum_{k < L2} (q L2 + k) R_{w S + q L2 + k}
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, 2) void window_seg2_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ in,
                                                                  unsigned W, unsigned S, unsigned L2,
                                                                  XYZZ<typename Curve::F>* __restrict__ out) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t S2 = S / L2;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W * S2) return;
  const uint32_t w = t / S2, q = t - w * S2;
  const Fb* src = reinterpret_cast<const Fb*>(in);
  const size_t b0 = (size_t)w * S + (size_t)q * L2;
  typename Ar::A R = Ar::zero(h != 0), acc = R;
  for (int k = (int)L2 - 1; k >= 0; --k) {  // acc before R: weights k, not k + 1
    acc = Ar::add(acc, R, h != 0);
    R = Ar::add(R, Ar::load(src, b0 + k, h), h != 0);
  }
  acc = Ar::add(acc, Ar::small_mul(R, q * L2, h != 0), h != 0);
  Ar::store(reinterpret_cast<Fb*>(out), t, h, acc);
}
// out[w] = a[w] + m b[w]
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, 2) void window_combine_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ a,
                                                                     const XYZZ<typename Curve::F>* __restrict__ b,
                                                                     unsigned W, unsigned m,
                                                                     XYZZ<typename Curve::F>* __restrict__ out) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W) return;
  const typename Ar::A x = Ar::load(reinterpret_cast<const Fb*>(a), t, h);
  const typename Ar::A y = Ar::load(reinterpret_cast<const Fb*>(b), t, h);
  Ar::store(reinterpret_cast<Fb*>(out), t, h, Ar::add(x, Ar::small_mul(y, m, h != 0), h != 0));
}

// The window segment sums in two passes (G2 lane pairs, set_variant bit 24):
// window_segment_pair_kernel holds R, the running sum and a loaded bucket
// (three G2 points, ~540 VGPRs of state for BLS12-381, spilled at the
// two-wave cap).  Pass 1 keeps R and the loaded bucket only and stores every
// suffix sum R_k = sum_{k' >= k} B_{j L + k'} of its segment; pass 2 sums a
// segment's stored R_k (the running sum's value), pass 3 adds the (j L) R_0
// fix-up -- the same segment sums, with two points live in each loop.
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, 2) void window_rsum_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ bucket_sum,
                                                                  unsigned W, unsigned B, unsigned L,
                                                                  XYZZ<typename Curve::F>* __restrict__ rs) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t S = B / L;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W * S) return;
  const uint32_t w = t / S, j = t - w * S;
  const Fb* bs = reinterpret_cast<const Fb*>(bucket_sum);
  Fb* out = reinterpret_cast<Fb*>(rs);
  const size_t b0 = (size_t)w * B + (size_t)j * L;
  typename Ar::A R = Ar::zero(h != 0);
  for (int k = (int)L - 1; k >= 0; --k) {
    R = Ar::add(R, Ar::load(bs, b0 + k, h), h != 0);
    Ar::store(out, b0 + k, h, R);
  }
}
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, 2) void window_rsum_total_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ rs,
                                                                        unsigned W, unsigned B, unsigned L,
                                                                        XYZZ<typename Curve::F>* __restrict__ out) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t S = B / L;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W * S) return;
  const uint32_t w = t / S, j = t - w * S;
  const Fb* src = reinterpret_cast<const Fb*>(rs);
  const size_t b0 = (size_t)w * B + (size_t)j * L;
  typename Ar::A acc = Ar::load(src, b0, h);
  for (uint32_t k = 1; k < L; ++k) acc = Ar::add(acc, Ar::load(src, b0 + k, h), h != 0);
  Ar::store(reinterpret_cast<Fb*>(out), t, h, acc);
}
// pass 3: the (j L) R_0 fix-ups, out[t] += (j L) rs[segment start] (apart,
// so the summing loop above keeps the scalar multiplication's registers free)
template <class Curve, class Ar>
__global__ __launch_bounds__(kBlock, 2) void window_rsum_fix_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ rs,
                                                                      unsigned W, unsigned B, unsigned L,
                                                                      XYZZ<typename Curve::F>* __restrict__ out) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t S = B / L;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W * S) return;
  const uint32_t w = t / S, j = t - w * S;
  if (j == 0) return;  // (both lanes of the pair)
  const typename Ar::A fix = Ar::small_mul(Ar::load(reinterpret_cast<const Fb*>(rs), (size_t)w * B + (size_t)j * L, h),
                                           j * L, h != 0);
  Fb* o = reinterpret_cast<Fb*>(out);
  Ar::store(o, t, h, Ar::add(Ar::load(o, t, h), fix, h != 0));
}

template <class Curve, class Ar = FipsPairArith<Curve>>
__global__ __launch_bounds__(kBlock, 2) void reduce_uniform_pair_kernel(const XYZZ<typename Curve::F>* __restrict__ in,
                                                                     unsigned W, unsigned S_in, unsigned K2,
                                                                     XYZZ<typename Curve::F>* __restrict__ out) {
  using Fb = typename Ar::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t S_out = (S_in + K2 - 1) / K2;
  const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) >> 1;
  if (t >= W * S_out) return;
  const uint32_t w = t / S_out, q = t - w * S_out;
  const uint32_t e0 = q * K2, e1 = min(S_in, e0 + K2);
  const Fb* src = reinterpret_cast<const Fb*>(in) + (size_t)8 * w * S_in;
  typename Ar::A acc = Ar::load(src, e0, h);
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = Ar::add(acc, Ar::load(src, e, h), h != 0);
  Ar::store(reinterpret_cast<Fb*>(out), t, h, acc);
}

// The BN254 G1 reductions over the 29-bit field (acc29::add / dbl; R-form
// arrays in and out, converted on load and store): the chain join and the
// window sums are chains of dependent point additions that run at one or two
// waves per SIMD, so an addition's instruction count is its latency.
template <bool kInRaw, bool kOutRaw>
__global__ __launch_bounds__(kBlock, 2) void seg_reduce29_kernel(const XYZZ<Bn254Fq>* __restrict__ in,
                                                                const uint32_t* __restrict__ beg,
                                                                const uint32_t* __restrict__ end,
                                                                const uint32_t* __restrict__ out_off, uint32_t nseg,
                                                                unsigned K2, XYZZ<Bn254Fq>* __restrict__ out,
                                                                const uint32_t* __restrict__ bucket,
                                                                XYZZ<Bn254Fq>* __restrict__ bucket_sum) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= out_off[nseg]) return;
  const uint32_t s = find_segment(out_off, nseg, t);
  const uint32_t e0 = beg[s] + (t - out_off[s]) * K2;
  const uint32_t e1 = min(end[s], e0 + K2);
  auto load = [&](uint32_t e) { return kInRaw ? acc29::load_raw(in, e) : acc29::load_pt(in, e); };
  acc29::Pt acc = load(e0);
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = acc29::add(acc, load(e));
  if (bucket) {
    if constexpr (kOutRaw) acc29::store_raw(bucket_sum, bucket[s], acc);
    else acc29::store_pt(bucket_sum, bucket[s], acc);
  } else {
    acc29::store_pt(out, t, acc);
  }
}
template <bool kRaw>
__global__ __launch_bounds__(kBlock, 2) void window_segment29_kernel(const XYZZ<Bn254Fq>* __restrict__ bucket_sum,
                                                                    unsigned W, unsigned B, unsigned L,
                                                                    XYZZ<Bn254Fq>* __restrict__ out) {
  const uint32_t S = B / L;
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S) return;
  const uint32_t w = t / S, j = t - w * S;
  const size_t b0 = (size_t)w * B + (size_t)j * L;
  acc29::Pt R{acc29::Acc{}, true}, acc = R;
  for (int k = (int)L - 1; k >= 0; --k) {
    R = acc29::add(R, kRaw ? acc29::load_raw(bucket_sum, b0 + k) : acc29::load_pt(bucket_sum, b0 + k));
    acc = acc29::add(acc, R);
  }
  acc = acc29::add(acc, acc29::small_mul(R, j * L));
  acc29::store_pt(out, t, acc);
}
// The last levels of the window sums in ONE launch per MSM: workgroup w
// reduces window w's S <= kBlock segment sums by a binary tree through LDS
// (log2 S dependent additions, as the one-launch-per-level binary tree,
// without a launch per level: 2^16 has S = 64 -> 6 launches of ~12 us, each
// mostly one latency-bound addition).  (Computing the segment sums in this
// kernel too, window_segment29_kernel's loop, gave wrong window sums on the
// GPU although the loop is the same code -- not understood, so not used.)
__global__ __launch_bounds__(kBlock, 2) void window_tree29_kernel(const XYZZ<Bn254Fq>* __restrict__ in, unsigned S,
                                                                 XYZZ<Bn254Fq>* __restrict__ out) {
  __shared__ acc29::Raw sh[kBlock];
  const uint32_t w = blockIdx.x, j = threadIdx.x;
  acc29::Pt v{acc29::Acc{}, true};
  if (j < S) v = acc29::load_pt(in, (size_t)w * S + j);
  unsigned span = 1;
  while (span < S) span <<= 1;
  for (unsigned half = span >> 1; half >= 1; half >>= 1) {
    if (j >= half && j < 2 * half) acc29::store_raw(sh, j - half, v);
    __syncthreads();
    if (j < half) v = acc29::add(v, acc29::load_raw(sh, j));
    __syncthreads();
  }
  if (j == 0) acc29::store_pt(out, w, v);
}
// window_segment29 + window_tree29 in one launch (S = B / L <= kBlock segment
// sums per window): thread j of workgroup w computes segment j's sum exactly
// as window_segment29_kernel does, then the LDS tree.  Every thread reaches
// every barrier (no early return).  set_variant bit 19 (A/B).
template <bool kRaw>
__global__ __launch_bounds__(kBlock, 2) void window_segtree29_kernel(const XYZZ<Bn254Fq>* __restrict__ bucket_sum,
                                                                    unsigned B, unsigned L,
                                                                    XYZZ<Bn254Fq>* __restrict__ out) {
  __shared__ acc29::Raw sh[kBlock];
  const uint32_t S = B / L;
  const uint32_t w = blockIdx.x, j = threadIdx.x;
  acc29::Pt v{acc29::Acc{}, true};
  if (j < S) {
    const size_t b0 = (size_t)w * B + (size_t)j * L;
    acc29::Pt R{acc29::Acc{}, true};
    v = R;
    for (int k = (int)L - 1; k >= 0; --k) {
      R = acc29::add(R, kRaw ? acc29::load_raw(bucket_sum, b0 + k) : acc29::load_pt(bucket_sum, b0 + k));
      v = acc29::add(v, R);
    }
    v = acc29::add(v, acc29::small_mul(R, j * L));
  }
  unsigned span = 1;
  while (span < S) span <<= 1;
  for (unsigned half = span >> 1; half >= 1; half >>= 1) {
    if (j >= half && j < 2 * half) acc29::store_raw(sh, j - half, v);
    __syncthreads();
    if (j < half) v = acc29::add(v, acc29::load_raw(sh, j));
    __syncthreads();
  }
  if (j == 0) acc29::store_pt(out, w, v);
}

// Window sums of windows with B <= kBlock buckets (c <= 9: the 2^16 MSM) in
// one launch, workgroup w = window w: sum_b (b + 1) B_b = sum_k T_k with the
// suffix sums T_k = sum_{b >= k} B_b, by a Hillis-Steele scan through LDS
// (log2 B levels of one addition) and a binary tree over the T_k (log2 B
// more): 14 dependent additions at B = 128 against window_segment29's L = 2
// running sums plus the (jL) R fix-up (~17) and the tree of the segment sums
// (6), and one launch instead of two.
template <bool kRaw>
__global__ __launch_bounds__(kBlock, 2) void window_scan29_kernel(const XYZZ<Bn254Fq>* __restrict__ bucket_sum,
                                                                 unsigned B, XYZZ<Bn254Fq>* __restrict__ out) {
  __shared__ acc29::Raw sh[kBlock];
  const uint32_t w = blockIdx.x, j = threadIdx.x;
  acc29::Pt v{acc29::Acc{}, true};
  if (j < B) v = kRaw ? acc29::load_raw(bucket_sum, (size_t)w * B + j) : acc29::load_pt(bucket_sum, (size_t)w * B + j);
  for (unsigned d = 1; d < B; d <<= 1) {  // v = T_j
    acc29::store_raw(sh, j, v);
    __syncthreads();
    if (j + d < B) v = acc29::add(v, acc29::load_raw(sh, j + d));
    __syncthreads();
  }
  unsigned span = 1;
  while (span < B) span <<= 1;
  for (unsigned half = span >> 1; half >= 1; half >>= 1) {
    if (j >= half && j < 2 * half) acc29::store_raw(sh, j - half, v);
    __syncthreads();
    if (j < half) v = acc29::add(v, acc29::load_raw(sh, j));
    __syncthreads();
  }
  if (j == 0) acc29::store_pt(out, w, v);
}

__global__ __launch_bounds__(kBlock, 2) void reduce_uniform29_kernel(const XYZZ<Bn254Fq>* __restrict__ in, unsigned W,
                                                                    unsigned S_in, unsigned K2,
                                                                    XYZZ<Bn254Fq>* __restrict__ out) {
  const uint32_t S_out = (S_in + K2 - 1) / K2;
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S_out) return;
  const uint32_t w = t / S_out, q = t - w * S_out;
  const uint32_t e0 = q * K2, e1 = min(S_in, e0 + K2);
  const XYZZ<Bn254Fq>* src = in + (size_t)w * S_in;
  acc29::Pt acc = acc29::load_pt(src, e0);
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = acc29::add(acc, acc29::load_pt(src, e));
  acc29::store_pt(out, t, acc);
}

// Window reduction, stage 2: sum K2 consecutive segment sums per window.
template <class Curve, class Ar = FipsArith<Curve>>
__global__ __launch_bounds__(kBlock, AccWaves<Curve>::value) void reduce_uniform_kernel(const XYZZ<typename Curve::F>* __restrict__ in,
                                                                unsigned W, unsigned S_in, unsigned K2,
                                                                XYZZ<typename Curve::F>* __restrict__ out) {
  uint32_t S_out = (S_in + K2 - 1) / K2;
  uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= W * S_out) return;
  uint32_t w = t / S_out, q = t - w * S_out;
  uint32_t e0 = q * K2, e1 = min(S_in, e0 + K2);
  const XYZZ<typename Curve::F>* src = in + (size_t)w * S_in;
  typename Ar::A acc = Ar::load(src, e0);
  for (uint32_t e = e0 + 1; e < e1; ++e) acc = Ar::add(acc, Ar::load(src, e));
  Ar::store(out, t, acc);
}

// Window reduction by workgroup trees (no per-segment (jL)*R fix-up, two
// launches instead of one per binary-tree level).  Units of a window are
// segments of L buckets; a node over the units [a, a + s) is
//   V  = sum_j [A_j + (j - a) L R_j],   Rs = s L sum_j R_j
// (A_j = sum_k (k + 1) B_{jL+k}, R_j = sum_k B_{jL+k}: the segment's running
// sums), so the root over all units is the window sum sum_b (b + 1) B_b
// (PippengerBase::AccumulateBuckets, pippenger_base.h:36-57).  Two adjacent
// nodes of equal size merge as V = V_l + V_r + Rs_r, Rs = 2 (Rs_l + Rs_r):
// three point operations per merge, none depending on the position.
// kLeafBuckets: leaves are segments read from bucket_sum (grid (groups, W));
// otherwise leaves are the nodes of the previous launch (`nodes_in`, `units`
// per window).  Each workgroup writes the node over its kWinBlock leaves
// (padding leaves are (0, 0): units past the end hold no buckets).
constexpr unsigned kWinBlock = 256;
template <class Curve, bool kLeafBuckets>
__global__ __launch_bounds__(kWinBlock, AccWaves<Curve>::value) void window_tree_kernel(
    const XYZZ<typename Curve::F>* __restrict__ bucket_sum, unsigned B, unsigned L, unsigned log_l,
    const XYZZ<typename Curve::F>* __restrict__ nodes_in, unsigned units, XYZZ<typename Curve::F>* __restrict__ nodes_out) {
  using F = typename HotOf<typename Curve::F>::type;
  using P = XYZZ<F>;
  extern __shared__ uint64_t win_lds[];
  P* lv = reinterpret_cast<P*>(win_lds);           // kWinBlock / 2 right-node V
  P* lr = lv + kWinBlock / 2;                      // and Rs
  const unsigned t = threadIdx.x, w = blockIdx.y;
  const unsigned u = blockIdx.x * kWinBlock + t;   // this thread's leaf unit
  P V = P::zero(), Rs = P::zero();
  if (u < units) {
    if constexpr (kLeafBuckets) {
      const P* bs = reinterpret_cast<const P*>(bucket_sum) + (size_t)w * B + (size_t)u * L;
      for (int k = (int)L - 1; k >= 0; --k) {
        Rs = Rs + bs[k];
        V = V + Rs;
      }
      for (unsigned k = 0; k < log_l; ++k) Rs = Rs.dbl();  // L R
    } else {
      const P* in = reinterpret_cast<const P*>(nodes_in) + 2 * ((size_t)w * units + u);
      V = in[0];
      Rs = in[1];
    }
  }
  for (unsigned k = 0; (1u << k) < kWinBlock; ++k) {
    const unsigned span = 1u << k;
    if ((t & (2 * span - 1)) == span) {  // a right node: hand it to its left neighbour
      lv[t >> (k + 1)] = V;
      lr[t >> (k + 1)] = Rs;
    }
    __syncthreads();
    if ((t & (2 * span - 1)) == 0) {
      const P rv = lv[t >> (k + 1)], rr = lr[t >> (k + 1)];
      V = V + rv + rr;
      Rs = (Rs + rr).dbl();
    }
    __syncthreads();
  }
  if (t == 0) {
    const unsigned groups = gridDim.x;
    P* o = reinterpret_cast<P*>(nodes_out) + 2 * ((size_t)w * groups + blockIdx.x);
    o[0] = V;
    o[1] = Rs;
  }
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
  TA_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_max_), 2 * sizeof(uint32_t), hipHostMallocDefault));
}

template <class Curve>
MsmGpu<Curve>::~MsmGpu() {
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
  for (auto* v : {&gev_sorted_, &gev_acc0_, &gev_acc1_})
    for (auto& e : *v) (void)hipEventDestroy(e);
  if (sort_stream_) (void)hipStreamDestroy(sort_stream_);
  if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
  if (copy_done_) (void)hipEventDestroy(copy_done_);
  for (auto e : chunk_ev_) (void)hipEventDestroy(e);
  if (h_max_) (void)hipHostFree(h_max_);
  if (own_stream_) (void)hipStreamDestroy(stream_);
}

template <class Curve>
void MsmGpu<Curve>::ensure_group_events(unsigned groups) {
  while (gev_sorted_.size() < groups) {
    hipEvent_t a, b, c;
    TA_HIP(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    TA_HIP(hipEventCreate(&b));
    TA_HIP(hipEventCreate(&c));
    gev_sorted_.push_back(a);
    gev_acc0_.push_back(b);
    gev_acc1_.push_back(c);
  }
}

// rocPRIM keys-only onesweep sort of the 64-bit entries on the key bits
// [begin_bit, end_bit) (entry bits 32 + those).  8-bit digits; the tile
// shape is set_variant bits 4-5 (A/B): 0 = 1024 threads x 8 items, 1 =
// rocPRIM's gfx950 default for 64-bit keys, 2 = 512 x 16, 3 = 1024 x 12.
// 2^26 sort: 11.0 / 12.2 / 11.7 ms (2^24: 2.72 / 3.07 / 2.95).  Sorting
// (key, val) u32 pairs took 12.7 ms and the accumulation read two words per
// entry: 2^26 MSM 95.0 -> 92.0 ms with the 64-bit entries.
template <unsigned Threads, unsigned Items>
using OnesweepCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<Threads, Items>, rocprim::kernel_config<Threads, Items>,
                                        8, rocprim::block_radix_rank_algorithm::match>>;

// One rocPRIM onesweep pass (keys only, 1024 x 8 tiles, 8-bit digits) over
// entry bits [bit, end_bit) from `in` to `out`, with the global digit offsets
// given: radix_sort_keys would first read all W*n entries once more for its
// digit histograms (2.4 ms at 2^26); the fused recode counts those digits as
// it computes them (recode_hist_kernel).  rocPRIM's own iteration entry point
// (lookback reset, ordered block ids, batching) does the rest.
namespace {
template <unsigned Threads, unsigned Items, rocprim::block_radix_rank_algorithm Rank>
using MsmOnesweep = rocprim::radix_sort_onesweep_config<rocprim::kernel_config<Threads, Items>,
                                                        rocprim::kernel_config<Threads, Items>, 8, Rank>;
using MsmBlockId = rocprim::detail::block_id_wrapper<unsigned int, true>;
constexpr uint32_t kOnesweepMinTile = 256 * 16;  // smallest tile below (sizes the lookback states)

template <class Cfg>
hipError_t onesweep_pass_cfg(const uint64_t* in, uint64_t* out, uint32_t size, unsigned bit, unsigned end_bit,
                             uint32_t* digit_offsets, uint32_t* offsets_tmp, void* lookback, void* block_id,
                             hipStream_t s) {
  rocprim::empty_type* none = nullptr;
  return rocprim::detail::radix_sort_onesweep_iteration<Cfg, false>(
      in, static_cast<uint64_t*>(nullptr), out, none, none, none, size, digit_offsets, offsets_tmp,
      static_cast<rocprim::detail::onesweep_lookback_state*>(lookback), true, true, rocprim::identity_decomposer{},
      bit, end_bit, MsmBlockId::create(block_id), s, false);
}

// tile shapes (set_variant bits 4-5, A/B): 0 = 1024 x 8 warp-match ranking
hipError_t onesweep_pass(unsigned cfg, const uint64_t* in, uint64_t* out, uint32_t size, unsigned bit,
                         unsigned end_bit, uint32_t* digit_offsets, uint32_t* offsets_tmp, void* lookback,
                         void* block_id, hipStream_t s) {
  using R = rocprim::block_radix_rank_algorithm;
  switch (cfg) {
    case 1:
      return onesweep_pass_cfg<MsmOnesweep<512, 8, R::match>>(in, out, size, bit, end_bit, digit_offsets,
                                                                offsets_tmp, lookback, block_id, s);
    case 2:
      return onesweep_pass_cfg<MsmOnesweep<256, 16, R::match>>(in, out, size, bit, end_bit, digit_offsets,
                                                                 offsets_tmp, lookback, block_id, s);
    case 3:
      return onesweep_pass_cfg<MsmOnesweep<1024, 12, R::match>>(in, out, size, bit, end_bit, digit_offsets,
                                                                  offsets_tmp, lookback, block_id, s);
#ifdef TACHYON_TUNING_KNOBS  // more tile shapes for A/B (TACHYON_ONESWEEP_CFG=4, 5; tuning builds only)
    case 4:
      return onesweep_pass_cfg<MsmOnesweep<1024, 16, R::match>>(in, out, size, bit, end_bit, digit_offsets,
                                                                  offsets_tmp, lookback, block_id, s);
    case 5:
      return onesweep_pass_cfg<MsmOnesweep<512, 16, R::match>>(in, out, size, bit, end_bit, digit_offsets,
                                                                 offsets_tmp, lookback, block_id, s);
#endif
    default:
      return onesweep_pass_cfg<MsmOnesweep<1024, 8, R::match>>(in, out, size, bit, end_bit, digit_offsets,
                                                                 offsets_tmp, lookback, block_id, s);
  }
}
}  // namespace

template <class Curve>
hipError_t MsmGpu<Curve>::sort_entries(void* tmp, size_t& bytes, const uint64_t* in, uint64_t* out, size_t count,
                                       unsigned begin_bit, unsigned end_bit, hipStream_t s) {
  begin_bit += 32;
  end_bit += 32;
  switch (sort_cfg_) {
    case 1:
      return rocprim::radix_sort_keys(tmp, bytes, in, out, count, begin_bit, end_bit, s);
    case 2:
      return rocprim::radix_sort_keys<OnesweepCfg<512, 16>>(tmp, bytes, in, out, count, begin_bit, end_bit, s);
    case 3:
      return rocprim::radix_sort_keys<OnesweepCfg<1024, 12>>(tmp, bytes, in, out, count, begin_bit, end_bit, s);
    default:
      return rocprim::radix_sort_keys<OnesweepCfg<1024, 8>>(tmp, bytes, in, out, count, begin_bit, end_bit, s);
  }
}

// Chain tables from the per-thread run flags: a chain = the pieces of one
// bucket across consecutive threads (head/tail pieces), numbered by a scan
// of the chain starts; then each chain's first-level piece count, the chain
// count and the longest chain, read back into h_max_ (pinned) on stream s.
template <class Curve>
void MsmGpu<Curve>::build_chains(const uint32_t* flags, const uint32_t* last, size_t T, unsigned K2,
                                 uint32_t* is_start, uint32_t* cid, uint32_t* cbeg, uint32_t* cend,
                                 uint32_t* cbucket, uint32_t* lcnt, uint32_t* dscal, hipStream_t s) {
  hipLaunchKernelGGL(chain_mark_kernel, dim3(grid_for(T + 1)), dim3(kBlock), 0, s, flags, (uint32_t)T, is_start,
                     dscal + 1);
  size_t scan_bytes = 0;
  TA_HIP(rocprim::exclusive_scan(nullptr, scan_bytes, is_start, cid, 0u, T + 1, rocprim::plus<uint32_t>(), s));
  void* scan_tmp = scan_tmp_.ensure(scan_bytes);
  TA_HIP(rocprim::exclusive_scan(scan_tmp, scan_bytes, is_start, cid, 0u, T + 1, rocprim::plus<uint32_t>(), s));
  hipLaunchKernelGGL(chain_build_kernel, dim3(grid_for(T)), dim3(kBlock), 0, s, flags, last, cid, (uint32_t)T, cbeg,
                     cend, cbucket, dscal);
  hipLaunchKernelGGL(seg_count_kernel, dim3(grid_for(T + 1)), dim3(kBlock), 0, s, cbeg, cend, dscal, (uint32_t)T, K2,
                     lcnt, dscal + 1);
  TA_HIP(hipGetLastError());
  TA_HIP(hipMemcpyAsync(h_max_, dscal, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
}

template <class Curve>
void MsmGpu<Curve>::enqueue(const Aff* d_bases, const Fr* d_scalars, size_t n, const MsmPlan& plan,
                            Point* d_windows) {
  // Ws = the windows each scalar emits (plan.active()); Wt = all windows of
  // the scalar (the recode's carry chain), the range starting at window w0;
  // W = the window sums this run computes: Ws, or Ws per MSM of a batch over
  // shared bases (run_batch: batch_ MSMs of n / batch_ points each, MSM g's
  // windows g Ws .. g Ws + Ws - 1 in the key space)
  const unsigned Ws = plan.active(), Wt = plan.windows, wr0 = plan.w_begin, B = plan.buckets, c = plan.c;
  // (a fold: Wt / fold_ key windows over fold_ copies of the bases, run_windows checked it)
  const unsigned W = (fold_ > 1 ? Wt / fold_ : Ws) * batch_;
  const uint32_t fold_w = fold_ > 1 ? Wt / fold_ : 0u;
  const uint32_t glen = batch_ > 1 ? (uint32_t)(n / batch_) : 0u;
  const uint32_t gstep = batch_distinct_ ? 0u : glen;  // shared bases (run_batch) or one array per MSM (run_groups)
  const uint32_t fold_n = gstep ? glen : (uint32_t)n;   // points per fold copy
  const size_t entries = n * Ws;
  const size_t nb = (size_t)W * B;
  if (n >= (size_t(1) << 31)) throw std::runtime_error("tachyon_mi355x: MSM size must be < 2^31 per device");
  if (((uint64_t)W << c) > (uint64_t(1) << 32))  // 32-bit keys (window << c | digit)
    throw std::runtime_error("tachyon_mi355x: too many windows for 32-bit bucket keys (MSM batch too large)");
  const uint32_t K = plan.K;
  // window groups: group g covers windows [g*G, min(W, (g+1)*G)), i.e. the
  // contiguous entry range [w0*n, w1*n); its sort (sort stream) overlaps the
  // accumulation of the previous group (MSM stream) -- the sort is HBM-bound,
  // the accumulation VALU-bound, so they share the CUs well
  // (a batch or a fold sorts all its windows together: the recode writes the
  // entries by scalar window, not by key window)
  const unsigned G = (batch_ > 1 || fold_ > 1) ? W : std::max(1u, std::min(plan.group, W));
  const unsigned ngroups = (W + G - 1) / G;
  const size_t epw = entries / W;  // entries per key window's share of the array (n without a batch)
  size_t T = 0;  // accumulation threads over all groups
  for (unsigned g = 0; g < ngroups; ++g) {
    const unsigned w0 = g * G, w1 = std::min(W, w0 + G);
    T += ((size_t)(w1 - w0) * epw + K - 1) / K;
  }
  if (T >= (size_t(1) << 31)) throw std::runtime_error("tachyon_mi355x: MSM too large for the chunking");
  ensure_group_events(ngroups);
  // the sort runs on its own stream only when the windows are pipelined
  // (created on first use: every extra stream may take one of the process's
  // few hardware queues)
  if (ngroups > 1 && !sort_stream_) TA_HIP(hipStreamCreateWithFlags(&sort_stream_, hipStreamNonBlocking));
  hipStream_t sort_stream = ngroups > 1 ? sort_stream_ : stream_;

  // (64 bytes of slack: the LDS-staged entry chunks read up to 7 entries past a lane's last)
  uint64_t* ents = static_cast<uint64_t*>(ents_.ensure(entries * 8 + 64));
  uint64_t* ents2 = static_cast<uint64_t*>(ents2_.ensure(entries * 8 + 64));
  // bucket sums and pieces in the 144-byte Raw format after the 29-bit
  // accumulation (not with the workgroup-tree window sums, an A/B path in R form)
  // (BLS12-381 G1: 224-byte Pol28::Raw after the 28-bit accumulation, read by
  // the 28-bit reductions -- not with the FIPS reductions of bit 22 or the
  // two-level window sums of bit 23; every join level raw, so the level buffer
  // takes the raw slot too)
  bool raw = false;
  size_t slot = sizeof(Point), lvl_slot = sizeof(Point);
  if constexpr (std::is_same_v<Curve, Bn254G1>) {
    raw = acc29_ && !tree_reduce_;
    if (raw) slot = sizeof(acc29::Raw);
  }
  if constexpr (std::is_same_v<Curve, Bls381G1>) {
    raw = acc28_ && !tree_reduce_ && !(variant_ & ((1 << 22) | (1 << 23)));
    if (raw) slot = lvl_slot = sizeof(Pol28::Raw);
  }
  // (G2 lane pairs over the limb fields: 8 raw components per point -- 448 B
  // BLS12-381, 288 B BN254 -- not with the FIPS pair reductions (bit 22), the
  // two-level (bit 23) or two-pass (bit 24) window sums)
  if constexpr (std::is_same_v<Curve, Bn254G2> || std::is_same_v<Curve, Bls381G2>) {
    using LimbPol = std::conditional_t<std::is_same_v<Curve, Bls381G2>, PairPol28, PairPol29>;
    raw = pair_acc_ && pair_limb_ && !tree_reduce_ && !(variant_ & ((1 << 22) | (1 << 23) | (1 << 24)));
    if (raw) slot = lvl_slot = 8 * sizeof(typename LimbPol::F);
  }
  Point* bucket_sum = static_cast<Point*>(buckets_.ensure(nb * slot));
  Point* pieces = static_cast<Point*>(part_a_.ensure(2 * T * slot));
  Point* lvl_buf = static_cast<Point*>(part_b_.ensure((2 * T / kJoinFanLong + T + 2) * lvl_slot));
  // Where the chain tables (and the join levels' offsets) are built -- they
  // depend only on the sorted keys (chain_flags_kernel), so they need not wait
  // for the accumulation:
  //  * kChainsInStream: windows with <= 16 K buckets in all (2^16, 2^17):
  //    before the accumulation, with every level's offsets by one workgroup
  //    from the device-side counts (join_offsets_all_kernel); the host reads
  //    the chain count back while the accumulation runs;
  //  * kChainsBefore: other MSMs of < 2^21 accumulation threads: the tables
  //    before the accumulation, the read-back during it, the offsets after;
  //  * kChainsAfter: from the accumulation's flags after it (large MSMs,
  //    where the tables cost more than the read-back gap they hide, and
  //    window-group pipelines).
  // All on the MSM's one stream: a second stream for the tables measured the
  // same alone, but it shifts the process's stream -> hardware-queue
  // round-robin (4 queues), which put the Groth16 prover's G1 and G2 MSM
  // streams on one queue and serialised them (2^20 proof 12.9 -> 14.3 ms,
  // profiles/r03e/ab_groth16_side_stream.log).
  const ChainMode chain_mode = ngroups != 1                                        ? kChainsAfter
                               : (size_t)W * B <= 16384 && T < (size_t(1) << 20) ? kChainsInStream
                               : T < (size_t(1) << 21)                            ? kChainsBefore
                                                                                  : kChainsAfter;
  const bool early_chains = chain_mode != kChainsAfter;
  const unsigned lv_max =
      chain_mode == kChainsInStream ? join_levels((uint32_t)std::min<size_t>(2 * T, ~0u), kJoinFanLong) + 1 : 0;
  uint32_t* early_ltab =
      chain_mode == kChainsInStream ? static_cast<uint32_t*>(lofs_.ensure(lv_max * (T + 2) * 4)) : nullptr;
  uint32_t* tflags = static_cast<uint32_t*>(start_.ensure(2 * T * 4));
  uint32_t* tlast = static_cast<uint32_t*>(end_.ensure(2 * T * 4));
  uint32_t* cflags = early_chains ? tflags + T : tflags;  // what the chain kernels read
  uint32_t* clast = early_chains ? tlast + T : tlast;
  uint32_t* is_start = static_cast<uint32_t*>(cnt_.ensure((T + 1) * 4));
  uint32_t* cid = static_cast<uint32_t*>(off_a_.ensure((T + 1) * 4));
  // chain tables: beg, end, bucket, level counts/offsets (<= T chains)
  uint32_t* ctab = static_cast<uint32_t*>(off_b_.ensure((6 * (T + 2) + 4) * 4));
  uint32_t* cbeg = ctab;
  uint32_t* cend = ctab + (T + 2);
  uint32_t* cbucket = ctab + 2 * (T + 2);
  uint32_t* lcnt = ctab + 3 * (T + 2);
  uint32_t* dscal = ctab + 6 * (T + 2);  // [0] nchains, [1] max chain length

  unsigned wbits = 0;
  while ((1u << wbits) < W) ++wbits;
  const unsigned key_bits = (G == 1) ? c : c + wbits;  // the window bits only matter within a multi-window group
  // recode fused with the first (low byte) radix pass; one sort group only
  // (the scatter stages a block's spt x 256 x W entries in LDS, <= 128 KiB)
  const uint32_t spt = recode_spt_;
  const bool narrow = key_bits <= 24 && !wide_stage_;  // 7-byte LDS staging in the scatter
  const size_t scatter_lds = (size_t)spt * kBlock * Ws * (narrow ? 7 : sizeof(uint64_t));
  const bool fused = fuse_recode_ && G == W && scatter_lds <= 128 * 1024;
  const unsigned sort_begin = fused ? std::min(8u, key_bits) : 0u;
  // onesweep passes fed with digit counts from the recode (places = the
  // 8-bit digits after the fused low byte); rocPRIM's radix_sort_keys
  // otherwise (set_variant bit 10, or other tile shapes, or > 2 places)
  const unsigned places = (key_bits - sort_begin + 7) / 8;
  const bool own_sort = fused && !rocprim_hist_ && places <= 2 && entries < (size_t(1) << 32);
  last_schedule_ = (fused ? kSchedFusedRecode : 0u) | (own_sort ? kSchedRecodeFedSort : 0u) |
                   (fused && narrow ? kSchedNarrowStaging : 0u);
  uint32_t* digit_off = nullptr;

  if (profile_) TA_HIP(hipEventRecord(ev_[1], stream_));
  if (fused) {
    const uint32_t nblocks = (uint32_t)((n + spt * kBlock - 1) / (spt * kBlock));
    const size_t hn = (size_t)256 * nblocks;
    const unsigned later_places = own_sort ? places : 0;
    // slot chunks: <= 1024 chunks of >= 4 blocks (bin_chunk_scan_kernel's loop, bin_offsets_kernel's rows)
    const uint32_t bper = std::max<uint32_t>(4, (nblocks + 1023) / 1024), bchunks = (nblocks + bper - 1) / bper;
    uint32_t* hist = static_cast<uint32_t*>(
        hist_.ensure(((2 + later_places) * hn + 5 * 256 + 2 * (size_t)bchunks * 256 + 256) * 4));
    uint32_t* hoff = hist + hn;
    uint32_t* later = hist + 2 * hn;
    uint32_t* digit_cnt = later + later_places * hn;  // 2 x 256 counts, 2 x 256 offsets, 256 spare
    uint32_t* bcsum = digit_cnt + 5 * 256;            // [chunk][bin] sums, then prefixes, then the bin totals
    uint32_t* bcpre = bcsum + (size_t)bchunks * 256;
    uint32_t* btotal = bcpre + (size_t)bchunks * 256;
    hipLaunchKernelGGL(recode_hist_kernel<Fr>, dim3(nblocks), dim3(kBlock), 0, stream_, d_scalars, (uint32_t)n, c,
                       Wt, wr0, Ws, nblocks, spt, later_places, hist, later, reinterpret_cast<uint4*>(bucket_sum),
                       nb * slot / 16, glen, gstep, fold_w, fold_n);
    TA_HIP(hipGetLastError());
    if (later_places > 0) {
      digit_off = digit_cnt + 2 * 256;
      TA_HIP(hipMemsetAsync(digit_cnt, 0, 2 * 256 * 4, stream_));
      // (>= 256 chunks: a 2^16 MSM's 128 recode blocks in one chunk took 17 us of serial loads)
      const uint32_t per_chunk = std::clamp<uint32_t>(nblocks / 256, 4, 128), chunks = (nblocks + per_chunk - 1) / per_chunk;
      hipLaunchKernelGGL(digit_count_kernel, dim3(chunks, later_places), dim3(kBlock), 0, stream_, later, nblocks,
                         per_chunk, digit_cnt);
      hipLaunchKernelGGL(digit_scan_kernel, dim3(later_places), dim3(kBlock), 0, stream_, digit_cnt, digit_off);
      TA_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(bin_chunk_sums_kernel, dim3(bchunks), dim3(kBlock), 0, stream_, hist, nblocks, bper, bcsum);
    hipLaunchKernelGGL(bin_chunk_scan_kernel, dim3(256), dim3(kBlock), 0, stream_, bcsum, bchunks, bcpre, btotal);
    hipLaunchKernelGGL(bin_offsets_kernel, dim3(bchunks), dim3(kBlock), 0, stream_, hist, nblocks, bper, bcpre, btotal,
                       hoff);
    TA_HIP(hipGetLastError());
    // the scattered entries are fully sorted when the key has <= 8 bits; the
    // own onesweep passes ping-pong from the scatter's output and end in ents2
    uint64_t* dst = own_sort ? (places % 2 == 0 ? ents2 : ents) : (sort_begin < key_bits ? ents : ents2);
    auto* scatter = narrow ? &recode_scatter_kernel<Fr, true> : &recode_scatter_kernel<Fr, false>;
    // dynamic LDS above 64 KiB: raise the launched instance's limit once (per instantiation)
    if (scatter_lds > 64 * 1024 && !scatter_lds_set_[narrow ? 1 : 0]) {
      TA_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(scatter), hipFuncAttributeMaxDynamicSharedMemorySize,
                                 128 * 1024));
      scatter_lds_set_[narrow ? 1 : 0] = true;
    }
    hipLaunchKernelGGL(scatter, dim3(nblocks), dim3(kBlock), scatter_lds, stream_, d_scalars, (uint32_t)n, c, Wt, wr0,
                       Ws, nblocks, spt, hist, hoff, dst, glen, gstep, fold_w, fold_n);
  } else {
    hipLaunchKernelGGL(recode_kernel<Fr>, dim3(grid_for(n)), dim3(kBlock), 0, stream_, d_scalars, (uint32_t)n, c,
                       Wt, wr0, Ws, ents, glen, gstep, fold_w, fold_n);
  }
  TA_HIP(hipGetLastError());
  // every bucket without an entry stays the identity (the fused recode clears them)
  if (!fused) TA_HIP(hipMemsetAsync(bucket_sum, 0, nb * slot, stream_));
  TA_HIP(hipEventRecord(ev_[2], stream_));  // recode done (also the profile mark)
  if (sort_stream != stream_) TA_HIP(hipStreamWaitEvent(sort_stream, ev_[2], 0));

  // ---- per group: radix sort of its (window, bucket, point) entries, then accumulation ----
  const size_t max_group_entries = (size_t)G * epw;
  size_t sort_bytes = 0;
  void* sort_tmp = nullptr;
  uint8_t* os_tmp = nullptr;  // own passes: lookback states, block id, spare offsets
  if (own_sort) {
    const size_t lookback_bytes = (size_t)256 * ((entries + kOnesweepMinTile - 1) / kOnesweepMinTile) * 4;
    os_tmp = static_cast<uint8_t*>(sort_tmp_.ensure(lookback_bytes + 1024 + 256 * 4));
  } else {
    TA_HIP(sort_entries(nullptr, sort_bytes, ents, ents2, max_group_entries, sort_begin, key_bits, sort_stream));
    sort_tmp = sort_tmp_.ensure(sort_bytes);
  }
  size_t tbase = 0;
  acc_launches_ = ngroups;
  for (unsigned g = 0; g < ngroups; ++g) {
    const unsigned w0 = g * G, w1 = std::min(W, w0 + G);
    const size_t e0 = (size_t)w0 * epw, ecount = (size_t)(w1 - w0) * epw;
    size_t bytes = sort_bytes;
    if (own_sort) {
      const size_t lookback_bytes = (size_t)256 * ((entries + kOnesweepMinTile - 1) / kOnesweepMinTile) * 4;
      const uint64_t* src = places % 2 == 0 ? ents2 : ents;
      uint64_t* out = places % 2 == 0 ? ents : ents2;
      for (unsigned q = 0; q < places; ++q) {
        TA_HIP(onesweep_pass(sort_cfg_, src, out, (uint32_t)entries, 32 + sort_begin + 8 * q, 32 + key_bits, digit_off + q * 256,
                             reinterpret_cast<uint32_t*>(os_tmp + lookback_bytes + 1024), os_tmp,
                             os_tmp + lookback_bytes, sort_stream));
        src = out;
        out = out == ents ? ents2 : ents;
      }
    } else if (sort_begin < key_bits) {
      TA_HIP(sort_entries(sort_tmp, bytes, ents + e0, ents2 + e0, ecount, sort_begin, key_bits, sort_stream));
    }
    if (profile_ && g + 1 == ngroups) TA_HIP(hipEventRecord(ev_[3], sort_stream));  // last sort done
    if (sort_stream != stream_) {
      TA_HIP(hipEventRecord(gev_sorted_[g], sort_stream));
      TA_HIP(hipStreamWaitEvent(stream_, gev_sorted_[g], 0));
    }
    if (g == 0 && pending_host_bases_) {
      // host-resident bases: their upload (the larger of the two) runs on its
      // own stream while the recode and the sort run; the host call returns
      // once the pageable copy is staged, i.e. with the GPU busy meanwhile
      if (!copy_stream_) TA_HIP(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
      if (!copy_done_) TA_HIP(hipEventCreateWithFlags(&copy_done_, hipEventDisableTiming));
      TA_HIP(hipMemcpyAsync(const_cast<Aff*>(d_bases), pending_host_bases_, n * sizeof(Aff), hipMemcpyHostToDevice,
                            copy_stream_));
      TA_HIP(hipEventRecord(copy_done_, copy_stream_));
      TA_HIP(hipStreamWaitEvent(stream_, copy_done_, 0));
      pending_host_bases_ = nullptr;
    }
    const size_t Tg = (ecount + K - 1) / K;
    if (chain_mode == kChainsInStream) {
      hipLaunchKernelGGL(chain_flags_kernel, dim3(grid_for(T)), dim3(kBlock), 0, stream_, ents2, c, (uint64_t)e0,
                         (uint64_t)(e0 + ecount), K, (uint32_t)T, cflags, clast);
      TA_HIP(hipGetLastError());
      build_chains(cflags, clast, T, plan.K2, is_start, cid, cbeg, cend, cbucket, lcnt, dscal, stream_);
      hipLaunchKernelGGL(join_offsets_all_kernel, dim3(1), dim3(kJoinOffBlock), 0, stream_, cbeg, cend, dscal,
                         plan.K2, (uint32_t)T, lv_max, (size_t)T + 2, early_ltab);
      TA_HIP(hipGetLastError());
      TA_HIP(hipEventRecord(ev_[7], stream_));  // chain count and longest chain read back
    } else if (chain_mode == kChainsBefore) {
      hipLaunchKernelGGL(chain_flags_kernel, dim3(grid_for(T)), dim3(kBlock), 0, stream_, ents2, c, (uint64_t)e0,
                         (uint64_t)(e0 + ecount), K, (uint32_t)T, cflags, clast);
      TA_HIP(hipGetLastError());
      build_chains(cflags, clast, T, plan.K2, is_start, cid, cbeg, cend, cbucket, lcnt, dscal, stream_);
      TA_HIP(hipEventRecord(ev_[7], stream_));
    }
    if (profile_) TA_HIP(hipEventRecord(gev_acc0_[g], stream_));
    // the entry reads of the limb-field accumulations (seg_acc_limb_body's
    // kEnt): LDS-staged chunks when every lane's first entry is 16-byte
    // aligned, else 16-byte pairs; set_variant bit 25: the 8-byte loads (A/B)
    const int ent_mode = (variant_ & (1u << 25)) ? 0 : (K % 2 == 0 && e0 % 2 == 0) ? 2 : 1;
    if constexpr (std::is_same_v<Curve, Bn254G1>) {
      if (acc29_) last_schedule_ |= kSchedAcc29;
      if (acc29_ && acc29_mode_ == 0 && ent_mode == 2) last_schedule_ |= kSchedEntStaged;
      using Acc29K = decltype(&seg_acc29_kernel<0, true, 0>);
      const Acc29K k0 = ent_mode == 2 ? (raw ? seg_acc29_kernel<0, true, 2> : seg_acc29_kernel<0, false, 2>)
                        : ent_mode == 1 ? (raw ? seg_acc29_kernel<0, true, 1> : seg_acc29_kernel<0, false, 1>)
                                        : (raw ? seg_acc29_kernel<0, true, 0> : seg_acc29_kernel<0, false, 0>);
      if (acc29_)  // 29-bit-limb accumulation (BN254 G1 default; set_variant bits 13 / 17: base prefetch A/B)
        hipLaunchKernelGGL(acc29_mode_ == 2 ? (raw ? seg_acc29_kernel<2, true, 0> : seg_acc29_kernel<2, false, 0>)
                           : acc29_mode_ == 1 ? (raw ? seg_acc29_kernel<1, true, 0> : seg_acc29_kernel<1, false, 0>)
                                              : k0,
                           dim3(grid_for(Tg)),
                           dim3(kBlock), 0, stream_, d_bases, ents2, c,
                           (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_, bucket_sum, pieces,
                           tflags, tlast);
      else
        hipLaunchKernelGGL(seg_acc_kernel<Curve>, dim3(grid_for(Tg)), dim3(kBlock), 0, stream_, d_bases, ents2, c,
                           (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_, bucket_sum, pieces,
                           tflags, tlast);
    } else if constexpr (std::is_same_v<Curve, Bls381G1>) {
      if (acc28_) {
        last_schedule_ |= kSchedAcc28;
        if (ent_mode == 2) last_schedule_ |= kSchedEntStaged;
        using Acc28K = decltype(&seg_acc28_kernel<0, false>);
        const Acc28K k28 = raw ? (ent_mode == 2 ? seg_acc28_kernel<2, true> : ent_mode == 1 ? seg_acc28_kernel<1, true>
                                                                                          : seg_acc28_kernel<0, true>)
                               : (ent_mode == 2 ? seg_acc28_kernel<2, false> : ent_mode == 1 ? seg_acc28_kernel<1, false>
                                                                                           : seg_acc28_kernel<0, false>);
        hipLaunchKernelGGL(k28, dim3(grid_for(Tg)), dim3(kBlock), 0, stream_, d_bases, ents2, c,
                           (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_, bucket_sum, pieces,
                           tflags, tlast);
      } else {
        hipLaunchKernelGGL(seg_acc_kernel<Curve>, dim3(grid_for(Tg)), dim3(kBlock), 0, stream_, d_bases, ents2, c,
                           (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_, bucket_sum, pieces,
                           tflags, tlast);
      }
    } else if constexpr (std::is_same_v<Curve, Bn254G2> || std::is_same_v<Curve, Bls381G2>) {
      // a lane pair per virtual thread (set_variant bit 15, A/B; bit 16: inline 12-limb products)
      constexpr bool kCallDefault = Curve::F::Base::N == 12;
      auto* pair_kernel = pair_inline_ ? &seg_acc_pair_kernel<Curve, false> : &seg_acc_pair_kernel<Curve, kCallDefault>;
      // (kCallDefault is false for 8-limb fields: both entries are the inline kernel there)
      if (pair_acc_) last_schedule_ |= kSchedLanePair;
      // the limb-field pairs (BLS12-381: 28-bit, BN254: 29-bit; bit 20 restores the FIPS pair)
      using LimbPol = std::conditional_t<std::is_same_v<Curve, Bls381G2>, PairPol28, PairPol29>;
      if (pair_acc_ && pair_limb_) {
        last_schedule_ |= std::is_same_v<Curve, Bls381G2> ? kSchedAcc28 : kSchedAcc29;
        // staged entries for BLS12-381 (2^24 accumulation 88.7 -> 88.0 ms); BN254 G2
        // measured 12.21 -> 12.32 ms at 2^22 with them (profiles/r06i/ab_entries_staged.log)
        const bool staged = ent_mode == 2 && std::is_same_v<Curve, Bls381G2>;
        if (staged) last_schedule_ |= kSchedEntStaged;
        auto* limb_kernel = staged ? (raw ? &seg_acc_pair_limb_kernel<LimbPol, true, true>
                                          : &seg_acc_pair_limb_kernel<LimbPol, true, false>)
                                   : (raw ? &seg_acc_pair_limb_kernel<LimbPol, false, true>
                                          : &seg_acc_pair_limb_kernel<LimbPol, false, false>);
        hipLaunchKernelGGL(limb_kernel, dim3(grid_for(2 * Tg)), dim3(kBlock), 0, stream_,
                           d_bases, ents2, c, (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_,
                           bucket_sum, pieces, tflags, tlast);
      } else if (pair_acc_)
        hipLaunchKernelGGL(pair_kernel, dim3(grid_for(2 * Tg)), dim3(kBlock), 0, stream_, d_bases,
                           ents2, c, (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_, bucket_sum,
                           pieces, tflags, tlast);
      else
        hipLaunchKernelGGL(seg_acc_kernel<Curve>, dim3(grid_for(Tg)), dim3(kBlock), 0, stream_, d_bases, ents2, c,
                           (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_, bucket_sum, pieces,
                           tflags, tlast);
    } else {
      hipLaunchKernelGGL(seg_acc_kernel<Curve>, dim3(grid_for(Tg)), dim3(kBlock), 0, stream_, d_bases, ents2, c,
                         (uint64_t)e0, (uint64_t)(e0 + ecount), (uint64_t)tbase, K, idx_mask_, bucket_sum, pieces,
                         tflags, tlast);
    }
    TA_HIP(hipGetLastError());
    if (profile_) TA_HIP(hipEventRecord(gev_acc1_[g], stream_));
    tbase += Tg;
  }
  if (profile_) TA_HIP(hipEventRecord(ev_[4], stream_));        // last accumulation done

  // G2: the lane-pair reductions with the lane-pair accumulation (set_variant bit 15 restores both)
  constexpr bool kG2 = std::is_same_v<Curve, Bn254G2> || std::is_same_v<Curve, Bls381G2>;
  const bool pair_reduce = kG2 && pair_acc_;
  const unsigned lanes = pair_reduce ? 2 : 1;  // threads per point
  auto* seg_reduce = &seg_reduce_kernel<Curve>;
  auto* win_segment = &window_segment_kernel<Curve>;
  auto* win_reduce = &reduce_uniform_kernel<Curve>;
  decltype(win_segment) rsum_pass1 = nullptr, rsum_pass2 = nullptr, rsum_fix = nullptr;  // G2 two-pass sums (bit 24)
  if constexpr (kG2) {
    if (pair_reduce) {
      using LimbPol = std::conditional_t<std::is_same_v<Curve, Bls381G2>, PairPol28, PairPol29>;
      if (pair_limb_ && !(variant_ & (1 << 22))) {  // the limb-field pair additions (bit 22: the FIPS pair)
        seg_reduce = raw ? &seg_reduce_pair_kernel<Curve, LimbPairArith<LimbPol, true, true>>
                         : &seg_reduce_pair_kernel<Curve, LimbPairArith<LimbPol>>;
        win_segment = raw ? &window_segment_pair_kernel<Curve, LimbPairArith<LimbPol, true, false>>
                          : &window_segment_pair_kernel<Curve, LimbPairArith<LimbPol>>;
        win_reduce = &reduce_uniform_pair_kernel<Curve, LimbPairArith<LimbPol>>;
        rsum_pass1 = &window_rsum_pair_kernel<Curve, LimbPairArith<LimbPol>>;
        rsum_pass2 = &window_rsum_total_pair_kernel<Curve, LimbPairArith<LimbPol>>;
        rsum_fix = &window_rsum_fix_pair_kernel<Curve, LimbPairArith<LimbPol>>;
      } else {
        seg_reduce = &seg_reduce_pair_kernel<Curve>;
        win_segment = &window_segment_pair_kernel<Curve>;
        win_reduce = &reduce_uniform_pair_kernel<Curve>;
        rsum_pass1 = &window_rsum_pair_kernel<Curve, FipsPairArith<Curve>>;
        rsum_pass2 = &window_rsum_total_pair_kernel<Curve, FipsPairArith<Curve>>;
        rsum_fix = &window_rsum_fix_pair_kernel<Curve, FipsPairArith<Curve>>;
      }
    }
  }
  // BLS12-381 G1: the reductions over the 28-bit field with the 28-bit accumulation
  // (set_variant bit 22: the FIPS reductions)
  if constexpr (std::is_same_v<Curve, Bls381G1>) {
    if (acc28_ && !(variant_ & (1 << 22))) {
      seg_reduce = raw ? &seg_reduce_kernel<Curve, Limb28ArithT<true, true>> : &seg_reduce_kernel<Curve, Limb28Arith>;
      win_segment = raw ? &window_segment_kernel<Curve, Limb28ArithT<true, false>>
                        : &window_segment_kernel<Curve, Limb28Arith>;
      win_reduce = &reduce_uniform_kernel<Curve, Limb28Arith>;
    }
  }
  // BN254 G1: the reductions over the 29-bit field with the 29-bit accumulation
  // (set_variant bit 18 restores the FIPS field for both)
  if constexpr (std::is_same_v<Curve, Bn254G1>) {
    if (acc29_) {
      seg_reduce = &seg_reduce29_kernel<false, false>;
      win_segment = raw ? &window_segment29_kernel<true> : &window_segment29_kernel<false>;
      win_reduce = &reduce_uniform29_kernel;
    }
  }
  // ---- join buckets that cross thread boundaries ----
  // (the chain count and the longest chain decide the levels: read back
  // while the accumulation runs when early_chains)
  if (early_chains && (variant_ & (1 << 21))) {  // debug: pre-derived flags == the accumulation's
    uint32_t* mism = static_cast<uint32_t*>(check_.ensure(sizeof(uint32_t)));
    TA_HIP(hipMemsetAsync(mism, 0, sizeof(uint32_t), stream_));
    hipLaunchKernelGGL(chain_flags_check_kernel, dim3(grid_for(T)), dim3(kBlock), 0, stream_, tflags, tlast, cflags,
                       clast, (uint32_t)T, mism);
    TA_HIP(hipGetLastError());
    uint32_t h = 0;
    TA_HIP(hipMemcpyAsync(&h, mism, sizeof(h), hipMemcpyDeviceToHost, stream_));
    TA_HIP(hipStreamSynchronize(stream_));
    if (h) throw std::runtime_error("tachyon_mi355x: chain flags derived before the accumulation differ from its own");
    last_schedule_ |= kSchedChainsChecked;
  }
  if (early_chains) {
    TA_HIP(hipEventSynchronize(ev_[7]));
  } else {
    build_chains(cflags, clast, T, plan.K2, is_start, cid, cbeg, cend, cbucket, lcnt, dscal, stream_);
    TA_HIP(hipStreamSynchronize(stream_));
  }
  const uint32_t nchains = h_max_[0], max_len = h_max_[1];
  const unsigned K2 = join_fan_in(max_len, plan.K2, T);
  const unsigned levels = join_levels(max_len, K2);
  last_levels_ = levels;
  if (nchains > 0 && levels > 0) {
    // phase 1: every level's output offsets (level l's table: segment s of
    // level l + 1 = [off_l[s], off_l[s + 1])), one table per level -- already
    // on the device for the small MSMs (join_offsets_all_kernel)
    const bool in_stream = chain_mode == kChainsInStream;
    if (in_stream && levels > lv_max) throw std::runtime_error("tachyon_mi355x: MSM join levels exceed their bound");
    const size_t stride = in_stream ? T + 2 : (size_t)nchains + 2;
    uint32_t* ltab = in_stream ? early_ltab : static_cast<uint32_t*>(lofs_.ensure(levels * stride * 4));
    hipStream_t off_stream = stream_;
    if (!in_stream) {
      const bool small = nchains <= kJoinSmallChains;  // offsets in one workgroup
      size_t scan2_bytes = 0;
      void* scan_tmp = nullptr;
      if (!small) {
        TA_HIP(rocprim::exclusive_scan(nullptr, scan2_bytes, lcnt, ltab, 0u, (size_t)nchains + 1,
                                       rocprim::plus<uint32_t>(), off_stream));
        scan_tmp = scan_tmp_.ensure(scan2_bytes);
      }
      for (unsigned l = 0; l < levels; ++l) {
        uint32_t* loff = ltab + l * stride;
        const uint32_t* pbeg = l == 0 ? cbeg : ltab + (l - 1) * stride;
        const uint32_t* pend = l == 0 ? cend : pbeg + 1;
        if (small) {
          hipLaunchKernelGGL(join_offsets_kernel, dim3(1), dim3(kJoinOffBlock), 0, off_stream, pbeg,
                             l == 0 ? pend : nullptr, nchains, K2, loff);
        } else {
          if (l > 0 || K2 != plan.K2)  // (level 0's counts came with the read-back, for plan.K2)
            hipLaunchKernelGGL(seg_count_kernel, dim3(grid_for((size_t)nchains + 1)), dim3(kBlock), 0, off_stream,
                               pbeg, pend, nullptr, nchains, K2, lcnt, nullptr);
          TA_HIP(rocprim::exclusive_scan(scan_tmp, scan2_bytes, lcnt, loff, 0u, (size_t)nchains + 1,
                                         rocprim::plus<uint32_t>(), off_stream));
        }
      }
      TA_HIP(hipGetLastError());
    }
    // phase 2: the levels, back to back on the MSM stream
    const Point* cur = pieces;
    size_t cur_items = 2 * T;
    Point* dst_bufs[2] = {lvl_buf, pieces};  // pieces is free once level 0 has read it
    for (unsigned l = 0; l < levels; ++l) {
      const bool last = (l + 1 == levels);
      const uint32_t* loff = ltab + l * stride;
      const uint32_t* cur_beg = l == 0 ? cbeg : ltab + (l - 1) * stride;
      const uint32_t* cur_end = l == 0 ? cend : cur_beg + 1;
      size_t out_items = cur_items / K2 + nchains + 1;
      Point* dst = dst_bufs[l & 1];
      auto* level_kernel = seg_reduce;
      if constexpr (std::is_same_v<Curve, Bn254G1>) {
        if (raw)  // Raw pieces into level 0, Raw bucket sums out of the last level
          level_kernel = l == 0 ? (last ? &seg_reduce29_kernel<true, true> : &seg_reduce29_kernel<true, false>)
                                : (last ? &seg_reduce29_kernel<false, true> : &seg_reduce29_kernel<false, false>);
      }
      hipLaunchKernelGGL(level_kernel, dim3(grid_for(lanes * out_items)), dim3(kBlock), 0, stream_, cur, cur_beg,
                         cur_end, loff, nchains, K2, dst, last ? cbucket : nullptr, bucket_sum);
      TA_HIP(hipGetLastError());
      cur = dst;
      cur_items = out_items;
    }
  }

  // ---- window sums ----
  // Two-level window sums (window_seg1/2 + combine) under set_variant bit 23,
  // for the G2 lane pairs and the one-lane BLS12-381 G1 / FIPS reductions: an
  // A/B that lost -- BLS12-381 G2 2^24 109.0 vs 106.2 ms (reduction 16.3 vs
  // 13.7), BN254 G2 2^20 6.6 vs 5.15 ms (2.18 vs 0.95), Groth16 2^20 12.8 vs
  // 11.4 ms (profiles/r05w/): the extra launches of two binary trees over
  // W x B/16 and W x B/1024 partial sums cost more than the fix-ups they save.
  // The one-level kernels (per-segment (jL) R fix-up) stay the default.
  using WinKernel1 = void (*)(const Point*, unsigned, unsigned, unsigned, Point*, Point*);
  using WinKernel2 = void (*)(const Point*, unsigned, unsigned, unsigned, Point*);
  using WinKernelC = void (*)(const Point*, const Point*, unsigned, unsigned, Point*);
  WinKernel1 seg1 = nullptr;
  WinKernel2 seg2 = nullptr;
  WinKernelC comb = nullptr;
  if constexpr (kG2) {
    if (pair_reduce) {
      using LimbPol = std::conditional_t<std::is_same_v<Curve, Bls381G2>, PairPol28, PairPol29>;
      if (pair_limb_ && !(variant_ & (1 << 22))) {
        seg1 = &window_seg1_pair_kernel<Curve, LimbPairArith<LimbPol>>;
        seg2 = &window_seg2_pair_kernel<Curve, LimbPairArith<LimbPol>>;
        comb = &window_combine_pair_kernel<Curve, LimbPairArith<LimbPol>>;
      } else {
        seg1 = &window_seg1_pair_kernel<Curve, FipsPairArith<Curve>>;
        seg2 = &window_seg2_pair_kernel<Curve, FipsPairArith<Curve>>;
        comb = &window_combine_pair_kernel<Curve, FipsPairArith<Curve>>;
      }
    }
  } else {
    bool fips = true;
    if constexpr (std::is_same_v<Curve, Bn254G1>) fips = !acc29_;  // the 29-bit raw path below
    if constexpr (std::is_same_v<Curve, Bls381G1>) {
      if (acc28_ && !(variant_ & (1 << 22))) {
        seg1 = &window_seg1_kernel<Curve, Limb28Arith>;
        seg2 = &window_seg2_kernel<Curve, Limb28Arith>;
        comb = &window_combine_kernel<Curve, Limb28Arith>;
        fips = false;
      }
    }
    if (fips) {
      seg1 = &window_seg1_kernel<Curve, FipsArith<Curve>>;
      seg2 = &window_seg2_kernel<Curve, FipsArith<Curve>>;
      comb = &window_combine_kernel<Curve, FipsArith<Curve>>;
    }
  }
  if (seg1 && (variant_ & (1 << 23)) && !tree_reduce_) {
    const unsigned L1 = std::min(16u, B), S1 = B / L1;
    const unsigned L2 = std::min(64u, S1), S2 = S1 / L2;
    // A_j, R_j (W S1 each), level-2 sums (W S2), two tree ping-pong halves, the two window sums
    const size_t tmp = (size_t)W * ((S1 + 1) / 2 + 1);
    Point* segA = static_cast<Point*>(
        seg_a_.ensure(((size_t)2 * W * S1 + (size_t)W * S2 + 2 * tmp + 2 * W) * sizeof(Point)));
    Point* segR = segA + (size_t)W * S1;
    Point* seg2o = segR + (size_t)W * S1;
    Point* tA = seg2o + (size_t)W * S2;
    Point* tB = tA + tmp;
    Point* winA = tB + tmp;
    Point* winB = winA + W;
    hipLaunchKernelGGL(seg1, dim3(grid_for(lanes * (size_t)W * S1)), dim3(kBlock), 0, stream_, bucket_sum, W, B, L1,
                       segA, segR);
    hipLaunchKernelGGL(seg2, dim3(grid_for(lanes * (size_t)W * S2)), dim3(kBlock), 0, stream_, segR, W, S1, L2, seg2o);
    TA_HIP(hipGetLastError());
    // binary trees (win_reduce) of the W x S arrays down to one point per window
    auto tree = [&](Point* src, unsigned S, Point* dst) {
      Point* cur = src;
      Point* bufs[2] = {tA, tB};
      int k = 0;
      while (S > 1) {
        const unsigned S_out = (S + 1) / 2;
        Point* o = (S_out == 1) ? dst : bufs[k];
        hipLaunchKernelGGL(win_reduce, dim3(grid_for(lanes * (size_t)W * S_out)), dim3(kBlock), 0, stream_, cur, W, S,
                           2u, o);
        TA_HIP(hipGetLastError());
        cur = o;
        k ^= 1;
        S = S_out;
      }
      if (cur != dst) TA_HIP(hipMemcpyAsync(dst, cur, W * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
    };
    tree(segA, S1, winA);
    tree(seg2o, S2, winB);
    hipLaunchKernelGGL(comb, dim3(grid_for(lanes * (size_t)W)), dim3(kBlock), 0, stream_, winA, winB, W, L1, d_windows);
    TA_HIP(hipGetLastError());
    if (profile_) TA_HIP(hipEventRecord(ev_[5], stream_));
    return;
  }
  if (tree_reduce_) {
    // segments of L buckets, workgroup trees of kWinBlock nodes, launches until one node per window
    unsigned L = plan.seg_tree, log_l = 0;
    while ((1u << log_l) < L) ++log_l;
    unsigned units = B / L;
    unsigned groups = (units + kWinBlock - 1) / kWinBlock;
    const size_t lds = (size_t)kWinBlock * sizeof(Point);  // kWinBlock / 2 (V, Rs) pairs
    Point* na = static_cast<Point*>(seg_a_.ensure((size_t)W * groups * 2 * sizeof(Point)));
    Point* nb_ = static_cast<Point*>(seg_b_.ensure((size_t)W * ((groups + kWinBlock - 1) / kWinBlock) * 2 * sizeof(Point)));
    hipLaunchKernelGGL((window_tree_kernel<Curve, true>), dim3(groups, W), dim3(kWinBlock), lds, stream_, bucket_sum, B,
                       L, log_l, nullptr, units, na);
    TA_HIP(hipGetLastError());
    Point* cur_n = na;
    Point* nxt_n = nb_;
    while (groups > 1) {
      units = groups;
      groups = (units + kWinBlock - 1) / kWinBlock;
      hipLaunchKernelGGL((window_tree_kernel<Curve, false>), dim3(groups, W), dim3(kWinBlock), lds, stream_, nullptr,
                         B, L, log_l, cur_n, units, nxt_n);
      TA_HIP(hipGetLastError());
      std::swap(cur_n, nxt_n);
    }
    // the root V of every window: node pairs (V, Rs), stride 2
    TA_HIP(hipMemcpy2DAsync(d_windows, sizeof(Point), cur_n, 2 * sizeof(Point), sizeof(Point), W,
                            hipMemcpyDeviceToDevice, stream_));
    if (profile_) TA_HIP(hipEventRecord(ev_[5], stream_));
    return;
  }
  unsigned S = B / plan.seg;
  // BN254 G1 (29-bit reductions): the binary levels until <= kBlock segment
  // sums per window are left, then one launch for the rest of the tree
  bool tree29 = false;
  if constexpr (std::is_same_v<Curve, Bn254G1>) {
    tree29 = acc29_;
    if (tree29 && B <= kBlock) {
      auto* scan = raw ? &window_scan29_kernel<true> : &window_scan29_kernel<false>;
      hipLaunchKernelGGL(scan, dim3(W), dim3(kBlock), 0, stream_, bucket_sum, B, d_windows);
      TA_HIP(hipGetLastError());
      if (profile_) TA_HIP(hipEventRecord(ev_[5], stream_));
      return;
    }
    if (tree29 && (variant_ & (1u << 19)) && S <= kBlock) {
      auto* segtree = raw ? &window_segtree29_kernel<true> : &window_segtree29_kernel<false>;
      hipLaunchKernelGGL(segtree, dim3(W), dim3(kBlock), 0, stream_, bucket_sum, B, plan.seg, d_windows);
      TA_HIP(hipGetLastError());
      if (profile_) TA_HIP(hipEventRecord(ev_[5], stream_));
      return;
    }
  }
  Point* seg_a = static_cast<Point*>(seg_a_.ensure((size_t)W * S * sizeof(Point)));
  Point* seg_b = static_cast<Point*>(seg_b_.ensure((size_t)W * S * sizeof(Point)));
  if (rsum_pass1 && (variant_ & (1 << 24))) {  // the two-pass segment sums (G2 lane pairs, A/B)
    Point* rs = static_cast<Point*>(rsum_.ensure((size_t)W * B * sizeof(Point)));
    hipLaunchKernelGGL(rsum_pass1, dim3(grid_for(lanes * (size_t)W * S)), dim3(kBlock), 0, stream_, bucket_sum, W, B,
                       plan.seg, rs);
    hipLaunchKernelGGL(rsum_pass2, dim3(grid_for(lanes * (size_t)W * S)), dim3(kBlock), 0, stream_, rs, W, B, plan.seg,
                       seg_a);
    hipLaunchKernelGGL(rsum_fix, dim3(grid_for(lanes * (size_t)W * S)), dim3(kBlock), 0, stream_, rs, W, B, plan.seg,
                       seg_a);
  } else {
    hipLaunchKernelGGL(win_segment, dim3(grid_for(lanes * (size_t)W * S)), dim3(kBlock), 0, stream_, bucket_sum, W, B,
                       plan.seg, seg_a);
  }
  TA_HIP(hipGetLastError());
  Point* s_cur = seg_a;
  Point* s_nxt = seg_b;
  // binary tree over the segment sums: these levels run a few hundred waves,
  // so they are latency-bound and the sequential adds per thread set the time
  // (fan-in 16 -> 2 saved ~0.4 ms at 2^21..2^23)
  constexpr unsigned KW = 2;
  while (S > 1) {
    if constexpr (std::is_same_v<Curve, Bn254G1>) {
      if (tree29 && S <= kBlock) {
        hipLaunchKernelGGL(window_tree29_kernel, dim3(W), dim3(kBlock), 0, stream_, s_cur, S, d_windows);
        TA_HIP(hipGetLastError());
        break;
      }
    }
    unsigned S_out = (S + KW - 1) / KW;
    Point* dst = (S_out == 1) ? d_windows : s_nxt;
    hipLaunchKernelGGL(win_reduce, dim3(grid_for(lanes * (size_t)W * S_out)), dim3(kBlock), 0, stream_, s_cur, W, S,
                       KW, dst);
    TA_HIP(hipGetLastError());
    std::swap(s_cur, s_nxt);
    S = S_out;
  }
  if (B / plan.seg == 1) {
    TA_HIP(hipMemcpyAsync(d_windows, seg_a, W * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
  }
  if (profile_) TA_HIP(hipEventRecord(ev_[5], stream_));
}

template <class Curve>
void MsmGpu<Curve>::run_windows(const void* bases, const void* scalars, size_t n, std::vector<Point>* out,
                                MsmPlan* plan_out) {
  MsmPlan plan = MsmPlan::make(n, Fr::Config::kModulusBits, force_c_, range_begin_, range_end_);
  // G2: running-sum segments twice the G1 rule's length -- a G2 fix-up costs
  // more against the latency-bound loop (BLS12-381 G2 2^24 reduction 13.7 ->
  // 13.0 ms at L = 128, BN254 G2 2^22 1.75 -> 1.64 ms at L = 32;
  // profiles/r05am, r05an)
  if constexpr (std::is_same_v<Curve, Bn254G2> || std::is_same_v<Curve, Bls381G2>) {
#ifdef TACHYON_TUNING_KNOBS
    if (!getenv("TACHYON_MSM_SEG"))
#endif
      plan.seg = std::min(plan.buckets, std::min(128u, plan.seg * 2));
  }
  switch (variant_ & 3) {  // accumulation chunk experiments
    case 1: plan.K = std::min(2048u, plan.K * 2); break;
    case 2: plan.K = std::min(2048u, plan.K * 4); break;
    case 3: plan.K = std::max(4u, plan.K / 2); break;
    default: break;
  }
  switch ((variant_ >> 2) & 3) {  // windows per sort/accumulate group
    case 1: plan.group = 1; break;
    case 2: plan.group = 2; break;
    case 3: plan.group = plan.active(); break;
    default: break;
  }
  idx_mask_ = ~kSignBit;
  fuse_recode_ = !(variant_ & 128);  // bit 7: the separate recode + full sort (A/B)
  static constexpr uint32_t kSpt[] = {kRecodeSpt, 1, 4, 3};
  recode_spt_ = kSpt[(variant_ >> 8) & 3];  // bits 8-9: scalars per thread of the fused recode
  sort_cfg_ = (variant_ >> 4) & 3;  // bits 4-5: onesweep tile shape
#ifdef TACHYON_TUNING_KNOBS
  if (const char* e = getenv("TACHYON_ONESWEEP_CFG")) sort_cfg_ = (unsigned)std::clamp(atoi(e), 0, 5);
#endif
  rocprim_hist_ = (variant_ & 1024) != 0;  // bit 10: rocPRIM's own digit histogram pass (A/B)
  wide_stage_ = (variant_ & 2048) != 0;    // bit 11: 8-byte LDS staging in the recode scatter (A/B)
  tree_reduce_ = (variant_ & 4096) != 0;   // bit 12: window sums by workgroup trees (A/B)
  // BN254 G1 accumulates over the 29-bit-limb field with hand-chained products
  // (field/f29_asm.h) and product-free conversions, the next base not
  // prefetched (3 waves per SIMD): 2^26 accumulation 67.3 -> 61.0 ms, faster
  // at every size from 2^16 (profiles/r03b/ab_acc29_conv.log).  Bit 18 forces
  // the 32-bit FIPS field; bits 13 / 17 prefetch the next base in registers
  // (2 waves) / through LDS by LDS-DMA (A/B); bit 14 is the default
  const bool acc29_default = std::is_same_v<Curve, Bn254G1>;
  acc29_ = !(variant_ & 262144) && ((variant_ & (8192 | 16384 | 131072)) != 0 || acc29_default);
  acc29_mode_ = (variant_ & 131072) ? 2 : (variant_ & 8192) ? 1 : 0;
  // BLS12-381 G1: the accumulation over 14 x 28-bit limbs (field/f28.h) by
  // default; bit 20 restores the 12 x 32-bit FIPS field (A/B)
  acc28_ = std::is_same_v<Curve, Bls381G1> && !(variant_ & (1 << 20));
  // G2: the lane pair over the 28-bit (BLS12-381, msm/pair28.h) / 29-bit
  // (BN254, msm/pair29.h) field; bit 20 restores the FIPS pair, bit 15 the
  // one-lane FIPS kernel
  pair_limb_ = (std::is_same_v<Curve, Bls381G2> || std::is_same_v<Curve, Bn254G2>) && !(variant_ & (1 << 20));
  // G2: a lane pair per point with inline products by default (BLS12-381 G2
  // 2^24 accumulation 129 -> 113 ms, BN254 G2 2^22 16.3 -> 15.7 ms); bit 15
  // restores the one-lane kernel, bit 16 the pair with out-of-line 12-limb products
  pair_acc_ = !(variant_ & 32768);
  pair_inline_ = !(variant_ & 65536);
  if (plan_out) *plan_out = plan;
  if (fold_ > 1 && (plan.w_begin != 0 || plan.w_end != plan.windows || plan.windows % fold_ != 0))
    throw std::runtime_error("tachyon_mi355x: an MSM fold must divide the plan's window count (all windows)");
  // window sums (per MSM of a batch, run_batch; W / fold of a folded run)
  const unsigned nwin = (fold_ > 1 ? plan.windows / fold_ : plan.active()) * batch_;
  out->assign(nwin, Point::zero());
  if (n == 0 || plan.active() == 0) return;
  if (profile_) TA_HIP(hipEventRecord(ev_[0], stream_));
  const Aff* d_bases = static_cast<const Aff*>(bases);
  const Fr* d_scalars = static_cast<const Fr*>(scalars);
  pending_host_bases_ = nullptr;
  if (!is_device_pointer(bases)) {  // uploaded inside enqueue(), overlapping the recode and the sort
    d_bases = static_cast<const Aff*>(bases_.ensure(n * sizeof(Aff)));
    pending_host_bases_ = bases;
  }
  if (!is_device_pointer(scalars)) {
    void* p = scalars_.ensure(n * sizeof(Fr));
    TA_HIP(hipMemcpyAsync(p, scalars, n * sizeof(Fr), hipMemcpyHostToDevice, stream_));
    d_scalars = static_cast<const Fr*>(p);
  }
  Point* d_windows = static_cast<Point*>(windows_.ensure(std::max(1u, nwin) * sizeof(Point)));
  enqueue(d_bases, d_scalars, n, plan, d_windows);
  TA_HIP(hipMemcpyAsync(out->data(), d_windows, nwin * sizeof(Point), hipMemcpyDeviceToHost, stream_));
  TA_HIP(hipStreamSynchronize(stream_));
  for (auto& p : *out) p = p.canonical();  // device values live in [0, 2p)
  if (profile_) {
    TA_HIP(hipEventElapsedTime(&timings_.h2d, ev_[0], ev_[1]));
    TA_HIP(hipEventElapsedTime(&timings_.recode, ev_[1], ev_[2]));
    TA_HIP(hipEventElapsedTime(&timings_.sort, ev_[2], ev_[3]));
    // sort: recode end -> last sort end; prep: recode end -> last accumulation end
    // (sort and accumulation overlap); acc: sum of the accumulation launches
    TA_HIP(hipEventElapsedTime(&timings_.prep, ev_[2], ev_[4]));
    timings_.acc = 0;
    for (unsigned g = 0; g < acc_launches_; ++g) {
      float ms = 0;
      TA_HIP(hipEventElapsedTime(&ms, gev_acc0_[g], gev_acc1_[g]));
      timings_.acc += ms;
    }
    timings_.acc_launches = (float)acc_launches_;
    TA_HIP(hipEventElapsedTime(&timings_.reduce, ev_[4], ev_[5]));
    TA_HIP(hipEventElapsedTime(&timings_.total, ev_[0], ev_[5]));
  }
}

// The accumulation's madd in registers: a chain of `iters` additions of one
// point per thread (no gathers, no bucket runs, 3 waves per SIMD as the
// accumulation kernels).  The result is stored so nothing is dead code.
namespace detail {
namespace {
__global__ __launch_bounds__(kBlock, 3) void madd_ceiling29_kernel(const Affine<Bn254Fq>* __restrict__ pts,
                                                                   XYZZ<Bn254Fq>* __restrict__ out, int iters) {
  using namespace acc29;
  const int t = blockIdx.x * kBlock + threadIdx.x;
  const Affine<Bn254Fq> p = pts[t & 1023], q = pts[(t + 5) & 1023];
  const F29 x2 = shl5_repack(q.x.v), y2 = shl5_repack(q.y.v);
  Acc acc = from_shifted(shl5_repack(p.x.v), shl5_repack(p.y.v));
  int special = 0;
  for (int i = 0; i < iters; ++i) acc = madd(acc, x2, y2, &special);
  XYZZ<Bn254Fq> r = to_xyzz(acc);
  r.zz.v[0] ^= (uint32_t)special;
  out[t] = r;
}
__global__ __launch_bounds__(kBlock, 3) void madd_ceiling32_kernel(const Affine<Bn254Fq>* __restrict__ pts,
                                                                   XYZZ<Bn254Fq>* __restrict__ out, int iters) {
  using F = HotFp<Bn254Fq>;
  const int t = blockIdx.x * kBlock + threadIdx.x;
  const Affine<F> p{pts[t & 1023].x, pts[t & 1023].y}, q{pts[(t + 5) & 1023].x, pts[(t + 5) & 1023].y};
  XYZZ<F> acc{p.x, p.y, F::one(), F::one()};
  bool zero = false;
  for (int i = 0; i < iters; ++i) acc = acc.madd_nz(q, &zero);
  out[t] = XYZZ<Bn254Fq>{acc.x, acc.y, zero ? Bn254Fq::zero() : Bn254Fq(acc.zz), acc.zzz};
}
// ... BLS12-381 G1's 14 x 28-bit field (Pol28), at seg_acc28_kernel's 2 waves per SIMD
__global__ __launch_bounds__(kBlock, 2) void madd_ceiling28_kernel(const Affine<Bls381Fq>* __restrict__ pts,
                                                                   XYZZ<Bls381Fq>* __restrict__ out, int iters) {
  const int t = blockIdx.x * kBlock + threadIdx.x;
  const Affine<Bls381Fq> p = pts[t & 1023], q = pts[(t + 5) & 1023];
  const Pol28::F x2 = Pol28::shift_repack(q.x.v), y2 = Pol28::shift_repack(q.y.v);
  Pol28::Acc acc = Pol28::from_shifted(Pol28::shift_repack(p.x.v), Pol28::shift_repack(p.y.v));
  int special = 0;
  for (int i = 0; i < iters; ++i) acc = Pol28::madd(acc, x2, y2, &special);
  XYZZ<Bls381Fq> r = Pol28::to_xyzz(acc);
  r.zz.v[0] ^= (uint32_t)special;
  out[t] = r;
}
// ... the G2 lane pairs over the limb fields (PairPol28 / PairPol29, as
// seg_acc_pair_limb_kernel): lane h of a pair holds component h; pts are Fq2
// affine points as 4 base-field components (x0 x1 y0 y1)
template <class Pol>
__global__ __launch_bounds__(kBlock) void madd_ceiling_pair_kernel(const typename Pol::Fb* __restrict__ comps,
                                                                   typename Pol::Fb* __restrict__ out, int iters) {
  using Fb = typename Pol::Fb;
  const uint32_t h = threadIdx.x & 1u;
  const int t = blockIdx.x * kBlock + threadIdx.x;
  const int pair = t >> 1;
  const Fb* p = comps + 4 * (pair & 1023);
  const Fb* q = comps + 4 * ((pair + 5) & 1023);
  const typename Pol::F x2 = Pol::repack(q[h].v), y2 = Pol::repack(q[2 + h].v);
  typename Pol::Acc acc = Pol::start(Pol::repack(p[h].v), Pol::repack(p[2 + h].v), h != 0);
  int special = 0;
  for (int i = 0; i < iters; ++i) acc = Pol::madd(acc, x2, y2, h != 0, &special);
  Fb v;
  Pol::to32(acc.x, v.v);
  v.v[0] ^= (uint32_t)special;
  out[4 * (size_t)t] = v;
  Pol::to32(acc.y, v.v);
  out[4 * (size_t)t + 1] = v;
  Pol::to32(acc.zz, v.v);
  out[4 * (size_t)t + 2] = v;
  Pol::to32(acc.zzz, v.v);
  out[4 * (size_t)t + 3] = v;
}

// Best-of-3 rate (G additions/s) of a ceiling kernel over `pts_words`
// pseudo-random field words below the modulus (not curve points: the formula
// does not care), `lanes_per_add` lanes per addition
template <class In, class Out, class Kern>
double time_ceiling(Kern kern, size_t in_words, size_t out_bytes_per_thread, unsigned top_mask_words,
                    uint32_t top_mask, unsigned lanes_per_add) {
  constexpr int kBlocks = 256 * 12, kIters = 400;
  std::vector<uint32_t> h(in_words);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < h.size(); ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h[i] = (uint32_t)(s >> 32);
    if (i % top_mask_words == top_mask_words - 1) h[i] &= top_mask;  // the top word of each element
  }
  void* pts = nullptr;
  void* out = nullptr;
  hipEvent_t e0, e1;
  TA_HIP(hipMalloc(&pts, h.size() * 4));
  TA_HIP(hipMalloc(&out, (size_t)kBlocks * kBlock * out_bytes_per_thread));
  TA_HIP(hipMemcpy(pts, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  TA_HIP(hipEventCreate(&e0));
  TA_HIP(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(kBlocks), dim3(kBlock), 0, 0, static_cast<const In*>(pts), static_cast<Out*>(out), 4);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    TA_HIP(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(kern, dim3(kBlocks), dim3(kBlock), 0, 0, static_cast<const In*>(pts), static_cast<Out*>(out),
                       kIters);
    TA_HIP(hipEventRecord(e1, 0));
    TA_HIP(hipEventSynchronize(e1));
    float ms = 0;
    TA_HIP(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  TA_HIP(hipGetLastError());
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(pts);
  (void)hipFree(out);
  return (double)kBlocks * kBlock / lanes_per_add * kIters / (best * 1e-3) / 1e9;
}
}  // namespace
}  // namespace detail

template <class Curve>
double MsmGpu<Curve>::madd_ceiling(int field_bits) {
  using namespace detail;
  if constexpr (std::is_same_v<Curve, Bn254G1>) {
    if (field_bits != 29 && field_bits != 32) return 0.0;
    require_gpu();
    auto* kern = field_bits == 29 ? &madd_ceiling29_kernel : &madd_ceiling32_kernel;
    return time_ceiling<Affine<Bn254Fq>, XYZZ<Bn254Fq>>(kern, 1024 * 16, sizeof(XYZZ<Bn254Fq>), 8, 0x0fffffffu, 1);
  } else if constexpr (std::is_same_v<Curve, Bls381G1>) {
    if (field_bits != 28) return 0.0;
    require_gpu();
    return time_ceiling<Affine<Bls381Fq>, XYZZ<Bls381Fq>>(&madd_ceiling28_kernel, 1024 * 24, sizeof(XYZZ<Bls381Fq>), 12, 0x0fffffffu, 1);
  } else if constexpr (std::is_same_v<Curve, Bls381G2>) {
    if (field_bits != 28) return 0.0;
    require_gpu();
    return time_ceiling<Bls381Fq, Bls381Fq>(&madd_ceiling_pair_kernel<PairPol28>, 1024 * 48, 4 * sizeof(Bls381Fq), 12,
                                  0x0fffffffu, 2);
  } else {
    if (field_bits != 29) return 0.0;
    require_gpu();
    return time_ceiling<Bn254Fq, Bn254Fq>(&madd_ceiling_pair_kernel<PairPol29>, 1024 * 32, 4 * sizeof(Bn254Fq), 8,
                                 0x0fffffffu, 2);
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

// Host-resident inputs of >= 2^24 points: the upload, not the GPU, is the
// bound (≈6.4 GB at ≈54 GB/s for 2^26 BN254 G1 against ≈95 ms of kernels),
// and the accumulation of a window needs every base, so a single MSM cannot
// start before the last byte arrives.  Split the points into chunks of
// ≥ 2^22 (the kParallelTerm decomposition, pippenger_adapter.h:82-113): a
// copy thread queues every chunk's H2D on copy_stream_ (recording one event
// per chunk) while this thread runs the MSM of chunk k as soon as its event
// is recorded, so the kernels of chunk k overlap the upload of k+1..; the
// chunk results are added on the host.  TACHYON_MSM_HOST_CHUNKS overrides
// the chunk count (1 = one MSM after one upload).  msm_benchmark_gpu sweep
// (host-resident, s): 2^26 chunks 1/4/6/8/12/16 -> 0.193/0.142/0.143/0.136/
// 0.140/0.140; 2^24 1/2/3/4/8 -> 0.053/0.046/0.043/0.042/0.043; 2^22 stays
// whole (1/3/4 -> 0.015/0.021/0.018: the per-chunk reduction dominates).
inline size_t host_chunk_count(size_t n) {
  if (const char* e = getenv("TACHYON_MSM_HOST_CHUNKS")) return std::clamp<size_t>(atoi(e), 1, 64);
  if (n < (size_t(1) << 24)) return 1;
  return std::min<size_t>(8, n >> 22);
}

template <class Curve>
typename MsmGpu<Curve>::Point MsmGpu<Curve>::run_host_pipelined(const void* bases, const void* scalars, size_t n,
                                                                size_t chunks) {
  const bool host_b = !is_device_pointer(bases), host_s = !is_device_pointer(scalars);
  Aff* d_b = host_b ? static_cast<Aff*>(bases_.ensure(n * sizeof(Aff))) : const_cast<Aff*>(static_cast<const Aff*>(bases));
  Fr* d_s = host_s ? static_cast<Fr*>(scalars_.ensure(n * sizeof(Fr))) : const_cast<Fr*>(static_cast<const Fr*>(scalars));
  if (!copy_stream_) TA_HIP(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  while (chunk_ev_.size() < chunks) {
    hipEvent_t e;
    TA_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    chunk_ev_.push_back(e);
  }
  const size_t step = (n + chunks - 1) / chunks;
  int device = 0;
  TA_HIP(hipGetDevice(&device));
  std::mutex mu;
  std::condition_variable cv;
  size_t ready = 0;  // chunks whose copies and event are queued
  bool failed = false;
  std::exception_ptr copy_error;
  std::thread copier([&] {
    try {
      TA_HIP(hipSetDevice(device));
      for (size_t k = 0; k < chunks; ++k) {
        const size_t lo = std::min(n, k * step), len = std::min(step, n - lo);
        if (host_b && len)
          TA_HIP(hipMemcpyAsync(d_b + lo, static_cast<const Aff*>(bases) + lo, len * sizeof(Aff),
                                hipMemcpyHostToDevice, copy_stream_));
        if (host_s && len)
          TA_HIP(hipMemcpyAsync(d_s + lo, static_cast<const Fr*>(scalars) + lo, len * sizeof(Fr),
                                hipMemcpyHostToDevice, copy_stream_));
        TA_HIP(hipEventRecord(chunk_ev_[k], copy_stream_));
        {
          std::lock_guard<std::mutex> lk(mu);
          ready = k + 1;
        }
        cv.notify_all();
      }
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      copy_error = std::current_exception();
      failed = true;
      cv.notify_all();
    }
  });
  struct Joiner {
    std::thread& t;
    ~Joiner() { if (t.joinable()) t.join(); }
  } joiner{copier};
  Point total = Point::zero();
  std::vector<Point> ws;
  MsmPlan plan;
  for (size_t k = 0; k < chunks; ++k) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return ready > k || failed; });
      if (failed) break;
    }
    const size_t lo = std::min(n, k * step), len = std::min(step, n - lo);
    if (!len) continue;
    TA_HIP(hipStreamWaitEvent(stream_, chunk_ev_[k], 0));
    run_windows(d_b + lo, d_s + lo, len, &ws, &plan);
    total = total + combine_windows(ws, plan.c);
  }
  copier.join();
  if (copy_error) std::rethrow_exception(copy_error);
  return total;
}

// Device bytes of the working buffers enqueue() grows for an n-point MSM
// (keys/values and their sort double buffers, sort scratch, accumulation
// pieces and chain tables, bucket and segment sums), plus 10 %.
template <class Curve>
size_t MsmGpu<Curve>::work_bytes(size_t n, unsigned c) const {
  const MsmPlan p = MsmPlan::make(n, Fr::Config::kModulusBits, c, range_begin_, range_end_);
  const size_t entries = n * p.active();
  const size_t T = (entries + p.K - 1) / p.K;
  size_t bytes = entries * 16 + entries / 2;                 // entries (x2) + onesweep scratch
  // (pieces and bucket sums in the 144-byte Raw format of the BN254 G1 accumulation)
  const size_t slot = std::is_same_v<Curve, Bn254G1> ? std::max<size_t>(sizeof(Point), 144) : sizeof(Point);
  bytes += 2 * T * slot + (2 * T / kJoinFanLong + T + 2) * sizeof(Point);  // pieces + first join level
  bytes += (T + 2) * 4 * 11;                                               // flags (x2), last bucket (x2), chain tables
  bytes += (T + 2) * 4 * 12;                                               // join-level offsets (<= 12 levels of <= T chains)
  bytes += (size_t)p.active() * p.buckets * slot;                           // bucket sums
  bytes += 2 * (size_t)p.active() * (p.buckets / p.seg) * sizeof(Point);
  return bytes + bytes / 10;
}

template <class Curve>
size_t MsmGpu<Curve>::held_bytes() const {
  const DeviceBuffer* bufs[] = {&ents_,  &ents2_, &sort_tmp_, &scan_tmp_, &start_, &end_,
                                &cnt_,   &off_a_, &off_b_, &part_a_, &part_b_,  &seg_a_,    &seg_b_, &buckets_,
                                &hist_, &lofs_};
  size_t s = 0;
  for (const DeviceBuffer* b : bufs) s += b->capacity();
  return s;
}

// Point chunks an n-point MSM runs in so that its working set fits the
// device: the analogue of DetermineMsmDivisionsForMemory
// (icicle_msm_utils.cc:10-68; halve the chunk until the estimate is below the
// free memory) for this backend's buffers.  `resident_bytes`: what the call
// itself must keep on the device for all chunks (uploaded host inputs).
// Free memory = hipMemGetInfo + the buffers this context already holds
// (they are reused); TACHYON_MSM_MEM_LIMIT (bytes) caps it for tests.
template <class Curve>
size_t MsmGpu<Curve>::device_budget() const {
  size_t free_b = 0, total_b = 0;
  TA_HIP(hipMemGetInfo(&free_b, &total_b));
  size_t avail = free_b + held_bytes();
  if (const char* e = getenv("TACHYON_MSM_MEM_LIMIT")) avail = std::min<size_t>(avail, strtoull(e, nullptr, 10));
  return avail / 10 * 9;
}

template <class Curve>
size_t MsmGpu<Curve>::memory_divisions(size_t n, size_t resident_bytes) const {
  const size_t avail = device_budget();
  size_t d = 1;
  while (resident_bytes + work_bytes((n + d - 1) / d, force_c_) > avail) {
    if ((n + d - 1) / d <= (size_t(1) << 16))
      throw std::runtime_error("tachyon_mi355x: not enough device memory for the MSM (need " +
                               std::to_string(resident_bytes + work_bytes((n + d - 1) / d, force_c_)) + " B, have " +
                               std::to_string(avail) + " B)");
    d *= 2;
  }
  return d;
}

template <class Curve>
size_t MsmGpu<Curve>::fold_staging_bytes(size_t points, unsigned fold) {
  const size_t per_point = (size_t)fold * 5 * sizeof(F);  // XYZZ copies + prefixes
  const size_t chunk = std::max<size_t>(1, std::min(points, kFoldChunkBytes / per_point));
  return chunk * per_point;
}

template <class Curve>
unsigned MsmGpu<Curve>::fit_fold(size_t points, unsigned windows, unsigned want, size_t run_b, size_t reusable) const {
  if (points == 0 || want <= 1) return 1;
  unsigned f = 1;
  while (f * 2 <= want) f *= 2;
  // the run may reuse this context's buffers; the table and its staging are
  // new allocations, so they must also fit the free memory alone
  const size_t avail = device_budget() + reusable;
  size_t free_b = 0, total_b = 0;
  TA_HIP(hipMemGetInfo(&free_b, &total_b));
  if (const char* e = getenv("TACHYON_MSM_MEM_LIMIT")) free_b = std::min<size_t>(free_b, strtoull(e, nullptr, 10));
  const size_t avail_new = free_b / 10 * 9 + reusable;
  for (; f > 1; f /= 2) {
    if (windows % f != 0 || (uint64_t)f * points >= (uint64_t(1) << 31)) continue;
    const size_t table = fold_table_bytes(points, f), staging = fold_staging_bytes(points, f);
    if (table + staging + run_b <= avail && table + staging <= avail_new) return f;
  }
  return 1;
}

template <class Curve>
typename MsmGpu<Curve>::Point MsmGpu<Curve>::run(const void* bases, const void* scalars, size_t n) {
  last_divisions_ = 1;
  if (n == 0) {
    std::vector<Point> ws;
    run_windows(bases, scalars, n, &ws, nullptr);
    return Point::zero();
  }
  const bool host_b = !is_device_pointer(bases), host_s = !is_device_pointer(scalars);
  const size_t resident = (host_b ? n * sizeof(Aff) : 0) + (host_s ? n * sizeof(Fr) : 0);
  const size_t divisions = memory_divisions(n, resident);
  if (host_b || host_s) {
    const size_t chunks = std::max(host_chunk_count(n), divisions);
    if (chunks > 1) {
      last_divisions_ = chunks;
      return run_host_pipelined(bases, scalars, n, chunks);
    }
  }
  std::vector<Point> ws;
  MsmPlan plan;
  if (divisions == 1) {
    run_windows(bases, scalars, n, &ws, &plan);
    return combine_windows(ws, plan.c);
  }
  // device-resident inputs larger than the working memory: consecutive point
  // chunks, results added (the kParallelTerm sum, pippenger_adapter.h:82-113)
  last_divisions_ = divisions;
  const size_t step = (n + divisions - 1) / divisions;
  Point total = Point::zero();
  for (size_t lo = 0; lo < n; lo += step) {
    const size_t len = std::min(step, n - lo);
    run_windows(static_cast<const Aff*>(bases) + lo, static_cast<const Fr*>(scalars) + lo, len, &ws, &plan);
    total = total + combine_windows(ws, plan.c);
  }
  return total;
}

template <class Curve>
const typename MsmGpu<Curve>::Aff* MsmGpu<Curve>::affine_bases(const void* bases, size_t n, int form) {
  if (form < 0 || form > 3) throw std::runtime_error("tachyon_mi355x: base form must be 0 affine, 1 projective, 2 jacobian or 3 xyzz");
  if (form == 0 || n == 0) return static_cast<const Aff*>(bases);
  const size_t in_bytes = n * (form == 3 ? 4 : 3) * sizeof(F);
  const F* d_in = static_cast<const F*>(bases);
  if (!is_device_pointer(bases)) {
    d_in = static_cast<const F*>(norm_in_.ensure(in_bytes));
    TA_HIP(hipMemcpyAsync(const_cast<F*>(d_in), bases, in_bytes, hipMemcpyHostToDevice, stream_));
  }
  Aff* out = static_cast<Aff*>(norm_out_.ensure(n * sizeof(Aff)));
  F* prefix = static_cast<F*>(norm_prefix_.ensure(n * sizeof(F)));
  constexpr uint32_t kChunk = 16;
  const size_t threads = (n + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(detail::points_to_affine_kernel<F>, dim3(ceil_div(threads, detail::kBlock)), dim3(detail::kBlock),
                     0, stream_, d_in, form, out, prefix, n, kChunk);
  TA_HIP(hipGetLastError());
  TA_HIP(hipStreamSynchronize(stream_));  // the caller may hand the array to another device's stream
  return out;
}

template <class Curve>
unsigned MsmGpu<Curve>::plan_windows(size_t n) const {
  return MsmPlan::make(n, Fr::Config::kModulusBits, force_c_).windows;
}

// The fold table of n device-resident bases: copy k = 2^(k c W / fold) P for
// the plan of n points (forced c or the size's default), fold x n affine
// points into `out` (device).
template <class Curve>
void MsmGpu<Curve>::fold_bases(const void* bases, size_t n, unsigned fold, void* out) {
  fold_bases_c(bases, n, fold, out, MsmPlan::make(n, Fr::Config::kModulusBits, force_c_).c);
}

// ... for run_groups_folded / run_batch_folded: count x len bases (the group
// arrays back to back), the window bits of a batch of len-point MSMs
template <class Curve>
void MsmGpu<Curve>::fold_bases_groups(const void* bases, size_t len, size_t count, unsigned fold, void* out) {
  fold_bases_c(bases, len * count, fold, out, batch_window_bits(len));
}

template <class Curve>
void MsmGpu<Curve>::fold_bases_c(const void* bases, size_t n, unsigned fold, void* out, unsigned c) {
  require_gpu();
  if (!is_device_pointer(bases) || !is_device_pointer(out))
    throw std::runtime_error("tachyon_mi355x: fold_bases takes device-resident bases and output");
  const MsmPlan plan = MsmPlan::make(n, Fr::Config::kModulusBits, c);
  if (fold < 1 || plan.windows % fold != 0)
    throw std::runtime_error("tachyon_mi355x: an MSM fold must divide the plan's window count");
  // (folded base indices vi + part n share the 32-bit entry value with the sign bit)
  if ((uint64_t)fold * n >= (uint64_t(1) << 31))
    throw std::runtime_error("tachyon_mi355x: fold x points must be < 2^31 (folded base indices)");
  if (n == 0) return;
  const unsigned shift = plan.c * (plan.windows / fold);
  // chunk by chunk of points, so the XYZZ staging stays <= kFoldChunkBytes
  // whatever the table size (copy k of point i lands at out[k n + i])
  const size_t m = fold_staging_bytes(n, fold) / ((size_t)fold * 5 * sizeof(F));
  F* xyzz = static_cast<F*>(norm_in_.ensure((size_t)fold * m * 4 * sizeof(F)));
  F* prefix = static_cast<F*>(norm_prefix_.ensure((size_t)fold * m * sizeof(F)));
  constexpr uint32_t kChunk = 16;
  for (size_t lo = 0; lo < n; lo += m) {
    const size_t len = std::min(m, n - lo);
    hipLaunchKernelGGL(detail::fold_points_kernel<F>, dim3(ceil_div(len, detail::kBlock)), dim3(detail::kBlock), 0,
                       stream_, static_cast<const Aff*>(bases) + lo, len, fold, shift, xyzz);
    for (unsigned k = 0; k < fold; ++k)
      hipLaunchKernelGGL(detail::points_to_affine_kernel<F>, dim3(ceil_div(ceil_div(len, kChunk), detail::kBlock)),
                         dim3(detail::kBlock), 0, stream_, xyzz + (size_t)k * len * 4, 3,
                         static_cast<Aff*>(out) + (size_t)k * n + lo, prefix + (size_t)k * len, len, kChunk);
    TA_HIP(hipGetLastError());
  }
  TA_HIP(hipStreamSynchronize(stream_));
  // a one-time build: its XYZZ staging is not kept
  norm_in_.release();
  norm_prefix_.release();
}

// The MSM of n scalars over a fold table (fold_bases of the same n, same
// window bits): W / fold window sums instead of W.
template <class Curve>
typename MsmGpu<Curve>::Point MsmGpu<Curve>::run_folded(const void* folded_bases, const void* scalars, size_t n,
                                                        unsigned fold) {
  last_divisions_ = 1;
  if (fold <= 1) return run(folded_bases, scalars, n);
  if (!is_device_pointer(folded_bases) || !is_device_pointer(scalars))
    throw std::runtime_error("tachyon_mi355x: a folded MSM takes device-resident bases and scalars");
  if ((uint64_t)fold * n >= (uint64_t(1) << 31))
    throw std::runtime_error("tachyon_mi355x: fold x points must be < 2^31 (folded base indices)");
  if (memory_divisions(n, 0) != 1)
    throw std::runtime_error("tachyon_mi355x: a folded MSM must fit the device in one piece");
  struct Reset {
    unsigned& f;
    ~Reset() { f = 1; }
  } reset{fold_};
  fold_ = fold;
  std::vector<Point> ws;
  MsmPlan plan;
  run_windows(folded_bases, scalars, n, &ws, &plan);
  return combine_windows(ws, plan.c);
}

// `count` MSMs over the same `len` device-resident bases in one recode, sort,
// accumulation and reduction: MSM g's scalars are scalars[g len, (g+1) len)
// (device or host; zero scalars pad shorter ones), its windows a block of
// the key space (recode_scalar's glen), its result the Horner combination of
// its own window sums.  One launch sequence instead of `count` -- the small
// MSMs of a KZG batch commitment are latency-bound one by one.
// window size from the length of one MSM, not the batch's total (windows
// sized for the total leave count x more buckets than entries per bucket:
// 2^14 x 32 MSMs 8.4 ms at the total's c = 15), but above one MSM's own
// default: the batch's count x W windows make the per-window work count
// times larger.  c = 8 up to len 2^13, 10 from 2^14 (c swept 5..16 over len
// 2^10..2^16 x count 8..128: 8 best or within noise at len <= 2^13, 10 at
// 2^14..2^16, odd 7 and 9 behind both neighbours;
// profiles/r04c/batch_probe_c_sweep*.log)
template <class Curve>
unsigned MsmGpu<Curve>::batch_window_bits(size_t len) const {
  if (force_c_) return force_c_;
  unsigned lg = 1;
  while ((size_t(1) << lg) < len) ++lg;
  return std::max(default_window_bits(lg, Fr::Config::kModulusBits), lg <= 13 ? std::min(lg + 1, 8u) : 10u);
}

template <class Curve>
size_t MsmGpu<Curve>::max_batch_count(size_t len) const {
  if (len == 0) return 0;
  const unsigned c = batch_window_bits(len);
  const uint64_t W = (Fr::Config::kModulusBits + 1 + c - 1) / c;
  const uint64_t by_keys = (uint64_t(1) << 32) / (W << c);
  const uint64_t by_total = ((uint64_t(1) << 31) - 1) / len;
  return (size_t)std::max<uint64_t>(1, std::min<uint64_t>({4096, by_keys, by_total}));
}

template <class Curve>
std::vector<typename MsmGpu<Curve>::Point> MsmGpu<Curve>::run_batch(const void* bases, const void* scalars,
                                                                    size_t len, size_t count) {
  return run_batch_impl(bases, scalars, len, count, false);
}

// `count` MSMs of `len` points each with their OWN bases -- MSM g over
// bases[g len, (g+1) len) and scalars[g len, (g+1) len) -- in one launch
// sequence, as run_batch (the recode's base index keeps the global i).  The
// Groth16 prover's A and witness + h MSMs run this way.
template <class Curve>
std::vector<typename MsmGpu<Curve>::Point> MsmGpu<Curve>::run_groups(const void* bases, const void* scalars,
                                                                     size_t len, size_t count) {
  return run_batch_impl(bases, scalars, len, count, true);
}

// run_groups over a fold table of the count x len bases (fold_bases_groups)
template <class Curve>
std::vector<typename MsmGpu<Curve>::Point> MsmGpu<Curve>::run_groups_folded(const void* folded_bases,
                                                                            const void* scalars, size_t len,
                                                                            size_t count, unsigned fold) {
  if (!is_device_pointer(folded_bases))
    throw std::runtime_error("tachyon_mi355x: a folded MSM takes a device-resident fold table");
  return run_batch_impl(folded_bases, scalars, len, count, true, fold);
}

template <class Curve>
std::vector<typename MsmGpu<Curve>::Point> MsmGpu<Curve>::run_batch_impl(const void* bases, const void* scalars,
                                                                         size_t len, size_t count, bool distinct,
                                                                         unsigned fold) {
  std::vector<Point> res(count, Point::zero());
  if (count == 0 || len == 0) return res;
  if (count == 1 && fold <= 1) {
    res[0] = run(bases, scalars, len);
    return res;
  }
  if (fold > 1 && !is_device_pointer(scalars))
    throw std::runtime_error("tachyon_mi355x: a folded MSM batch takes device-resident scalars");
  if (!is_device_pointer(bases)) throw std::runtime_error("tachyon_mi355x: run_batch needs device-resident bases");
  const size_t total = len * count;
  if (total >= (size_t(1) << 31) || count > 4096)
    throw std::runtime_error("tachyon_mi355x: MSM batch too large (< 2^31 scalars, <= 4096 MSMs)");
  if (fold > 1 && (uint64_t)fold * total >= (uint64_t(1) << 31))
    throw std::runtime_error("tachyon_mi355x: fold x points must be < 2^31 (folded base indices)");
  // (window size: batch_window_bits)
  struct Reset {
    MsmGpu* m;
    unsigned c;
    ~Reset() {
      m->batch_ = 1;
      m->batch_distinct_ = false;
      m->force_c_ = c;
      m->fold_ = 1;
    }
  } reset{this, force_c_};
  force_c_ = batch_window_bits(len);
  batch_distinct_ = distinct;
  batch_ = (unsigned)count;
  fold_ = std::max(1u, fold);
  last_divisions_ = 1;
  std::vector<Point> ws;
  MsmPlan plan;
  run_windows(bases, scalars, total, &ws, &plan);
  // each MSM's Horner combination of its windows on the host (W c doublings
  // apiece), spread over a few host threads for larger batches
  const unsigned Ws = fold_ > 1 ? plan.windows / fold_ : plan.active();  // window sums per MSM
  auto combine = [&](size_t g0, size_t g1) {
    for (size_t g = g0; g < g1; ++g) {
      std::vector<Point> one(ws.begin() + g * Ws, ws.begin() + (g + 1) * Ws);
      res[g] = combine_windows(one, plan.c);
    }
  };
  const size_t nth = std::min<size_t>({count / 4, 16, std::max(1u, std::thread::hardware_concurrency())});
  if (nth <= 1) {
    combine(0, count);
  } else {
    std::vector<std::thread> th;
    const size_t step = (count + nth - 1) / nth;
    for (size_t g0 = 0; g0 < count; g0 += step) th.emplace_back(combine, g0, std::min(count, g0 + step));
    for (auto& t : th) t.join();
  }
  return res;
}

// The windows [w_begin, w_end) alone (PippengerBase::AccumulateWindowSums
// restricted to them): Horner over the range, then c * w_begin doublings.
template <class Curve>
typename MsmGpu<Curve>::Point MsmGpu<Curve>::run_window_range(const void* bases, const void* scalars, size_t n,
                                                              unsigned w_begin, unsigned w_end) {
  struct Reset {
    MsmGpu* m;
    ~Reset() { m->range_begin_ = 0; m->range_end_ = ~0u; }
  } reset{this};
  range_begin_ = w_begin;
  range_end_ = w_end;
  last_divisions_ = 1;
  std::vector<Point> ws;
  MsmPlan plan;
  // the window range of every point chunk run() would use for memory
  // (DetermineMsmDivisionsForMemory), partials added; host inputs stay on the
  // host and each chunk uploads its own slice (counted as resident: a
  // conservative bound).  The window bits must not depend on the chunk size,
  // so the whole input's plan is forced on the chunks.
  if (n == 0) {
    run_windows(bases, scalars, 0, &ws, &plan);
    return Point::zero();
  }
  const size_t resident = (is_device_pointer(bases) ? 0 : n * sizeof(Aff)) +
                          (is_device_pointer(scalars) ? 0 : n * sizeof(Fr));
  const size_t divisions = memory_divisions(n, resident);
  struct RestoreC {
    MsmGpu* m;
    unsigned c;
    ~RestoreC() { m->force_c_ = c; }
  } restore_c{this, force_c_};
  if (divisions > 1 && !force_c_) force_c_ = MsmPlan::make(n, Fr::Config::kModulusBits).c;
  last_divisions_ = divisions;
  const size_t step = (n + divisions - 1) / divisions;
  Point total = Point::zero();
  for (size_t lo = 0; lo < n; lo += step) {
    const size_t len = std::min(step, n - lo);
    run_windows(static_cast<const Aff*>(bases) + lo, static_cast<const Fr*>(scalars) + lo, len, &ws, &plan);
    if (plan.active() == 0) return Point::zero();
    Point p = combine_windows(ws, plan.c);
    for (unsigned k = 0; k < plan.c * plan.w_begin; ++k) p = p.dbl();
    total = total + p;
  }
  return total;
}

}  // namespace tachyon_amd::msm
