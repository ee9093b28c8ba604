// Radix-2 NTT kernels for MI355X (gfx950) and the NttDomain host driver.
// Reference semantics: radix2_evaluation_domain.h:213-333,
// univariate_evaluation_domain.h:141-232,464-489,518-566, radix2_twiddle_cache.h:57-121.
#include "ntt.h"

#include "../field/fr29.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

namespace tachyon_amd::ntt {

namespace {

constexpr unsigned kBlock = 256;
constexpr uint32_t kMaxPassStages = 8;
// Elements per workgroup: 1024 (32 KiB of LDS) = 256 threads x 2^2, so every
// thread owns one radix-4 group per register step and 5 workgroups fit a CU
// (5 waves per SIMD at 88 VGPRs).  2^24 sweep (tools/tune_ntt.py,
// TACHYON_NTT_LDS_ELEMS x TACHYON_NTT_RADIX_LOG): 2048/r3 2.43, 2048/r2 2.44,
// 1024/r2 1.95, 1024/r3 2.82 (half the threads idle), 512/r2 2.54 ms.
constexpr uint32_t kMaxLdsElems = 1024;

enum : uint32_t {
  kLoadCoset = 1,
  kStoreScale = 2,
  kStoreCoset = 4,
  kLoadTw4 = 8,
  kStoreTw4 = 16,
  kLoadXch = 32,
  kStoreXch = 64
};

// Twiddle tables.  BN254 Fr butterflies multiply by a Shoup product
// (Fp::mul_shoup, mont_asm.h shoup_mul_8): an entry is the plain twiddle and
// its quotient floor(w 2^256 / p), 64 bytes -- 13 fewer v_mad_u64_u32, 29
// fewer carry adds and no Montgomery digits per butterfly than a Montgomery
// product by a 32-byte Montgomery twiddle.  BLS12-381 Fr (3p > 2^256) keeps
// Montgomery twiddles.
template <class Fr>
struct ShoupTw {
  Fr w, wq;
};
template <class Fr>
struct NttTw {
  using type = Fr;
};
template <>
struct NttTw<Bn254Fr> {
  using type = ShoupTw<Bn254Fr>;
};
template <class Fr>
__device__ __forceinline__ Fr tw_mul(const Fr& x, const Fr& w) {
  return x * w;
}
template <class Fr>
__device__ __forceinline__ Fr tw_mul(const Fr& x, const ShoupTw<Fr>& t) {
  return x.mul_shoup(t.w, t.wq);
}

template <class Fr>
struct PassArgs {
  uint32_t L, s0, k, log_m, final_pass, mode, pow_bits;
  const Fr* load_lo;
  const Fr* load_hi;
  const Fr* store_lo;
  const Fr* store_hi;
  Fr scale;
  // four-step exchange (kStoreTw4: the forward stage 1's last pass; kLoadTw4:
  // the inverse stage 2's first pass): element k of batch entry b (the local
  // column c_l) times w_N^(+-(c0 + b) k), at its packed send / recv position
  FourStepTw<Fr> fs;
  // single-pass transforms smaller than a tile: 2^pack batch entries per
  // workgroup, set m = entry (blockIdx.y << pack) + m (0: one entry per blockIdx.y)
  uint32_t pack;
};

// The exchange layout of the fused stages: chunk h (n/G^2 elements, to / from
// rank h) holds [k1_l][c_l], row-major -- so the row NTTs read (forward
// stage 2) and write (inverse stage 1) Cg-element runs and need no transpose.
// Column side: element k1 of local column c_l at (h Rg + k1_l) Cg + c_l =
// k1 Cg + c_l (h = k1 >> log_rg).  (The unfused round-4 stages keep
// twiddle_exchange_kernel's [c_l][k1_l] chunks and the transposes.)
template <class Fr>
__device__ __forceinline__ size_t fs_packed(const FourStepTw<Fr>& f, uint32_t k1, uint32_t c_l) {
  return ((size_t)k1 << f.log_cg) + c_l;
}
// Row side: element c (column, c = g Cg + c_l) of local row j at (g Rg + j) Cg + c_l
template <class Fr>
__device__ __forceinline__ size_t xch_pos(const FourStepTw<Fr>& f, uint32_t c, uint32_t j) {
  return ((((size_t)(c >> f.log_cg) << f.log_rg) + j) << f.log_cg) + (c & ((1u << f.log_cg) - 1));
}
// w_N^((c0 + c_l) k1) from the two-level power tables of the four-step's root
template <class Fr>
__device__ __forceinline__ Fr fs_twiddle(const FourStepTw<Fr>& f, uint32_t k1, uint32_t c_l) {
  const uint64_t e = ((uint64_t)(f.c0 + c_l) * k1) & ((uint64_t(1) << f.log_n) - 1);
  return f.lo[e & ((1u << f.bits) - 1)] * f.hi[e >> f.bits];
}

__device__ __forceinline__ uint32_t bitrev(uint32_t x, uint32_t bits) {
  return bits == 0 ? 0u : (__brev(x) >> (32 - bits));
}

// One pass of k DIF stages (s0 .. s0+k-1) over M sets of 2^k elements held in
// LDS.  Non-final passes are in place (each workgroup reads and writes the
// same positions); the final pass (s0 + k == L) writes natural order through
// the bit-reversal permutation, M bit-reversed-consecutive sets per workgroup
// so every store row is M contiguous elements.
// R DIF stages (t .. t+R-1 of the pass) on groups of 2^R elements held in
// registers.  Group g covers set m = g mod M and the positions
// a0 + j q (j < 2^R, q = 2^(k-t-R)); stage t+u pairs j with j + 2^(R-1-u).
// Twiddle of the butterfly whose low element has global index i at global
// stage s: w_s^(i mod 2^(L-s-1)) (the reference's Radix2TwiddleCache row s).
// kLast: the transform's last R stages (final pass, t + R == k).
template <int R, bool kLast, bool kPrefetch, class Fr, class Tw, class IndexFn>
__device__ __forceinline__ void radix_step(Fr* __restrict__ lds, const Tw* __restrict__ tw, const PassArgs<Fr>& a,
                                           uint32_t t, IndexFn index) {
  constexpr int E = 1 << R;
  const uint32_t log_m = a.log_m, M = 1u << log_m;
  const uint32_t n = 1u << a.L;
  const uint32_t groups = (M << a.k) >> R;
  const uint32_t qlog = a.k - t - R;
  for (uint32_t g = threadIdx.x; g < groups; g += kBlock) {
    const uint32_t m = g & (M - 1);
    const uint32_t rr = g >> log_m;
    const uint32_t off = rr & ((1u << qlog) - 1);
    const uint32_t a0 = ((rr >> qlog) << (qlog + R)) + off;
    // the step's twiddles first: their global loads overlap the LDS reads
    // and the first butterflies instead of stalling each product
    Tw wv[R][E / 2];
    if constexpr (!kLast && kPrefetch) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const uint32_t st = a.s0 + t + u;
        const uint32_t gap_mask = (1u << (a.L - st - 1)) - 1;
        const Tw* tws = tw + (n - (n >> st));
        const int half = E >> (u + 1);
        int c = 0;
#pragma unroll
        for (int j = 0; j < E; ++j) {
          if (j & half) continue;
          wv[u][c++] = tws[index(a0 + ((uint32_t)j << qlog), m) & gap_mask];
        }
      }
    }
    Fr x[E];
#pragma unroll
    for (int j = 0; j < E; ++j) x[j] = lds[((a0 + ((uint32_t)j << qlog)) << log_m) + m];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const uint32_t st = a.s0 + t + u;
      const Tw* tws = tw + (n - (n >> st));
      const int half = E >> (u + 1);
      int c = 0;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j & half) continue;
        const Fr lo = x[j], hi = x[j + half];
        // ButterflyFnInOut: lo = lo + hi; hi = (lo - hi) * w
        x[j] = lo + hi;
        if constexpr (kLast) {
          // the transform's last R stages: the twiddle index is j mod 2^(R-1-u)
          // (a0 and the set base are multiples of 2^R), known at compile time;
          // index 0 is w = 1 -- the whole last stage and half the one before
          const uint32_t idx = (uint32_t)j & ((1u << (R - 1 - u)) - 1);
          x[j + half] = idx ? tw_mul(lo.sub_unreduced(hi), tws[idx]) : (lo - hi);
        } else {
          // twiddles are canonical, so lo - hi + 2p needs no borrow test
          if constexpr (kPrefetch) {
            x[j + half] = tw_mul(lo.sub_unreduced(hi), wv[u][c++]);
          } else {
            const uint32_t gap_mask = (1u << (a.L - st - 1)) - 1;
            x[j + half] = tw_mul(lo.sub_unreduced(hi), tws[index(a0 + ((uint32_t)j << qlog), m) & gap_mask]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < E; ++j) lds[((a0 + ((uint32_t)j << qlog)) << log_m) + m] = x[j];
  }
}

template <class Fr, class Tw, int MaxR, bool kPrefetch = true, int kWaves = 1>
__global__ __launch_bounds__(kBlock, kWaves) void dif_pass_kernel(const Fr* __restrict__ in, Fr* __restrict__ out,
                                                          const Tw* __restrict__ tw, PassArgs<Fr> a) {
  extern __shared__ uint4 smem_raw[];
  Fr* lds = reinterpret_cast<Fr*>(smem_raw);
  const uint32_t L = a.L, k = a.k, log_m = a.log_m;
  const uint32_t M = 1u << log_m;
  const uint32_t elems = M << k;
  const uint32_t b = blockIdx.x;
  // batch of independent contiguous transforms (the packed four-step
  // layouts address the whole buffer themselves); with a.pack the workgroup's
  // sets are 2^pack whole transforms, entries ybase + m
  const uint32_t pk = a.pack, ybase = blockIdx.y << pk;
  if (!(a.mode & (kLoadTw4 | kLoadXch))) in += (size_t)ybase << L;
  if (!(a.mode & (kStoreTw4 | kStoreXch))) out += (size_t)ybase << L;

  // index(mid, m) of element m of the block's set, position mid in the set
  uint32_t hi_shift = L - a.s0;            // set stride in the hi dimension
  uint32_t mid_shift = L - a.s0 - k;       // stride between set members
  uint32_t hi = 0, lo_base = 0, r0 = 0;
  if (!a.final_pass) {
    uint32_t lo_blocks = (1u << mid_shift) >> log_m;
    hi = b / lo_blocks;
    lo_base = (b - hi * lo_blocks) << log_m;
  } else {
    r0 = b << log_m;
  }
  auto index = [&](uint32_t mid, uint32_t m) -> uint32_t {
    if (!a.final_pass) return (hi << hi_shift) + (mid << mid_shift) + lo_base + m;
    uint32_t h = bitrev(r0 + m, L - k);
    return (h << k) + mid;
  };

  // ---- load ----
  for (uint32_t e = threadIdx.x; e < elems; e += kBlock) {
    uint32_t mid = e >> log_m, m = e & (M - 1);
    uint32_t i = index(mid, m);
    const uint32_t ent = pk ? m : 0u;
    Fr v;
    if (a.mode & kLoadTw4) {
      v = in[fs_packed(a.fs, i, ybase + ent)] * fs_twiddle(a.fs, i, ybase + ent);
    } else if (a.mode & kLoadXch) {
      v = in[xch_pos(a.fs, i, ybase + ent)];
    } else {
      v = in[((size_t)ent << L) + i];
      if (a.mode & kLoadCoset) v = v * (a.load_lo[i & ((1u << a.pow_bits) - 1)] * a.load_hi[i >> a.pow_bits]);
    }
    lds[e] = v;
  }
  __syncthreads();

  // ---- k butterfly stages, up to MaxR per LDS round trip ----
  // A step of R stages loads 2^R elements of one set into registers, runs
  // the R * 2^(R-1) butterflies there (2^(R-1) independent ones per stage,
  // which the scheduler interleaves) and writes them back: one LDS round
  // trip and one barrier per R stages instead of per stage.
  for (uint32_t t = 0; t < k;) {
    const uint32_t R = min((uint32_t)MaxR, k - t);
    const bool last = a.final_pass && t + R == k;
    if (MaxR >= 3 && R == 3) {
      if (last) radix_step<3, true, kPrefetch>(lds, tw, a, t, index);
      else radix_step<3, false, kPrefetch>(lds, tw, a, t, index);
    } else if (MaxR >= 2 && R == 2) {
      if (last) radix_step<2, true, kPrefetch>(lds, tw, a, t, index);
      else radix_step<2, false, kPrefetch>(lds, tw, a, t, index);
    } else {
      if (last) radix_step<1, true, kPrefetch>(lds, tw, a, t, index);
      else radix_step<1, false, kPrefetch>(lds, tw, a, t, index);
    }
    t += R;
    __syncthreads();
  }

  // ---- store ----
  if (!a.final_pass) {
    for (uint32_t e = threadIdx.x; e < elems; e += kBlock) {
      uint32_t mid = e >> log_m, m = e & (M - 1);
      out[index(mid, m)] = lds[e];
    }
  } else {
    for (uint32_t e = threadIdx.x; e < elems; e += kBlock) {
      uint32_t q = e >> log_m, m = e & (M - 1);
      uint32_t mid = bitrev(q, k);
      Fr v = lds[(mid << log_m) + m];
      const uint32_t o = pk ? q : (q << (L - k)) + r0 + m, ent = pk ? m : 0u;
      if (a.mode & kStoreCoset) v = v * (a.store_lo[o & ((1u << a.pow_bits) - 1)] * a.store_hi[o >> a.pow_bits]);
      else if (a.mode & kStoreScale) v = v * a.scale;
      if (a.mode & kStoreTw4) out[fs_packed(a.fs, o, ybase + ent)] = (v * fs_twiddle(a.fs, o, ybase + ent)).canonical();
      else if (a.mode & kStoreXch) out[xch_pos(a.fs, o, ybase + ent)] = v.canonical();
      else out[((size_t)ent << L) + o] = v.canonical();
    }
  }
}

// ---------------------------------------------------------------------------
// BN254 Fr passes over 9 x 29-bit limbs (field/fr29.h): the same DIF network,
// pass plan, index maps, bit reversal and fused scalings as dif_pass_kernel,
// with the butterflies of fr29::radix4 / radix2 (carry-free products, limb-wise
// sums and differences).  Elements between passes are 36-byte F29 (normalized,
// < 8p); the first pass reads the 32-byte Montgomery input, the final pass
// writes canonical 32-byte values.  LDS holds the elements as 9 limb planes
// of kMaxLdsElems words (a plane stride fixed at compile time: one ds_read_b32
// per limb with an immediate offset).  Twiddles: R'-form (36 B) in the first
// pass, whose stage tables stream from HBM; Shoup (72 B) in the later ones.
using fr29::F29;
template <class TwT>
struct Tw29Table {
  const TwT* tw;  // entry of (stage s, index j) at tw[(n - (n >> s)) - off + j]
  uint32_t off;
};

// kSwz: positions XOR-swizzled so that the 32-lane groups of a ds_read_b32 /
// ds_write_b32 (bank = word mod 32) hit 32 distinct banks in every register
// step of the 8-stage, 4-set passes (2^24: qlog = 6, 4, 2, 0): bit 2 ^= bit 5,
// bits 3, 4 ^= bit 6.  Without it the qlog = 2 / 0 steps are 2- / 4-way
// conflicted on all 72 LDS accesses of a group.
template <bool kSwz>
__device__ __forceinline__ uint32_t swz29(uint32_t p) {
  if constexpr (kSwz) return p ^ ((p >> 3) & 4u) ^ (((p >> 6) & 1u) * 0x18u);
  else return p;
}
template <bool kSwz>
__device__ __forceinline__ F29 lds29_load(const uint32_t* __restrict__ lds, uint32_t pos) {
  F29 v;
  pos = swz29<kSwz>(pos);
#pragma unroll
  for (int i = 0; i < 9; ++i) v.l[i] = lds[i * kMaxLdsElems + pos];
  return v;
}
template <bool kSwz>
__device__ __forceinline__ void lds29_store(uint32_t* __restrict__ lds, uint32_t pos, const F29& v) {
  pos = swz29<kSwz>(pos);
#pragma unroll
  for (int i = 0; i < 9; ++i) lds[i * kMaxLdsElems + pos] = v.l[i];
}

template <int R, bool kLast, bool kSwz, class TwT, class IndexFn>
__device__ __forceinline__ void radix29_step(uint32_t* __restrict__ lds, Tw29Table<TwT> tt,
                                             const PassArgs<Bn254Fr>& a, uint32_t t, IndexFn index) {
  constexpr int E = 1 << R;
  const uint32_t log_m = a.log_m, M = 1u << log_m;
  const uint32_t n = 1u << a.L;
  const uint32_t groups = (M << a.k) >> R;
  const uint32_t qlog = a.k - t - R;
  const uint32_t st = a.s0 + t;
  const TwT* twA = tt.tw + ((n - (n >> st)) - tt.off);
  const uint32_t gapA = (1u << (a.L - st - 1)) - 1;
  for (uint32_t g = threadIdx.x; g < groups; g += kBlock) {
    const uint32_t m = g & (M - 1);
    const uint32_t rr = g >> log_m;
    const uint32_t off = rr & ((1u << qlog) - 1);
    const uint32_t a0 = ((rr >> qlog) << (qlog + R)) + off;
    if constexpr (R == 2) {
      // twiddles first: their loads overlap the LDS reads
      TwT tA0, tA1, tB0, tB1;
      if constexpr (kLast) {
        tA1 = twA[1];  // stage L - 2 has the two entries {1, w_4}; everything else is 1
      } else {
        const TwT* twB = tt.tw + ((n - (n >> (st + 1))) - tt.off);
        const uint32_t gapB = (1u << (a.L - st - 2)) - 1;
        tA0 = twA[index(a0, m) & gapA];
        tA1 = twA[index(a0 + (1u << qlog), m) & gapA];
        tB0 = twB[index(a0, m) & gapB];
        tB1 = twB[index(a0 + (2u << qlog), m) & gapB];
      }
      F29 x[4];
#pragma unroll
      for (int j = 0; j < E; ++j) x[j] = lds29_load<kSwz>(lds, ((a0 + ((uint32_t)j << qlog)) << log_m) + m);
      if constexpr (kLast) fr29::radix4_last(x, tA1);
      else fr29::radix4(x, tA0, tA1, tB0, tB1);
#pragma unroll
      for (int j = 0; j < E; ++j) lds29_store<kSwz>(lds, ((a0 + ((uint32_t)j << qlog)) << log_m) + m, x[j]);
    } else {
      TwT tA;
      if constexpr (!kLast) tA = twA[index(a0, m) & gapA];
      F29 x[2];
#pragma unroll
      for (int j = 0; j < E; ++j) x[j] = lds29_load<kSwz>(lds, ((a0 + ((uint32_t)j << qlog)) << log_m) + m);
      if constexpr (kLast) fr29::radix2_last(x);
      else fr29::radix2(x, tA);
#pragma unroll
      for (int j = 0; j < E; ++j) lds29_store<kSwz>(lds, ((a0 + ((uint32_t)j << qlog)) << log_m) + m, x[j]);
    }
  }
}

// kFirst: the input is the 32-byte Montgomery array (the transform's first
// pass, R'-form twiddles); otherwise 36-byte F29 from the previous pass.
template <bool kFirst, bool kSwz, class TwT>
__global__ __launch_bounds__(kBlock) void dif29_pass_kernel(const void* __restrict__ in_v, void* __restrict__ out_v,
                                                            Tw29Table<TwT> tt, PassArgs<Bn254Fr> a) {
  __shared__ uint32_t lds[9 * kMaxLdsElems];
  const uint32_t L = a.L, k = a.k, log_m = a.log_m;
  const uint32_t M = 1u << log_m;
  const uint32_t elems = M << k;
  const uint32_t b = blockIdx.x;
  uint32_t hi_shift = L - a.s0;
  uint32_t mid_shift = L - a.s0 - k;
  uint32_t hi = 0, lo_base = 0, r0 = 0;
  if (!a.final_pass) {
    uint32_t lo_blocks = (1u << mid_shift) >> log_m;
    hi = b / lo_blocks;
    lo_base = (b - hi * lo_blocks) << log_m;
  } else {
    r0 = b << log_m;
  }
  auto index = [&](uint32_t mid, uint32_t m) -> uint32_t {
    if (!a.final_pass) return (hi << hi_shift) + (mid << mid_shift) + lo_base + m;
    uint32_t h = bitrev(r0 + m, L - k);
    return (h << k) + mid;
  };

  // ---- load ----
  // (a.pack: the workgroup's sets are 2^pack whole transforms, entries ybase + m)
  const uint32_t pk = a.pack, ybase = blockIdx.y << pk;
  const size_t batch_off = (size_t)ybase << L;
  for (uint32_t e = threadIdx.x; e < elems; e += kBlock) {
    const uint32_t mid = e >> log_m, m = e & (M - 1);
    const uint32_t i = index(mid, m);
    const uint32_t ent = pk ? m : 0u;
    F29 v;
    if constexpr (kFirst) {
      Bn254Fr x;
      if ((a.mode & kLoadTw4) && a.fs.tab29) {  // the precomputed R'-form twiddle: one product
        const Bn254Fr raw = static_cast<const Bn254Fr*>(in_v)[fs_packed(a.fs, i, ybase + ent)];
        const auto* t29 = static_cast<const fr29::TwMont29*>(a.fs.tab29);
        v = fr29::tw_prod(fr29::from_words(raw.v), t29[((size_t)(ybase + ent) << a.fs.log_r) + i]);
        lds29_store<kSwz>(lds, e, v);
        continue;
      }
      if (a.mode & kLoadTw4) {
        x = static_cast<const Bn254Fr*>(in_v)[fs_packed(a.fs, i, ybase + ent)] * fs_twiddle(a.fs, i, ybase + ent);
      } else if (a.mode & kLoadXch) {
        x = static_cast<const Bn254Fr*>(in_v)[xch_pos(a.fs, i, ybase + ent)];
      } else {
        x = static_cast<const Bn254Fr*>(in_v)[batch_off + ((size_t)ent << L) + i];
        if (a.mode & kLoadCoset) x = x * (a.load_lo[i & ((1u << a.pow_bits) - 1)] * a.load_hi[i >> a.pow_bits]);
      }
      v = fr29::from_words(x.v);
    } else {
      v = static_cast<const F29*>(in_v)[batch_off + ((size_t)ent << L) + i];
    }
    lds29_store<kSwz>(lds, e, v);
  }
  __syncthreads();

  for (uint32_t t = 0; t < k;) {
    const uint32_t R = min(2u, k - t);
    const bool last = a.final_pass && t + R == k;
    if (R == 2) {
      if (last) radix29_step<2, true, kSwz>(lds, tt, a, t, index);
      else radix29_step<2, false, kSwz>(lds, tt, a, t, index);
    } else {
      if (last) radix29_step<1, true, kSwz>(lds, tt, a, t, index);
      else radix29_step<1, false, kSwz>(lds, tt, a, t, index);
    }
    t += R;
    __syncthreads();
  }

  // ---- store ----
  if (!a.final_pass) {
    F29* out = static_cast<F29*>(out_v) + batch_off;
    for (uint32_t e = threadIdx.x; e < elems; e += kBlock) {
      const uint32_t mid = e >> log_m, m = e & (M - 1);
      out[index(mid, m)] = lds29_load<kSwz>(lds, e);
    }
  } else {
    Bn254Fr* out = static_cast<Bn254Fr*>(out_v) + ((a.mode & (kStoreTw4 | kStoreXch)) ? 0 : batch_off);
    for (uint32_t e = threadIdx.x; e < elems; e += kBlock) {
      const uint32_t q = e >> log_m, m = e & (M - 1);
      const uint32_t mid = bitrev(q, k);
      Bn254Fr v;
      const uint32_t o = pk ? q : (q << (L - k)) + r0 + m, ent = pk ? m : 0u;
      if ((a.mode & kStoreTw4) && a.fs.tab29) {  // the precomputed R'-form twiddle: one product
        const auto* t29 = static_cast<const fr29::TwMont29*>(a.fs.tab29);
        const F29 y = fr29::tw_prod(lds29_load<kSwz>(lds, (mid << log_m) + m),
                                    t29[((size_t)(ybase + ent) << a.fs.log_r) + o]);
        fr29::to_canonical_words(y, v.v);
        out[fs_packed(a.fs, o, ybase + ent)] = v;
        continue;
      }
      fr29::to_canonical_words(lds29_load<kSwz>(lds, (mid << log_m) + m), v.v);
      if (a.mode & kStoreCoset) v = (v * (a.store_lo[o & ((1u << a.pow_bits) - 1)] * a.store_hi[o >> a.pow_bits])).canonical();
      else if (a.mode & kStoreScale) v = (v * a.scale).canonical();
      if (a.mode & kStoreTw4) out[fs_packed(a.fs, o, ybase + ent)] = (v * fs_twiddle(a.fs, o, ybase + ent)).canonical();
      else if (a.mode & kStoreXch) out[xch_pos(a.fs, o, ybase + ent)] = v;
      else out[((size_t)ent << L) + o] = v;
    }
  }
}

// Montgomery twiddles (canonical w 2^256 mod p) -> the 29-bit tables: entries
// [0, split) R'-form (w 2^261 mod p = 32 W mod p), entries [split, count)
// Shoup {w, floor(w 2^261 / p)} with floor(w 2^261 / p) = 32 floor(w 2^256 /
// p) + floor(32 W / p) (W = w 2^256 mod p, the Montgomery entry).
__global__ __launch_bounds__(kBlock) void tw29_table_kernel(fr29::TwMont29* __restrict__ mont29,
                                                            fr29::TwShoup29* __restrict__ shoup29,
                                                            const Bn254Fr* __restrict__ in, uint32_t split,
                                                            uint32_t count) {
  const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= count) return;
  const Bn254Fr W = in[j].canonical();
  if (j < split) {
    Bn254Fr x = W;
#pragma unroll
    for (int i = 0; i < 5; ++i) x = (x + x).canonical();
    mont29[j].w = fr29::from_words(x.v);
  } else {
    const Bn254Fr w = W.from_mont();
    const Bn254Fr q32 = Bn254Fr::shoup_quotient(w);
    // t = floor(32 W / p): five doublings of W (< p, so 2r < 2p < 2^256),
    // each followed by a subtraction of p when 2r >= p (one quotient bit)
    uint32_t t = 0;
    uint32_t r[8];
    for (int i = 0; i < 8; ++i) r[i] = W.v[i];
    for (int bit = 0; bit < 5; ++bit) {
      uint32_t c = 0;
      for (int i = 0; i < 8; ++i) {
        const uint32_t nc = r[i] >> 31;
        r[i] = (r[i] << 1) | c;
        c = nc;
      }
      uint32_t d[8], borrow = 0;
      for (int i = 0; i < 8; ++i) {
        const uint64_t s = (uint64_t)r[i] - fr29::kPWords[i] - borrow;
        d[i] = (uint32_t)s;
        borrow = (uint32_t)(s >> 63);
      }
      t = 2 * t + (borrow ? 0u : 1u);
      if (!borrow)
        for (int i = 0; i < 8; ++i) r[i] = d[i];
    }
    fr29::TwShoup29 e;
    e.w = fr29::from_words(w.v);
    e.wq = f29::shl5_repack(q32.v);
    e.wq.l[0] |= t;  // the low 5 bits of 32 q32 are zero
    shoup29[j - split] = e;
  }
}

// T0[j] = w^j for j < n/2 from two small power tables: lo[j & mask] * hi[j >> bits]
template <class Fr>
__global__ __launch_bounds__(kBlock) void twiddle_base_kernel(Fr* __restrict__ t0, uint32_t count,
                                                              const Fr* __restrict__ lo, const Fr* __restrict__ hi,
                                                              uint32_t bits) {
  uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= count) return;
  t0[j] = (lo[j & ((1u << bits) - 1)] * hi[j >> bits]).canonical();  // canonical: see radix_step
}

// Montgomery twiddle table -> Shoup entries {plain w, floor(w 2^256 / p)}
template <class Fr>
__global__ __launch_bounds__(kBlock) void shoup_table_kernel(ShoupTw<Fr>* __restrict__ out,
                                                             const Fr* __restrict__ in, uint32_t count) {
  uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= count) return;
  const Fr w = in[j].from_mont();
  out[j] = ShoupTw<Fr>{w, Fr::shoup_quotient(w)};
}

// T_s[j] = T_0[j << s]  (the strided sub-sampling of radix2_twiddle_cache.h:105-117)
template <class T>
__global__ __launch_bounds__(kBlock) void twiddle_stage_kernel(T* __restrict__ ts, const T* __restrict__ t0,
                                                               uint32_t count, uint32_t s) {
  uint32_t j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= count) return;
  ts[j] = t0[(size_t)j << s];
}

template <class Fr>
Fr fr_from_u64(uint64_t v) {
  Fr x = Fr::zero();
  x.v[0] = (uint32_t)v;
  x.v[1] = (uint32_t)(v >> 32);
  return x.to_mont();
}

// halo2curves' BN254 Fr two-adic root of unity 7^((r-1)/2^28), Montgomery limbs
// exactly as OverrideSubgroupGenerator writes kTwoAdicRootOfUnity
// (bn/bn254/halo2/bn254.cc:18-23).  GetRootOfUnity's large-subgroup branch
// (large^(3^2), bn254.cc:24-29) lands on the same element.
constexpr uint64_t kBn254FrHalo2TwoAdicRootMont64[4] = {10822932506504462008ULL, 10978899855858987673ULL,
                                                        12888607242213977304ULL, 2119232853909229097ULL};
std::atomic<bool> g_bn254_fr_halo2{false};

template <class Fr>
Fr two_adic_root() {
  Fr r;
  const uint64_t* src = Fr::Config::kTwoAdicRootMont64;
  if constexpr (std::is_same_v<Fr, Bn254Fr>) {
    if (g_bn254_fr_halo2.load()) src = kBn254FrHalo2TwoAdicRootMont64;
  }
  for (int i = 0; i < Fr::N / 2; ++i) {
    r.v[2 * i] = (uint32_t)src[i];
    r.v[2 * i + 1] = (uint32_t)(src[i] >> 32);
  }
  return r;
}

template <class Fr>
std::vector<Fr> host_powers(const Fr& base, const Fr& scale, size_t count) {
  std::vector<Fr> out(count);
  Fr p = scale;
  for (size_t i = 0; i < count; ++i) {
    out[i] = p;
    p = p * base;
  }
  return out;
}

// FourStepTw::tab29: entry (c_l << log_r) + k1 = w_N^((c0 + c_l) k1) of this
// rank (the direction's power tables in f) in R'-form (32 W mod p, W the
// canonical Montgomery value: five doublings, as tw29_table_kernel)
__global__ __launch_bounds__(kBlock) void fs_table29_kernel(FourStepTw<Bn254Fr> f, uint32_t log_r, size_t count,
                                                            fr29::TwMont29* __restrict__ out) {
  const size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= count) return;
  const uint32_t c_l = (uint32_t)(j >> log_r), k1 = (uint32_t)(j & ((size_t(1) << log_r) - 1));
  Bn254Fr x = fs_twiddle(f, k1, c_l).canonical();
#pragma unroll
  for (int i = 0; i < 5; ++i) x = (x + x).canonical();
  out[j].w = fr29::from_words(x.v);
}

// out[c][r] = in[r][c] for a rows x cols row-major matrix, through 32 x 32 LDS tiles
template <class Fr>
__global__ __launch_bounds__(kBlock) void transpose_kernel(const Fr* __restrict__ in, Fr* __restrict__ out,
                                                           uint32_t rows, uint32_t cols) {
  __shared__ Fr tile[32][33];
  const uint32_t c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const uint32_t tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (uint32_t j = ty; j < 32; j += 8) {
    const uint32_t r = r0 + j, c = c0 + tx;
    if (r < rows && c < cols) tile[j][tx] = in[(size_t)r * cols + c];
  }
  __syncthreads();
  for (uint32_t j = ty; j < 32; j += 8) {
    const uint32_t c = c0 + j, r = r0 + tx;
    if (r < rows && c < cols) out[(size_t)c * rows + r] = tile[tx][j];
  }
}

// forward: send[(h * Cg + c_l) * Rg + k1_l] = work[c_l * R + k1] * w^((c0 + c_l) k1), k1 = h Rg + k1_l
// inverse (unpack = true): out[c_l * R + k1] = recv[(h * Cg + c_l) * Rg + k1_l] * w^-((c0 + c_l) k1)
template <class Fr>
__global__ __launch_bounds__(kBlock) void twiddle_exchange_kernel(const Fr* __restrict__ in, Fr* __restrict__ out,
                                                                  uint32_t log_r, uint32_t log_rg, uint32_t log_cg,
                                                                  uint32_t c0, uint32_t log_n, const Fr* __restrict__ lo,
                                                                  const Fr* __restrict__ hi, uint32_t pow_bits,
                                                                  uint32_t unpack) {
  const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;  // position in the [c_l][k1] view
  if (i >= ((size_t)1 << (log_cg + log_r))) return;
  const uint32_t c_l = (uint32_t)(i >> log_r), k1 = (uint32_t)(i & ((1u << log_r) - 1));
  const uint32_t h = k1 >> log_rg, k1_l = k1 & ((1u << log_rg) - 1);
  const size_t j = (((size_t)h << log_cg) + c_l) * ((size_t)1 << log_rg) + k1_l;  // packed position
  const uint64_t e = ((uint64_t)(c0 + c_l) * k1) & ((uint64_t(1) << log_n) - 1);
  const Fr w = lo[e & ((1u << pow_bits) - 1)] * hi[e >> pow_bits];
  if (!unpack) out[j] = in[i] * w;
  else out[i] = in[j] * w;
}

}  // namespace

template <class Fr>
NttDomain<Fr>::NttDomain(size_t num_coeffs, hipStream_t stream) : stream_(stream) {
  require_gpu();
  log_n_ = 0;
  while ((size_t(1) << log_n_) < std::max<size_t>(num_coeffs, 1)) ++log_n_;
  if (log_n_ > (uint32_t)Fr::Config::kTwoAdicity || log_n_ > 30)
    throw std::runtime_error("tachyon_mi355x: NTT size exceeds the field's two-adicity");
  n_ = size_t(1) << log_n_;
  if (!stream_) {
    TA_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    own_stream_ = true;
  }
  // w_n = root^(2^(s - log n))  (PrimeFieldBase::GetRootOfUnity, prime_field_base.h:90-130)
  omega_ = two_adic_root<Fr>();
  for (uint32_t i = log_n_; i < (uint32_t)Fr::Config::kTwoAdicity; ++i) omega_ = omega_.sqr();
  omega_inv_ = omega_.inverse();
  size_inv_ = fr_from_u64<Fr>(n_).inverse();
  offset_ = Fr::one();
  offset_inv_ = Fr::one();

  // elements per workgroup (LDS footprint); TACHYON_NTT_LDS_ELEMS overrides it
  // in tuning builds only (-DTACHYON_TUNING_KNOBS, tools/tune_ntt.py)
  uint32_t lds_elems = kMaxLdsElems;
  uint32_t max_stages = kMaxPassStages;
#ifdef TACHYON_TUNING_KNOBS
  if (const char* e = getenv("TACHYON_NTT_LDS_ELEMS")) lds_elems = std::clamp<uint32_t>(atoi(e), 256, 4096);
  // (A/B of fewer, longer passes: 12 stages with 4096-element tiles = the
  // 2-pass 2^12 x 2^12 plan of 2^24, 128 KiB of LDS per workgroup)
  if (const char* e = getenv("TACHYON_NTT_PASS_STAGES")) max_stages = std::clamp<uint32_t>(atoi(e), 4, 12);
#endif
  // pass plan: ceil(L / 8) passes, stages split evenly
  if (log_n_ > 0) {
    uint32_t P = (log_n_ + max_stages - 1) / max_stages;
    uint32_t s0 = 0;
    for (uint32_t p = 0; p < P; ++p) {
      uint32_t k = (log_n_ - s0) / (P - p);
      Pass ps;
      ps.s0 = s0;
      ps.k = k;
      ps.final_pass = (s0 + k == log_n_);
      uint32_t avail = ps.final_pass ? (log_n_ - k) : (log_n_ - s0 - k);  // log2 of sets available
      uint32_t log_m = 0;
      while (log_m < avail && ((2u << log_m) << k) <= lds_elems) ++log_m;
      ps.log_m = log_m;
      plan_.push_back(ps);
      s0 += k;
    }
  }
  pow_bits_ = (log_n_ + 1) / 2;
  // stages per register step (1 = radix-2 through LDS every stage) and the
  // other schedule overrides: A/B measurements in tuning builds only
#ifdef TACHYON_TUNING_KNOBS
  if (const char* e = getenv("TACHYON_NTT_RADIX_LOG")) radix_ = std::clamp(atoi(e), 1, 3);
  if (const char* e = getenv("TACHYON_NTT_SHOUP")) shoup_mode_ = std::clamp(atoi(e), 0, 2);
  if (const char* e = getenv("TACHYON_NTT_VARIANT")) ntt_variant_ = std::clamp(atoi(e), 0, 3);
#endif
  ev_.resize(plan_.size() + 1);
  for (auto& e : ev_) TA_HIP(hipEventCreate(&e));
  build_twiddles();
  // BN254 Fr up to 2^20: the 29-bit passes by default -- fewer instructions
  // win while the clock holds (2^20 forward 0.126 -> 0.118 ms, inverse 0.133 ->
  // 0.127); from 2^22 the 32-bit ones are faster (2^24 1.78 vs 1.88 ms
  // forward; profiles/r04b/ntt_ab_32_vs_29_2_20_24.log).  set_variant(0)
  // forces the 32-bit passes.
  if constexpr (std::is_same_v<Fr, Bn254Fr>) {
    if (log_n_ >= 1 && log_n_ <= 20) {
      variant_ = 1;
      build_tables29();
    }
  }
}

template <class Fr>
NttDomain<Fr>::~NttDomain() {
  for (auto& e : ev_) (void)hipEventDestroy(e);
  if (own_stream_) (void)hipStreamDestroy(stream_);
}

template <class Fr>
void NttDomain<Fr>::build_twiddles() {
  if (log_n_ == 0) return;
  const uint32_t half = (uint32_t)(n_ / 2);
  const uint32_t lb = (log_n_ - 1 + 1) / 2;  // lo bits of the base table split
  const size_t lo_cnt = size_t(1) << lb;
  const size_t hi_cnt = std::max<size_t>(1, half >> lb);
  using Tw = typename NttTw<Fr>::type;
  constexpr bool kShoup = !std::is_same_v<Tw, Fr>;
  // Montgomery stage tables (stage s holds w^(j 2^s), j < n / 2^(s+1), at
  // offset n - (n >> s)): the twiddles of the 32-bit passes for fields without
  // Shoup entries, and the source of every other table (BN254 Fr: the 29-bit
  // tables now, the 32-bit Shoup ones on first use of set_variant bit 0)
  Fr* monts[2] = {kShoup ? static_cast<Fr*>(twm_fwd_.ensure(n_ * sizeof(Fr)))
                         : static_cast<Fr*>(tw_fwd_.ensure(n_ * sizeof(Tw))),
                  kShoup ? static_cast<Fr*>(twm_inv_.ensure(n_ * sizeof(Fr)))
                         : static_cast<Fr*>(tw_inv_.ensure(n_ * sizeof(Tw)))};
  DeviceBuffer lo_d, hi_d;
  Fr* lo = static_cast<Fr*>(lo_d.ensure(lo_cnt * sizeof(Fr)));
  Fr* hi = static_cast<Fr*>(hi_d.ensure(hi_cnt * sizeof(Fr)));
  for (int dir = 0; dir < 2; ++dir) {
    Fr w = dir == 0 ? omega_ : omega_inv_;
    std::vector<Fr> lo_h = host_powers(w, Fr::one(), lo_cnt);
    Fr w_step = w;
    for (uint32_t i = 0; i < lb; ++i) w_step = w_step.sqr();
    std::vector<Fr> hi_h = host_powers(w_step, Fr::one(), hi_cnt);
    TA_HIP(hipMemcpyAsync(lo, lo_h.data(), lo_cnt * sizeof(Fr), hipMemcpyHostToDevice, stream_));
    TA_HIP(hipMemcpyAsync(hi, hi_h.data(), hi_cnt * sizeof(Fr), hipMemcpyHostToDevice, stream_));
    Fr* mont = monts[dir];
    hipLaunchKernelGGL(twiddle_base_kernel<Fr>, dim3(ceil_div(half, kBlock)), dim3(kBlock), 0, stream_, mont, half,
                       lo, hi, lb);
    for (uint32_t s = 1; s < log_n_; ++s) {
      uint32_t cnt = (uint32_t)(n_ >> (s + 1));
      hipLaunchKernelGGL(twiddle_stage_kernel<Fr>, dim3(ceil_div(cnt, kBlock)), dim3(kBlock), 0, stream_,
                         mont + (n_ - (n_ >> s)), mont, cnt, s);
    }
    TA_HIP(hipGetLastError());
    TA_HIP(hipStreamSynchronize(stream_));  // host vectors go out of scope
  }
  if constexpr (kShoup) ensure_tables32();  // (the 29-bit tables are built on first use of variant bit 0)
}

// BN254 Fr: the 29-bit tables from the Montgomery stage tables (tw29_table_kernel)
template <class Fr>
void NttDomain<Fr>::build_tables29() {
  if constexpr (std::is_same_v<Fr, Bn254Fr>) {
    if (tables29_ || log_n_ == 0) return;
    tables29_ = true;
    const uint32_t k0 = plan_.empty() ? log_n_ : plan_[0].k;
    const size_t count = n_ - 1;  // all stage tables
    split29_ = n_ - (n_ >> k0);
    const size_t nshoup = count - split29_;
    DeviceBuffer* bm[2] = {&t29m_fwd_, &t29m_inv_};
    DeviceBuffer* bs[2] = {&t29s_fwd_, &t29s_inv_};
    const Fr* mont[2] = {twm_fwd_.as<Fr>(), twm_inv_.as<Fr>()};
    for (int dir = 0; dir < 2; ++dir) {
      auto* m29 = static_cast<fr29::TwMont29*>(bm[dir]->ensure(std::max<size_t>(1, split29_) * sizeof(fr29::TwMont29)));
      auto* s29 = static_cast<fr29::TwShoup29*>(bs[dir]->ensure(std::max<size_t>(1, nshoup) * sizeof(fr29::TwShoup29)));
      hipLaunchKernelGGL(tw29_table_kernel, dim3(ceil_div(count, kBlock)), dim3(kBlock), 0, stream_, m29, s29,
                         mont[dir], (uint32_t)split29_, (uint32_t)count);
    }
    TA_HIP(hipGetLastError());
    TA_HIP(hipStreamSynchronize(stream_));
  }
}

// The 32-bit Shoup tables {plain w, floor(w 2^256 / p)} of dif_pass_kernel's
// later passes (BN254 Fr under set_variant bit 0)
template <class Fr>
void NttDomain<Fr>::ensure_tables32() {
  using Tw = typename NttTw<Fr>::type;
  if constexpr (!std::is_same_v<Tw, Fr>) {
    if (tables32_ || log_n_ == 0) return;
    const uint32_t count = (uint32_t)(n_ - 1);
    Tw* tab[2] = {static_cast<Tw*>(tw_fwd_.ensure(n_ * sizeof(Tw))), static_cast<Tw*>(tw_inv_.ensure(n_ * sizeof(Tw)))};
    const Fr* mont[2] = {twm_fwd_.as<Fr>(), twm_inv_.as<Fr>()};
    for (int dir = 0; dir < 2; ++dir)
      hipLaunchKernelGGL(shoup_table_kernel<Fr>, dim3(ceil_div(count, kBlock)), dim3(kBlock), 0, stream_, tab[dir],
                         mont[dir], count);
    TA_HIP(hipGetLastError());
    TA_HIP(hipStreamSynchronize(stream_));
    tables32_ = true;
  }
}

template <class Fr>
bool NttDomain<Fr>::set_variant(int v) {
  if (v < 0 || v > 7 || (v & 3) == 2) return false;  // bit 1 (the LDS swizzle) modifies bit 0
  if ((v & 3) != 0 && !std::is_same_v<Fr, Bn254Fr>) return false;
  variant_ = v;
  if (v & 1) build_tables29();
  return true;
}

// A one-pass transform (<= 8 stages) smaller than a tile of kMaxLdsElems: 2^p
// batch entries per workgroup (the largest p with 2^p | batch and 2^(L + p)
// elements in the tile) instead of one entry using 2^L / 4 of its 256 threads
// -- the 2^8-point column NTTs of the four-step's 2^8 x 2^16 split.  Variant
// bit 2 turns it off (A/B).
template <class Fr>
uint32_t NttDomain<Fr>::pack_log(size_t batch) const {
  if (plan_.size() != 1 || batch < 2 || (variant_ & 4)) return 0;
  uint32_t p = 0;
  while (batch % (size_t(2) << p) == 0 && (n_ << (p + 1)) <= kMaxLdsElems) ++p;
  return p;
}

template <class Fr>
void NttDomain<Fr>::build_powers(const Fr& base, const Fr& scale, Fr* d_lo, Fr* d_hi) {
  const size_t lo_cnt = size_t(1) << pow_bits_;
  const size_t hi_cnt = std::max<size_t>(1, n_ >> pow_bits_);
  std::vector<Fr> lo_h = host_powers(base, scale, lo_cnt);
  Fr step = base;
  for (uint32_t i = 0; i < pow_bits_; ++i) step = step.sqr();
  std::vector<Fr> hi_h = host_powers(step, Fr::one(), hi_cnt);
  TA_HIP(hipMemcpyAsync(d_lo, lo_h.data(), lo_cnt * sizeof(Fr), hipMemcpyHostToDevice, stream_));
  TA_HIP(hipMemcpyAsync(d_hi, hi_h.data(), hi_cnt * sizeof(Fr), hipMemcpyHostToDevice, stream_));
  TA_HIP(hipStreamSynchronize(stream_));
}

template <class Fr>
void NttDomain<Fr>::set_offset(const Fr& h) {
  offset_ = h;
  has_offset_ = !h.is_one();
  offset_inv_ = has_offset_ ? h.inverse() : Fr::one();
  if (!has_offset_) return;
  const size_t lo_cnt = size_t(1) << pow_bits_;
  const size_t hi_cnt = std::max<size_t>(1, n_ >> pow_bits_);
  // forward: multiply input i by h^i ; inverse: output i by n^-1 h^-i
  build_powers(h, Fr::one(), static_cast<Fr*>(coset_lo_.ensure(lo_cnt * sizeof(Fr))),
               static_cast<Fr*>(coset_hi_.ensure(hi_cnt * sizeof(Fr))));
  build_powers(offset_inv_, size_inv_, static_cast<Fr*>(icoset_lo_.ensure(lo_cnt * sizeof(Fr))),
               static_cast<Fr*>(icoset_hi_.ensure(hi_cnt * sizeof(Fr))));
}

template <class Fr>
void NttDomain<Fr>::run(Fr* d_data, bool inverse, size_t batch, const Fr* src_in, const FourStepTw<Fr>* fs) {
  if (log_n_ == 0 || batch == 0) {
    // size-1 domain: forward is the identity (h^0 = 1); inverse scales by n^-1 = 1
    if (fs) throw std::runtime_error("tachyon_mi355x: four-step sub-transforms need >= 2 points");
    if (src_in && src_in != d_data && batch)
      TA_HIP(hipMemcpyAsync(d_data, src_in, batch * n_ * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
    return;
  }
  if (batch > 65535) throw std::runtime_error("tachyon_mi355x: NTT batch exceeds the grid limit");
  if constexpr (std::is_same_v<Fr, Bn254Fr>) {
    if (variant_ & 1) return run29(d_data, inverse, batch, src_in, fs);
  }
  using Tw = typename NttTw<Fr>::type;
  constexpr bool kShoup = !std::is_same_v<Tw, Fr>;
  const Tw* tw = inverse ? tw_inv_.as<Tw>() : tw_fwd_.as<Tw>();
  const Fr* twm = kShoup ? (inverse ? twm_inv_.as<Fr>() : twm_fwd_.as<Fr>()) : reinterpret_cast<const Fr*>(tw);
  Fr* scratch = plan_.size() > 1 ? static_cast<Fr*>(scratch_.ensure(batch * n_ * sizeof(Fr))) : d_data;
  if (profile_) TA_HIP(hipEventRecord(ev_[0], stream_));
  for (size_t p = 0; p < plan_.size(); ++p) {
    const Pass& ps = plan_[p];
    PassArgs<Fr> a{};
    a.L = log_n_;
    a.s0 = ps.s0;
    a.k = ps.k;
    a.log_m = ps.log_m;
    a.final_pass = ps.final_pass ? 1u : 0u;
    a.pow_bits = pow_bits_;
    a.mode = 0;
    if (p == 0 && !inverse && has_offset_) {
      a.mode |= kLoadCoset;
      a.load_lo = coset_lo_.as<Fr>();
      a.load_hi = coset_hi_.as<Fr>();
    }
    if (ps.final_pass && inverse) {
      if (has_offset_) {
        a.mode |= kStoreCoset;
        a.store_lo = icoset_lo_.as<Fr>();
        a.store_hi = icoset_hi_.as<Fr>();
      } else {
        a.mode |= kStoreScale;
        a.scale = size_inv_;
      }
    }
    if (fs) {
      a.fs = *fs;
      if (fs->rows) {
        if (p == 0 && !inverse) a.mode |= kLoadXch;
        if (ps.final_pass && inverse) a.mode |= kStoreXch;
      } else {
        if (p == 0 && inverse) a.mode |= kLoadTw4;
        if (ps.final_pass && !inverse) a.mode |= kStoreTw4;
      }
    }
    // first pass: data (or src_in) -> scratch; middle: scratch in place; last: scratch -> data
    const Fr* src = (p == 0) ? (src_in ? src_in : d_data) : scratch;
    Fr* dst = ps.final_pass ? d_data : scratch;
    // a one-pass transform smaller than a tile: several batch entries per workgroup
    a.pack = pack_log(batch);
    if (a.pack) a.log_m = a.pack;
    uint32_t elems = (1u << a.log_m) << ps.k;
    uint32_t blocks = a.pack ? 1u : (uint32_t)(n_ / elems);
    const uint32_t gy = (uint32_t)(batch >> a.pack);
    size_t lds = (size_t)elems * sizeof(Fr);
    // Shoup twiddles (64 B) in the passes whose stage tables are small and
    // cache-resident; Montgomery twiddles (32 B) where the tables stream from
    // HBM -- the first pass reads the big tables of stages 0.. once each
    // (TACHYON_NTT_SHOUP: 0 = Montgomery everywhere, 1 = Shoup everywhere)
    const bool shoup = kShoup && (shoup_mode_ == 1 || (shoup_mode_ == 2 && p > 0));
    // (A/B, TACHYON_NTT_VARIANT: bit 0 = the Montgomery radix-4 pass at >= 5
    // waves/SIMD, bit 1 = the Shoup radix-4 passes without the twiddle
    // prefetch at >= 5 waves/SIMD)
#ifdef TACHYON_TUNING_KNOBS
    // tiles above 64 KiB (TACHYON_NTT_LDS_ELEMS > 2048) need the kernel's dynamic-LDS limit raised
    auto allow = [&](const void* k) {
      if (lds > 64 * 1024) TA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    };
    if (shoup) {
      auto kern = radix_ == 1 ? dif_pass_kernel<Fr, Tw, 1> : radix_ == 2 ? dif_pass_kernel<Fr, Tw, 2>
                                                                         : dif_pass_kernel<Fr, Tw, 3>;
      if (radix_ == 2 && (ntt_variant_ & 2)) kern = dif_pass_kernel<Fr, Tw, 2, false, 5>;
      allow(reinterpret_cast<const void*>(kern));
      hipLaunchKernelGGL(kern, dim3(blocks, gy), dim3(kBlock), lds, stream_, src, dst, tw, a);
    } else {
      auto kern = radix_ == 1 ? dif_pass_kernel<Fr, Fr, 1> : radix_ == 2 ? dif_pass_kernel<Fr, Fr, 2>
                                                                         : dif_pass_kernel<Fr, Fr, 3>;
      if (radix_ == 2 && (ntt_variant_ & 1)) kern = dif_pass_kernel<Fr, Fr, 2, true, 5>;
      allow(reinterpret_cast<const void*>(kern));
      hipLaunchKernelGGL(kern, dim3(blocks, gy), dim3(kBlock), lds, stream_, src, dst, twm, a);
    }
#else
    // release schedule: radix-4 register steps (2 DIF stages per LDS round trip)
    if (lds > 64 * 1024) throw std::runtime_error("tachyon_mi355x: NTT pass tile above 64 KiB in a release build");
    if (shoup)
      hipLaunchKernelGGL((dif_pass_kernel<Fr, Tw, 2>), dim3(blocks, gy), dim3(kBlock), lds, stream_, src,
                         dst, tw, a);
    else
      hipLaunchKernelGGL((dif_pass_kernel<Fr, Fr, 2>), dim3(blocks, gy), dim3(kBlock), lds, stream_, src,
                         dst, twm, a);
#endif
    TA_HIP(hipGetLastError());
    if (profile_) TA_HIP(hipEventRecord(ev_[p + 1], stream_));
  }
  if (profile_) {
    TA_HIP(hipEventSynchronize(ev_[plan_.size()]));
    timings_.passes.assign(plan_.size(), 0.f);
    for (size_t p = 0; p < plan_.size(); ++p) TA_HIP(hipEventElapsedTime(&timings_.passes[p], ev_[p], ev_[p + 1]));
    TA_HIP(hipEventElapsedTime(&timings_.total, ev_[0], ev_[plan_.size()]));
  }
}


// BN254 Fr: the passes over 9 x 29-bit limbs (dif29_pass_kernel); the same
// pass plan, modes and scratch discipline as run()
template <class Fr>
void NttDomain<Fr>::run29(Fr* d_data, bool inverse, size_t batch, const Fr* src_in, const FourStepTw<Fr>* fs) {
  if constexpr (std::is_same_v<Fr, Bn254Fr>) {
    const auto* tm = (inverse ? t29m_inv_ : t29m_fwd_).template as<fr29::TwMont29>();
    const auto* ts = (inverse ? t29s_inv_ : t29s_fwd_).template as<fr29::TwShoup29>();
    F29* scratch = plan_.size() > 1 ? static_cast<F29*>(scratch29_.ensure(batch * n_ * sizeof(F29))) : nullptr;
    if (profile_) TA_HIP(hipEventRecord(ev_[0], stream_));
    for (size_t p = 0; p < plan_.size(); ++p) {
      const Pass& ps = plan_[p];
      PassArgs<Fr> a{};
      a.L = log_n_;
      a.s0 = ps.s0;
      a.k = ps.k;
      a.log_m = ps.log_m;
      a.final_pass = ps.final_pass ? 1u : 0u;
      a.pow_bits = pow_bits_;
      a.mode = 0;
      if (p == 0 && !inverse && has_offset_) {
        a.mode |= kLoadCoset;
        a.load_lo = coset_lo_.as<Fr>();
        a.load_hi = coset_hi_.as<Fr>();
      }
      if (ps.final_pass && inverse) {
        if (has_offset_) {
          a.mode |= kStoreCoset;
          a.store_lo = icoset_lo_.as<Fr>();
          a.store_hi = icoset_hi_.as<Fr>();
        } else {
          a.mode |= kStoreScale;
          a.scale = size_inv_;
        }
      }
      if (fs) {
        a.fs = *fs;
        if (fs->rows) {
          if (p == 0 && !inverse) a.mode |= kLoadXch;
          if (ps.final_pass && inverse) a.mode |= kStoreXch;
        } else {
          if (p == 0 && inverse) a.mode |= kLoadTw4;
          if (ps.final_pass && !inverse) a.mode |= kStoreTw4;
        }
      }
      // first pass: data / src_in (32 B) -> scratch (36 B); middle: scratch in place; last: scratch -> data
      const void* src = (p == 0) ? static_cast<const void*>(src_in ? src_in : d_data) : scratch;
      void* dst = ps.final_pass ? static_cast<void*>(d_data) : scratch;
      a.pack = pack_log(batch);  // a one-pass transform smaller than a tile: several entries per workgroup
      if (a.pack) a.log_m = a.pack;
      const uint32_t elems = (1u << a.log_m) << ps.k;
      const uint32_t blocks = a.pack ? 1u : (uint32_t)(n_ / elems);
      const uint32_t gy = (uint32_t)(batch >> a.pack);
      // the 29-bit kernel's LDS planes are sized for kMaxLdsElems (tuning plans with larger tiles: 32-bit only)
      if (elems > kMaxLdsElems) throw std::runtime_error("tachyon_mi355x: 29-bit NTT pass tile above its LDS planes");
      const bool swz = (variant_ & 2) != 0;
      if (p == 0) {
        auto* k0 = swz ? &dif29_pass_kernel<true, true, fr29::TwMont29> : &dif29_pass_kernel<true, false, fr29::TwMont29>;
        hipLaunchKernelGGL(k0, dim3(blocks, gy), dim3(kBlock), 0, stream_, src, dst,
                           Tw29Table<fr29::TwMont29>{tm, 0u}, a);
      } else {
        auto* k1 = swz ? &dif29_pass_kernel<false, true, fr29::TwShoup29>
                       : &dif29_pass_kernel<false, false, fr29::TwShoup29>;
        hipLaunchKernelGGL(k1, dim3(blocks, gy), dim3(kBlock), 0, stream_, src, dst,
                           Tw29Table<fr29::TwShoup29>{ts, (uint32_t)split29_}, a);
      }
      TA_HIP(hipGetLastError());
      if (profile_) TA_HIP(hipEventRecord(ev_[p + 1], stream_));
    }
    if (profile_) {
      TA_HIP(hipEventSynchronize(ev_[plan_.size()]));
      timings_.passes.assign(plan_.size(), 0.f);
      for (size_t p = 0; p < plan_.size(); ++p) TA_HIP(hipEventElapsedTime(&timings_.passes[p], ev_[p], ev_[p + 1]));
      TA_HIP(hipEventElapsedTime(&timings_.total, ev_[0], ev_[plan_.size()]));
    }
  }
}

template <class Fr>
void NttDomain<Fr>::forward_device(Fr* d_data, size_t batch) { run(d_data, false, batch); }

template <class Fr>
void NttDomain<Fr>::transform_device(const Fr* src, Fr* dst, bool inverse, size_t batch, const FourStepTw<Fr>* fs) {
  run(dst, inverse, batch, src, fs);
}

template <class Fr>
void NttDomain<Fr>::inverse_device(Fr* d_data, size_t batch) { run(d_data, true, batch); }

template <class Fr>
void NttDomain<Fr>::forward_host(const Fr* in, size_t len, Fr* out) {
  if (len > n_) throw std::runtime_error("tachyon_mi355x: FFT input longer than the domain");
  Fr* d = static_cast<Fr*>(io_.ensure(n_ * sizeof(Fr)));
  TA_HIP(hipMemcpyAsync(d, in, len * sizeof(Fr), hipMemcpyHostToDevice, stream_));
  if (len < n_) TA_HIP(hipMemsetAsync(d + len, 0, (n_ - len) * sizeof(Fr), stream_));
  run(d, false, 1);
  TA_HIP(hipMemcpyAsync(out, d, n_ * sizeof(Fr), hipMemcpyDeviceToHost, stream_));
  TA_HIP(hipStreamSynchronize(stream_));
}

template <class Fr>
void NttDomain<Fr>::inverse_host(const Fr* in, size_t len, Fr* out) {
  if (len > n_) throw std::runtime_error("tachyon_mi355x: IFFT input longer than the domain");
  Fr* d = static_cast<Fr*>(io_.ensure(n_ * sizeof(Fr)));
  TA_HIP(hipMemcpyAsync(d, in, len * sizeof(Fr), hipMemcpyHostToDevice, stream_));
  if (len < n_) TA_HIP(hipMemsetAsync(d + len, 0, (n_ - len) * sizeof(Fr), stream_));
  run(d, true, 1);
  TA_HIP(hipMemcpyAsync(out, d, n_ * sizeof(Fr), hipMemcpyDeviceToHost, stream_));
  TA_HIP(hipStreamSynchronize(stream_));
}

template <class Fr>
Ntt4Step<Fr>::Ntt4Step(uint32_t log_n, uint32_t log_world, uint32_t rank, hipStream_t stream, uint32_t log_r)
    : log_n_(log_n), log_g_(log_world), rank_(rank), n_(size_t(1) << log_n), stream_(stream) {
  require_gpu();
  log_r_ = log_r ? log_r : log_n / 2;
  if (log_r_ >= log_n) throw std::runtime_error("tachyon_mi355x: four-step NTT needs 1 <= log R < log n");
  log_c_ = log_n - log_r_;
  if (log_g_ > log_r_ || log_g_ > log_c_ || rank >= (1u << log_g_) || log_n > (uint32_t)Fr::Config::kTwoAdicity ||
      log_n > 30)
    throw std::runtime_error("tachyon_mi355x: four-step NTT needs R, C >= world size");
  if (!stream_) {
    TA_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    own_stream_ = true;
  }
  dom_r_ = new NttDomain<Fr>(size_t(1) << log_r_, stream_);
  dom_c_ = new NttDomain<Fr>(size_t(1) << log_c_, stream_);
  // w_n and its two-level power tables (w_n^e = lo[e & mask] * hi[e >> bits])
  Fr w = two_adic_root<Fr>();
  for (uint32_t i = log_n; i < (uint32_t)Fr::Config::kTwoAdicity; ++i) w = w.sqr();
  w_ = w;
  pow_bits_ = (log_n + 1) / 2;
  const size_t lo_cnt = size_t(1) << pow_bits_, hi_cnt = size_t(1) << (log_n - pow_bits_);
  const Fr wi = w.inverse();
  DeviceBuffer* bufs[4] = {&w_lo_, &w_hi_, &wi_lo_, &wi_hi_};
  const Fr bases[2] = {w, wi};
  for (int d = 0; d < 2; ++d) {
    Fr step = bases[d];
    for (uint32_t i = 0; i < pow_bits_; ++i) step = step.sqr();
    std::vector<Fr> lo_h = host_powers(bases[d], Fr::one(), lo_cnt);
    std::vector<Fr> hi_h = host_powers(step, Fr::one(), hi_cnt);
    TA_HIP(hipMemcpyAsync(bufs[2 * d]->ensure(lo_cnt * sizeof(Fr)), lo_h.data(), lo_cnt * sizeof(Fr),
                          hipMemcpyHostToDevice, stream_));
    TA_HIP(hipMemcpyAsync(bufs[2 * d + 1]->ensure(hi_cnt * sizeof(Fr)), hi_h.data(), hi_cnt * sizeof(Fr),
                          hipMemcpyHostToDevice, stream_));
    TA_HIP(hipStreamSynchronize(stream_));
  }
}

template <class Fr>
Ntt4Step<Fr>::~Ntt4Step() {
  delete dom_r_;
  delete dom_c_;
  if (own_stream_) (void)hipStreamDestroy(stream_);
}

// Stage 1 forward: the R-point NTTs of the local columns read `in` directly
// (no copy) and their last pass multiplies by w_n^(c k1) and writes the packed
// send layout (no separate twiddle kernel): two HBM round trips for R <= 2^16.
// (Before round 5: a copy, the passes, and twiddle_exchange_kernel -- kept as
// the unfused path, fused_ = false, for A/B.)
// The exchange twiddles of one direction as FourStepTw::tab29, built on first
// use when the column NTTs run on the 29-bit passes (nullptr otherwise: the
// 32-bit passes compute them)
template <class Fr>
const void* Ntt4Step<Fr>::exchange_table(bool inverse) {
  if constexpr (!std::is_same_v<Fr, Bn254Fr>) {
    (void)inverse;
    return nullptr;
  } else {
    if (!(dom_r_->variant() & 1) || no_table_) return nullptr;
    DeviceBuffer& t = inverse ? tab29_inv_ : tab29_fwd_;
    if (!t.capacity()) {
      const uint32_t log_cg = log_c_ - log_g_, log_rg = log_r_ - log_g_;
      const FourStepTw<Fr> f{inverse ? wi_lo_.as<Fr>() : w_lo_.as<Fr>(), inverse ? wi_hi_.as<Fr>() : w_hi_.as<Fr>(),
                             pow_bits_, log_n_, log_rg, log_cg, rank_ << log_cg};
      const size_t count = local_size();
      auto* out = static_cast<fr29::TwMont29*>(t.ensure(count * sizeof(fr29::TwMont29)));
      hipLaunchKernelGGL(fs_table29_kernel, dim3(ceil_div(count, kBlock)), dim3(kBlock), 0, stream_, f, log_r_, count,
                         out);
      TA_HIP(hipGetLastError());
    }
    return t.as<void>();
  }
}

template <class Fr>
void Ntt4Step<Fr>::forward_stage1(const Fr* in, Fr* send) {
  const size_t m = local_size();
  const uint32_t log_cg = log_c_ - log_g_, log_rg = log_r_ - log_g_;
  if (fused_) {
    FourStepTw<Fr> fs{w_lo_.as<Fr>(), w_hi_.as<Fr>(), pow_bits_, log_n_, log_rg, log_cg, rank_ << log_cg};
    fs.tab29 = exchange_table(false);
    fs.log_r = log_r_;
    dom_r_->transform_device(in, send, false, size_t(1) << log_cg, &fs);
    return;
  }
  Fr* work = static_cast<Fr*>(work_.ensure(m * sizeof(Fr)));
  TA_HIP(hipMemcpyAsync(work, in, m * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
  dom_r_->forward_device(work, size_t(1) << log_cg);
  hipLaunchKernelGGL(twiddle_exchange_kernel<Fr>, dim3(ceil_div(m, kBlock)), dim3(kBlock), 0, stream_, work, send,
                     log_r_, log_rg, log_cg, rank_ << log_cg, log_n_, w_lo_.as<Fr>(), w_hi_.as<Fr>(), pow_bits_, 0u);
  TA_HIP(hipGetLastError());
}

template <class Fr>
void Ntt4Step<Fr>::forward_stage2(const Fr* recv, Fr* out) {
  const uint32_t log_cg = log_c_ - log_g_, log_rg = log_r_ - log_g_;
  if (fused_) {
    // recv = G chunks [k1_l][c_l] (fs_packed): the C-point NTTs' first pass
    // reads each local row k1_l as G runs of Cg elements (kLoadXch) -- no
    // transpose.  A one-pass C NTT in place would read what other workgroups
    // write: recv goes through the work buffer then.
    FourStepTw<Fr> fs{};
    fs.log_rg = log_rg;
    fs.log_cg = log_cg;
    fs.rows = 1;
    const Fr* src = recv;
    if (recv == out && dom_c_->plan().size() == 1) {
      Fr* work = static_cast<Fr*>(work_.ensure(local_size() * sizeof(Fr)));
      TA_HIP(hipMemcpyAsync(work, recv, local_size() * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
      src = work;
    }
    dom_c_->transform_device(src, out, false, size_t(1) << log_rg, &fs);
    return;
  }
  // round 4: recv = [c][k1_l] (C x Rg) -> out = [k1_l][c], then C-point NTTs on the rows
  const uint32_t rows = 1u << log_c_, cols = 1u << log_rg;
  hipLaunchKernelGGL(transpose_kernel<Fr>, dim3(ceil_div(cols, 32), ceil_div(rows, 32)), dim3(kBlock), 0, stream_,
                     recv, out, rows, cols);
  TA_HIP(hipGetLastError());
  dom_c_->forward_device(out, cols);
}

template <class Fr>
void Ntt4Step<Fr>::inverse_stage1(const Fr* in, Fr* send) {
  // in = [k1_l][k2] (Rg x C): inverse C-point NTTs on the rows
  const size_t m = local_size();
  const uint32_t log_cg = log_c_ - log_g_, log_rg = log_r_ - log_g_;
  const uint32_t rows = 1u << log_rg, cols = 1u << log_c_;
  if (fused_) {
    // the last pass writes the exchange layout, G chunks [k1_l][c_l]
    // (kStoreXch) -- no transpose; in place (in == send) through the work buffer
    FourStepTw<Fr> fs{};
    fs.log_rg = log_rg;
    fs.log_cg = log_cg;
    fs.rows = 1;
    if (in == send) {
      Fr* work = static_cast<Fr*>(work_.ensure(m * sizeof(Fr)));
      dom_c_->transform_device(in, work, true, rows, &fs);
      TA_HIP(hipMemcpyAsync(send, work, m * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
    } else {
      dom_c_->transform_device(in, send, true, rows, &fs);
    }
    return;
  }
  // round 4: a copy, the inverse passes, then the transpose to [c][k1_l] = G chunks [c_l][k1_l]
  Fr* work = static_cast<Fr*>(work_.ensure(m * sizeof(Fr)));
  TA_HIP(hipMemcpyAsync(work, in, m * sizeof(Fr), hipMemcpyDeviceToDevice, stream_));
  dom_c_->inverse_device(work, rows);
  hipLaunchKernelGGL(transpose_kernel<Fr>, dim3(ceil_div(cols, 32), ceil_div(rows, 32)), dim3(kBlock), 0, stream_,
                     work, send, rows, cols);
  TA_HIP(hipGetLastError());
}

template <class Fr>
void Ntt4Step<Fr>::inverse_stage2(const Fr* recv, Fr* out) {
  const size_t m = local_size();
  const uint32_t log_cg = log_c_ - log_g_, log_rg = log_r_ - log_g_;
  if (fused_) {  // the unpack and w_n^-(c k1) in the first pass's load
    FourStepTw<Fr> fs{wi_lo_.as<Fr>(), wi_hi_.as<Fr>(), pow_bits_, log_n_, log_rg, log_cg, rank_ << log_cg};
    fs.tab29 = exchange_table(true);
    fs.log_r = log_r_;
    dom_r_->transform_device(recv, out, true, size_t(1) << log_cg, &fs);
    return;
  }
  hipLaunchKernelGGL(twiddle_exchange_kernel<Fr>, dim3(ceil_div(m, kBlock)), dim3(kBlock), 0, stream_, recv, out,
                     log_r_, log_rg, log_cg, rank_ << log_cg, log_n_, wi_lo_.as<Fr>(), wi_hi_.as<Fr>(), pow_bits_, 1u);
  TA_HIP(hipGetLastError());
  dom_r_->inverse_device(out, size_t(1) << log_cg);
}

template <class Fr>
NttMultiDevice<Fr>::NttMultiDevice(uint32_t log_n, const std::vector<int>& devices, int primary,
                                   hipStream_t primary_stream)
    : log_n_(log_n), n_(size_t(1) << log_n), primary_(primary), s0_(primary_stream), ids_(devices) {
  const size_t G = devices.size();
  if (G < 2 || (G & (G - 1))) throw std::runtime_error("tachyon_mi355x: multi-device NTT needs 2^k >= 2 devices");
  log_g_ = (uint32_t)__builtin_ctzll(G);
  log_r_ = ntt4_split_log_r(log_n, log_g_);  // the fewest pass launches (2^24: 2^8 x 2^16)
  log_c_ = log_n - log_r_;
  if (log_g_ > log_r_ || log_g_ > log_c_)
    throw std::runtime_error("tachyon_mi355x: multi-device NTT needs R, C >= devices");
  int count = 0, prev = 0;
  TA_HIP(hipGetDeviceCount(&count));
  for (int d : devices)
    if (d < 0 || d >= count) throw std::runtime_error("tachyon_mi355x: device id out of range");
  TA_HIP(hipGetDevice(&prev));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  TA_HIP(hipSetDevice(primary_));
  TA_HIP(hipEventCreateWithFlags(&ev0_, hipEventDisableTiming));
  for (int d : devices)  // xGMI peer access where the pair supports it (copies work without it)
    if (d != primary_) {
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, primary_, d) == hipSuccess && ok) (void)hipDeviceEnablePeerAccess(d, 0);
      (void)hipGetLastError();
    }
  for (size_t g = 0; g < G; ++g) {
    TA_HIP(hipSetDevice(devices[g]));
    auto p = std::make_unique<Part>();
    p->device = devices[g];
    TA_HIP(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    TA_HIP(hipEventCreateWithFlags(&p->ev1, hipEventDisableTiming));
    TA_HIP(hipEventCreateWithFlags(&p->ev2, hipEventDisableTiming));
    p->plan = std::make_unique<Ntt4Step<Fr>>(log_n, log_g_, (uint32_t)g, p->stream, log_r_);
    const size_t m = n_ >> log_g_;
    p->in.ensure(m * sizeof(Fr));
    p->send.ensure(m * sizeof(Fr));
    p->recv.ensure(m * sizeof(Fr));
    p->out.ensure(m * sizeof(Fr));
    for (int e : devices)
      if (e != devices[g]) {
        int ok = 0;
        if (hipDeviceCanAccessPeer(&ok, devices[g], e) == hipSuccess && ok) (void)hipDeviceEnablePeerAccess(e, 0);
        (void)hipGetLastError();
      }
    parts_.push_back(std::move(p));
  }
  TA_HIP(hipSetDevice(primary_));
  stage_.ensure(n_ * sizeof(Fr));
}

template <class Fr>
NttMultiDevice<Fr>::~NttMultiDevice() {
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) prev = 0;
  for (auto& p : parts_) {  // each part's stream, events and buffers on its own device
    (void)hipSetDevice(p->device);
    (void)hipStreamSynchronize(p->stream);
    p->plan.reset();
    p->in.release();
    p->send.release();
    p->recv.release();
    p->out.release();
    (void)hipEventDestroy(p->ev1);
    (void)hipEventDestroy(p->ev2);
    (void)hipStreamDestroy(p->stream);
  }
  (void)hipSetDevice(primary_);
  (void)hipStreamSynchronize(s0_);
  stage_.release();
  io_.release();
  if (ev0_) (void)hipEventDestroy(ev0_);
  (void)hipSetDevice(prev);
}

// forward: stage = x^T (x as R x C), part g's input = stage chunk g (its
//   columns, column-major); stage 1; all-to-all; stage 2 -> rows [g R/G,
//   (g+1) R/G) of Z[k1][k2] = X[k1 + R k2]; the parts' rows = Z (R x C) in
//   stage; y = Z^T.  Both transposes take an R x C matrix.
// inverse: stage = Z = y^T (y as C x R), part g's input = rows chunk g;
//   inverse stages 1, 2 -> columns; the parts' columns = x^T (C x R); x = its
//   transpose.  Both transposes take a C x R matrix.
template <class Fr>
void NttMultiDevice<Fr>::run(const Fr* x, Fr* y, bool inverse) {
  const size_t G = parts_.size(), m = n_ >> log_g_, chunk = m >> log_g_;
  const uint32_t R = 1u << log_r_, C = 1u << log_c_;
  const uint32_t rows_in = inverse ? C : R, cols_in = inverse ? R : C;
  int prev = 0;
  TA_HIP(hipGetDevice(&prev));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  TA_HIP(hipSetDevice(primary_));
  Fr* stage = stage_.as<Fr>();
  hipLaunchKernelGGL(transpose_kernel<Fr>, dim3(ceil_div(cols_in, 32), ceil_div(rows_in, 32)), dim3(kBlock), 0, s0_,
                     x, stage, rows_in, cols_in);
  TA_HIP(hipGetLastError());
  TA_HIP(hipEventRecord(ev0_, s0_));
  for (size_t g = 0; g < G; ++g) {  // scatter + stage 1
    Part& p = *parts_[g];
    TA_HIP(hipSetDevice(p.device));
    TA_HIP(hipStreamWaitEvent(p.stream, ev0_, 0));
    TA_HIP(hipMemcpyPeerAsync(p.in.template as<void>(), p.device, stage + g * m, primary_, m * sizeof(Fr), p.stream));
    if (inverse) p.plan->inverse_stage1(p.in.template as<Fr>(), p.send.template as<Fr>());
    else p.plan->forward_stage1(p.in.template as<Fr>(), p.send.template as<Fr>());
    TA_HIP(hipEventRecord(p.ev1, p.stream));
  }
  for (size_t h = 0; h < G; ++h) {  // all-to-all: chunk h of every part's send -> part h's recv + stage 2
    Part& q = *parts_[h];
    TA_HIP(hipSetDevice(q.device));
    for (size_t g = 0; g < G; ++g) TA_HIP(hipStreamWaitEvent(q.stream, parts_[g]->ev1, 0));
    for (size_t g = 0; g < G; ++g)
      TA_HIP(hipMemcpyPeerAsync(q.recv.template as<Fr>() + g * chunk, q.device, parts_[g]->send.template as<Fr>() + h * chunk,
                                parts_[g]->device, chunk * sizeof(Fr), q.stream));
    if (inverse) q.plan->inverse_stage2(q.recv.template as<Fr>(), q.out.template as<Fr>());
    else q.plan->forward_stage2(q.recv.template as<Fr>(), q.out.template as<Fr>());
    TA_HIP(hipEventRecord(q.ev2, q.stream));
  }
  TA_HIP(hipSetDevice(primary_));
  for (size_t g = 0; g < G; ++g) {  // gather on the primary stream
    Part& p = *parts_[g];
    TA_HIP(hipStreamWaitEvent(s0_, p.ev2, 0));
    TA_HIP(hipMemcpyPeerAsync(stage + g * m, primary_, p.out.template as<void>(), p.device, m * sizeof(Fr), s0_));
  }
  hipLaunchKernelGGL(transpose_kernel<Fr>, dim3(ceil_div(cols_in, 32), ceil_div(rows_in, 32)), dim3(kBlock), 0, s0_,
                     stage, y, rows_in, cols_in);
  TA_HIP(hipGetLastError());
}

template <class Fr>
void NttMultiDevice<Fr>::host(const Fr* in, size_t len, Fr* out, bool inverse) {
  if (len > n_) throw std::runtime_error("tachyon_mi355x: more inputs than the domain size");
  int prev = 0;
  TA_HIP(hipGetDevice(&prev));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  TA_HIP(hipSetDevice(primary_));
  Fr* d = static_cast<Fr*>(io_.ensure(n_ * sizeof(Fr)));
  TA_HIP(hipMemcpyAsync(d, in, len * sizeof(Fr), hipMemcpyHostToDevice, s0_));
  if (len < n_) TA_HIP(hipMemsetAsync(d + len, 0, (n_ - len) * sizeof(Fr), s0_));
  run(d, d, inverse);
  TA_HIP(hipMemcpyAsync(out, d, n_ * sizeof(Fr), hipMemcpyDeviceToHost, s0_));
  TA_HIP(hipStreamSynchronize(s0_));
}

template <class Fr>
Fr root_of_unity(uint32_t log_n) {
  if (log_n > (uint32_t)Fr::Config::kTwoAdicity)
    throw std::runtime_error("tachyon_mi355x: no root of unity of that order in the field");
  Fr w = two_adic_root<Fr>();
  for (uint32_t i = log_n; i < (uint32_t)Fr::Config::kTwoAdicity; ++i) w = w.sqr();
  return w;
}
bool set_bn254_fr_halo2_generator(bool on) { return g_bn254_fr_halo2.exchange(on); }
bool bn254_fr_halo2_generator() { return g_bn254_fr_halo2.load(); }

template <class Fr>
Fr field_from_u64(uint64_t v) {
  return fr_from_u64<Fr>(v);
}

template class NttDomain<Bn254Fr>;
template class NttDomain<Bls381Fr>;
template Bn254Fr root_of_unity<Bn254Fr>(uint32_t);
template Bls381Fr root_of_unity<Bls381Fr>(uint32_t);
template Bn254Fr field_from_u64<Bn254Fr>(uint64_t);
template Bls381Fr field_from_u64<Bls381Fr>(uint64_t);
template class Ntt4Step<Bn254Fr>;

uint32_t ntt4_split_log_r(uint32_t log_n, uint32_t log_world) {
  auto passes = [](uint32_t k) { return (k + kMaxPassStages - 1) / kMaxPassStages; };
  uint32_t best = 0, best_cost = ~0u;
  for (uint32_t r = std::max(1u, log_world); r < log_n; ++r) {
    const uint32_t c = log_n - r;
    if (c < log_world || r > c) continue;
    const uint32_t cost = passes(r) + passes(c);
    if (cost <= best_cost) {  // ties: the larger R (up to C)
      best_cost = cost;
      best = r;
    }
  }
  return best ? best : log_n / 2;
}
template class NttMultiDevice<Bn254Fr>;

}  // namespace tachyon_amd::ntt
