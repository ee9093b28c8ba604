// Variable-base MSM on MI355X: host driver interface.
//
// Drop-in for tachyon::math::VariableBaseMSMGpu<Point> (variable_base_msm_gpu.h:11-30)
// whose GPU work the reference delegates to icicle (icicle_msm.h:19-100).
// Pipeline (one HIP stream, no host sync until the final window sums):
//   recode   scalars (Montgomery -> canonical -> signed c-bit digits), one
//            64-bit entry per (window, point): key (window, |digit|) << 32 |
//            point index | sign<<31
//   sort     per-window radix sort of the (bucket, point) pairs (rocPRIM)
//   bounds   bucket [start, end) from the sorted keys
//   acc      bucket sums as XYZZ, split into chunks of <= K entries so that a
//            skewed bucket (NonUniform test set) is spread over many threads
//   levels   tree-reduce per-bucket chunk partials (K2-ary) until one per bucket
//   window   sum_b b * B_b per window via per-segment running sums
//   host     Horner over windows (c doublings each) -> one point
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "../common/hip_util.h"
#include "../ec/point.h"

namespace tachyon_amd::msm {

// MsmGpu::set_variant bits that exist (A/B tuning only; all compute the same MSM)
constexpr int kMsmVariantMask = 0x3FFFFBF;  // bits 0-25 except 6 (21: a debug check, not a schedule)
// schedule of the last run (last_schedule()): the recode fused with the first
// radix pass, the onesweep passes fed by the recode's digit counts, 7-byte LDS
// staging in the recode scatter, the 29-bit-limb G1 accumulation, the lane-pair
// G2 accumulation, the 28-bit-limb BLS12-381 G1 accumulation, the pre-derived
// chain flags checked, the limb-field accumulation's entries staged in LDS
constexpr unsigned kSchedFusedRecode = 1, kSchedRecodeFedSort = 2, kSchedNarrowStaging = 4, kSchedAcc29 = 8,
                   kSchedLanePair = 16, kSchedAcc28 = 32, kSchedChainsChecked = 64, kSchedEntStaged = 128;

struct MsmPlan {
  unsigned c = 0;        // window bits
  unsigned windows = 0;  // W
  unsigned buckets = 0;  // B = 2^(c-1) buckets per window (|digit| in [1, B])
  unsigned K = 0;        // entries per accumulation chunk
  unsigned K2 = 16;      // fan-in of the partial-reduction levels (4 for long chains at run time)
  unsigned levels = 0;   // number of K2 levels
  unsigned seg = 0;      // buckets per running-sum segment
  unsigned seg_tree = 0; // the same for the workgroup-tree window reduction (no fix-up: shorter)
  unsigned group = 0;    // windows per sort/accumulate pipeline stage
  // the windows this run computes, [w_begin, w_end) of the W (default all):
  // a window-range MSM is the sum over those windows of 2^(c w) S_w, so the
  // windows of one MSM can be split across devices (run_window_range)
  unsigned w_begin = 0, w_end = 0;
  unsigned active() const { return w_end - w_begin; }
  static inline MsmPlan make(size_t n, unsigned scalar_bits, unsigned force_c = 0, unsigned w_begin = 0,
                             unsigned w_end = ~0u);
};

// Window size: more bits -> fewer windows (fewer madds, fewer sort passes)
// but more buckets to reduce.  n*W madds dominate at large n; below ~2^20 the
// latency of the bucket/window reduction sets a ~1 ms floor, which favours
// few windows.  Table = fastest c of the BN254 G1 sweeps on MI355X
// (tools/tune_msm.py); only c with a distinct window count
// (W = ceil(255/c)) are candidates.  For another scalar width a c whose
// window count c - 1 also gives is one bit of buckets too many: BLS12-381's
// 255-bit Fr has W = 16 at c = 16 and at c = 17, and c = 16 measured faster at
// 2^22 / 2^23 (G1 12.8 vs 14.1 / 23.4 vs 25.5 ms, G2 31.7 vs 34.5 / 60.3 vs
// 64.1; profiles/r04b/tune_bls_*.log).
inline unsigned default_window_bits(unsigned lg, unsigned scalar_bits = 254) {
  static constexpr unsigned kBest[] = {8, 10, 13, 15, 16, 16, 17, 17, 20, 20, 20};  // lg = 16 .. 26
  unsigned c = lg < 16 ? (unsigned)std::max<int>(4, (int)lg - 7) : kBest[std::min<unsigned>(lg, 26) - 16];
  const unsigned d = scalar_bits + 1;  // signed digits: W c >= bits + 1
  while (c > 4 && (d + c - 2) / (c - 1) == (d + c - 1) / c) --c;
  return c;
}

inline MsmPlan MsmPlan::make(size_t n, unsigned scalar_bits, unsigned force_c, unsigned w_begin, unsigned w_end) {
  MsmPlan p;
  unsigned lg = 1;
  while ((size_t(1) << lg) < n) ++lg;
  unsigned c = force_c ? force_c : default_window_bits(lg, scalar_bits);
  p.c = c;
  p.windows = (scalar_bits + 1 + c - 1) / c;  // W*c >= bits+1
  p.buckets = 1u << (c - 1);
  p.w_end = std::min(w_end, p.windows);
  p.w_begin = std::min(w_begin, p.w_end);
  size_t entries = (size_t)n * p.active();
  // One sort + one accumulation launch over all windows.  (Pipelining one
  // window at a time -- window w+1 sorting on a second stream while window w
  // accumulates -- measured slower at 2^26: 108 vs 99 ms; the onesweep sort
  // and the accumulation slow each other down by about the time they
  // overlap.  set_variant bits 2-3 keep it for experiments.)
  p.group = p.active();
  // entries per accumulation thread: ~2^18 threads with K in [16, 64] below
  // 2^26 entries, then 128, and 256 from 2^29 entries.  Longer runs per
  // thread leave fewer bucket pieces for the chain join, which dominates the
  // small sizes (tools/tune_msm.py; old rule K = entries/2^20 at 1x/2x/4x, ms:
  // 2^18 1.63/1.59/1.66, 2^19 2.14/2.08/2.10, 2^20 2.94/2.89/2.77,
  // 2^21 4.72/4.71/4.66, 2^22 8.14/8.10/8.24; one box, K = 128 vs 64: 2^20
  // 2.88 (K 64) vs 2.94 (K 32), 2^22 8.87 vs 8.57, 2^23 15.56 vs 15.77;
  // 2^26: K = 128/256/512/1024 -> 99.9/98.9/99.1/99.3)
  // Round 4 (29-bit and limb-pair reductions): twice that K for 2^22 < entries
  // <= 2^25 -- 2^18 1.19 -> 1.17, 2^19 1.53 -> 1.48, 2^21 3.82 -> 3.62 ms, 2^20
  // even, 2^22 and up slower (profiles/r04b/tune_k_bn254_g1_2_18_25.log)
  size_t k = entries >= (size_t(1) << 29)   ? 256
             : entries >= (size_t(1) << 26) ? 128
             : entries > (size_t(1) << 25)  ? std::clamp<size_t>(entries >> 18, 16, 64)
             : entries > (size_t(1) << 22)  ? std::clamp<size_t>(entries >> 17, 32, 128)
                                            : std::clamp<size_t>(entries >> 18, 16, 64);
  if (p.group == 1) k = n >> 18;  // ~1024 workgroups per window launch
  p.K = (unsigned)std::clamp<size_t>(k, 8, 256);
  p.K += p.K & 1;  // even: every lane's first entry 16-byte aligned (the LDS-staged entry reads)
  // first-level fan-in; the join drops to 4-ary levels when the longest chain
  // is longer than 16 pieces (kJoinFanLong, chosen after the chain read-back)
  p.K2 = 16;
  size_t maxchunks = (n + p.K - 1) / p.K;  // worst case: all entries of a window in one bucket
  p.levels = 0;
  while (maxchunks > 1) {
    maxchunks = (maxchunks + p.K2 - 1) / p.K2;
    ++p.levels;
  }
  // running-sum segment length: long segments amortise the (jL)*R fix-up, but
  // small MSMs need >= ~48K segment threads to fill the chip (a 2^16 MSM with
  // 64-bucket segments ran 208 threads of ~2000 serial mulmods each).
  // TACHYON_MSM_SEG sweep (ms): 2^20 L = 8/16/32 2.83/2.97/3.29; 2^22 8/16/32
  // 7.99/7.84/8.30; 2^24 16/32/64 26.3/26.2/26.3
  size_t nb = (size_t)p.active() * p.buckets;
  unsigned seg = 2;
  while (seg < 64 && ((nb / (seg * 2)) >= 49152)) seg *= 2;
  p.seg = std::min<unsigned>(p.buckets, seg);
  // workgroup-tree reduction: no per-segment fix-up, so shorter segments (more
  // threads, shorter serial chains) until ~128 K segment threads
  unsigned st = 2;
  while (st < 64 && (nb / (st * 2)) >= 131072) st *= 2;
  p.seg_tree = std::min<unsigned>(p.buckets, st);
#ifdef TACHYON_TUNING_KNOBS
  if (const char* e = getenv("TACHYON_MSM_SEG"); e && atoi(e) > 0)  // A/B override (tuning builds only)
    p.seg = std::clamp<unsigned>(atoi(e), 2, p.buckets);
#endif
  return p;
}

// Per-phase device timings of the last run (ms), filled when profiling is on.
struct MsmTimings {
  float h2d = 0, recode = 0, sort = 0, prep = 0, acc = 0, reduce = 0, total = 0;
  float acc_launches = 0;  // acc = sum over this many accumulation launches
};

template <class Curve>
class MsmGpu {
 public:
  using F = typename Curve::F;
  using Fr = typename Curve::Fr;
  using Point = XYZZ<F>;
  using Aff = Affine<F>;

  explicit MsmGpu(hipStream_t stream = nullptr);
  ~MsmGpu();
  MsmGpu(const MsmGpu&) = delete;
  MsmGpu& operator=(const MsmGpu&) = delete;

  // bases: n affine points (Montgomery, (0,0) = identity); scalars: n Fr in
  // Montgomery form.  Either may live on the host or on the current device.
  // Returns the MSM as an XYZZ point (host memory).
  Point run(const void* bases, const void* scalars, size_t n);

  // Window sums only -- device work identical to run(); `out` gets
  // plan.active() points (the windows of the range set by run_window_range,
  // all W otherwise).
  void run_windows(const void* bases, const void* scalars, size_t n, std::vector<Point>* out,
                   MsmPlan* plan_out);

  // `count` MSMs over the same `len` device-resident bases (scalars: count x
  // len, host or device, zero-padded) as one recode / sort / accumulation /
  // reduction with a block of windows per MSM; returns the count results.
  std::vector<Point> run_batch(const void* bases, const void* scalars, size_t len, size_t count);
  // The largest count run_batch takes for MSMs of `len` points (at most 4096
  // MSMs, count x len < 2^31 scalars, count x W windows << c within the 32-bit
  // bucket keys); 0 when len == 0.
  size_t max_batch_count(size_t len) const;
  // `count` MSMs of `len` points with their own device-resident bases: MSM g
  // over bases[g len, (g+1) len) and scalars[g len, (g+1) len), one launch
  // sequence (same limits as run_batch).
  std::vector<Point> run_groups(const void* bases, const void* scalars, size_t len, size_t count);

  // The windows [w_begin, w_end) of the MSM only: sum_w 2^(c w) S_w over
  // them (c = the forced window bits or the size's default).  Summing the
  // results of ranges that tile [0, W) gives run(); multi-GPU window split.
  Point run_window_range(const void* bases, const void* scalars, size_t n, unsigned w_begin, unsigned w_end);

  // Bases given as projective (form 1), Jacobian (2) or XYZZ (3) points (host or
  // device) normalised to affine on the device; returns the device array of n
  // affine points (valid until the next call).  Form 0 returns `bases` as is.
  const Aff* affine_bases(const void* bases, size_t n, int form);

  // Fixed bases (a proving key's): with the plan's W windows of c bits and a
  // fold F dividing W, fold_bases builds F copies of the n bases, copy k =
  // 2^(k c W / F) P_i (device, F n affine points), and run_folded adds window
  // w's digit to copy w / (W / F) in key window w mod (W / F): the same n W
  // entries, W / F window sums -- 1 / F of the bucket reduction and of the
  // host Horner.  Both take device-resident arrays; the plan (forced c or the
  // size's default) must be the same for both calls.
  void fold_bases(const void* bases, size_t n, unsigned fold, void* out);
  Point run_folded(const void* folded_bases, const void* scalars, size_t n, unsigned fold);
  // The same for run_groups: the table of the count x len bases (window bits
  // of a batch of len-point MSMs, batch_window_bits), then the grouped MSMs
  // over it (device scalars); copy k of the whole array at k count len.
  void fold_bases_groups(const void* bases, size_t len, size_t count, unsigned fold, void* out);
  std::vector<Point> run_groups_folded(const void* folded_bases, const void* scalars, size_t len, size_t count,
                                       unsigned fold);
  unsigned plan_windows(size_t n) const;  // W of the plan for n points
  unsigned batch_windows(size_t len) const {  // W of run_batch / run_groups over len-point MSMs
    const unsigned c = batch_window_bits(len);
    return (Fr::Config::kModulusBits + 1 + c - 1) / c;
  }
  // Memory planning for fixed-base callers (a proving key's fold tables):
  //  * device_budget: the bytes one run may use -- free device memory plus
  //    the buffers this context already holds (they are reused), capped by
  //    TACHYON_MSM_MEM_LIMIT, minus 10 % (memory_divisions uses the same);
  //  * run_bytes / batch_run_bytes: the working set of an n-point run, and of
  //    run_groups / run_batch over count x len points;
  //  * fit_fold(points, windows, want, reusable): the largest power of two <=
  //    want dividing `windows` whose table (fold x points affine bases), its
  //    build staging and the run's working set fit device_budget() +
  //    `reusable` (an older table the caller will drop), with fold x points <
  //    2^31 base indices; 1 = no table (run / run_groups instead).
  size_t device_budget() const;
  size_t run_bytes(size_t n) const { return work_bytes(n, force_c_); }
  size_t batch_run_bytes(size_t len, size_t count) const { return work_bytes(len * count, batch_window_bits(len)); }
  unsigned fit_fold(size_t points, unsigned windows, unsigned want, size_t run_bytes, size_t reusable = 0) const;
  static size_t fold_table_bytes(size_t points, unsigned fold) { return (size_t)fold * points * sizeof(Aff); }
  // staging of fold_bases: XYZZ copies + Montgomery-trick prefixes of one
  // point chunk (the table is built chunk by chunk, kFoldChunkBytes at most)
  static size_t fold_staging_bytes(size_t points, unsigned fold);
  static constexpr size_t kFoldChunkBytes = size_t(1) << 30;

  static Point combine_windows(const std::vector<Point>& window_sums, unsigned c);
  // Mixed additions per second (G/s) of this curve's accumulation field code
  // in registers on the current device -- no gathers, no run logic: the VALU
  // ceiling the bench prices the accumulation against, measured on the same
  // box.  field_bits: BN254 G1 29 (its default field) or 32 (FIPS); BLS12-381
  // G1 28; G2 the lane-pair limb fields, BN254 29 / BLS12-381 28 (G additions
  // of whole G2 points, two lanes each); 0.0 for other values.
  static double madd_ceiling(int field_bits);

  void set_force_window_bits(unsigned c) { force_c_ = c; }
  // kernel-variant bits for in-process A/B tuning (0 = default)
  // A/B tuning knobs (bits 0-5, 7-20, 22 -- the FIPS reductions instead of
  // the limb-field ones; see run_windows --, 23 two-level and 24 two-pass
  // window sums) and bit 21, a debug check (the small-MSM chain flags vs the
  // accumulation's).  Every variant computes the same MSM; bit 6 (once a
  // wrong-result gather-locality experiment) and anything above bit 24 are
  // refused.
  void set_variant(int v) {
    if (v < 0 || (v & ~kMsmVariantMask)) throw std::runtime_error("tachyon_mi355x: unknown MSM variant bits");
    variant_ = v;
  }
  void set_profile(bool on) { profile_ = on; }
  unsigned force_window_bits() const { return force_c_; }
  int variant() const { return variant_; }
  bool profile() const { return profile_; }
  const MsmTimings& timings() const { return timings_; }
  hipStream_t stream() const { return stream_; }
  unsigned last_levels() const { return last_levels_; }
  // number of point chunks the last run() was split into for device memory
  // (DetermineMsmDivisionsForMemory) or for the host-upload pipeline
  size_t last_divisions() const { return last_divisions_; }
  unsigned last_schedule() const { return last_schedule_; }  // kSched* bits of the last run

 private:
  unsigned batch_window_bits(size_t len) const;
  std::vector<Point> run_batch_impl(const void* bases, const void* scalars, size_t len, size_t count, bool distinct,
                                    unsigned fold = 1);
  void fold_bases_c(const void* bases, size_t n, unsigned fold, void* out, unsigned c);
  void enqueue(const Aff* d_bases, const Fr* d_scalars, size_t n, const MsmPlan& plan, Point* d_windows);
  Point run_host_pipelined(const void* bases, const void* scalars, size_t n, size_t chunks);
  size_t work_bytes(size_t n, unsigned c) const;
  size_t held_bytes() const;
  size_t memory_divisions(size_t n, size_t resident_bytes) const;
  void ensure_group_events(unsigned groups);
  void build_chains(const uint32_t* flags, const uint32_t* last, size_t T, unsigned K2, uint32_t* is_start,
                    uint32_t* cid, uint32_t* cbeg, uint32_t* cend, uint32_t* cbucket, uint32_t* lcnt, uint32_t* dscal,
                    hipStream_t s);
  hipError_t sort_entries(void* tmp, size_t& bytes, const uint64_t* in, uint64_t* out, size_t count,
                          unsigned begin_bit, unsigned end_bit, hipStream_t s);

  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  bool profile_ = false;
  unsigned force_c_ = 0;
  int variant_ = 0;
  MsmTimings timings_;
  DeviceBuffer bases_, scalars_, ents_, ents2_, sort_tmp_, scan_tmp_, check_;
  DeviceBuffer start_, end_, cnt_, off_a_, off_b_, part_a_, part_b_, seg_a_, seg_b_, windows_, buckets_;
  hipEvent_t ev_[8] = {};  // 0-5 phase marks, 7 chain count read back (early chain tables)
  hipStream_t sort_stream_ = nullptr;  // group sorts run here, overlapping the accumulation on stream_
  std::vector<hipEvent_t> gev_sorted_, gev_acc0_, gev_acc1_;
  unsigned acc_launches_ = 0;
  unsigned sort_cfg_ = 0;  // onesweep tile shape (set_variant bits 4-5)
  bool rocprim_hist_ = false;  // rocPRIM's digit histogram pass instead of the recode's counts (bit 10)
  bool wide_stage_ = false;    // 8-byte entries in the recode scatter's LDS staging (bit 11)
  bool tree_reduce_ = false;   // window sums by workgroup trees (bit 12)
  bool acc29_ = false;         // BN254 G1 accumulation over 29-bit limbs (default; bit 18: FIPS 32-bit)
  int acc29_mode_ = 0;         // ... next base: 0 not prefetched, 1 in registers (bit 13), 2 via LDS-DMA (bit 17)
  bool pair_acc_ = false;      // G2 accumulation with a lane pair per point (bit 15)
  bool acc28_ = false;         // BLS12-381 G1 accumulation over 28-bit limbs (default; bit 20: FIPS 32-bit)
  bool pair_limb_ = false;     // G2 lane pair over 28-bit (BLS12-381) / 29-bit (BN254) limbs (default; bit 20: FIPS pair)
  bool pair_inline_ = false;   // ... its 12-limb products inline (bit 16)
  uint32_t idx_mask_ = 0x7FFFFFFFu;  // base-index mask of the accumulation gathers (strips the sign bit)
  bool fuse_recode_ = true;          // recode fused with the low-byte radix pass
  uint32_t recode_spt_ = 2;          // scalars per thread of the fused recode
  bool scatter_lds_set_[2] = {false, false};  // 128 KiB dynamic LDS allowed: wide / narrow scatter
  const void* pending_host_bases_ = nullptr;  // host bases still to upload (see enqueue)
  hipStream_t copy_stream_ = nullptr;
  hipEvent_t copy_done_ = nullptr;
  std::vector<hipEvent_t> chunk_ev_;  // host-resident pipeline: chunk k uploaded
  DeviceBuffer hist_;
  DeviceBuffer rsum_;  // the two-pass G2 window sums' suffix sums (set_variant bit 24)
  DeviceBuffer norm_in_, norm_out_, norm_prefix_;  // affine_bases
  DeviceBuffer maxlen_, lofs_;  // lofs_: every join level's output offsets
  uint32_t* h_max_ = nullptr;  // pinned read-back of the largest bucket
  unsigned last_levels_ = 0;
  size_t last_divisions_ = 1;
  unsigned last_schedule_ = 0;
  unsigned range_begin_ = 0, range_end_ = ~0u;  // window range of the next run_windows
  unsigned batch_ = 1;                           // MSMs in the next run_windows (run_batch)
  bool batch_distinct_ = false;                  // ... each over its own bases (run_groups)
  unsigned fold_ = 1;                            // base copies of the next run_windows (run_folded)
};

extern template class MsmGpu<Bn254G1>;
extern template class MsmGpu<Bn254G2>;
extern template class MsmGpu<Bls381G1>;
extern template class MsmGpu<Bls381G2>;

}  // namespace tachyon_amd::msm
