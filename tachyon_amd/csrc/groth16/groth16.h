// Groth16 prover on MI355X: the circom witness map (QAP) and the five MSMs of
// CreateProofWithAssignment on the GPU, behind one host object per proving key.
//
// Reference path restated:
//   vendors/circom/prover_main.cc:82-160 (CreateProof: zkey -> proving key,
//     wtns -> full assignments, WitnessMapFromMatrices, NoZK / ZK proof)
//   vendors/circom/circomlib/circuit/quadratic_arithmetic_program.h:24-113
//     (a, b from the A/B coefficients, c = a * b, IFFT x3, DistributePowers by
//     the 2n-th root of unity, FFT x3, h = a * b - c on the coset)
//   tachyon/zk/r1cs/groth16/prove.h:33-165 (CalculateCoeff and
//     CreateProofWithAssignment: A, B in G2, B in G1 when r != 0, C)
//   vendors/circom/circomlib/zkey/proving_key.h:42-52 (ToNativeProvingKey:
//     l_g1_query = points C1, h_g1_query = points H1)
//
// Device residency: the proving key's points and the coefficient matrices
// (CSR by constraint) are uploaded once in the constructor -- the analogue of
// the device-resident bases the reference keeps for KZG (kzg.h:90-114); a
// proof uploads only the m witness values.  The QAP is three kernels plus
// six batched NTT launches; every MSM takes device pointers (no copies).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "../common/hip_util.h"
#include "../msm/msm.h"
#include "../ntt/ntt.h"
#include "circom_io.h"

namespace tachyon_amd::groth16 {

template <class G1, class G2>
struct Proof {
  Affine<typename G1::F> a;
  Affine<typename G2::F> b;
  Affine<typename G1::F> c;
};

// One rank's share of the MSMs of CreateProofWithAssignment
// (prove.h:95-146) as XYZZ sums: rank k of `world` takes the contiguous
// ceil(count / world) chunk k of every MSM's point range (the kParallelTerm
// split, pippenger_adapter.h:82-113).  The partials of all ranks added
// together are the single-GPU MSM results, whatever the split.
template <class G1, class G2>
struct ProofPartials {
  // layout tag of the C-ABI blob: bump the magic whenever the fields change
  // ("G262": a, b1, merged lh, b2); `bytes` catches a size mismatch as well
  uint32_t magic = 0x32363247;
  uint32_t bytes = sizeof(ProofPartials);
  uint32_t with_b1 = 0;  // the B-in-G1 MSM was run (needed when r != 0)
  uint32_t rank = 0, world = 1;
  XYZZ<typename G1::F> a, b1, lh;  // lh: the witness (C1) and h (H1) MSMs, merged
  XYZZ<typename G2::F> b2;
};

// Per-phase device timings of the last prove (ms), when profiling is on.
struct ProveTimings {
  float upload = 0, qap = 0, msm_a = 0, msm_b2 = 0, msm_b1 = 0, msm_l = 0, msm_h = 0, total = 0;
};

template <class G1, class G2>
class Groth16Prover {
 public:
  using G1Type = G1;
  using G2Type = G2;
  using Fr = typename G1::Fr;
  using F1 = typename G1::F;
  using F2 = typename G2::F;
  using Key = circom::ZKey<G1, G2>;

  explicit Groth16Prover(const Key& key, hipStream_t stream = nullptr);
  // a copy of src (whose buffers live on src_device) on the current device,
  // the proving key copied peer to peer (one-process multi-device proofs)
  Groth16Prover(const Groth16Prover& src, int src_device, hipStream_t stream = nullptr);
  ~Groth16Prover();
  Groth16Prover(const Groth16Prover&) = delete;  // (the device copy above takes a source device)
  Groth16Prover& operator=(const Groth16Prover&) = delete;

  // full: num_vars Montgomery-form assignments (full[0] = 1), host or device.
  // r, s: the blinding scalars (Montgomery); null = zero (the NoZK proof,
  // prove.h:178-186).  Returns canonical affine points.
  Proof<G1, G2> prove(const Fr* full, size_t count, const Fr* r, const Fr* s);

  // The multi-GPU split of prove(): every rank runs the witness map (it is a
  // few percent of the proof) and its shard of the MSMs; the partials of
  // all ranks are exchanged (one all-gather) and assemble() adds them and
  // applies r, s and the key's alpha/beta/delta terms on the host.
  // prove(full, r, s) == assemble({partials(full, r != 0, 0, 1)}, r, s).
  ProofPartials<G1, G2> partials(const Fr* full, size_t count, bool with_b1, uint32_t rank, uint32_t world);
  Proof<G1, G2> assemble(const ProofPartials<G1, G2>* parts, size_t world, const Fr* r, const Fr* s) const;

  // The witness map alone: h evaluations on the coset (domain_size values,
  // canonical Montgomery) written to `d_h` (device) -- for parity tests.
  void witness_map(const Fr* d_full, Fr* d_h);

  // Proving-key setup (the fold tables of the fixed queries, built here
  // instead of inside the first proof): the tables the proofs of shard
  // (rank, world) use, each the largest fold up to the variant's that fits
  // the device next to the MSM's working set (MsmGpu::fit_fold; fold 1 =
  // plain MSMs, and the grouped G1 MSM falls back to separate MSMs when its
  // working set does not fit).  Returns the table bytes held afterwards.
  // A proof after prepare() builds nothing; one without it prepares itself.
  size_t prepare(uint32_t rank, uint32_t world, bool with_b1);
  size_t fold_table_bytes() const;
  // the folds the last prepare chose: B2, the grouped G1 (0 = separate
  // MSMs), A, B1, witness + h
  void last_folds(unsigned out[5]) const;

  const Key& key() const { return key_; }
  void set_profile(bool on) { profile_ = on; }
  // window bits of the proof's MSMs (0 = each MSM's default): A (and B in G1),
  // the merged witness + h MSM, B in G2 -- tuning and A/B only
  // A/B: bit 0 = A and the witness + h MSM as two MSMs (round 4) instead of
  // one grouped MSM (MsmGpu::run_groups, one process one device); bits 1-3 =
  // the fold of the G2 B MSM's fixed bases (MsmGpu::run_folded), bits 4-6 the
  // fold of the grouped G1 MSM's (run_groups_folded): 0 the default (kB2Fold
  // / kG1Fold), k = 1..5 2^(k-1) copies at most (1 = none); valid_variant checks
  static bool valid_variant(int v) { return v >= 0 && v < 128 && ((v >> 1) & 7) <= 5 && ((v >> 4) & 7) <= 5; }
  void set_variant(int v) { variant_ = v; }
  unsigned b2_fold() const { return fold_of((variant_ >> 1) & 7, kB2Fold); }
  unsigned g1_fold() const { return fold_of((variant_ >> 4) & 7, kG1Fold); }
  // (the largest power of two up to these that divides the MSM's W).
  // profiles/r05ai: B2 x16 + G1 x4 10.06 ms per 2^20 proof, B2 x8 10.13, B2
  // x4 10.33, G1 x2 10.34, no tables 11.11; r05ah: both x8 10.27, G1 x8 10.41
  static constexpr unsigned kB2Fold = 16, kG1Fold = 4;
  int variant() const { return variant_; }
  void set_msm_window_bits(unsigned c_a, unsigned c_lh, unsigned c_b2) {
    c_a_ = c_a;
    c_lh_ = c_lh;
    c_b2_ = c_b2;
  }
  const ProveTimings& timings() const { return timings_; }
  hipStream_t stream() const { return stream_; }

 private:
  static unsigned fold_of(unsigned sel, unsigned dflt) { return sel == 0 ? dflt : 1u << (sel - 1); }
  struct FoldTable;
  // one rank's point ranges of the proof's MSMs, and whether A and the
  // witness + h MSM run as one grouped MSM
  struct ShardPlan {
    size_t q_lo = 0, q_len = 0;    // queries 1 .. m-1 of A, B1, B2
    size_t lh_lo = 0, lh_len = 0;  // the merged witness + h MSM (ungrouped)
    bool grouped = false;
  };
  ShardPlan shard_plan(uint32_t rank, uint32_t world) const;
  // the fold table of `tab` for these bases, (re)built when they, the length,
  // the window bits or the fold the memory allows changed; returns its fold
  // (1: no table, the MSM runs plain)
  template <class G>
  unsigned ensure_table(msm::MsmGpu<G>& msm, FoldTable& tab, const Affine<typename G::F>* bases, size_t len,
                        unsigned fold, unsigned c);
  template <class G>
  XYZZ<typename G::F> fixed_msm(msm::MsmGpu<G>& msm, FoldTable& tab, const Affine<typename G::F>* bases,
                                const Fr* scalars, size_t len, unsigned fold, unsigned c);
  // the grouped G1 MSM's table (fold 1 = none); false when the grouped MSM
  // itself does not fit the device (separate MSMs then)
  bool ensure_group_table(unsigned* fold_out);
  void init_device_state();
  void build_groups();
  Key key_;  // host copy: verifying-key points and the query heads used on the host
  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  bool profile_ = false;
  unsigned c_a_ = 0, c_lh_ = 0, c_b2_ = 0;  // set_msm_window_bits
  int variant_ = 0;
  size_t glen_ = 0;                          // build_groups: points per group (0 = no grouped MSM)
  DeviceBuffer gbases_, gscalars_;           // 3 x glen_ bases / scalars of the grouped MSM
  size_t n_ = 0;  // domain size
  std::unique_ptr<ntt::NttDomain<Fr>> dom_, coset_;
  std::unique_ptr<msm::MsmGpu<G1>> msm1_;
  std::unique_ptr<msm::MsmGpu<G2>> msm2_;
  DeviceBuffer a1_, b1_, lh1_, b2_;              // query points (lh1 = C1 | H1)
  // fold tables of the fixed queries (built on first use): the table, and
  // the bases / length / fold / window bits it was built for (fold 0: none)
  struct FoldTable {
    DeviceBuffer buf;
    const void* src = nullptr;
    size_t len = 0;
    unsigned want = 0, c = 0;  // the fold asked for and the window bits of the last decision
    unsigned fold = 0;         // the fold built (1: none fits, plain MSM; 0: not decided)
  };
  FoldTable b2_tab_, a_tab_, b1_tab_, lh_tab_;   // G2 B; A, B in G1, witness + h (ungrouped / shards)
  FoldTable g1_tab_;                             // the grouped G1 MSM's table (over gbases_)
  bool group_fits_ = true;                       // the grouped G1 MSM fits the device (ensure_group_table)
  unsigned folds_[5] = {0, 0, 0, 0, 0};          // last_folds
  DeviceBuffer lh_;                              // scalars of the merged MSM: witness | h
  DeviceBuffer row_a_, row_b_, col_, val_;       // CSR of the A and B matrices
  DeviceBuffer full_, abc_;                      // witness, 3 x n work vectors
  ProveTimings timings_;
  hipEvent_t ev_[4] = {};
};

extern template class Groth16Prover<Bn254G1, Bn254G2>;
extern template class Groth16Prover<Bls381G1, Bls381G2>;

}  // namespace tachyon_amd::groth16
