// Communicators for the library-level sharded entry points (one process per
// MI355X).  The reference's multi-GPU callers (benchmark/msm/msm_benchmark_gpu.cc:57-69,
// vendors/circom/prover_main.cc:116-128 under a launcher) would hand the
// library a communicator and let it do the exchange; the two exchanges of this
// path are
//   * all_gather_host: the per-rank partial results (one XYZZ point per MSM,
//     the Groth16 partials blob) -- bytes, gathered in rank order;
//   * all_to_all_device: the four-step NTT's transpose, block h of the send
//     buffer to rank h, on the plan's stream.
// Backends:
//   * RcclComm -- RCCL (ncclComm_t) over xGMI: ncclAllGather, and the
//     all-to-all as one ncclGroupStart/End of ncclSend/ncclRecv pairs, both
//     enqueued on the caller's stream.
//   * HostComm -- the HOST-STAGED FALLBACK: the caller supplies two callbacks
//     that exchange host buffers (e.g. torch.distributed over gloo, or ranks
//     sharing one GPU, which RCCL refuses: "Duplicate GPU detected").  Device
//     data are copied to the host, exchanged, and copied back.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <cstdint>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../common/hip_util.h"

namespace tachyon_amd::dist {

class Comm {
 public:
  Comm(int world, int rank);
  virtual ~Comm() = default;
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;
  int world() const { return world_; }
  int rank() const { return rank_; }
  virtual const char* backend() const = 0;
  // every rank's `bytes` of host memory `send`, gathered in rank order into
  // host `recv` (world * bytes); returns when recv is filled
  virtual void all_gather_host(const void* send, void* recv, size_t bytes) = 0;
  // device buffers of world blocks of `bytes`: send block h goes to rank h,
  // recv block h comes from rank h; ordered on `stream` (the HostComm
  // fallback synchronises it)
  virtual void all_to_all_device(const void* send, void* recv, size_t bytes, hipStream_t stream) = 0;

 protected:
  int world_, rank_;
};

class RcclComm : public Comm {
 public:
  // wrap a communicator the caller owns (world and rank read from it)
  explicit RcclComm(ncclComm_t comm);
  // ncclCommInitRank on the current device (collective over the ranks)
  RcclComm(const ncclUniqueId& id, int world, int rank);
  ~RcclComm() override;
  const char* backend() const override { return "rccl"; }
  void all_gather_host(const void* send, void* recv, size_t bytes) override;
  void all_to_all_device(const void* send, void* recv, size_t bytes, hipStream_t stream) override;
  ncclComm_t handle() const { return comm_; }

 private:
  void ensure_stream();
  ncclComm_t comm_ = nullptr;
  bool owned_ = false;
  hipStream_t stream_ = nullptr;  // the small host all-gathers
  DeviceBuffer stage_;
};

// Callback signatures (C-ABI, include/tachyon_mi355x.h): host buffers; return 0 on success.
using AllGatherFn = int (*)(void* user, const void* send, void* recv, size_t bytes);
using AllToAllFn = int (*)(void* user, const void* send, void* recv, size_t bytes);

class HostComm : public Comm {
 public:
  HostComm(int world, int rank, AllGatherFn ag, AllToAllFn a2a, void* user);
  const char* backend() const override { return "host"; }
  void all_gather_host(const void* send, void* recv, size_t bytes) override;
  void all_to_all_device(const void* send, void* recv, size_t bytes, hipStream_t stream) override;

 private:
  AllGatherFn ag_;
  AllToAllFn a2a_;
  void* user_;
  std::vector<uint8_t> hsend_, hrecv_;
};

ncclUniqueId rccl_unique_id();

// One fixed-size record per rank, gathered in rank order, with a status
// word: `local()` computes this rank's record; if it throws, the rank still
// enters the all-gather (with a failure flag) so that no other rank is left
// blocked in the collective, and after the exchange EVERY rank throws when
// any rank failed (its own error first).
template <class T, class Fn>
std::vector<T> gather_checked(Comm* comm, Fn&& local) {
  struct Rec {
    uint32_t ok = 0, rank = 0;
    T v{};
  };
  static_assert(std::is_trivially_copyable_v<Rec>);
  Rec mine;
  mine.rank = (uint32_t)comm->rank();
  std::exception_ptr err;
  try {
    mine.v = local();
    mine.ok = 1;
  } catch (...) {
    err = std::current_exception();
  }
  std::vector<Rec> all((size_t)comm->world());
  comm->all_gather_host(&mine, all.data(), sizeof(Rec));
  if (err) std::rethrow_exception(err);
  std::vector<T> out;
  out.reserve(all.size());
  for (const Rec& r : all) {
    if (!r.ok)
      throw std::runtime_error("tachyon_mi355x: rank " + std::to_string(r.rank) +
                               " failed its local part of a sharded call");
    out.push_back(r.v);
  }
  return out;
}

}  // namespace tachyon_amd::dist

// the C-ABI handle (include/tachyon_mi355x.h, "Communicators")
struct tachyon_mi355x_comm {
  std::unique_ptr<tachyon_amd::dist::Comm> impl;
};
