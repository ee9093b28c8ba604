// Communicator backends (see comm.h).
#include "comm.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace tachyon_amd::dist {

namespace {

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("tachyon_mi355x: RCCL ") + what + " failed: " + ncclGetErrorString(r));
}

}  // namespace

Comm::Comm(int world, int rank) : world_(world), rank_(rank) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("tachyon_mi355x: communicator rank outside [0, world)");
}

ncclUniqueId rccl_unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return id;
}

namespace {
int nccl_count(ncclComm_t c) {
  int n = 0;
  nccl_check(ncclCommCount(c, &n), "ncclCommCount");
  return n;
}
int nccl_rank(ncclComm_t c) {
  int r = 0;
  nccl_check(ncclCommUserRank(c, &r), "ncclCommUserRank");
  return r;
}
}  // namespace

RcclComm::RcclComm(ncclComm_t comm) : Comm(nccl_count(comm), nccl_rank(comm)), comm_(comm), owned_(false) {}

RcclComm::RcclComm(const ncclUniqueId& id, int world, int rank) : Comm(world, rank), owned_(true) {
  nccl_check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
}

RcclComm::~RcclComm() {
  if (stream_) (void)hipStreamDestroy(stream_);
  if (owned_ && comm_) (void)ncclCommDestroy(comm_);
}

void RcclComm::ensure_stream() {
  if (!stream_) TA_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
}

void RcclComm::all_gather_host(const void* send, void* recv, size_t bytes) {
  if (bytes == 0) return;
  ensure_stream();
  uint8_t* d = static_cast<uint8_t*>(stage_.ensure((size_t)(world_ + 1) * bytes));
  TA_HIP(hipMemcpyAsync(d, send, bytes, hipMemcpyHostToDevice, stream_));
  nccl_check(ncclAllGather(d, d + bytes, bytes, ncclUint8, comm_, stream_), "ncclAllGather");
  TA_HIP(hipMemcpyAsync(recv, d + bytes, (size_t)world_ * bytes, hipMemcpyDeviceToHost, stream_));
  TA_HIP(hipStreamSynchronize(stream_));
}

void RcclComm::all_to_all_device(const void* send, void* recv, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return;
  const uint8_t* s = static_cast<const uint8_t*>(send);
  uint8_t* r = static_cast<uint8_t*>(recv);
  nccl_check(ncclGroupStart(), "ncclGroupStart");
  for (int h = 0; h < world_; ++h) {
    nccl_check(ncclSend(s + (size_t)h * bytes, bytes, ncclUint8, h, comm_, stream), "ncclSend");
    nccl_check(ncclRecv(r + (size_t)h * bytes, bytes, ncclUint8, h, comm_, stream), "ncclRecv");
  }
  nccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

HostComm::HostComm(int world, int rank, AllGatherFn ag, AllToAllFn a2a, void* user)
    : Comm(world, rank), ag_(ag), a2a_(a2a), user_(user) {
  if (!ag_) throw std::runtime_error("tachyon_mi355x: host communicator needs an all-gather callback");
}

void HostComm::all_gather_host(const void* send, void* recv, size_t bytes) {
  if (bytes == 0) return;
  if (world_ == 1) {
    memcpy(recv, send, bytes);
    return;
  }
  if (ag_(user_, send, recv, bytes) != 0) throw std::runtime_error("tachyon_mi355x: host all-gather callback failed");
}

// host-staged: device -> host, exchange by callback, host -> device
void HostComm::all_to_all_device(const void* send, void* recv, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return;
  const size_t total = (size_t)world_ * bytes;
  if (world_ == 1) {
    TA_HIP(hipMemcpyAsync(recv, send, total, hipMemcpyDeviceToDevice, stream));
    return;
  }
  if (!a2a_) throw std::runtime_error("tachyon_mi355x: host communicator has no all-to-all callback");
  hsend_.resize(total);
  hrecv_.resize(total);
  TA_HIP(hipMemcpyAsync(hsend_.data(), send, total, hipMemcpyDeviceToHost, stream));
  TA_HIP(hipStreamSynchronize(stream));
  if (a2a_(user_, hsend_.data(), hrecv_.data(), bytes) != 0)
    throw std::runtime_error("tachyon_mi355x: host all-to-all callback failed");
  TA_HIP(hipMemcpyAsync(recv, hrecv_.data(), total, hipMemcpyHostToDevice, stream));
  TA_HIP(hipStreamSynchronize(stream));  // the host staging buffer is reused
}

}  // namespace tachyon_amd::dist
