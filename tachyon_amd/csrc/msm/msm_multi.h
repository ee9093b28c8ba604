// One-process multi-device MSM: the reference's kParallelTerm decomposition
// (pippenger_adapter.h:82-113: split the points into contiguous chunks, one
// independent MSM per chunk, add the chunk results) with one chunk per device,
// so a single-process caller of the C-ABI (benchmark/msm msm_benchmark_gpu.cc:
// 57-69, the scroll_halo2 bridge bn254_msm_gpu.cc:11-35, both of which the
// reference pins to device 0, msm_gpu.h:54-56) uses several MI355X.
//
// Each shard runs the single-device MsmGpu on its own device, from its own
// host thread and on its own stream: host-resident inputs are uploaded per
// shard over that device's own PCIe link (MsmGpu::run pipelines the upload of
// large shards with their kernels); device-resident inputs on another device
// are copied peer-to-peer (xGMI) into the shard's device first.  The shard
// results (XYZZ) are added on the host -- EC addition is not a reduction
// operator of any collective, and the partials are n_devices points.
//
// Device ids may repeat ("logical devices"): several shards then share one
// GPU on separate streams, which is how the one-GPU test box exercises the
// N-shard path.
#pragma once
#include <chrono>
#include <exception>
#include <memory>
#include <thread>
#include <vector>

#include "msm.h"

namespace tachyon_amd::msm {

template <class Curve>
class MsmMultiDevice {
 public:
  using Point = typename MsmGpu<Curve>::Point;
  using Aff = typename MsmGpu<Curve>::Aff;
  using Fr = typename MsmGpu<Curve>::Fr;

  explicit MsmMultiDevice(const std::vector<int>& devices) {
    if (devices.empty()) throw std::runtime_error("tachyon_mi355x: empty device list");
    int count = 0;
    TA_HIP(hipGetDeviceCount(&count));
    for (int d : devices)
      if (d < 0 || d >= count)
        throw std::runtime_error("tachyon_mi355x: device id " + std::to_string(d) + " out of range (" +
                                 std::to_string(count) + " devices)");
    int prev = 0;
    TA_HIP(hipGetDevice(&prev));
    struct Restore {
      int d;
      ~Restore() { (void)hipSetDevice(d); }
    } restore{prev};
    for (int d : devices) {
      TA_HIP(hipSetDevice(d));
      auto s = std::make_unique<Shard>();
      s->device = d;
      s->msm = std::make_unique<MsmGpu<Curve>>(nullptr);
      shards_.push_back(std::move(s));
    }
  }

  ~MsmMultiDevice() {
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) prev = 0;
    for (auto& s : shards_) {  // free each shard's stream and buffers on its own device
      (void)hipSetDevice(s->device);
      s.reset();
    }
    (void)hipSetDevice(prev);
  }

  size_t devices() const { return shards_.size(); }
  const std::vector<int> device_ids() const {
    std::vector<int> ids;
    for (auto& s : shards_) ids.push_back(s->device);
    return ids;
  }
  // per shard: wall ms of its upload/copy + MSM, and its point count (last run)
  const std::vector<float>& last_shard_ms() const { return shard_ms_; }
  const std::vector<size_t>& last_shard_points() const { return shard_n_; }

  // The single-device settings reach every shard (set_devices copies the
  // context's current ones in with copy_settings).
  void set_force_window_bits(unsigned c) {
    for (auto& s : shards_) s->msm->set_force_window_bits(c);
  }
  void set_variant(int v) {
    for (auto& s : shards_) s->msm->set_variant(v);
  }
  void set_profile(bool on) {
    for (auto& s : shards_) s->msm->set_profile(on);
  }
  void copy_settings(const MsmGpu<Curve>& from) {
    set_force_window_bits(from.force_window_bits());
    set_variant(from.variant());
    set_profile(from.profile());
  }
  // The shard that ran the most points in the last run (shard 0 unless it was
  // empty): its timings / schedule stand for the run.
  const MsmGpu<Curve>& lead() const {
    size_t best = 0;
    for (size_t k = 1; k < shard_n_.size(); ++k)
      if (shard_n_[k] > shard_n_[best]) best = k;
    return *shards_[best]->msm;
  }
  size_t last_divisions() const {
    size_t d = 0;
    for (auto& s : shards_) d = std::max(d, s->msm->last_divisions());
    return d;
  }

  Point run(const void* bases, const void* scalars, size_t n) {
    const size_t N = shards_.size();
    const size_t step = (n + N - 1) / N;
    const int src_b = device_of(bases), src_s = device_of(scalars);
    std::vector<Point> part(N, Point::zero());
    std::vector<std::exception_ptr> err(N);
    shard_ms_.assign(N, 0.f);
    shard_n_.assign(N, 0);
    std::vector<std::thread> th;
    th.reserve(N);
    for (size_t k = 0; k < N; ++k) {
      const size_t lo = std::min(n, k * step), len = std::min(step, n - lo);
      shard_n_[k] = len;
      th.emplace_back([&, k, lo, len] {
        try {
          if (len == 0) return;
          Shard& s = *shards_[k];
          TA_HIP(hipSetDevice(s.device));
          const auto t0 = std::chrono::steady_clock::now();
          const void* b = static_cast<const Aff*>(bases) + lo;
          const void* sc = static_cast<const Fr*>(scalars) + lo;
          // device inputs owned by another device: one peer copy of this shard over xGMI
          if (src_b >= 0 && src_b != s.device) b = peer_copy(s.bases, b, src_b, s.device, len * sizeof(Aff));
          if (src_s >= 0 && src_s != s.device) sc = peer_copy(s.scalars, sc, src_s, s.device, len * sizeof(Fr));
          part[k] = s.msm->run(b, sc, len);
          shard_ms_[k] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        } catch (...) {
          err[k] = std::current_exception();
        }
      });
    }
    for (auto& t : th) t.join();
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
    Point total = Point::zero();
    for (const Point& p : part) total = total + p;
    return total;
  }

 private:
  struct Shard {
    int device = 0;
    std::unique_ptr<MsmGpu<Curve>> msm;
    DeviceBuffer bases, scalars;  // this shard's copy of device inputs owned by another device
  };

  // owning device of a device pointer, -1 for host memory
  static int device_of(const void* p) {
    if (!p) return -1;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    return (attr.type == hipMemoryTypeDevice || attr.isManaged) ? attr.device : -1;
  }

  static const void* peer_copy(DeviceBuffer& dst, const void* src, int src_dev, int dst_dev, size_t bytes) {
    void* d = dst.ensure(bytes);
    TA_HIP(hipMemcpyPeer(d, dst_dev, src, src_dev, bytes));
    return d;
  }

  std::vector<std::unique_ptr<Shard>> shards_;
  std::vector<float> shard_ms_;
  std::vector<size_t> shard_n_;
};

// "0,1,2,3" -> {0, 1, 2, 3} (TACHYON_MSM_GPU_DEVICES); empty on a malformed list
inline std::vector<int> parse_device_list(const char* s) {
  std::vector<int> out;
  if (!s) return out;
  const char* p = s;
  while (*p) {
    char* end = nullptr;
    long v = strtol(p, &end, 10);
    if (end == p || v < 0 || v > 1024) return {};
    out.push_back((int)v);
    p = end;
    if (*p == ',') ++p;
    else if (*p) return {};
  }
  return out;
}

}  // namespace tachyon_amd::msm
