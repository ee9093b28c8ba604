// Small HIP runtime helpers shared by the MSM and NTT drivers.
// (The reference's thin runtime layer is tachyon/device/gpu/: gpuStream /
// gpuMemPool aliases, GpuMemory RAII, GpuPointerGetAttributes.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace tachyon_amd {

[[noreturn]] inline void hip_fail(hipError_t e, const char* what, const char* file, int line) {
  char buf[512];
  snprintf(buf, sizeof buf, "tachyon_mi355x: HIP error '%s' (%d) in %s at %s:%d", hipGetErrorString(e),
           (int)e, what, file, line);
  throw std::runtime_error(buf);
}

#define TA_HIP(expr)                                                \
  do {                                                              \
    hipError_t _e = (expr);                                         \
    if (_e != hipSuccess) ::tachyon_amd::hip_fail(_e, #expr, __FILE__, __LINE__); \
  } while (0)

// Device-resident scratch that only grows; reused across calls so the hot path
// never allocates (allocation is not capturable and costs ~100 us at GB sizes).
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  ~DeviceBuffer() { release(); }

  void* ensure(size_t bytes) {
    if (bytes > cap_) {
      release();
      size_t want = bytes < 256 ? 256 : bytes;
      TA_HIP(hipMalloc(&ptr_, want));
      cap_ = want;
    }
    return ptr_;
  }
  template <class T>
  T* as() const { return static_cast<T*>(ptr_); }
  size_t capacity() const { return cap_; }
  void release() {
    if (ptr_) (void)hipFree(ptr_);
    ptr_ = nullptr;
    cap_ = 0;
  }

 private:
  void* ptr_ = nullptr;
  size_t cap_ = 0;
};

// True if `p` is device (or managed) memory visible to the current device --
// the analogue of the reference's GpuPointerGetAttributes check
// (icicle_msm_bn254_g1.cc:37-45).
inline bool is_device_pointer(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeDevice || attr.isManaged;
}

// The device that owns `p` (device or managed memory), or -1 for host memory.
inline int pointer_device(const void* p) {
  if (!p) return -1;
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return (attr.type == hipMemoryTypeDevice || attr.isManaged) ? attr.device : -1;
}

inline unsigned ceil_div(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

inline void require_gpu() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    throw std::runtime_error("tachyon_mi355x: no HIP device available (the MI355X backend has no CPU fallback)");
}

}  // namespace tachyon_amd
