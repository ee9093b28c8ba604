// A C++ multi-process caller of the library-level sharded entry points (the
// shape of benchmark/msm/msm_benchmark_gpu.cc:57-69 or vendors/circom/
// prover_main.cc under a launcher, one process per GPU), without torch:
//
//   comm_check <log_n> <world> <rank> <uid_file>
//
// Rank 0 writes the RCCL unique id (tachyon_mi355x_comm_unique_id) to
// uid_file, the other ranks wait for it; every rank then joins the
// communicator (tachyon_mi355x_comm_init_rccl), computes its contiguous shard
// of ONE seeded global input (tachyon_mi355x_gen_bases_at / gen_scalars with
// the shard's start) and calls tachyon_mi355x_msm_gpu_sharded_affine, and runs
// the four-step NTT of its slab through tachyon_mi355x_bn254_ntt4_run
// (forward, then inverse back to the slab).  Prints one JSON line: the MSM
// (hex, every rank the same), whether the NTT round trip returned the slab,
// the communicator's backend.  World 1 runs on the one-GPU test box (RCCL
// refuses two ranks on one GPU); tests/test_gpu_comm.py compares the MSM with
// the oracle.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/tachyon_mi355x.h"

namespace {

std::string hex(const void* p, size_t n) {
  static const char* d = "0123456789abcdef";
  const unsigned char* b = static_cast<const unsigned char*>(p);
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += d[b[i] >> 4];
    s += d[b[i] & 15];
  }
  return s;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: comm_check <log_n> <world> <rank> <uid_file>\n");
    return 2;
  }
  const unsigned log_n = (unsigned)atoi(argv[1]);
  const int world = atoi(argv[2]), rank = atoi(argv[3]);
  const std::string uid_file = argv[4];
  if (world < 1 || rank < 0 || rank >= world || (world & (world - 1)) || log_n < 2 || log_n > 26) return 2;
  unsigned char uid[128];
  if (rank == 0) {
    if (tachyon_mi355x_comm_unique_id(uid, sizeof uid) != (int)sizeof uid) return 3;
    FILE* f = fopen((uid_file + ".tmp").c_str(), "wb");
    if (!f || fwrite(uid, 1, sizeof uid, f) != sizeof uid) return 3;
    fclose(f);
    if (rename((uid_file + ".tmp").c_str(), uid_file.c_str()) != 0) return 3;
  } else {
    for (int i = 0;; ++i) {
      FILE* f = fopen(uid_file.c_str(), "rb");
      if (f && fread(uid, 1, sizeof uid, f) == sizeof uid) {
        fclose(f);
        break;
      }
      if (f) fclose(f);
      if (i > 6000) return 3;  // 60 s
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  tachyon_mi355x_comm* comm = tachyon_mi355x_comm_init_rccl(uid, world, rank);
  if (!comm) return 4;

  // MSM: this rank's contiguous shard of one global seeded input
  const size_t n = size_t(1) << log_n, chunk = (n + world - 1) / world;
  const size_t start = std::min(n, (size_t)rank * chunk), len = std::min(chunk, n - start);
  void *d_bases = nullptr, *d_scalars = nullptr;
  if (hipMalloc(&d_bases, std::max<size_t>(1, len) * 64) != hipSuccess) return 5;
  if (hipMalloc(&d_scalars, std::max<size_t>(1, len) * 32) != hipSuccess) return 5;
  const uint64_t seed = 0xC0FFEE;
  if (len) {
    tachyon_mi355x_gen_bases_at(0, seed, start, len, 16, d_bases, nullptr);
    tachyon_mi355x_gen_scalars(1, seed, start, len, d_scalars, nullptr);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  void* ctx = tachyon_mi355x_msm_gpu_create(0, nullptr);
  unsigned char msm[64];
  tachyon_mi355x_msm_gpu_sharded_affine(0, ctx, comm, d_bases, d_scalars, len, msm);
  tachyon_mi355x_msm_gpu_destroy(0, ctx);

  // NTT: the four-step of this rank's slab, forward then inverse
  unsigned log_world = 0;
  while ((1 << log_world) < world) ++log_world;
  tachyon_mi355x_bn254_ntt4* plan = tachyon_mi355x_bn254_ntt4_create(log_n, log_world, (uint32_t)rank, nullptr);
  const size_t m = tachyon_mi355x_bn254_ntt4_local_size(plan);
  tachyon_bn254_fr *x = nullptr, *y = nullptr, *z = nullptr;
  if (hipMalloc(&x, m * 32) != hipSuccess || hipMalloc(&y, m * 32) != hipSuccess || hipMalloc(&z, m * 32) != hipSuccess)
    return 5;
  tachyon_mi355x_gen_scalars(1, seed + 1, (size_t)rank * m, m, x, nullptr);
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  tachyon_mi355x_bn254_ntt4_run(plan, comm, 0, x, y);
  tachyon_mi355x_bn254_ntt4_run(plan, comm, 1, y, z);
  tachyon_mi355x_bn254_ntt4_synchronize(plan);
  std::vector<unsigned char> hx(m * 32), hz(m * 32);
  if (hipMemcpy(hx.data(), x, m * 32, hipMemcpyDeviceToHost) != hipSuccess) return 5;
  if (hipMemcpy(hz.data(), z, m * 32, hipMemcpyDeviceToHost) != hipSuccess) return 5;
  const bool round_trip = hx == hz;
  tachyon_mi355x_bn254_ntt4_destroy(plan);
  printf("{\"log_n\": %u, \"world\": %d, \"rank\": %d, \"backend\": \"%s\", \"msm\": \"%s\", \"ntt_round_trip\": %s}\n",
         log_n, world, rank, tachyon_mi355x_comm_backend(comm), hex(msm, 64).c_str(), round_trip ? "true" : "false");
  tachyon_mi355x_comm_destroy(comm);
  (void)hipFree(d_bases);
  (void)hipFree(d_scalars);
  (void)hipFree(x);
  (void)hipFree(y);
  (void)hipFree(z);
  return round_trip ? 0 : 1;
}
