// Device helpers: synthetic inputs and elementwise parity kernels (see device_ops.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../ec/point.h"

namespace tachyon_amd::util {

void gen_scalars(int field, uint64_t seed, size_t start, size_t n, void* d_out, hipStream_t stream);
// points [start, start + n) of the seeded sequence (any start)
void gen_bases(int curve, uint64_t seed, size_t start, size_t n, size_t chunk, void* d_out, hipStream_t stream);
void field_op(int field, int op, const void* a, const void* b, void* out, size_t count);
// out[i] = num[i] / den[i] (0 where den[i] == 0) for n BN254 Fr in Montgomery
// form, host buffers (RationalField::BatchEvaluate on the GPU)
void batch_evaluate_bn254_fr(const void* num, const void* den, void* out, size_t n);
void ec_op(int curve, int op, const void* a, const void* b, void* out, size_t count);

}  // namespace tachyon_amd::util
