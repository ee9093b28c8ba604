// Instantiation of the MSM pipeline for bn254_g1 (kernels in msm_impl.h).
#include "msm_impl.h"

namespace tachyon_amd::msm {
template class MsmGpu<Bn254G1>;
}  // namespace tachyon_amd::msm
