// Instantiation of the MSM pipeline for bls12_381_g1 (kernels in msm_impl.h).
#include "msm_impl.h"

namespace tachyon_amd::msm {
template class MsmGpu<Bls381G1>;
}  // namespace tachyon_amd::msm
