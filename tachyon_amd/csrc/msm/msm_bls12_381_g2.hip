// Instantiation of the MSM pipeline for bls12_381_g2 (kernels in msm_impl.h).
#include "msm_impl.h"

namespace tachyon_amd::msm {
template class MsmGpu<Bls381G2>;
}  // namespace tachyon_amd::msm
