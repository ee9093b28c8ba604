"""tachyon_amd -- MI355X-native MSM + NTT backend for Tachyon.

The product is libtachyon_mi355x.so (hand-written HIP for gfx950 behind
Tachyon's tachyon/c C-ABI, declared in include/tachyon_mi355x.h).  This
package is its host-side Python mirror:
  tachyon_amd.msm.VariableBaseMSMGpu        ~ tachyon::math::VariableBaseMSMGpu<Point>
  tachyon_amd.ntt.Radix2EvaluationDomain    ~ tachyon::math::Radix2EvaluationDomain<bn254::Fr>
  tachyon_amd.dist                          one-process-per-GPU sharded MSM / NTT
Nothing here computes on the CPU; the library is loaded lazily so that
importing the package works on a build host without a GPU.
"""
__all__ = ["msm", "ntt", "params"]
