"""ctypes binding of libtachyon_mi355x.so (the C-ABI in include/tachyon_mi355x.h).

The library is built in-tree by `tachyon_amd.build.build()` (hipcc, gfx950).
There is no CPU fallback: if the shared library is missing this module raises,
and every compute entry point of the library aborts without a HIP device.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# TACHYON_MI355X_LIB: alternative build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("TACHYON_MI355X_LIB") or os.path.join(HERE, "libtachyon_mi355x.so")

CURVES = {"bn254_g1": 0, "bn254_g2": 1, "bls12_381_g1": 2, "bls12_381_g2": 3}
FIELDS = {"bn254_fq": 0, "bn254_fr": 1, "bls12_381_fq": 2, "bls12_381_fr": 3}
FIELD_BYTES = {"bn254_fq": 32, "bn254_fr": 32, "bls12_381_fq": 48, "bls12_381_fr": 32}
# curve -> (affine point bytes, scalar field)
CURVE_INFO = {
    "bn254_g1": (64, "bn254_fr"),
    "bn254_g2": (128, "bn254_fr"),
    "bls12_381_g1": (96, "bls12_381_fr"),
    "bls12_381_g2": (192, "bls12_381_fr"),
}

_lib = None

# (name, restype, argtypes) of every entry point declared in include/tachyon_mi355x.h
vp, sz, i32, u8, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint8, ctypes.c_uint64
fp = ctypes.POINTER(ctypes.c_float)
# tachyon_mi355x_all_gather_fn / _all_to_all_fn: (user, send, recv, bytes) -> 0 on success
COMM_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


class MsmShard(ctypes.Structure):
    """tachyon_mi355x_msm_shard: one rank's part of a sharded MSM plan."""
    _fields_ = [("start", ctypes.c_size_t), ("count", ctypes.c_size_t), ("point_groups", ctypes.c_uint),
                ("window_groups", ctypes.c_uint), ("window_bits", ctypes.c_uint), ("w_begin", ctypes.c_uint),
                ("w_end", ctypes.c_uint)]
SIGNATURES = [
    # reference C-ABI: MSM
    ("tachyon_bn254_g1_init", None, []),
    ("tachyon_bls12_381_g1_init", None, []),
    ("tachyon_bn254_g2_init", None, []),
    ("tachyon_bls12_381_g2_init", None, []),
    ("tachyon_bn254_g1_create_msm", vp, [u8]),
    ("tachyon_bn254_g1_destroy_msm", None, [vp]),
    ("tachyon_bn254_g1_point2_msm", vp, [vp, vp, vp, sz]),
    ("tachyon_bn254_g1_affine_msm", vp, [vp, vp, vp, sz]),
    ("tachyon_bn254_g1_create_msm_gpu", vp, [u8]),
    ("tachyon_bn254_g1_destroy_msm_gpu", None, [vp]),
    ("tachyon_bn254_g1_point2_msm_gpu", vp, [vp, vp, vp, sz]),
    ("tachyon_bn254_g1_affine_msm_gpu", vp, [vp, vp, vp, sz]),
    ("tachyon_bls12_381_g1_create_msm", vp, [u8]),
    ("tachyon_bls12_381_g1_destroy_msm", None, [vp]),
    ("tachyon_bls12_381_g1_point2_msm", vp, [vp, vp, vp, sz]),
    ("tachyon_bls12_381_g1_affine_msm", vp, [vp, vp, vp, sz]),
    ("tachyon_bls12_381_g1_create_msm_gpu", vp, [u8]),
    ("tachyon_bls12_381_g1_destroy_msm_gpu", None, [vp]),
    ("tachyon_bls12_381_g1_point2_msm_gpu", vp, [vp, vp, vp, sz]),
    ("tachyon_bls12_381_g1_affine_msm_gpu", vp, [vp, vp, vp, sz]),
    # reference C-ABI: univariate domain / containers
    ("tachyon_bn254_univariate_evaluation_domain_create", vp, [sz]),
    ("tachyon_bn254_univariate_evaluation_domain_destroy", None, [vp]),
    ("tachyon_bn254_univariate_evaluation_domain_empty_evals", vp, [vp]),
    ("tachyon_bn254_univariate_evaluation_domain_empty_poly", vp, [vp]),
    ("tachyon_bn254_univariate_evaluation_domain_fft", vp, [vp, vp]),
    ("tachyon_bn254_univariate_evaluation_domain_fft_inplace", vp, [vp, vp]),
    ("tachyon_bn254_univariate_evaluation_domain_ifft", vp, [vp, vp]),
    ("tachyon_bn254_univariate_evaluation_domain_ifft_inplace", vp, [vp, vp]),
    ("tachyon_bn254_univariate_evaluations_create", vp, []),
    ("tachyon_bn254_univariate_evaluations_clone", vp, [vp]),
    ("tachyon_bn254_univariate_evaluations_destroy", None, [vp]),
    ("tachyon_bn254_univariate_evaluations_len", sz, [vp]),
    ("tachyon_bn254_univariate_evaluations_set_value", None, [vp, sz, vp]),
    ("tachyon_bn254_univariate_evaluation_domain_empty_rational_evals", vp, [vp]),
    ("tachyon_bn254_univariate_rational_evaluations_create", vp, []),
    ("tachyon_bn254_univariate_rational_evaluations_clone", vp, [vp]),
    ("tachyon_bn254_univariate_rational_evaluations_destroy", None, [vp]),
    ("tachyon_bn254_univariate_rational_evaluations_len", sz, [vp]),
    ("tachyon_bn254_univariate_rational_evaluations_set_zero", None, [vp, sz]),
    ("tachyon_bn254_univariate_rational_evaluations_set_trivial", None, [vp, sz, vp]),
    ("tachyon_bn254_univariate_rational_evaluations_set_rational", None, [vp, sz, vp, vp]),
    ("tachyon_bn254_univariate_rational_evaluations_evaluate", None, [vp, sz, vp]),
    ("tachyon_bn254_univariate_rational_evaluations_batch_evaluate", vp, [vp]),
    ("tachyon_bn254_univariate_dense_polynomial_create", vp, []),
    ("tachyon_bn254_univariate_dense_polynomial_clone", vp, [vp]),
    ("tachyon_bn254_univariate_dense_polynomial_destroy", None, [vp]),
    # extensions
    ("tachyon_mi355x_bn254_univariate_evaluations_get_value", None, [vp, sz, vp]),
    ("tachyon_mi355x_bn254_univariate_evaluations_data", vp, [vp]),
    ("tachyon_mi355x_bn254_univariate_evaluations_resize", None, [vp, sz]),
    ("tachyon_mi355x_bn254_univariate_dense_polynomial_len", sz, [vp]),
    ("tachyon_mi355x_bn254_univariate_dense_polynomial_resize", None, [vp, sz]),
    ("tachyon_mi355x_bn254_univariate_dense_polynomial_set_value", None, [vp, sz, vp]),
    ("tachyon_mi355x_bn254_univariate_dense_polynomial_get_value", None, [vp, sz, vp]),
    ("tachyon_mi355x_bn254_univariate_dense_polynomial_data", vp, [vp]),
    ("tachyon_mi355x_bn254_univariate_rational_evaluations_resize", None, [vp, sz]),
    ("tachyon_mi355x_bn254_univariate_rational_evaluations_get", None, [vp, sz, vp, vp]),
    ("tachyon_mi355x_bn254_halo2_override_subgroup_generator", None, []),
    ("tachyon_mi355x_bn254_halo2_restore_subgroup_generator", None, []),
    ("tachyon_mi355x_bn254_halo2_subgroup_generator_active", i32, []),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_size", sz, [vp]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_group_gen", None, [vp, vp]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_set_offset", None, [vp, vp]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_transform_device", None, [vp, vp, i32]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_transform_host", None, [vp, vp, sz, i32]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_transform_batch_device", None, [vp, vp, sz, i32]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_stream", vp, [vp]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_set_profile", None, [vp, i32]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_set_variant", i32, [vp, i32]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_set_devices", i32, [vp, vp, sz]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_devices", sz, [vp, vp, sz]),
    ("tachyon_mi355x_bn254_univariate_evaluation_domain_last_timings", i32, [vp, fp, fp, i32]),
    ("tachyon_mi355x_bn254_ntt4_create", vp, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp]),
    ("tachyon_mi355x_bn254_ntt4_destroy", None, [vp]),
    ("tachyon_mi355x_bn254_ntt4_local_size", sz, [vp]),
    ("tachyon_mi355x_bn254_ntt4_create_split", vp, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                    vp]),
    ("tachyon_mi355x_bn254_ntt4_log_rows", ctypes.c_uint32, [vp]),
    ("tachyon_mi355x_ntt4_split_log_r", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32]),
    ("tachyon_mi355x_bn254_ntt4_stage", None, [vp, i32, i32, vp, vp]),
    ("tachyon_mi355x_bn254_ntt4_synchronize", None, [vp]),
    ("tachyon_mi355x_bn254_ntt4_stream", vp, [vp]),
    ("tachyon_bn254_g2_create_msm_gpu", vp, [u8]),
    ("tachyon_bn254_g2_destroy_msm_gpu", None, [vp]),
    ("tachyon_bn254_g2_affine_msm_gpu", vp, [vp, vp, vp, sz]),
    ("tachyon_bls12_381_g2_create_msm_gpu", vp, [u8]),
    ("tachyon_bls12_381_g2_destroy_msm_gpu", None, [vp]),
    ("tachyon_bls12_381_g2_affine_msm_gpu", vp, [vp, vp, vp, sz]),
    ("tachyon_mi355x_msm_gpu_affine", None, [i32, vp, vp, vp, sz, vp]),
    ("tachyon_mi355x_msm_gpu_window_range_affine", None, [i32, vp, vp, vp, sz, ctypes.c_uint, ctypes.c_uint, vp]),
    ("tachyon_mi355x_msm_gpu_batch_affine", i32, [i32, vp, vp, sz, vp, sz, vp]),
    ("tachyon_mi355x_msm_gpu_plan_windows", ctypes.c_uint, [i32, vp, sz]),
    ("tachyon_mi355x_msm_gpu_fold_bases", i32, [i32, vp, vp, sz, ctypes.c_uint, vp]),
    ("tachyon_mi355x_msm_gpu_folded_affine", i32, [i32, vp, vp, vp, sz, ctypes.c_uint, vp]),
    ("tachyon_mi355x_msm_gpu_create", vp, [i32, vp]),
    ("tachyon_mi355x_msm_gpu_destroy", None, [i32, vp]),
    ("tachyon_mi355x_msm_gpu_run", i32, [i32, vp, vp, sz, vp, sz, i32, vp]),
    ("tachyon_mi355x_msm_gpu_run_points", i32, [i32, vp, vp, sz, i32, vp, sz, i32, vp]),
    ("tachyon_mi355x_msm_gpu_set_window_bits", None, [i32, vp, ctypes.c_uint]),
    ("tachyon_mi355x_msm_gpu_set_profile", None, [i32, vp, i32]),
    ("tachyon_mi355x_msm_gpu_set_variant", i32, [i32, vp, i32]),
    ("tachyon_mi355x_msm_gpu_last_divisions", sz, [i32, vp]),
    ("tachyon_mi355x_msm_gpu_last_schedule", ctypes.c_uint, [i32, vp]),
    ("tachyon_mi355x_msm_madd_ceiling", ctypes.c_double, [i32, i32]),
    ("tachyon_mi355x_msm_gpu_set_devices", i32, [i32, vp, ctypes.POINTER(ctypes.c_int), sz]),
    ("tachyon_mi355x_msm_gpu_last_shards", sz, [i32, vp, fp, ctypes.POINTER(ctypes.c_size_t),
                                              ctypes.POINTER(ctypes.c_int), sz]),
    ("tachyon_mi355x_msm_gpu_last_timings", None, [i32, vp, fp]),
    ("tachyon_mi355x_msm_plan", None, [i32, sz, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint)]),
    ("tachyon_mi355x_affine_sum", None, [i32, vp, sz, vp]),
    ("tachyon_mi355x_jacobian_to_affine", None, [i32, vp, vp]),
    ("tachyon_mi355x_gen_scalars", None, [i32, u64, sz, sz, vp, vp]),
    ("tachyon_mi355x_gen_bases", None, [i32, u64, sz, sz, vp, vp]),
    ("tachyon_mi355x_gen_bases_at", None, [i32, u64, sz, sz, sz, vp, vp]),
    ("tachyon_mi355x_field_op", None, [i32, i32, vp, vp, vp, sz]),
    ("tachyon_mi355x_ec_op", None, [i32, i32, vp, vp, vp, sz]),
    ("tachyon_mi355x_groth16_prover_create", vp, [vp, sz]),
    ("tachyon_mi355x_groth16_prover_destroy", None, [vp]),
    ("tachyon_mi355x_groth16_prover_info", None, [vp, ctypes.POINTER(ctypes.c_uint32)]),
    ("tachyon_mi355x_groth16_prove", None, [vp, vp, sz, vp, vp, vp, vp, vp]),
    ("tachyon_mi355x_groth16_witness_map", None, [vp, vp, sz, vp]),
    ("tachyon_mi355x_groth16_partials_size", sz, [vp]),
    ("tachyon_mi355x_groth16_prove_partials", None, [vp, vp, sz, i32, ctypes.c_uint32, ctypes.c_uint32, vp]),
    ("tachyon_mi355x_groth16_assemble", None, [vp, vp, sz, vp, vp, vp, vp, vp]),
    ("tachyon_mi355x_groth16_set_profile", None, [vp, i32]),
    ("tachyon_mi355x_groth16_set_msm_window_bits", None, [vp, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]),
    ("tachyon_mi355x_groth16_set_variant", i32, [vp, i32]),
    ("tachyon_mi355x_groth16_set_devices", i32, [vp, vp, sz]),
    ("tachyon_mi355x_groth16_last_timings", None, [vp, fp]),
    ("tachyon_mi355x_zkey_curve", i32, [vp, sz]),
    ("tachyon_mi355x_wtns_parse", sz, [i32, vp, sz, vp, sz]),
    ("tachyon_mi355x_kzg_create", vp, [i32]),
    ("tachyon_mi355x_kzg_destroy", None, [vp]),
    ("tachyon_mi355x_kzg_unsafe_setup", None, [vp, sz, vp]),
    ("tachyon_mi355x_kzg_n", sz, [vp]),
    ("tachyon_mi355x_kzg_downsize", i32, [vp, sz]),
    ("tachyon_mi355x_kzg_get_srs", None, [vp, i32, vp]),
    ("tachyon_mi355x_kzg_commit", i32, [vp, i32, vp, sz, vp]),
    ("tachyon_mi355x_kzg_commit_batch", i32, [vp, i32, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.POINTER(ctypes.c_size_t), sz, vp]),
    # field-generic NTT domains
    ("tachyon_mi355x_ntt_domain_create", vp, [i32, sz]),
    ("tachyon_mi355x_ntt_domain_destroy", None, [vp]),
    ("tachyon_mi355x_ntt_domain_size", sz, [vp]),
    ("tachyon_mi355x_ntt_domain_field", i32, [vp]),
    ("tachyon_mi355x_ntt_domain_group_gen", None, [vp, vp]),
    ("tachyon_mi355x_ntt_domain_set_offset", None, [vp, vp]),
    ("tachyon_mi355x_ntt_domain_transform_host", None, [vp, vp, sz, i32]),
    ("tachyon_mi355x_ntt_domain_transform_device", None, [vp, vp, sz, i32]),
    ("tachyon_mi355x_ntt_domain_stream", vp, [vp]),
    # communicators and library-level sharded entry points
    ("tachyon_mi355x_comm_unique_id", i32, [vp, sz]),
    ("tachyon_mi355x_comm_init_rccl", vp, [vp, i32, i32]),
    ("tachyon_mi355x_comm_from_rccl", vp, [vp]),
    ("tachyon_mi355x_comm_create_host", vp, [i32, i32, COMM_FN, COMM_FN, vp]),
    ("tachyon_mi355x_comm_destroy", None, [vp]),
    ("tachyon_mi355x_comm_all_gather", None, [vp, vp, vp, sz]),
    ("tachyon_mi355x_comm_world", i32, [vp]),
    ("tachyon_mi355x_comm_rank", i32, [vp]),
    ("tachyon_mi355x_comm_backend", ctypes.c_char_p, [vp]),
    ("tachyon_mi355x_msm_gpu_sharded_affine", None, [i32, vp, vp, vp, vp, sz, vp]),
    ("tachyon_mi355x_msm_shard_plan", i32, [i32, sz, i32, i32, vp]),
    ("tachyon_mi355x_msm_gpu_sharded_plan_affine", i32, [i32, vp, vp, vp, vp, vp, vp]),
    ("tachyon_mi355x_bn254_ntt4_run", None, [vp, vp, i32, vp, vp]),
    ("tachyon_mi355x_bn254_ntt4_set_variant", i32, [vp, i32]),
    ("tachyon_mi355x_groth16_prove_sharded", None, [vp, vp, vp, sz, vp, vp, vp, vp, vp]),
    ("tachyon_mi355x_groth16_prepare", sz, [vp, ctypes.c_uint32, ctypes.c_uint32, i32]),
    ("tachyon_mi355x_groth16_prover_folds", None, [vp, ctypes.POINTER(ctypes.c_uint32)]),
    ("tachyon_mi355x_jacobian_destroy", None, [i32, vp]),
    ("tachyon_mi355x_version", ctypes.c_char_p, []),
    ("tachyon_mi355x_device_count", i32, []),
]


def lib():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: PyTorch-ROCm bundles its own
        # libamdhip64 (SONAME libamdhip64.so.7) and cannot initialise the GPU
        # once /opt/rocm's copy is loaded.  Importing torch first makes this
        # library bind to the runtime torch already loaded, so HBM buffers,
        # streams and RCCL from torch interoperate with the C-ABI.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(the MI355X backend has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            try:
                f = getattr(L, name)
            except AttributeError:
                # an A/B build from an older commit (TACHYON_MI355X_LIB) may
                # predate an entry point; the in-tree library must have all
                if os.environ.get("TACHYON_MI355X_LIB"):
                    continue
                raise
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib
