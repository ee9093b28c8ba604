"""Host mirror of tachyon::math::VariableBaseMSMGpu<Point> over the C-ABI.

Reference: tachyon/math/elliptic_curves/msm/variable_base_msm_gpu.h:11-30
(ctor(mem_pool, stream); Run(bases, scalars, &ret) -> bool) and the C-ABI
tachyon_<curve>_g1_{create,destroy}_msm_gpu / _affine_msm_gpu
(tachyon/c/math/elliptic_curves/generator/msm_gpu.h.tpl:26-54).

Inputs may be `bytes`, contiguous numpy arrays (host memory) or torch CUDA
tensors (device memory, used in place -- the analogue of the reference's
device-pointer detection, icicle_msm_bn254_g1.cc:37-45).
"""
import ctypes

import numpy as np

from ._lib import CURVE_INFO, CURVES, FIELD_BYTES, MsmShard, lib

_CREATE = {
    "bn254_g1": ("tachyon_bn254_g1_create_msm_gpu", "tachyon_bn254_g1_destroy_msm_gpu", "tachyon_bn254_g1_affine_msm_gpu"),
    "bn254_g2": ("tachyon_bn254_g2_create_msm_gpu", "tachyon_bn254_g2_destroy_msm_gpu", "tachyon_bn254_g2_affine_msm_gpu"),
    "bls12_381_g1": ("tachyon_bls12_381_g1_create_msm_gpu", "tachyon_bls12_381_g1_destroy_msm_gpu",
                     "tachyon_bls12_381_g1_affine_msm_gpu"),
    "bls12_381_g2": ("tachyon_bls12_381_g2_create_msm_gpu", "tachyon_bls12_381_g2_destroy_msm_gpu",
                     "tachyon_bls12_381_g2_affine_msm_gpu"),
}


def _ptr(x):
    """(pointer, nbytes, keepalive) of bytes / numpy / torch tensor."""
    if isinstance(x, (bytes, bytearray)):
        buf = ctypes.create_string_buffer(bytes(x), max(1, len(x)))
        return ctypes.addressof(buf), len(x), buf
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"]:
            x = np.ascontiguousarray(x)
        return x.ctypes.data, x.nbytes, x
    if hasattr(x, "data_ptr"):  # torch tensor (host or device)
        if not x.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return x.data_ptr(), x.numel() * x.element_size(), x
    raise TypeError(f"unsupported buffer type {type(x)}")


class VariableBaseMSMGpu:
    def __init__(self, curve: str = "bn254_g1", degree: int = 0):
        if curve not in CURVES:
            raise ValueError(f"unknown curve {curve}")
        self.curve = curve
        self.curve_id = CURVES[curve]
        self.window_bits = 0  # forced window bits (set_window_bits), 0 = the size's default
        self.point_bytes, self.scalar_field = CURVE_INFO[curve]
        self.scalar_bytes = FIELD_BYTES[self.scalar_field]
        create, self._destroy, self._affine_msm = _CREATE[curve]
        self._ctx = getattr(lib(), create)(degree)
        if not self._ctx:
            raise RuntimeError("failed to create MSM context")

    def close(self):
        if self._ctx:
            getattr(lib(), self._destroy)(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _args(self, bases, scalars, n):
        pb, bn, kb = _ptr(bases)
        ps, sn, ks = _ptr(scalars)
        if n is None:
            n = bn // self.point_bytes
        if bn < n * self.point_bytes or sn < n * self.scalar_bytes:
            raise ValueError("bases/scalars shorter than n")
        return pb, ps, n, (kb, ks)

    def run(self, bases, scalars, n=None) -> bytes:
        """MSM sum_i scalars[i] * bases[i]; returns affine (x, y) Montgomery bytes."""
        pb, ps, n, keep = self._args(bases, scalars, n)
        out = ctypes.create_string_buffer(self.point_bytes)
        lib().tachyon_mi355x_msm_gpu_affine(self.curve_id, self._ctx, pb, ps, n, out)
        del keep
        return out.raw

    def run_sharded(self, comm, bases, scalars, n=None) -> bytes:
        """This rank's shard of an MSM over a library communicator
        (tachyon_amd.dist.LibComm): the local partial, the all-gather and the
        group sum inside the library (tachyon_mi355x_msm_gpu_sharded_affine);
        every rank returns the whole MSM (affine bytes)."""
        pb, ps, n, keep = self._args(bases, scalars, n)
        out = ctypes.create_string_buffer(self.point_bytes)
        lib().tachyon_mi355x_msm_gpu_sharded_affine(self.curve_id, self._ctx, comm.handle, pb, ps, n, out)
        del keep
        return out.raw

    def run_sharded_plan(self, comm, shard, bases, scalars) -> bytes:
        """This rank's part of a shard_plan() partition (its point group's
        bases / scalars over its window range) over a library communicator:
        partial, all-gather and group sum inside the library
        (tachyon_mi355x_msm_gpu_sharded_plan_affine); every rank returns the
        whole MSM (affine bytes)."""
        pb, ps, _, keep = self._args(bases, scalars, shard.count)
        out = ctypes.create_string_buffer(self.point_bytes)
        ok = lib().tachyon_mi355x_msm_gpu_sharded_plan_affine(self.curve_id, self._ctx, comm.handle,
                                                              ctypes.byref(shard), pb, ps, out)
        del keep
        if not ok:
            raise RuntimeError("sharded MSM failed on some rank (see stderr)")
        return out.raw

    def run_batch(self, d_bases, scalars, length: int, count: int) -> list:
        """`count` MSMs over the same `length` device-resident bases (a CUDA
        tensor or device pointer) in one launch sequence: MSM g takes
        scalars[g length .. (g+1) length) (host or device; zero-padded);
        returns count affine results -- tachyon_mi355x_msm_gpu_batch_affine."""
        pb = d_bases if isinstance(d_bases, int) else d_bases.data_ptr()
        ps, sn, ks = _ptr(scalars)
        if sn < length * count * self.scalar_bytes:
            raise ValueError("scalars shorter than count x length")
        out = ctypes.create_string_buffer(self.point_bytes * max(1, count))
        if not lib().tachyon_mi355x_msm_gpu_batch_affine(self.curve_id, self._ctx, pb, length, ps, count, out):
            raise ValueError("run_batch needs device-resident bases")
        del ks
        return [out.raw[g * self.point_bytes:(g + 1) * self.point_bytes] for g in range(count)]

    def plan_windows(self, n: int) -> int:
        """W of the plan for n points under this context's window bits."""
        return lib().tachyon_mi355x_msm_gpu_plan_windows(self.curve_id, self._ctx, n)

    def fold_bases(self, d_bases, n: int, fold: int, d_out):
        """Fixed-base table for run_folded: `fold` x n affine points into the
        device buffer d_out, copy k = 2^(k c W / fold) P_i (device tensors or
        pointers) -- tachyon_mi355x_msm_gpu_fold_bases."""
        pb = d_bases if isinstance(d_bases, int) else d_bases.data_ptr()
        po = d_out if isinstance(d_out, int) else d_out.data_ptr()
        if not isinstance(d_out, int) and d_out.numel() * d_out.element_size() < fold * n * self.point_bytes:
            raise ValueError("d_out shorter than fold x n points")
        if not lib().tachyon_mi355x_msm_gpu_fold_bases(self.curve_id, self._ctx, pb, n, fold, po):
            raise ValueError(f"fold {fold} refused (must divide W = {self.plan_windows(n)}; device arrays only)")

    def run_folded(self, d_folded, d_scalars, n: int, fold: int) -> bytes:
        """The MSM of n device scalars over a fold_bases table (same n, same
        window bits); affine bytes -- tachyon_mi355x_msm_gpu_folded_affine."""
        pb = d_folded if isinstance(d_folded, int) else d_folded.data_ptr()
        ps = d_scalars if isinstance(d_scalars, int) else d_scalars.data_ptr()
        out = ctypes.create_string_buffer(self.point_bytes)
        if not lib().tachyon_mi355x_msm_gpu_folded_affine(self.curve_id, self._ctx, pb, ps, n, fold, out):
            raise ValueError(f"fold {fold} refused (must divide W = {self.plan_windows(n)}; device arrays only)")
        return out.raw

    def run_window_range(self, bases, scalars, w_begin: int, w_end: int, n=None) -> bytes:
        """The windows [w_begin, w_end) of the MSM only: sum_w 2^(c w) S_w
        (affine).  Ranges tiling [0, W) add up to run(); see
        dist.window_split_msm."""
        pb, ps, n, keep = self._args(bases, scalars, n)
        out = ctypes.create_string_buffer(self.point_bytes)
        lib().tachyon_mi355x_msm_gpu_window_range_affine(self.curve_id, self._ctx, pb, ps, n, w_begin, w_end, out)
        del keep
        return out.raw

    def run_jacobian(self, bases, scalars, n=None) -> bytes:
        """Through the reference entry point (*_affine_msm_gpu): returns the
        Jacobian the C-ABI allocates (copied, then freed)."""
        pb, ps, n, keep = self._args(bases, scalars, n)
        p = getattr(lib(), self._affine_msm)(self._ctx, pb, ps, n)
        nbytes = self.point_bytes // 2 * 3
        data = ctypes.string_at(p, nbytes)
        lib().tachyon_mi355x_jacobian_destroy(self.curve_id, p)
        del keep
        return data

    def set_window_bits(self, c: int):
        """Force the window bits of later runs (0 = the size's default)."""
        lib().tachyon_mi355x_msm_gpu_set_window_bits(self.curve_id, self._ctx, c)
        self.window_bits = c

    def set_profile(self, on: bool):
        lib().tachyon_mi355x_msm_gpu_set_profile(self.curve_id, self._ctx, 1 if on else 0)

    def set_variant(self, variant: int):
        if not lib().tachyon_mi355x_msm_gpu_set_variant(self.curve_id, self._ctx, variant):
            raise ValueError(f"unknown MSM variant bits in {variant:#x}")

    def set_devices(self, device_ids):
        """Shard every later MSM over these devices (one point chunk per entry,
        ids may repeat; [] or one id = single device), results added on the
        host -- tachyon_mi355x_msm_gpu_set_devices."""
        ids = list(device_ids)
        arr = (ctypes.c_int * max(1, len(ids)))(*ids)
        if not lib().tachyon_mi355x_msm_gpu_set_devices(self.curve_id, self._ctx, arr, len(ids)):
            raise ValueError(f"device ids out of range: {ids}")

    def last_shards(self) -> list:
        """[(device, points, wall ms)] of the last multi-device run ([] if single device)."""
        cap = 64
        ms, pts, dev = (ctypes.c_float * cap)(), (ctypes.c_size_t * cap)(), (ctypes.c_int * cap)()
        k = lib().tachyon_mi355x_msm_gpu_last_shards(self.curve_id, self._ctx, ms, pts, dev, cap)
        return [(dev[i], pts[i], ms[i]) for i in range(min(k, cap))]

    def madd_ceiling(self, field_bits: int = 29) -> float:
        """In-register mixed additions/s (G) of this curve's accumulation field
        code on the current device (tachyon_mi355x_msm_madd_ceiling): 29 = the
        29-bit-limb field, 32 = FIPS; 0.0 where not provided."""
        return float(lib().tachyon_mi355x_msm_madd_ceiling(self.curve_id, int(field_bits)))

    def last_schedule(self) -> dict:
        """Schedule of the last run: fused recode + first radix pass, recode-fed
        onesweep passes, 7-byte LDS staging (tachyon_mi355x_msm_gpu_last_schedule)."""
        b = lib().tachyon_mi355x_msm_gpu_last_schedule(self.curve_id, self._ctx)
        return {"fused_recode": bool(b & 1), "recode_fed_sort": bool(b & 2), "narrow_staging": bool(b & 4),
                "acc29": bool(b & 8), "lane_pair": bool(b & 16), "acc28": bool(b & 32),
                "chains_checked": bool(b & 64), "entries_staged": bool(b & 128)}

    def last_divisions(self) -> int:
        """Point chunks the last run was split into (device memory or host-upload pipeline)."""
        return lib().tachyon_mi355x_msm_gpu_last_divisions(self.curve_id, self._ctx)

    def last_timings(self) -> dict:
        out = (ctypes.c_float * 8)()
        lib().tachyon_mi355x_msm_gpu_last_timings(self.curve_id, self._ctx, out)
        return dict(zip(("h2d", "recode", "sort", "prep", "acc", "reduce", "total", "acc_launches"), list(out)))


def shard_plan(curve: str, n_total: int, world: int, rank: int) -> MsmShard:
    """The library's partition of an n_total-point MSM over `world` ranks for
    `rank` (tachyon_mi355x_msm_shard_plan): point shards, or the hybrid point
    group x window range where it measured faster."""
    s = MsmShard()
    if not lib().tachyon_mi355x_msm_shard_plan(CURVES[curve], n_total, world, rank, ctypes.byref(s)):
        raise ValueError(f"rank {rank} outside a world of {world}")
    return s


def plan(curve: str, n: int):
    c, w = ctypes.c_uint(), ctypes.c_uint()
    lib().tachyon_mi355x_msm_plan(CURVES[curve], n, ctypes.byref(c), ctypes.byref(w))
    return c.value, w.value


def affine_sum(curve: str, points: bytes) -> bytes:
    """Group sum of affine points on the host (combines per-GPU partial MSMs)."""
    pbytes = CURVE_INFO[curve][0]
    n = len(points) // pbytes
    src = ctypes.create_string_buffer(points, max(1, len(points)))
    out = ctypes.create_string_buffer(pbytes)
    lib().tachyon_mi355x_affine_sum(CURVES[curve], src, n, out)
    return out.raw


def jacobian_to_affine(curve: str, jac: bytes) -> bytes:
    pbytes = CURVE_INFO[curve][0]
    src = ctypes.create_string_buffer(jac, len(jac))
    out = ctypes.create_string_buffer(pbytes)
    lib().tachyon_mi355x_jacobian_to_affine(CURVES[curve], src, out)
    return out.raw


def gen_scalars(field: str, seed: int, n: int, d_out_ptr: int, start: int = 0, stream=None):
    lib().tachyon_mi355x_gen_scalars({"bn254_fr": 1, "bls12_381_fr": 3}[field], seed, start, n, d_out_ptr, stream)


def gen_bases(curve: str, seed: int, n: int, chunk: int, d_out_ptr: int, stream=None, start: int = 0):
    """Points [start, start + n) of the seeded doubling-chain sequence (any start): every rank can generate its shard of one global input."""
    lib().tachyon_mi355x_gen_bases_at(CURVES[curve], seed, start, n, chunk, d_out_ptr, stream)
