"""Host mirror of tachyon::math::Radix2EvaluationDomain<bn254::Fr> over the C-ABI.

Reference: tachyon/c/math/polynomials/univariate/bn254_univariate_evaluation_domain.h:38-136
(create / fft / ifft returning new containers) and
tachyon/math/polynomials/univariate/univariate_evaluation_domain.h
(FFT/IFFT semantics, GetCoset :102-117).
Elements are BN254 Fr in Montgomery form, 32 bytes each.
"""
import ctypes

from ._lib import lib

FR_BYTES = 32


def override_subgroup_generator():
    """math::halo2::OverrideSubgroupGenerator() (bn/bn254/halo2/bn254.cc:7-30):
    BN254 Fr domains created afterwards use halo2curves' generator 7."""
    lib().tachyon_mi355x_bn254_halo2_override_subgroup_generator()


def restore_subgroup_generator():
    lib().tachyon_mi355x_bn254_halo2_restore_subgroup_generator()


def halo2_subgroup_generator_active() -> bool:
    return bool(lib().tachyon_mi355x_bn254_halo2_subgroup_generator_active())


class ScopedSubgroupGeneratorOverrider:
    """math::halo2::ScopedSubgroupGeneratorOverrider (bn254.cc:32-44) as a
    context manager: installs the halo2 set, restores the previous one on exit."""

    def __enter__(self):
        self._prev = halo2_subgroup_generator_active()
        override_subgroup_generator()
        return self

    def __exit__(self, *exc):
        if not self._prev:
            restore_subgroup_generator()
        return False


class Radix2EvaluationDomain:
    def __init__(self, num_coeffs: int, _handle=None):
        L = lib()
        self._d = _handle or L.tachyon_bn254_univariate_evaluation_domain_create(num_coeffs)
        if not self._d:
            raise RuntimeError("domain creation failed")
        self.size = L.tachyon_mi355x_bn254_univariate_evaluation_domain_size(self._d)
        self.log_size_of_group = self.size.bit_length() - 1
        self.offset = None

    @classmethod
    def create(cls, num_coeffs: int):
        return cls(num_coeffs)

    def close(self):
        if self._d:
            lib().tachyon_bn254_univariate_evaluation_domain_destroy(self._d)
            self._d = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def group_gen(self) -> bytes:
        out = ctypes.create_string_buffer(FR_BYTES)
        lib().tachyon_mi355x_bn254_univariate_evaluation_domain_group_gen(self._d, out)
        return out.raw

    def set_offset(self, offset_mont: bytes):
        """Coset h*<w> (GetCoset); offset = Montgomery bytes of h."""
        buf = ctypes.create_string_buffer(offset_mont, FR_BYTES)
        lib().tachyon_mi355x_bn254_univariate_evaluation_domain_set_offset(self._d, buf)
        self.offset = offset_mont

    def _poly(self, coeffs: bytes):
        L = lib()
        p = L.tachyon_bn254_univariate_dense_polynomial_create()
        n = len(coeffs) // FR_BYTES
        L.tachyon_mi355x_bn254_univariate_dense_polynomial_resize(p, n)
        if n:
            ctypes.memmove(L.tachyon_mi355x_bn254_univariate_dense_polynomial_data(p), coeffs, n * FR_BYTES)
        return p

    def _evals(self, evals: bytes):
        L = lib()
        e = L.tachyon_bn254_univariate_evaluations_create()
        n = len(evals) // FR_BYTES
        L.tachyon_mi355x_bn254_univariate_evaluations_resize(e, n)
        if n:
            ctypes.memmove(L.tachyon_mi355x_bn254_univariate_evaluations_data(e), evals, n * FR_BYTES)
        return e

    def fft(self, coeffs: bytes) -> bytes:
        """tachyon_bn254_univariate_evaluation_domain_fft: coefficients -> evaluations."""
        L = lib()
        p = self._poly(coeffs)
        e = L.tachyon_bn254_univariate_evaluation_domain_fft(self._d, p)
        n = L.tachyon_bn254_univariate_evaluations_len(e)
        out = ctypes.string_at(L.tachyon_mi355x_bn254_univariate_evaluations_data(e), n * FR_BYTES) if n else b""
        L.tachyon_bn254_univariate_evaluations_destroy(e)
        L.tachyon_bn254_univariate_dense_polynomial_destroy(p)
        return out

    def ifft(self, evals: bytes) -> bytes:
        """tachyon_bn254_univariate_evaluation_domain_ifft: evaluations -> coefficients
        (trailing zero coefficients removed, like the reference CPU path)."""
        L = lib()
        e = self._evals(evals)
        p = L.tachyon_bn254_univariate_evaluation_domain_ifft(self._d, e)
        n = L.tachyon_mi355x_bn254_univariate_dense_polynomial_len(p)
        out = ctypes.string_at(L.tachyon_mi355x_bn254_univariate_dense_polynomial_data(p), n * FR_BYTES) if n else b""
        L.tachyon_bn254_univariate_dense_polynomial_destroy(p)
        L.tachyon_bn254_univariate_evaluations_destroy(e)
        return out

    def transform_device(self, d_ptr: int, inverse: bool = False):
        """In-place transform of `size` elements already in HBM (not synchronised;
        runs on self.stream)."""
        lib().tachyon_mi355x_bn254_univariate_evaluation_domain_transform_device(self._d, d_ptr, 1 if inverse else 0)

    def transform_host(self, buf, inverse: bool = False):
        """IcicleNTT::Run semantics (icicle_ntt.h:53-142): in place on a writable
        host buffer (ctypes buffer / numpy array) of exactly `size` Montgomery
        elements, natural order, on the domain's coset; synchronous."""
        import numpy as np
        if isinstance(buf, np.ndarray):
            ptr, nbytes = buf.ctypes.data, buf.nbytes
        else:
            ptr, nbytes = ctypes.addressof(buf), ctypes.sizeof(buf)
        lib().tachyon_mi355x_bn254_univariate_evaluation_domain_transform_host(self._d, ptr, nbytes // 32,
                                                                              1 if inverse else 0)

    @property
    def stream(self) -> int:
        return lib().tachyon_mi355x_bn254_univariate_evaluation_domain_stream(self._d)

    def set_profile(self, on: bool):
        lib().tachyon_mi355x_bn254_univariate_evaluation_domain_set_profile(self._d, 1 if on else 0)

    def set_variant(self, variant: int):
        """Kernel variant: 0 = the 8 x 32-bit-limb passes, 1 = the 9 x 29-bit-limb
        passes, 3 = the 29-bit passes with swizzled LDS positions (a new domain
        uses 1 up to 2^20 elements, 0 above); all give the same canonical
        outputs."""
        if not lib().tachyon_mi355x_bn254_univariate_evaluation_domain_set_variant(self._d, variant):
            raise ValueError(f"unknown NTT variant {variant}")

    def set_devices(self, device_ids):
        """Run later transforms of the plain domain as a four-step NTT over these
        devices, one process (ids may repeat; the first 2^k of them are used,
        see devices(); [] or one id = single device) --
        tachyon_mi355x_bn254_univariate_evaluation_domain_set_devices."""
        ids = list(device_ids)
        arr = (ctypes.c_int * max(1, len(ids)))(*ids)
        if not lib().tachyon_mi355x_bn254_univariate_evaluation_domain_set_devices(self._d, arr, len(ids)):
            raise ValueError(f"device list refused for a 2^{self.size.bit_length() - 1} domain: {ids}")

    def devices(self) -> list:
        arr = (ctypes.c_int * 64)()
        k = lib().tachyon_mi355x_bn254_univariate_evaluation_domain_devices(self._d, arr, 64)
        return list(arr)[:min(k, 64)]

    def last_timings(self):
        total = ctypes.c_float()
        passes = (ctypes.c_float * 16)()
        k = lib().tachyon_mi355x_bn254_univariate_evaluation_domain_last_timings(self._d, ctypes.byref(total), passes, 16)
        return total.value, list(passes)[:k]

    def transform_batch_device(self, d_ptr: int, batch: int, inverse: bool = False):
        """In-place transform of `batch` consecutive arrays of `size` elements in HBM."""
        lib().tachyon_mi355x_bn254_univariate_evaluation_domain_transform_batch_device(
            self._d, d_ptr, batch, 1 if inverse else 0)


NTT_FIELDS = {"bn254_fr": 1, "bls12_381_fr": 3}


class FieldEvaluationDomain:
    """Radix2EvaluationDomain<F> for F = bn254 Fr or bls12_381 Fr over the
    field-generic C-ABI domain (tachyon_mi355x_ntt_domain_*): the engine of
    IcicleNTT<bls12_381::Fr> (icicle_ntt_bls12_381.cc:31-115).  fft / ifft
    take and return the full domain (size x 32 Montgomery bytes; shorter
    inputs are zero-padded), natural order, on the domain's coset."""

    def __init__(self, field: str, num_coeffs: int):
        if field not in NTT_FIELDS:
            raise ValueError(f"no GPU NTT for {field}")
        self.field = field
        self._d = lib().tachyon_mi355x_ntt_domain_create(NTT_FIELDS[field], num_coeffs)
        if not self._d:
            raise RuntimeError("domain creation failed")
        self.size = lib().tachyon_mi355x_ntt_domain_size(self._d)
        self.log_size_of_group = self.size.bit_length() - 1

    def close(self):
        if self._d:
            lib().tachyon_mi355x_ntt_domain_destroy(self._d)
            self._d = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def group_gen(self) -> bytes:
        out = ctypes.create_string_buffer(FR_BYTES)
        lib().tachyon_mi355x_ntt_domain_group_gen(self._d, out)
        return out.raw

    def set_offset(self, offset_mont: bytes = None):
        """Coset h*<w> of later transforms (GetCoset); None = the plain domain."""
        buf = ctypes.create_string_buffer(offset_mont, FR_BYTES) if offset_mont is not None else None
        lib().tachyon_mi355x_ntt_domain_set_offset(self._d, buf)

    def _host(self, data: bytes, inverse: bool) -> bytes:
        if len(data) > self.size * FR_BYTES:
            raise ValueError("more elements than the domain size")
        buf = ctypes.create_string_buffer(bytes(data) + b"\x00" * (self.size * FR_BYTES - len(data)),
                                          self.size * FR_BYTES)
        lib().tachyon_mi355x_ntt_domain_transform_host(self._d, buf, self.size, 1 if inverse else 0)
        return buf.raw

    def fft(self, coeffs: bytes) -> bytes:
        return self._host(coeffs, False)

    def ifft(self, evals: bytes) -> bytes:
        return self._host(evals, True)

    def transform_device(self, d_ptr: int, batch: int = 1, inverse: bool = False):
        """In place on `batch` device arrays of size elements (on self.stream, not synchronised)."""
        lib().tachyon_mi355x_ntt_domain_transform_device(self._d, d_ptr, batch, 1 if inverse else 0)

    @property
    def stream(self) -> int:
        return lib().tachyon_mi355x_ntt_domain_stream(self._d)


class FourStepNtt:
    """One rank's plan of the distributed four-step NTT (include/tachyon_mi355x.h,
    tachyon_mi355x_bn254_ntt4_*).  n = 2^log_n = R*C, R = 2^floor(log_n/2), or
    R = 2^log_r when given (split_log_r: the split with the fewest passes).

    Layouts (see input_indices / output_indices): rank r holds the columns
    [r C/G, (r+1) C/G) of the R x C view of x, column-major, and produces the
    rows [r R/G, (r+1) R/G) of X, row-major.  The inverse maps back.
    """

    def __init__(self, log_n: int, world: int, rank: int, stream=None, log_r: int = None):
        """stream: a torch.cuda.Stream (or None for a new one).  The plan's
        kernels run on it; callers run the exchange and any tensor work between
        the stages under `with torch.cuda.stream(plan.torch_stream)` so that one
        stream orders everything.  (PyTorch's default stream is the legacy null
        stream, which does not order against the non-blocking streams HIP
        libraries create -- a raw handle 0 is therefore not accepted.)"""
        import torch
        if world & (world - 1):
            raise ValueError("world size must be a power of two")
        if stream is None:
            stream = torch.cuda.Stream()
        if not isinstance(stream, torch.cuda.Stream) or stream.cuda_stream == 0:
            raise ValueError("FourStepNtt needs a non-default torch.cuda.Stream")
        self.torch_stream = stream
        self.log_n, self.world, self.rank = log_n, world, rank
        if log_r:
            self._p = lib().tachyon_mi355x_bn254_ntt4_create_split(log_n, log_r, world.bit_length() - 1, rank,
                                                                   stream.cuda_stream)
        else:
            self._p = lib().tachyon_mi355x_bn254_ntt4_create(log_n, world.bit_length() - 1, rank, stream.cuda_stream)
        if not self._p:
            raise RuntimeError("four-step NTT plan creation failed")
        self.log_r = lib().tachyon_mi355x_bn254_ntt4_log_rows(self._p)
        self.local_size = lib().tachyon_mi355x_bn254_ntt4_local_size(self._p)

    def close(self):
        if self._p:
            lib().tachyon_mi355x_bn254_ntt4_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stage(self, stage: int, inverse: bool, d_in: int, d_out: int):
        """Enqueue stage 1 (in -> send) or 2 (recv -> out) on the plan's stream."""
        lib().tachyon_mi355x_bn254_ntt4_stage(self._p, stage, 1 if inverse else 0, d_in, d_out)

    def run_stage(self, stage: int, inverse: bool, src, dst):
        """Tensor form of stage() for tachyon_amd.dist.sharded_ntt (device tensors)."""
        self.stage(stage, inverse, src.data_ptr(), dst.data_ptr())

    def run(self, comm, src, dst, inverse: bool = False):
        """Both stages and the all-to-all between them inside the library
        (tachyon_mi355x_bn254_ntt4_run) over a tachyon_amd.dist.LibComm whose
        world / rank are this plan's; src / dst: device tensors of local_size
        elements, ordered on the plan's stream."""
        if comm.world != self.world or comm.rank != self.rank:
            raise ValueError("communicator world/rank differ from the plan's")
        lib().tachyon_mi355x_bn254_ntt4_run(self._p, comm.handle, 1 if inverse else 0, src.data_ptr(), dst.data_ptr())

    def set_variant(self, variant: int):
        """A/B (same bytes): bit 0 = the round-4 stages (copy + passes +
        separate twiddle kernel) instead of the fused exchange; bit 1 = the
        32-bit-limb passes for the sub-transforms; bit 2 = one column per
        workgroup in one-pass sub-transforms (no packing); bit 3 = the
        exchange twiddles computed in the pass (no precomputed table)."""
        if not lib().tachyon_mi355x_bn254_ntt4_set_variant(self._p, variant):
            raise ValueError(f"unknown four-step variant {variant}")

    def synchronize(self):
        lib().tachyon_mi355x_bn254_ntt4_synchronize(self._p)

    @staticmethod
    def split_log_r(log_n: int, world: int) -> int:
        """log R of the split with the fewest pass launches (tachyon_mi355x_ntt4_split_log_r)."""
        return lib().tachyon_mi355x_ntt4_split_log_r(log_n, world.bit_length() - 1)

    @staticmethod
    def input_indices(log_n: int, world: int, rank: int, log_r: int = None):
        """Global index of each local input element: in[c_l*R + r] = x[C*r + c]."""
        import numpy as np
        lr = log_r or log_n // 2
        R, C = 1 << lr, 1 << (log_n - lr)
        cg = C // world
        c = rank * cg + np.arange(cg)[:, None]
        r = np.arange(R)[None, :]
        return (C * r + c).reshape(-1)

    @staticmethod
    def output_indices(log_n: int, world: int, rank: int, log_r: int = None):
        """Global index of each local output element: out[k1_l*C + k2] = X[k1 + R*k2]."""
        import numpy as np
        lr = log_r or log_n // 2
        R, C = 1 << lr, 1 << (log_n - lr)
        rg = R // world
        k1 = rank * rg + np.arange(rg)[:, None]
        k2 = np.arange(C)[None, :]
        return (k1 + R * k2).reshape(-1)


class RationalEvaluations:
    """UnivariateEvaluations<RationalField<bn254::Fr>> over the C-ABI
    (tachyon/c/math/polynomials/univariate/bn254_univariate_rational_evaluations.h):
    numerator / denominator pairs; batch_evaluate() runs on the GPU."""

    def __init__(self, _handle=None):
        self._h = _handle or lib().tachyon_bn254_univariate_rational_evaluations_create()

    @classmethod
    def empty(cls, domain: "Radix2EvaluationDomain"):
        """domain->Empty<RationalEvals>(): size() zeros (0 / 1)."""
        return cls(lib().tachyon_bn254_univariate_evaluation_domain_empty_rational_evals(domain._d))

    def close(self):
        if self._h:
            lib().tachyon_bn254_univariate_rational_evaluations_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return lib().tachyon_bn254_univariate_rational_evaluations_len(self._h)

    def clone(self):
        return RationalEvaluations(lib().tachyon_bn254_univariate_rational_evaluations_clone(self._h))

    def resize(self, n: int):
        lib().tachyon_mi355x_bn254_univariate_rational_evaluations_resize(self._h, n)

    def set_zero(self, i: int):
        lib().tachyon_bn254_univariate_rational_evaluations_set_zero(self._h, i)

    def set_trivial(self, i: int, numerator: bytes):
        lib().tachyon_bn254_univariate_rational_evaluations_set_trivial(
            self._h, i, ctypes.create_string_buffer(numerator, FR_BYTES))

    def set_rational(self, i: int, numerator: bytes, denominator: bytes):
        lib().tachyon_bn254_univariate_rational_evaluations_set_rational(
            self._h, i, ctypes.create_string_buffer(numerator, FR_BYTES),
            ctypes.create_string_buffer(denominator, FR_BYTES))

    def get(self, i: int):
        n, d = ctypes.create_string_buffer(FR_BYTES), ctypes.create_string_buffer(FR_BYTES)
        lib().tachyon_mi355x_bn254_univariate_rational_evaluations_get(self._h, i, n, d)
        return n.raw, d.raw

    def evaluate(self, i: int) -> bytes:
        out = ctypes.create_string_buffer(FR_BYTES)
        lib().tachyon_bn254_univariate_rational_evaluations_evaluate(self._h, i, out)
        return out.raw

    def batch_evaluate(self) -> bytes:
        L = lib()
        e = L.tachyon_bn254_univariate_rational_evaluations_batch_evaluate(self._h)
        n = L.tachyon_bn254_univariate_evaluations_len(e)
        out = ctypes.string_at(L.tachyon_mi355x_bn254_univariate_evaluations_data(e), n * FR_BYTES) if n else b""
        L.tachyon_bn254_univariate_evaluations_destroy(e)
        return out
