"""Host mirror of tachyon::crypto::KZG<G1Point, MaxDegree, Commitment> over the C-ABI.

Reference: tachyon/crypto/commitments/kzg/kzg.h -- UnsafeSetup(size[, tau])
(:169-207), N() (:167), Downsize (:210-215), Commit / CommitLagrange
(:217-258), batch commitments ResizeBatchCommitments / GetBatchCommitments
(:116-165, here `commit_batch`), g1_powers_of_tau[_lagrange] (:70-76).  The
SRS is generated and kept on the GPU (SetupForGpu, :90-114); commitments are
MSMs over it.  Scalars: Montgomery bytes / numpy (host) or CUDA tensors.
"""
import ctypes
import secrets

from ._lib import lib
from .msm import _ptr

CURVES = {"bn254_g1": (0, 64, "bn254_fr"), "bls12_381_g1": (2, 96, "bls12_381_fr")}


class KZG:
    def __init__(self, curve: str = "bn254_g1"):
        self.curve = curve
        self._cid, self.point_bytes, self.scalar_field = CURVES[curve]
        self._h = lib().tachyon_mi355x_kzg_create(self._cid)

    def close(self):
        if self._h:
            lib().tachyon_mi355x_kzg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def unsafe_setup(self, size: int, tau: bytes = None) -> bool:
        """tau: Montgomery bytes of the trapdoor; random (F::Random) if None."""
        if tau is None:
            from . import params as P
            r = P.FIELDS[self.scalar_field][0]
            tau = P.mont(secrets.randbelow(r), r, 4).to_bytes(32, "little")
        buf = ctypes.create_string_buffer(tau, 32)
        lib().tachyon_mi355x_kzg_unsafe_setup(self._h, size, buf)
        return True

    def N(self) -> int:
        return lib().tachyon_mi355x_kzg_n(self._h)

    def downsize(self, n: int) -> bool:
        return bool(lib().tachyon_mi355x_kzg_downsize(self._h, n))

    def _srs(self, lagrange: bool) -> bytes:
        out = ctypes.create_string_buffer(max(1, self.N() * self.point_bytes))
        lib().tachyon_mi355x_kzg_get_srs(self._h, 1 if lagrange else 0, out)
        return out.raw[:self.N() * self.point_bytes]

    def g1_powers_of_tau(self) -> bytes:
        return self._srs(False)

    def g1_powers_of_tau_lagrange(self) -> bytes:
        return self._srs(True)

    def _commit(self, scalars, lagrange: bool):
        p, n, keep = _ptr(scalars)
        out = ctypes.create_string_buffer(self.point_bytes)
        if not lib().tachyon_mi355x_kzg_commit(self._h, 1 if lagrange else 0, p, n // 32, out):
            return None
        return out.raw

    def commit(self, coeffs):
        """Commit(poly coefficients) -> affine commitment bytes, or None where
        the reference returns false (more coefficients than N, kzg.h:217-226)."""
        return self._commit(coeffs, False)

    def commit_lagrange(self, evals):
        """CommitLagrange(evaluations over the size-N domain) -> affine bytes,
        or None when |evals| > N (kzg.h:239-248)."""
        return self._commit(evals, True)

    def commit_batch(self, polys, lagrange: bool = False):
        """Batch mode (ResizeBatchCommitments + Commit(v, state, i) +
        GetBatchCommitments, kzg.h:116-165): one MSM per polynomial, the
        commitments normalised together with one inversion
        (tachyon_mi355x_kzg_commit_batch).  A list of affine bytes, or None
        when any polynomial has more than N elements."""
        if not polys:
            return []
        ptrs = [_ptr(p) for p in polys]
        arr = (ctypes.c_void_p * len(ptrs))(*[p for p, _, _ in ptrs])
        lens = (ctypes.c_size_t * len(ptrs))(*[nb // 32 for _, nb, _ in ptrs])
        out = ctypes.create_string_buffer(len(ptrs) * self.point_bytes)
        if not lib().tachyon_mi355x_kzg_commit_batch(self._h, 1 if lagrange else 0, arr, lens, len(ptrs), out):
            return None
        pb = self.point_bytes
        return [out.raw[i * pb:(i + 1) * pb] for i in range(len(ptrs))]
