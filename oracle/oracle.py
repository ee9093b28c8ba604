"""ORACLE (test infrastructure only): ctypes wrapper of oracle/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module -- as the checker / the CPU baseline, never as the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

FIELDS = {"bn254_fq": 0, "bn254_fr": 1, "bls12_381_fq": 2, "bls12_381_fr": 3}
FIELD_BYTES = {"bn254_fq": 32, "bn254_fr": 32, "bls12_381_fq": 48, "bls12_381_fr": 32}
CURVES = {"bn254_g1": 0, "bn254_g2": 1, "bls12_381_g1": 2, "bls12_381_g2": 3}
# affine point bytes, scalar field
CURVE_INFO = {
    "bn254_g1": (64, "bn254_fr"),
    "bn254_g2": (128, "bn254_fr"),
    "bls12_381_g1": (96, "bls12_381_fr"),
    "bls12_381_g2": (192, "bls12_381_fr"),
}
FIELD_OPS = {"add": 0, "sub": 1, "mul": 2, "sqr": 3, "neg": 4, "inv": 5, "to_mont": 6,
             "from_mont": 7, "dbl": 8}
MSM_METHODS = {"parallel_term": 0, "pippenger": 1, "naive": 2}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
        L.oracle_field_op.argtypes = [i, i, vp, vp, vp, sz]
        L.oracle_field_op.restype = i
        L.oracle_msm.argtypes = [i, vp, vp, sz, i, i, vp, vp]
        L.oracle_msm.restype = i
        L.oracle_fft.argtypes = [i, sz, vp, vp, sz]
        L.oracle_fft.restype = ctypes.c_long
        L.oracle_ifft.argtypes = [i, sz, vp, vp, sz]
        L.oracle_ifft.restype = ctypes.c_long
        L.oracle_gen_scalars.argtypes = [i, u64, sz, sz, vp]
        L.oracle_gen_scalars.restype = i
        L.oracle_gen_bases.argtypes = [i, u64, sz, sz, vp]
        L.oracle_gen_bases.restype = i
        L.oracle_ec_op.argtypes = [i, i, vp, vp, vp]
        L.oracle_ec_op.restype = i
        L.oracle_rand_u64.argtypes = [u64, u64]
        L.oracle_rand_u64.restype = u64
        L.oracle_domain_info.argtypes = [i, sz, vp]
        L.oracle_domain_info.restype = i
        L.oracle_max_threads.restype = i
        L.oracle_eval_at_powers.argtypes = [i, vp, sz, vp, vp, sz, vp]
        L.oracle_eval_at_powers.restype = i
        L.oracle_dlog_dot.argtypes = [i, u64, sz, sz, sz, vp, vp]
        L.oracle_dlog_dot.restype = i
        L.oracle_groth16_witness_map.argtypes = [i, sz, vp, sz, vp, sz, vp]
        L.oracle_groth16_witness_map.restype = i
        L.oracle_bn254_fr_set_halo2.argtypes = [i]
        L.oracle_bn254_fr_set_halo2.restype = i
        L.oracle_bn254_fr_large_subgroup_root.argtypes = [vp]
        L.oracle_bn254_fr_large_subgroup_root.restype = None
        _lib = L
    return _lib


def _buf(b):
    return ctypes.create_string_buffer(bytes(b), len(b)) if len(b) else ctypes.create_string_buffer(1)


def field_op(field, op, a: bytes, b: bytes = None) -> bytes:
    nb = FIELD_BYTES[field]
    count = len(a) // nb
    A = _buf(a)
    B = _buf(b if b is not None else a)
    out = ctypes.create_string_buffer(max(1, count * nb))
    rc = lib().oracle_field_op(FIELDS[field], FIELD_OPS[op], A, B, out, count)
    assert rc == 0
    return out.raw[:count * nb]


def msm(curve, bases: bytes, scalars: bytes, method="parallel_term", threads=0):
    """Returns (affine_bytes, jacobian_bytes)."""
    pb, sf = CURVE_INFO[curve]
    n = len(bases) // pb
    assert len(scalars) == n * FIELD_BYTES[sf]
    out = ctypes.create_string_buffer(pb)
    jac = ctypes.create_string_buffer(pb // 2 * 3)
    bb = np.frombuffer(bases, dtype=np.uint8) if n else np.zeros(1, np.uint8)
    ss = np.frombuffer(scalars, dtype=np.uint8) if n else np.zeros(1, np.uint8)
    rc = lib().oracle_msm(CURVES[curve], bb.ctypes.data, ss.ctypes.data, n, MSM_METHODS[method],
                          threads, out, jac)
    assert rc == 0
    return out.raw, jac.raw


def msm_np(curve, bases: np.ndarray, scalars: np.ndarray, method="parallel_term", threads=0):
    """Zero-copy variant for large numpy inputs (uint8/uint64 contiguous)."""
    pb, sf = CURVE_INFO[curve]
    n = bases.nbytes // pb
    out = ctypes.create_string_buffer(pb)
    rc = lib().oracle_msm(CURVES[curve], bases.ctypes.data, scalars.ctypes.data, n,
                          MSM_METHODS[method], threads, out, None)
    assert rc == 0
    return out.raw


def gen_scalars(field, seed, n, start=0) -> np.ndarray:
    out = np.empty(n * 4, dtype=np.uint64)
    rc = lib().oracle_gen_scalars(FIELDS[field], seed, start, n, out.ctypes.data)
    assert rc == 0
    return out


def gen_bases(curve, seed, n, chunk) -> np.ndarray:
    pb, _ = CURVE_INFO[curve]
    out = np.empty(n * pb // 8, dtype=np.uint64)
    rc = lib().oracle_gen_bases(CURVES[curve], seed, n, chunk, out.ctypes.data)
    assert rc == 0
    return out


def dlog_dot(field, seed, chunk, scalars, start=0) -> int:
    """sum_i s_i k_j 2^t mod r over the synthetic bases' known discrete logs
    (oracle_dlog_dot): MSM(gen_bases(seed, chunk) [start, start + n), scalars)
    = dlog_dot(...) * G.  `scalars`: Montgomery bytes / uint8 or uint64 array."""
    buf = np.ascontiguousarray(np.frombuffer(bytes(scalars), np.uint8) if isinstance(scalars, (bytes, bytearray))
                               else scalars)
    n = buf.nbytes // 32
    out = (ctypes.c_uint64 * 4)()
    fid = {"bn254_fr": 1, "bls12_381_fr": 3}[field]
    rc = lib().oracle_dlog_dot(fid, seed, start, n, chunk, buf.ctypes.data, out)
    assert rc == 0
    return sum(int(out[k]) << (64 * k) for k in range(4))


def eval_at_powers(coeffs, w_mont: bytes, indices, field="bn254_fr") -> list:
    """[sum_j c_j (w^i)^j for i in indices] as Montgomery bytes (oracle_eval_at_powers):
    the FFT's outputs at those indices without the butterfly network."""
    buf = np.ascontiguousarray(np.frombuffer(bytes(coeffs), np.uint8) if isinstance(coeffs, (bytes, bytearray))
                               else coeffs)
    n = buf.nbytes // 32
    idx = np.ascontiguousarray(np.array(indices, dtype=np.uint64))
    out = ctypes.create_string_buffer(32 * max(1, len(idx)))
    rc = lib().oracle_eval_at_powers(FIELDS[field], buf.ctypes.data, n, _buf(w_mont), idx.ctypes.data, len(idx), out)
    assert rc == 0
    return [out.raw[32 * q:32 * (q + 1)] for q in range(len(idx))]


def fft(coeffs: bytes, domain_num_coeffs, offset_mont: bytes = None, field="bn254_fr"):
    nb = FIELD_BYTES[field]
    size = 1 << max(0, (domain_num_coeffs - 1).bit_length())
    v = ctypes.create_string_buffer(bytes(coeffs) + b"\x00" * (size * nb - len(coeffs)), size * nb)
    off = _buf(offset_mont) if offset_mont else None
    r = lib().oracle_fft(FIELDS[field], domain_num_coeffs, off, v, len(coeffs) // nb)
    assert r >= 0
    return v.raw[:r * nb]


def ifft(evals: bytes, domain_num_coeffs, offset_mont: bytes = None, field="bn254_fr"):
    nb = FIELD_BYTES[field]
    size = 1 << max(0, (domain_num_coeffs - 1).bit_length())
    v = ctypes.create_string_buffer(bytes(evals) + b"\x00" * (size * nb - len(evals)), size * nb)
    off = _buf(offset_mont) if offset_mont else None
    r = lib().oracle_ifft(FIELDS[field], domain_num_coeffs, off, v, len(evals) // nb)
    assert r >= 0
    return v.raw[:r * nb]


def fft_np(v: np.ndarray, inverse=False, field="bn254_fr"):
    """In-place transform of a full-domain numpy array (uint64, 4 limbs/elt)."""
    n = v.size // 4
    f = lib().oracle_ifft if inverse else lib().oracle_fft
    r = f(FIELDS[field], n, None, v.ctypes.data, n)
    assert r >= 0
    return r


def ec_op(curve, op, p: bytes, q: bytes = None):
    pb, _ = CURVE_INFO[curve]
    ops = {"add": 0, "dbl": 1, "on_curve": 2, "mul": 3, "jac_to_affine": 4}
    out = ctypes.create_string_buffer(pb)
    P_ = _buf(p)
    Q_ = _buf(q) if q is not None else None
    r = lib().oracle_ec_op(CURVES[curve], ops[op], P_, Q_, out)
    if op == "on_curve":
        return bool(r)
    assert r == 0
    return out.raw


def max_threads():
    return lib().oracle_max_threads()


def bn254_fr_set_halo2(on: bool) -> bool:
    """OverrideSubgroupGenerator (on) / restore (off) for domains created
    afterwards (bn/bn254/halo2/bn254.cc:7-30).  Returns the previous state."""
    return bool(lib().oracle_bn254_fr_set_halo2(1 if on else 0))


def bn254_fr_large_subgroup_root() -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_bn254_fr_large_subgroup_root(out)
    return out.raw


class halo2_domain:
    """with halo2_domain(): ...  -- ScopedSubgroupGeneratorOverrider (bn254.cc:32-44)."""

    def __enter__(self):
        self._prev = bn254_fr_set_halo2(True)
        return self

    def __exit__(self, *exc):
        bn254_fr_set_halo2(self._prev)
        return False
