"""Test-side CPU mirror of the four-step plan (tachyon_amd.ntt.FourStepNtt):
the same stage-1 / stage-2 layouts, computed with the oracle's FFT and field
multiply.  Used only as the checker-side stand-in for the per-rank GPU kernels
in the gloo tests (the CPU container has no GPU); the GPU plan itself is
checked against the oracle in tests/test_gpu_ntt.py."""
import numpy as np

from oracle import oracle as O


def _mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = O.field_op("bn254_fr", "mul", np.ascontiguousarray(a).tobytes(), np.ascontiguousarray(b).tobytes())
    return np.frombuffer(out, dtype=np.uint64).reshape(-1, 4)


def _ntt_rows(m: np.ndarray, inverse: bool) -> np.ndarray:
    out = np.array(m, dtype=np.uint64, copy=True)
    for row in out:
        buf = np.ascontiguousarray(row)
        O.fft_np(buf, inverse=inverse)
        row[:] = buf
    return out


class CpuFourStepPlan:
    def __init__(self, log_n: int, world: int, rank: int):
        self.log_n, self.world, self.rank = log_n, world, rank
        self.n = 1 << log_n
        self.R, self.C = 1 << (log_n // 2), 1 << (log_n - log_n // 2)
        self.Rg, self.Cg = self.R // world, self.C // world
        self.local_size = self.n // world
        e1 = np.zeros((self.n, 4), dtype=np.uint64)
        e1[1] = np.frombuffer(O.field_op("bn254_fr", "to_mont", (1).to_bytes(32, "little")), dtype=np.uint64)
        O.fft_np(e1.reshape(-1))  # FFT of x: w^i, the power table of w_n
        self.pw = e1

    def _tw(self, inverse: bool) -> np.ndarray:
        c = self.rank * self.Cg + np.arange(self.Cg)[:, None]
        k1 = np.arange(self.R)[None, :]
        e = (c * k1) % self.n
        if inverse:
            e = (self.n - e) % self.n
        return self.pw[e.reshape(-1)]

    def _pack_index(self):
        c_l = np.arange(self.Cg)[:, None]
        k1 = np.arange(self.R)[None, :]
        h, k1_l = k1 // self.Rg, k1 % self.Rg
        return ((h * self.Cg + c_l) * self.Rg + k1_l).reshape(-1)

    def run_stage(self, stage: int, inverse: bool, src, dst):
        d = src.numpy().view(np.uint64).reshape(-1, 4)
        if not inverse and stage == 1:
            y = _ntt_rows(d.reshape(self.Cg, self.R, 4).reshape(self.Cg, -1), False).reshape(-1, 4)
            y = _mul(y, self._tw(False))
            out = np.empty_like(y)
            out[self._pack_index()] = y
        elif not inverse and stage == 2:
            t = d.reshape(self.C, self.Rg, 4).transpose(1, 0, 2).reshape(self.Rg, -1)
            out = _ntt_rows(t, False).reshape(-1, 4)
        elif inverse and stage == 1:
            y = _ntt_rows(d.reshape(self.Rg, -1), True).reshape(self.Rg, self.C, 4)
            out = y.transpose(1, 0, 2).reshape(-1, 4)
        else:
            y = d[self._pack_index()]
            y = _mul(y, self._tw(True))
            out = _ntt_rows(y.reshape(self.Cg, -1), True).reshape(-1, 4)
        dst.copy_(__import__("torch").from_numpy(np.ascontiguousarray(out).view(np.uint8).reshape(-1)))
