"""Host mirror of the circom Groth16 prover over the C-ABI.

Reference interfaces mirrored (names and argument meaning):
  vendors/circom/prover_main.cc:82-160  CreateProof(zkey, wtns): ParseZKey,
      ParseWtns, then per run WitnessMapFromMatrices + CreateProofWithAssignment(NoZK|ZK)
  vendors/circom/circomlib/circuit/quadratic_arithmetic_program.h:24-113
      QuadraticArithmeticProgram::WitnessMapFromMatrices -> `witness_map`
  tachyon/zk/r1cs/groth16/prove.h:52-186
      CreateProofWithAssignment(pk, r, s, ...) / ...NoZK / ...ZK -> `prove`
All compute runs in libtachyon_mi355x.so on the GPU (the proving key is
uploaded once per Groth16Prover); there is no CPU fallback.

Field elements cross the boundary as Montgomery-form little-endian bytes (the
reference's in-memory layout); proofs come back as affine point bytes
(G1: 2 x Fq, G2: 2 x Fq2; identity = all zero bytes).
"""
import ctypes

from ._lib import lib
from .msm import _ptr

CURVE_NAMES = {0: "bn254", 1: "bls12_381"}
POINT_BYTES = {"bn254": (64, 128), "bls12_381": (96, 192)}


def wtns_parse(data: bytes, curve: str = "bn254") -> bytes:
    """wtns v2 -> Montgomery Fr bytes (wtns.h:99-117: canonical in, Montgomery out)."""
    cid = {v: k for k, v in CURVE_NAMES.items()}[curve]
    p, n, keep = _ptr(data)
    count = lib().tachyon_mi355x_wtns_parse(cid, p, n, None, 0)
    out = ctypes.create_string_buffer(max(1, count * 32))
    lib().tachyon_mi355x_wtns_parse(cid, p, n, out, count)
    return out.raw[:count * 32]


def zkey_curve(data: bytes) -> str:
    p, n, keep = _ptr(data)
    return CURVE_NAMES[lib().tachyon_mi355x_zkey_curve(p, n)]


class Groth16Prover:
    """ParseZKey + GetProvingKey().ToNativeProvingKey(), resident on the GPU."""

    def __init__(self, zkey: bytes):
        p, n, keep = _ptr(zkey)
        self._h = lib().tachyon_mi355x_groth16_prover_create(p, n)
        if not self._h:
            raise RuntimeError("failed to create the Groth16 prover")
        info = (ctypes.c_uint32 * 4)()
        lib().tachyon_mi355x_groth16_prover_info(self._h, info)
        self.curve = CURVE_NAMES[info[0]]
        self.num_vars, self.num_public, self.domain_size = info[1], info[2], info[3]
        self.g1_bytes, self.g2_bytes = POINT_BYTES[self.curve]

    @property
    def num_instance_variables(self):  # ZKey::GetNumInstanceVariables
        return self.num_public + 1

    def close(self):
        if self._h:
            lib().tachyon_mi355x_groth16_prover_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def witness_map(self, full) -> bytes:
        """WitnessMapFromMatrices: h evaluations on the coset (domain_size x 32 B)."""
        p, n, keep = _ptr(full)
        out = ctypes.create_string_buffer(self.domain_size * 32)
        lib().tachyon_mi355x_groth16_witness_map(self._h, p, n // 32, out)
        return out.raw

    def prove(self, full, r: bytes = None, s: bytes = None):
        """CreateProofWithAssignment(pk, r, s, h, instance, witness, full[1:]);
        r = s = None is CreateProofWithAssignmentNoZK.  `full` may be host
        bytes/numpy or a CUDA tensor.  Returns (A, B, C) affine bytes."""
        p, n, keep = _ptr(full)
        a = ctypes.create_string_buffer(self.g1_bytes)
        b = ctypes.create_string_buffer(self.g2_bytes)
        c = ctypes.create_string_buffer(self.g1_bytes)
        rb = ctypes.create_string_buffer(r, 32) if r is not None else None
        sb = ctypes.create_string_buffer(s, 32) if s is not None else None
        lib().tachyon_mi355x_groth16_prove(self._h, p, n // 32, rb, sb, a, b, c)
        return a.raw, b.raw, c.raw

    # ---- multi-GPU split (one process per GPU) ----
    def partials_size(self) -> int:
        return lib().tachyon_mi355x_groth16_partials_size(self._h)

    def prove_partials(self, full, rank: int, world: int, with_b1: bool = False) -> bytes:
        """This rank's shard of the proof's MSMs (after the full witness map) as an
        opaque blob of partials_size() bytes; with_b1 is required when the
        proof will be assembled with r != 0."""
        p, n, keep = _ptr(full)
        out = ctypes.create_string_buffer(self.partials_size())
        lib().tachyon_mi355x_groth16_prove_partials(self._h, p, n // 32, 1 if with_b1 else 0, rank, world, out)
        return out.raw

    def assemble(self, parts: bytes, r: bytes = None, s: bytes = None):
        """Sum the per-rank partials (concatenated blobs, one per rank) and
        apply r, s and the key's alpha/beta/delta terms -> (A, B, C)."""
        size = self.partials_size()
        if len(parts) % size:
            raise ValueError("partials blob length is not a multiple of partials_size()")
        p, n, keep = _ptr(parts)
        a = ctypes.create_string_buffer(self.g1_bytes)
        b = ctypes.create_string_buffer(self.g2_bytes)
        c = ctypes.create_string_buffer(self.g1_bytes)
        rb = ctypes.create_string_buffer(r, 32) if r is not None else None
        sb = ctypes.create_string_buffer(s, 32) if s is not None else None
        lib().tachyon_mi355x_groth16_assemble(self._h, p, len(parts) // size, rb, sb, a, b, c)
        return a.raw, b.raw, c.raw

    def prove_sharded(self, full, r: bytes = None, s: bytes = None, group=None, device=None, comm=None):
        """prove() across the ranks of `group`: every rank runs the witness map
        and its MSM shard, one all-gather exchanges the partials, every rank
        assembles the same proof.  World size 1 (or no process group) is prove().
        With `comm` (a tachyon_amd.dist.LibComm) the whole flow runs inside the
        library (tachyon_mi355x_groth16_prove_sharded) over that communicator."""
        import torch.distributed as dist
        from .dist import all_gather_bytes
        if comm is not None:
            p, n, keep = _ptr(full)
            a = ctypes.create_string_buffer(self.g1_bytes)
            b = ctypes.create_string_buffer(self.g2_bytes)
            c = ctypes.create_string_buffer(self.g1_bytes)
            rb = ctypes.create_string_buffer(r, 32) if r is not None else None
            sb = ctypes.create_string_buffer(s, 32) if s is not None else None
            lib().tachyon_mi355x_groth16_prove_sharded(self._h, comm.handle, p, n // 32, rb, sb, a, b, c)
            return a.raw, b.raw, c.raw
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
            return self.prove(full, r, s)
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        with_b1 = r is not None and any(r)
        part = self.prove_partials(full, rank, world, with_b1)
        return self.assemble(all_gather_bytes(part, group, device), r, s)

    def prepare(self, rank: int = 0, world: int = 1, with_b1: bool = False) -> int:
        """Proving-key setup: build the fixed-base fold tables the proofs of
        shard (rank, world) use, each the largest fold that fits the device
        beside the MSM's working set (tachyon_mi355x_groth16_prepare); returns
        the table bytes held.  A proof without it prepares itself."""
        return lib().tachyon_mi355x_groth16_prepare(self._h, rank, world, 1 if with_b1 else 0)

    def folds(self) -> dict:
        """Folds the last prepare chose (1 = no table; grouped_g1 0 = A and the
        witness + h MSM ran as separate MSMs; a1 / b1 / lh 0 = not built)."""
        out = (ctypes.c_uint32 * 5)()
        lib().tachyon_mi355x_groth16_prover_folds(self._h, out)
        return dict(zip(("b2", "grouped_g1", "a1", "b1", "lh"), list(out)))

    def set_devices(self, device_ids):
        """One-process multi-device proofs: every later prove() runs the
        multi-rank split with one host thread per device entry (ids may
        repeat; [] or one id = single device) -- tachyon_mi355x_groth16_set_devices."""
        ids = list(device_ids)
        arr = (ctypes.c_int * max(1, len(ids)))(*ids)
        if not lib().tachyon_mi355x_groth16_set_devices(self._h, arr, len(ids)):
            raise ValueError(f"device ids out of range: {ids}")

    def set_variant(self, variant: int):
        """A/B: bit 0 = A and the witness + h MSM as two MSMs (round 4), clear =
        one grouped MSM (default); bits 1-3 = the G2 B query's fold table,
        bits 4-6 the grouped G1 MSM's (0 = the default, B2 16 copies and G1 4;
        k = 1..5: up to 2^(k-1) copies, 1 = none); same proof."""
        if not lib().tachyon_mi355x_groth16_set_variant(self._h, variant):
            raise ValueError(f"unknown Groth16 variant {variant}")

    def set_msm_window_bits(self, c_a: int = 0, c_lh: int = 0, c_b2: int = 0):
        """Window bits of the proof's MSMs (0 = default): A / B in G1, the merged
        witness + h MSM, B in G2 (tuning; same proof)."""
        lib().tachyon_mi355x_groth16_set_msm_window_bits(self._h, c_a, c_lh, c_b2)

    def set_profile(self, on: bool):
        lib().tachyon_mi355x_groth16_set_profile(self._h, 1 if on else 0)

    def last_timings(self) -> dict:
        """ms per phase of the last prove with profiling on; msm_l is the merged
        witness + h MSM (msm_h stays 0)."""
        out = (ctypes.c_float * 8)()
        lib().tachyon_mi355x_groth16_last_timings(self._h, out)
        return dict(zip(("upload", "qap", "msm_a", "msm_b2", "msm_b1", "msm_l", "msm_h", "total"), list(out)))


def create_proof_with_assignment_no_zk(prover: Groth16Prover, full):
    return prover.prove(full)


def create_proof_with_assignment(prover: Groth16Prover, r: bytes, s: bytes, full):
    return prover.prove(full, r, s)
