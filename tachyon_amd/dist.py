"""One-process-per-GPU sharding of the MSM (torch.distributed; backend "nccl" = RCCL).

The reference's kParallelTerm strategy (pippenger_adapter.h:82-113) splits the
points into contiguous chunks, runs one Pippenger per chunk and adds the chunk
results; the multi-GPU MSM is the same decomposition with one chunk per rank.
The only exchange is one all-gather of the per-rank partial points (affine,
64 B for BN254 G1) followed by a group sum on every rank -- elliptic-curve
addition is not an RCCL reduction operator.

The NTT shards as a four-step (Bailey) transform with ONE all-to-all
(sharded_ntt): local R-point NTTs on column slabs, twiddles,
all-to-all transpose, local C-point NTTs on row slabs.
"""
import ctypes
import sys
import traceback
from typing import Callable

import numpy as np

from ._lib import COMM_FN, CURVE_INFO, lib
from .msm import affine_sum


class LibComm:
    """A communicator of the library (tachyon_mi355x_comm, include/tachyon_mi355x.h
    "communicators"): the sharded entry points -- msm.VariableBaseMSMGpu.run_sharded,
    ntt.FourStepNtt.run, groth16.Groth16Prover.prove_sharded(comm=...) -- do
    their exchange inside the C++ library through it.

    * LibComm.rccl(group): RCCL over xGMI, ncclCommInitRank from a unique id
      that rank 0 creates and broadcasts over the torch process group (one
      GPU per rank; RCCL refuses two ranks on one GPU).
    * LibComm.from_process_group(group): the HOST-STAGED FALLBACK -- the
      library calls back into torch.distributed (gloo: host tensors; nccl:
      device tensors) with host buffers.
    """

    def __init__(self, handle, keep=()):
        if not handle:
            raise RuntimeError("communicator creation failed")
        self._h = handle
        self._keep = keep  # the ctypes callbacks must outlive the handle

    @property
    def handle(self):
        return self._h

    @property
    def world(self) -> int:
        return lib().tachyon_mi355x_comm_world(self._h)

    @property
    def rank(self) -> int:
        return lib().tachyon_mi355x_comm_rank(self._h)

    @property
    def backend(self) -> str:
        return lib().tachyon_mi355x_comm_backend(self._h).decode()

    def all_gather(self, blob: bytes) -> bytes:
        """Every rank's equal-length blob, concatenated in rank order
        (tachyon_mi355x_comm_all_gather)."""
        out = ctypes.create_string_buffer(max(1, len(blob) * self.world))
        lib().tachyon_mi355x_comm_all_gather(self._h, ctypes.create_string_buffer(blob, max(1, len(blob))), out,
                                             len(blob))
        return out.raw[:len(blob) * self.world]

    def close(self):
        if self._h:
            lib().tachyon_mi355x_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @classmethod
    def rccl(cls, group=None):
        """RCCL communicator over the ranks of `group` (world 1 without a group)."""
        import torch.distributed as dist
        multi = dist.is_available() and dist.is_initialized()
        world = dist.get_world_size(group) if multi else 1
        rank = dist.get_rank(group) if multi else 0
        uid = ctypes.create_string_buffer(128)
        if rank == 0 and lib().tachyon_mi355x_comm_unique_id(uid, 128) != 128:
            raise RuntimeError("ncclGetUniqueId failed")
        raw = uid.raw
        if world > 1:
            obj = [raw if rank == 0 else None]
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(obj, src=src, group=group)
            raw = obj[0]
        return cls(lib().tachyon_mi355x_comm_init_rccl(ctypes.create_string_buffer(raw, 128), world, rank))

    @classmethod
    def from_process_group(cls, group=None):
        """Host-staged communicator whose exchanges are torch.distributed collectives."""
        import torch
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        device = None if _host_collectives(group) else torch.device("cuda", torch.cuda.current_device())

        def tensor(ptr, nbytes):
            t = torch.frombuffer(bytearray(ctypes.string_at(ptr, nbytes)), dtype=torch.uint8)
            return t.to(device) if device is not None else t

        def store(ptr, t):
            h = t.cpu().numpy()
            ctypes.memmove(ptr, h.ctypes.data, h.nbytes)

        def all_gather(_user, send, recv, nbytes):
            try:
                t = tensor(send, nbytes)
                out = torch.empty(world * nbytes, dtype=torch.uint8, device=t.device)
                dist.all_gather_into_tensor(out, t, group=group)
                store(recv, out)
                return 0
            except Exception:
                traceback.print_exc(file=sys.stderr)
                return 1

        def all_to_all(_user, send, recv, nbytes):
            try:
                t = tensor(send, world * nbytes)
                out = torch.empty_like(t)
                dist.all_to_all_single(out, t, group=group)
                store(recv, out)
                return 0
            except Exception:
                traceback.print_exc(file=sys.stderr)
                return 1

        ag, a2a = COMM_FN(all_gather), COMM_FN(all_to_all)
        return cls(lib().tachyon_mi355x_comm_create_host(world, rank, ag, a2a, None), keep=(ag, a2a))


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous shard [start, start + n) of rank (ceil split, like
    base::ParallelizeMap's ceil(n / T) chunking)."""
    chunk = (n_total + world - 1) // world
    start = min(rank * chunk, n_total)
    return start, max(0, min(chunk, n_total - start))


def combine_partials(curve: str, partials: bytes) -> bytes:
    """Sum of the per-rank affine partials (host group arithmetic of the product library)."""
    return affine_sum(curve, partials)


def _host_collectives(group=None) -> bool:
    """gloo takes host tensors: it is the CPU rehearsal backend of the multi-rank
    path (tests, or bench.py with TACHYON_DIST_BACKEND=gloo on a one-GPU box);
    nccl (= RCCL on ROCm) moves device tensors over xGMI."""
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"


def all_gather_bytes(blob: bytes, group=None, device=None) -> bytes:
    """All-gather one equal-length byte blob per rank; returns the concatenation
    in rank order (device tensors over RCCL when `device` is given, host
    tensors under gloo)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    if device is not None and not _host_collectives(group):
        t = t.to(device)
    out = torch.empty(world * len(blob), dtype=torch.uint8, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu().numpy().tobytes()


def all_gather_partials(curve: str, partial: bytes, group=None, device=None) -> bytes:
    """All-gather every rank's affine partial; returns the concatenation in rank order."""
    if len(partial) != CURVE_INFO[curve][0]:
        raise ValueError(f"{curve} partial must be one affine point")
    return all_gather_bytes(partial, group, device)


def sharded_msm(curve: str, local_msm: Callable[[], bytes], group=None, device=None) -> bytes:
    """Run `local_msm()` (this rank's shard -> affine partial) and combine across ranks."""
    import torch.distributed as dist
    part = local_msm()
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return part
    return combine_partials(curve, all_gather_partials(curve, part, group, device))


def window_range(windows: int, rank: int, world: int):
    """Rank's contiguous window range [w0, w1) of W windows (the window split)."""
    base, extra = divmod(windows, world)
    w0 = rank * base + min(rank, extra)
    return w0, w0 + base + (1 if rank < extra else 0)


def window_split_msm(curve: str, msm, bases, scalars, n: int, c: int, group=None, device=None) -> bytes:
    """The MSM split by WINDOWS across ranks: every rank holds all n points and
    computes sum_{w in its range} 2^(c w) S_w (msm.run_window_range with c-bit
    windows); one all-gather of the affine partials and a host group sum, as
    for the point split.  With W a multiple of the world size (c = 16: W = 16
    for 254-bit scalars) every rank does n * W / N additions over a W/N-window
    bucket set.  Measured per rank at 2^26 (tools/split_probe.py): 16.2 ms at
    N = 8 (2 windows) vs 14.4 ms for a 2^23-point shard -- every rank recodes
    all n scalars, and 2 x 2^26 additions exceed the shard's 15 x 2^23 -- so
    the bench keeps the point split; this is the option for inputs that are
    already replicated."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    windows = _windows_for(curve, c)
    w0, w1 = window_range(windows, rank, world)
    prev = getattr(msm, "window_bits", 0)
    msm.set_window_bits(c)
    try:
        part = msm.run_window_range(bases, scalars, w0, w1, n)
    finally:  # the caller's context keeps its own window choice
        msm.set_window_bits(prev)
    if world == 1:
        return part
    return combine_partials(curve, all_gather_partials(curve, part, group, device))


def _windows_for(curve: str, c: int) -> int:
    bits = 254 if curve.startswith("bn254") else 255  # Fr modulus bits (BN254 / BLS12-381)
    return (bits + 1 + c - 1) // c


def sharded_ntt(plan, local, inverse: bool = False, group=None):
    """Distributed NTT of this rank's slab (tachyon_amd.ntt.FourStepNtt layouts).

    `local` is a uint8 tensor of plan.local_size * 32 bytes (device tensor for
    the GPU plan); returns the output slab.  The plan's kernels and the RCCL
    all-to-all run on the plan's stream (plan.torch_stream), so no host
    synchronisation is needed between the stages; the result is ready on that
    stream (the caller's stream waits for it on the next sharded_ntt call or
    should call plan.torch_stream.synchronize()).
    """
    import torch
    import torch.distributed as dist
    stream = getattr(plan, "torch_stream", None)
    if stream is None or not local.is_cuda:  # host plan (CPU rehearsal)
        return _sharded_ntt_on_stream(plan, local, inverse, group)
    # one stream orders the stages, the collective and the allocations
    # (the caller's tensor must be ready on the plan's stream)
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        return _sharded_ntt_on_stream(plan, local, inverse, group)


def _sharded_ntt_on_stream(plan, local, inverse, group):
    import torch
    import torch.distributed as dist
    send = torch.empty_like(local)
    out = torch.empty_like(local)
    plan.run_stage(1, inverse, local, send)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if send.is_cuda and _host_collectives(group):
            recv_h = torch.empty(send.shape, dtype=send.dtype)
            dist.all_to_all_single(recv_h, send.cpu(), group=group)
            recv = recv_h.to(send.device)
        else:
            recv = torch.empty_like(local)
            dist.all_to_all_single(recv, send, group=group)
    else:
        recv = send
    plan.run_stage(2, inverse, recv, out)
    return out
