"""Multi-rank MSM sharding on CPU (gloo, world_size 2..8): the shard split, the
all-gather of per-rank partial points and the product's host-side group sum
(tachyon_mi355x_affine_sum, no GPU needed) reproduce the single-process MSM.
The per-rank local MSM is the oracle here (the CPU box has no GPU); on the GPU
box bench.py runs the same code with the HIP MSM and RCCL."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tachyon_amd",
                   "libtachyon_mi355x.so")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, curve, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from tachyon_amd import dist as D
        pb, sf = O.CURVE_INFO[curve]
        bases = O.gen_bases(curve, 99, n, 16).tobytes()
        scalars = O.gen_scalars(sf, 99, n).tobytes()
        start, m = D.shard_range(n, rank, world)
        local = lambda: O.msm(curve, bases[start * pb:(start + m) * pb], scalars[start * 32:(start + m) * 32])[0]
        got = D.sharded_msm(curve, local)
        if rank == 0:
            q.put((got, O.msm(curve, bases, scalars)[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not os.path.exists(LIB), reason="libtachyon_mi355x.so not built")
@pytest.mark.parametrize("curve,n,world", [("bn254_g1", 301, 2), ("bls12_381_g1", 64, 2), ("bn254_g1", 203, 8),
                                           ("bn254_g2", 67, 4)])
def test_sharded_msm_gloo(curve, n, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, curve, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, expect = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == expect


def test_shard_range_covers():
    from tachyon_amd.dist import shard_range
    for n in (0, 1, 7, 64, 1 << 26):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert sum(m for _, m in spans) == n
            pos = 0
            for s, m in spans:
                if m:
                    assert s == pos
                pos = s + m if m else pos


def test_window_range_tiles():
    """dist.window_range: contiguous, ordered ranges tiling [0, W), sizes
    differing by at most one (W = 16 at c = 16 splits 2 per rank at N = 8)."""
    from tachyon_amd.dist import _windows_for, window_range
    assert _windows_for("bn254_g1", 16) == 16 and _windows_for("bn254_g1", 20) == 13
    assert _windows_for("bls12_381_g1", 16) == 16
    for W in (1, 5, 13, 16, 26):
        for world in (1, 2, 3, 4, 8, 16):
            spans = [window_range(W, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == W
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [w1 - w0 for w0, w1 in spans]
            assert max(sizes) - min(sizes) <= 1
    assert [window_range(16, r, 8) for r in range(8)] == [(2 * r, 2 * r + 2) for r in range(8)]


def _ntt_worker(rank, world, port, log_n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import numpy as np
        from oracle import oracle as O
        from tachyon_amd import dist as D
        from tachyon_amd.ntt import FourStepNtt
        from tests.ntt4_cpu_plan import CpuFourStepPlan
        n = 1 << log_n
        x = O.gen_scalars("bn254_fr", 4242 + log_n, n).reshape(n, 4)
        X = x.copy().reshape(-1)
        O.fft_np(X)
        X = X.reshape(n, 4)
        plan = CpuFourStepPlan(log_n, world, rank)
        local = torch.from_numpy(np.ascontiguousarray(x[FourStepNtt.input_indices(log_n, world, rank)]).view(np.uint8).reshape(-1))
        out = D.sharded_ntt(plan, local)
        ok_fwd = out.numpy().tobytes() == X[FourStepNtt.output_indices(log_n, world, rank)].tobytes()
        back = D.sharded_ntt(plan, out, inverse=True)
        ok_inv = back.numpy().tobytes() == local.numpy().tobytes()
        q.put((rank, ok_fwd, ok_inv))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,log_n", [(2, 4), (2, 7), (4, 8), (8, 8)])
def test_sharded_ntt_gloo(world, log_n):
    """Four-step distributed NTT orchestration (layouts + one all-to-all) over
    gloo; per-rank stages from the CPU mirror plan, result = the full oracle FFT
    (world 8 = the driver's 8-GPU layout)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ntt_worker, args=(r, world, port, log_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(r, True, True) for r in range(world)]


def test_four_step_layouts_partition():
    import numpy as np
    from tachyon_amd.ntt import FourStepNtt
    for log_n in (2, 5, 12):
        for world in (1, 2, 4, 8):
            if (1 << (log_n // 2)) < world:
                continue
            for f in (FourStepNtt.input_indices, FourStepNtt.output_indices):
                idx = np.concatenate([f(log_n, world, r) for r in range(world)])
                assert sorted(idx.tolist()) == list(range(1 << log_n))


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tachyon_amd import dist as D
        blob = bytes((rank * 37 + i) & 0xFF for i in range(1000))
        got = D.all_gather_bytes(blob)
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


def test_all_gather_bytes_world3():
    """The exchange of the multi-GPU Groth16 split (Groth16Prover.prove_sharded):
    one equal-length opaque blob per rank, concatenated in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == b"".join(bytes((r * 37 + i) & 0xFF for i in range(1000)) for r in range(3))


def _g16_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tachyon_amd.groth16 import Groth16Prover

        class HostOnly(Groth16Prover):
            """prove_sharded's host logic with the library calls stubbed out."""
            def __init__(self):
                self._h = None
                self.calls = []

            def partials_size(self):
                return 48

            def prove_partials(self, full, rank, world, with_b1=False):
                self.calls.append(("partials", rank, world, with_b1))
                return bytes([rank]) * 48

            def assemble(self, parts, r=None, s=None):
                self.calls.append(("assemble", parts, r, s))
                return (b"A", b"B", b"C")

        p = HostOnly()
        r = (7).to_bytes(32, "little")
        proof = p.prove_sharded(b"\0" * 64, r, r)
        q.put((rank, proof, p.calls))
    finally:
        dist.destroy_process_group()


def test_groth16_prove_sharded_world2():
    """Groth16Prover.prove_sharded: each rank computes its own shard (rank,
    world, B1 when r != 0), one all-gather hands every rank the blobs in rank
    order, every rank assembles the same proof."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_g16_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r = (7).to_bytes(32, "little")
    for rank, proof, calls in got:
        assert proof == (b"A", b"B", b"C")
        assert calls[0] == ("partials", rank, 2, True)
        assert calls[1] == ("assemble", bytes([0]) * 48 + bytes([1]) * 48, r, r)


def _lib_comm_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tachyon_amd import dist as D
        comm = D.LibComm.from_process_group()
        blob = bytes((rank * 53 + i) & 0xFF for i in range(777))
        got = (comm.backend, comm.world, comm.rank, comm.all_gather(blob), comm.all_gather(b""))
        comm.close()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_library_host_comm_world3():
    """The host-staged communicator of the library (tachyon_mi355x_comm_create_host
    with torch.distributed callbacks; no GPU work): tachyon_mi355x_comm_all_gather
    -- the exchange of the library's sharded MSM / Groth16 entries -- returns
    every rank's blob in rank order on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lib_comm_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=240) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = b"".join(bytes((r * 53 + i) & 0xFF for i in range(777)) for r in range(3))
    for rank, (backend, world, rk, g, empty) in got:
        assert (backend, world, rk) == ("host", 3, rank) and g == want and empty == b""


def _plan_worker(rank, world, port, curve, n, q):
    """One rank of the LIBRARY's partition (tachyon_mi355x_msm_shard_plan):
    its point group over its window range.  The window-range partial
    sum_{w in [w0, w1)} 2^(c w) S_w is the MSM of the scalars' c-bit digits of
    that range (the oracle computes it here -- no GPU on this box); the
    partials go through the library's host-staged communicator
    (tachyon_mi355x_comm_all_gather, the exchange of
    tachyon_mi355x_msm_gpu_sharded_plan_affine) and the library's host group
    sum."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from tachyon_amd import dist as D
        from tachyon_amd import msm as M
        pb, sf = O.CURVE_INFO[curve]
        bases = O.gen_bases(curve, 123, n, 16).tobytes()
        scalars = O.gen_scalars(sf, 123, n).tobytes()
        s = M.shard_plan(curve, n, world, rank)
        lo, m = s.start, s.count
        sc = scalars[lo * 32:(lo + m) * 32]
        if s.window_groups > 1:  # keep the digits of [w_begin, w_end) of every scalar of the group
            mask = sum(((1 << s.window_bits) - 1) << (s.window_bits * w) for w in range(s.w_begin, s.w_end))
            out = b""
            for i in range(m):
                k = int.from_bytes(O.field_op(sf, "from_mont", sc[32 * i:32 * (i + 1)]), "little") & mask
                out += O.field_op(sf, "to_mont", k.to_bytes(32, "little"))
            sc = out
        part = O.msm(curve, bases[lo * pb:(lo + m) * pb], sc)[0] if m else bytes(pb)
        comm = D.LibComm.from_process_group()
        total = M.affine_sum(curve, comm.all_gather(part))
        comm.close()
        q.put((rank, (s.point_groups, s.window_groups), total, O.msm(curve, bases, scalars)[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not os.path.exists(LIB), reason="libtachyon_mi355x.so not built")
@pytest.mark.parametrize("curve,n,world,groups", [("bn254_g1", 90, 8, (4, 2)), ("bls12_381_g2", 21, 4, (2, 2)),
                                                  ("bn254_g1", 50, 4, (4, 1))])
def test_library_shard_plan_gloo(curve, n, world, groups):
    """The hybrid point x window partition the library runs at N = 8 (BN254
    G1: 4 point groups x 2 window ranges, c = 19) and N = 4 (BLS12-381 G2),
    and point shards elsewhere: every rank's partial through the library's
    communicator sums to the oracle's MSM on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, curve, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, g, total, want in got:
        assert g == groups and total == want, rank
