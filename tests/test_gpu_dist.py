"""Multi-rank flows with the real HIP library: two gloo ranks that share the
one GPU of the box (the 8-GPU RCCL runs are the driver's).

* Groth16Prover.prove_sharded: each rank computes its real partial blob
  (tachyon_mi355x_groth16_prove_partials), one all-gather, every rank
  assembles -- the proof equals prove() on one process and the oracle.
* tachyon_amd.dist.sharded_ntt: the input slab is produced by work on another
  stream than the plan's (the ordering contract of the four-step C-ABI: the
  plan's stream waits for the caller's), and the distributed transform equals
  the oracle's FFT of the global vector; the inverse returns the input.
"""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(target, world, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=timeout) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(got, key=lambda t: t[0])


def _g16_worker(rank, world, port, q, zbytes, fb, r, s):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tachyon_amd.groth16 import Groth16Prover
        prover = Groth16Prover(zbytes)
        nozk = prover.prove_sharded(fb)
        zk = prover.prove_sharded(fb, r, s)
        prover.close()
        q.put((rank, nozk, zk))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("curve,log_n", [("bn254", 8), ("bls12_381", 6)])
def test_groth16_prove_sharded_real_partials_world2(curve, log_n):
    from groth16_synth import synth_zkey
    from oracle import circom_format as CF
    from oracle import groth16 as OG
    from oracle import pyref
    from tachyon_amd.groth16 import Groth16Prover
    zbytes, full = synth_zkey(curve, log_n=log_n, num_public=2, seed=77)
    Fr = pyref.Field("bn254_fr" if curve == "bn254" else "bls12_381_fr")
    fb = b"".join(Fr.to_bytes(v) for v in full)
    r_int, s_int = 0x1234567, Fr.p - 3
    r, s = Fr.to_bytes(r_int), Fr.to_bytes(s_int)
    got = _run(_g16_worker, 2, zbytes, fb, r, s)
    zk = CF.parse_zkey(zbytes)
    want_nozk, want_zk = list(OG.prove(zk, full)), list(OG.prove(zk, full, r_int, s_int))
    single = Groth16Prover(zbytes)
    assert list(single.prove(fb)) == want_nozk
    single.close()
    for rank, nozk, zkp in got:
        assert list(nozk) == want_nozk, rank
        assert list(zkp) == want_zk, rank


def _ntt_worker(rank, world, port, q, log_n):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import numpy as np
        from oracle import oracle as O
        from tachyon_amd import dist as D
        from tachyon_amd.ntt import FourStepNtt
        n = 1 << log_n
        x = O.gen_scalars("bn254_fr", 606, n).view(np.uint8).reshape(n, 32)
        plan = FourStepNtt(log_n, world, rank)
        idx = FourStepNtt.input_indices(log_n, world, rank)
        host = torch.from_numpy(np.ascontiguousarray(x[idx]).reshape(-1))
        # produce the slab on a side stream, after a delay kernel there, so a
        # plan that did not wait for the caller's stream would read garbage
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            big = torch.ones(1 << 24, device="cuda")
            for _ in range(20):
                big = big * 1.0001
            local = torch.zeros(host.numel(), dtype=torch.uint8, device="cuda")
            local.copy_(host.cuda(non_blocking=False))
            out = D.sharded_ntt(plan, local)
            back = D.sharded_ntt(plan, out, inverse=True)
        plan.torch_stream.synchronize()
        oidx = FourStepNtt.output_indices(log_n, world, rank)
        q.put((rank, out.cpu().numpy().tobytes(), oidx.tolist(), back.cpu().numpy().tobytes() == host.numpy().tobytes()))
        plan.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("log_n", [10, 15])
def test_sharded_ntt_cross_stream_world2(log_n):
    import numpy as np
    from oracle import oracle as O
    n = 1 << log_n
    got = _run(_ntt_worker, 2, log_n)
    x = O.gen_scalars("bn254_fr", 606, n).tobytes()
    want = np.frombuffer(O.fft(x, n), dtype=np.uint8).reshape(n, 32)
    for rank, out, oidx, round_trip in got:
        assert round_trip, rank
        assert out == np.ascontiguousarray(want[oidx]).tobytes(), rank


def _window_split_worker(rank, world, port, q, n, c):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from tachyon_amd import dist as D
        from tachyon_amd.msm import VariableBaseMSMGpu
        bases = O.gen_bases("bn254_g1", 5, n, 64).tobytes()
        scalars = O.gen_scalars("bn254_fr", 5, n).tobytes()
        m = VariableBaseMSMGpu("bn254_g1")
        got = D.window_split_msm("bn254_g1", m, bases, scalars, n, c)
        m.close()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,c", [(2, 16), (3, 12)])
def test_window_split_msm_gloo(world, c):
    """dist.window_split_msm: every rank holds all points and computes its
    window range (tachyon_mi355x_msm_gpu_window_range_affine); the all-gathered
    partials sum to the oracle's MSM on every rank."""
    from oracle import oracle as O
    n = 3000
    bases = O.gen_bases("bn254_g1", 5, n, 64).tobytes()
    scalars = O.gen_scalars("bn254_fr", 5, n).tobytes()
    want, _ = O.msm("bn254_g1", bases, scalars)
    for rank, got in _run(_window_split_worker, world, n, c):
        assert got == want, rank
