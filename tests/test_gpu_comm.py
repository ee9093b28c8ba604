"""Library-level sharded entry points (include/tachyon_mi355x.h "communicators"):
the exchange of the multi-process MSM, four-step NTT and Groth16 runs inside
libtachyon_mi355x.so over a tachyon_mi355x_comm.

* RCCL backend, world 1 (the box has one GPU; RCCL refuses two ranks on one
  GPU, "Duplicate GPU detected"): ncclCommInitRank, ncclAllGather and the
  ncclSend/ncclRecv all-to-all on the real library, results equal to the
  unsharded MSM / the oracle's FFT / prove().
* Host-staged backend, world 2: two gloo ranks sharing the GPU, the library
  calling back into torch.distributed -- each rank's shard through the C
  entry, every rank's result equal to the unsharded MSM, the oracle's FFT slab
  and the single-process proof.
The reference caller shape is benchmark/msm/msm_benchmark_gpu.cc:57-69 under a
launcher (one process per GPU).
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402

import torch.multiprocessing as mp  # noqa: E402

from test_gpu_dist import _free_port, _run  # noqa: E402  (spawned gloo ranks on the one GPU)


def _g16_inputs(curve="bn254", log_n=7):
    from groth16_synth import synth_zkey
    from oracle import pyref
    zbytes, full = synth_zkey(curve, log_n=log_n, num_public=2, seed=91)
    Fr = pyref.Field("bn254_fr" if curve == "bn254" else "bls12_381_fr")
    fb = b"".join(Fr.to_bytes(v) for v in full)
    return zbytes, fb, Fr.to_bytes(0x55AA), Fr.to_bytes(Fr.p - 9)


def test_rccl_comm_world1():
    from tachyon_amd import dist as D
    from tachyon_amd.groth16 import Groth16Prover
    from tachyon_amd.msm import VariableBaseMSMGpu
    from tachyon_amd.ntt import FourStepNtt
    comm = D.LibComm.rccl()
    assert (comm.backend, comm.world, comm.rank) == ("rccl", 1, 0)
    # MSM: the sharded entry with one rank is the MSM
    n = 5000
    bases = O.gen_bases("bn254_g1", 3, n, 64).tobytes()
    scalars = O.gen_scalars("bn254_fr", 3, n).tobytes()
    m = VariableBaseMSMGpu("bn254_g1")
    assert m.run_sharded(comm, bases, scalars) == O.msm("bn254_g1", bases, scalars)[0]
    assert m.run_sharded(comm, b"", b"", 0) == bytes(64)  # an empty shard: the identity
    m.close()
    # NTT: stage 1, the ncclSend/ncclRecv all-to-all (to itself), stage 2
    log_n = 12
    x = O.gen_scalars("bn254_fr", 12, 1 << log_n)
    plan = FourStepNtt(log_n, 1, 0)
    idx = FourStepNtt.input_indices(log_n, 1, 0)
    src = torch.from_numpy(np.ascontiguousarray(x.reshape(-1, 4)[idx]).view(np.uint8).reshape(-1)).cuda()
    dst, back = torch.empty_like(src), torch.empty_like(src)
    torch.cuda.synchronize()
    plan.run(comm, src, dst)
    plan.run(comm, dst, back, inverse=True)
    plan.synchronize()
    want = np.frombuffer(O.fft(x.tobytes(), 1 << log_n), dtype=np.uint8).reshape(-1, 32)
    assert dst.cpu().numpy().tobytes() == np.ascontiguousarray(want[FourStepNtt.output_indices(log_n, 1, 0)]).tobytes()
    assert torch.equal(back, src)
    plan.close()
    # Groth16 through the library's sharded entry
    zbytes, fb, r, s = _g16_inputs()
    p = Groth16Prover(zbytes)
    assert p.prove_sharded(fb, r, s, comm=comm) == p.prove(fb, r, s)
    p.close()
    comm.close()


def _host_comm_worker(rank, world, port, q, log_n_ntt, g16):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tachyon_amd import dist as D
        from tachyon_amd.groth16 import Groth16Prover
        from tachyon_amd.msm import VariableBaseMSMGpu
        from tachyon_amd.ntt import FourStepNtt
        comm = D.LibComm.from_process_group()
        info = (comm.backend, comm.world, comm.rank)
        # MSM: rank's contiguous shard of one global input (device-resident)
        n = 7001
        bases = O.gen_bases("bn254_g1", 4, n, 64).view(np.uint8).reshape(n, 64)
        scalars = O.gen_scalars("bn254_fr", 4, n).view(np.uint8).reshape(n, 32)
        lo, cnt = D.shard_range(n, rank, world)
        db = torch.from_numpy(np.ascontiguousarray(bases[lo:lo + cnt]).reshape(-1)).cuda()
        ds = torch.from_numpy(np.ascontiguousarray(scalars[lo:lo + cnt]).reshape(-1)).cuda()
        m = VariableBaseMSMGpu("bn254_g1")
        msm = m.run_sharded(comm, db, ds, cnt)
        m.close()
        # NTT: the four-step with the host-staged all-to-all inside the library
        x = O.gen_scalars("bn254_fr", 707, 1 << log_n_ntt).reshape(-1, 4)
        plan = FourStepNtt(log_n_ntt, world, rank)
        idx = FourStepNtt.input_indices(log_n_ntt, world, rank)
        src = torch.from_numpy(np.ascontiguousarray(x[idx]).view(np.uint8).reshape(-1)).cuda()
        dst, back = torch.empty_like(src), torch.empty_like(src)
        torch.cuda.synchronize()
        plan.run(comm, src, dst)
        plan.run(comm, dst, back, inverse=True)
        plan.synchronize()
        ntt = (dst.cpu().numpy().tobytes(), FourStepNtt.output_indices(log_n_ntt, world, rank).tolist(),
               torch.equal(back, src))
        plan.close()
        # Groth16: partials, all-gather and assembly inside the library
        zbytes, fb, r, s = g16
        p = Groth16Prover(zbytes)
        proofs = (p.prove_sharded(fb, comm=comm), p.prove_sharded(fb, r, s, comm=comm))
        p.close()
        comm.close()
        q.put((rank, info, msm, ntt, proofs))
    finally:
        dist.destroy_process_group()


def test_host_staged_comm_world2():
    from tachyon_amd.groth16 import Groth16Prover
    log_n = 11
    g16 = _g16_inputs()
    got = _run(_host_comm_worker, 2, log_n, g16)
    n = 7001
    want_msm = O.msm("bn254_g1", O.gen_bases("bn254_g1", 4, n, 64).tobytes(), O.gen_scalars("bn254_fr", 4, n).tobytes())[0]
    x = O.gen_scalars("bn254_fr", 707, 1 << log_n).tobytes()
    want_ntt = np.frombuffer(O.fft(x, 1 << log_n), dtype=np.uint8).reshape(-1, 32)
    zbytes, fb, r, s = g16
    single = Groth16Prover(zbytes)
    want_proofs = (single.prove(fb), single.prove(fb, r, s))
    single.close()
    for rank, info, msm, (out, oidx, round_trip), proofs in got:
        assert info == ("host", 2, rank)
        assert msm == want_msm, rank
        assert out == np.ascontiguousarray(want_ntt[oidx]).tobytes() and round_trip, rank
        assert proofs == want_proofs, rank


def test_cpp_sharded_client_world1(tmp_path):
    """bin/comm_check: a C++ caller of the communicator entry points without
    torch (the rank writes / reads the RCCL unique id through a file, joins with
    tachyon_mi355x_comm_init_rccl, runs tachyon_mi355x_msm_gpu_sharded_affine on
    its shard of one seeded input and the four-step round trip through
    tachyon_mi355x_bn254_ntt4_run).  World 1 on the box's GPU: the MSM equals
    the oracle's and the discrete-log identity of the inputs."""
    import json
    import subprocess
    from oracle import pyref
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tachyon_amd", "bin", "comm_check")
    log_n = 12
    r = subprocess.run([exe, str(log_n), "1", "0", str(tmp_path / "uid")], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["backend"] == "rccl" and res["ntt_round_trip"]
    n, seed = 1 << log_n, 0xC0FFEE
    bases = O.gen_bases("bn254_g1", seed, n, 16).tobytes()
    scalars = O.gen_scalars("bn254_fr", seed, n).tobytes()
    want = O.msm("bn254_g1", bases, scalars)[0]
    assert bytes.fromhex(res["msm"]) == want
    C = pyref.Curve("bn254_g1")
    assert want == C.to_bytes(C.mul(C.G, O.dlog_dot("bn254_fr", seed, 16, scalars)))


def test_rccl_sharded_plan_entry_world1():
    """tachyon_mi355x_msm_gpu_sharded_plan_affine over the RCCL communicator at
    world 1: the library's own plan (one point shard: the whole MSM), and a
    hybrid shard of two window ranges (each range's partial is the window-range
    MSM at the shard's window bits; the two partials add up to the MSM)."""
    from tachyon_amd import dist as D
    from tachyon_amd import msm as M
    from tachyon_amd._lib import MsmShard
    comm = D.LibComm.rccl()
    n = 6000
    bases = O.gen_bases("bn254_g1", 8, n, 64).tobytes()
    scalars = O.gen_scalars("bn254_fr", 8, n).tobytes()
    want = O.msm("bn254_g1", bases, scalars)[0]
    db = torch.frombuffer(bytearray(bases), dtype=torch.uint8).cuda()
    ds = torch.frombuffer(bytearray(scalars), dtype=torch.uint8).cuda()
    m = M.VariableBaseMSMGpu("bn254_g1")
    s = M.shard_plan("bn254_g1", n, 1, 0)
    assert (s.start, s.count, s.window_groups) == (0, n, 1)
    assert m.run_sharded_plan(comm, s, db, ds) == want
    c = 13
    W = D._windows_for("bn254_g1", c)
    parts = []
    for w0, w1 in (D.window_range(W, 0, 2), D.window_range(W, 1, 2)):
        got = m.run_sharded_plan(comm, MsmShard(0, n, 1, 2, c, w0, w1), db, ds)
        m.set_window_bits(c)
        assert got == m.run_window_range(db, ds, w0, w1, n), (w0, w1)
        m.set_window_bits(0)
        parts.append(got)
    assert M.affine_sum("bn254_g1", b"".join(parts)) == want
    assert m.window_bits == 0 and m.run(db, ds) == want  # the entry restored the context's window bits
    m.close()
    comm.close()


def _hybrid_worker(rank, world, port, q, curve, n):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tachyon_amd import dist as D
        from tachyon_amd import msm as M
        from tachyon_amd._lib import MsmShard
        pb, sf = O.CURVE_INFO[curve]
        bases = O.gen_bases(curve, 31, n, 64).view(np.uint8).reshape(n, pb)
        scalars = O.gen_scalars(sf, 31, n).view(np.uint8).reshape(n, 32)
        comm = D.LibComm.from_process_group()
        # the hybrid at world 2: one point group (all points) x two window ranges, c = 16
        c = 16
        w0, w1 = D.window_range(D._windows_for(curve, c), rank, world)
        shard = MsmShard(0, n, 1, world, c, w0, w1)
        db = torch.from_numpy(np.ascontiguousarray(bases).reshape(-1)).cuda()
        ds = torch.from_numpy(np.ascontiguousarray(scalars).reshape(-1)).cuda()
        m = M.VariableBaseMSMGpu(curve)
        got = m.run_sharded_plan(comm, shard, db, ds)
        # and the library's own plan at world 2 (point shards)
        s = M.shard_plan(curve, n, world, rank)
        db2 = torch.from_numpy(np.ascontiguousarray(bases[s.start:s.start + s.count]).reshape(-1)).cuda()
        ds2 = torch.from_numpy(np.ascontiguousarray(scalars[s.start:s.start + s.count]).reshape(-1)).cuda()
        got2 = m.run_sharded_plan(comm, s, db2, ds2)
        m.close()
        comm.close()
        q.put((rank, got, got2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("curve,n", [("bn254_g1", 5000), ("bls12_381_g2", 700)])
def test_host_staged_sharded_plan_world2(curve, n):
    """Two gloo ranks sharing the GPU through the library's host-staged
    communicator: a hybrid shard (window ranges of all points) and the
    library's own world-2 plan; every rank's result is the oracle's MSM."""
    got = _run(_hybrid_worker, 2, curve, n)
    pb, sf = O.CURVE_INFO[curve]
    want = O.msm(curve, O.gen_bases(curve, 31, n, 64).tobytes(), O.gen_scalars(sf, 31, n).tobytes())[0]
    for rank, hyb, pts in got:
        assert hyb == want and pts == want, rank


def _failing_rank_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes
        import time
        from tachyon_amd import dist as D
        from tachyon_amd import msm as M
        from tachyon_amd._lib import lib
        comm = D.LibComm.from_process_group()
        n = 3000
        bases = O.gen_bases("bn254_g1", 5, n, 64).tobytes()
        scalars = O.gen_scalars("bn254_fr", 5, n).tobytes()
        s = M.shard_plan("bn254_g1", n, world, rank)
        m = M.VariableBaseMSMGpu("bn254_g1")
        ctx = m._ctx if rank == 0 else None  # rank 1's local part fails (null context)
        out = ctypes.create_string_buffer(64)
        t0 = time.time()
        rc = lib().tachyon_mi355x_msm_gpu_sharded_plan_affine(0, ctx, comm.handle, ctypes.byref(s),
                                                             bases[s.start * 64:], scalars[s.start * 32:], out)
        dt = time.time() - t0
        # the communicator still works after the failed call
        after = comm.all_gather(bytes([rank]))
        m.close()
        comm.close()
        q.put((rank, rc, out.raw == bytes(64), dt, after))
    finally:
        dist.destroy_process_group()


def test_failing_rank_does_not_hang_the_others():
    """A rank whose local part throws still enters the all-gather with a
    failure flag, so rank 0 -- whose MSM succeeded -- is not left waiting in
    the collective: tachyon_mi355x_msm_gpu_sharded_plan_affine returns 0 on
    BOTH ranks (out untouched, no abort) and the communicator stays usable."""
    got = _run(_failing_rank_worker, 2, timeout=180)
    for rank, rc, untouched, dt, after in got:
        assert rc == 0 and untouched and after == bytes([0, 1]), rank
        assert dt < 120, rank
