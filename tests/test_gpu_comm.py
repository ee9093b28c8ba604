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

from test_gpu_dist import _run  # noqa: E402  (spawned gloo ranks on the one GPU)


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
