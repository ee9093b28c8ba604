"""Parity at the BASELINE sizes (BASELINE.json configs[1] "MSM 2^20 -> 2^26 sweep,
bit-exact vs CPU" and configs[2] "NTT 2^20 -> 2^24"): the GPU results on the
bench's own synthetic inputs (device-generated, the same seeds and schemes as
bench.py) equal the CPU oracle's bit for bit -- the oracle is the C
restatement of PippengerAdapter kParallelTerm / Radix2EvaluationDomain run
with all host threads (about 25 s of CPU at 2^26)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
SEED = 0x7AC40001  # bench.py's seed


@pytest.mark.timeout(400)
@pytest.mark.parametrize("logn", [20, 22, 24, 26])
def test_msm_sweep_vs_oracle(logn):
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = 1 << logn
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", SEED, n, 1 << 10, d_b.data_ptr())
    M.gen_scalars("bn254_fr", SEED, n, d_s.data_ptr())
    torch.cuda.synchronize()
    m = M.VariableBaseMSMGpu("bn254_g1")
    got = m.run(d_b, d_s)
    hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
    del d_b, d_s
    m.close()
    assert O.msm_np("bn254_g1", hb, hs) == got


def non_uniform_scalars(torch, M, field, n, seed=SEED + 3):
    """NonUniform(n, 1) (variable_base_msm_test_set.h:43-53; the reference's
    published GPU table, benchmark/msm --test_set non_uniform): one seeded
    random scalar repeated n times, on the device."""
    one = torch.empty(32, dtype=torch.uint8, device="cuda")
    M.gen_scalars(field, seed, 1, one.data_ptr())
    torch.cuda.synchronize()
    return one.repeat(n)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("logn", [23, 26])
def test_msm_non_uniform_vs_oracle(logn):
    """Every scalar equal: every window puts all n points into ONE bucket, so
    at 2^26 one bucket spans ~262 K accumulation threads and the chain join
    runs at its full depth.  Equals the oracle's kParallelTerm MSM on the same
    inputs, and s * (sum of the bases) -- the oracle's MSM with unit scalars
    (one digit per point) scaled by s -- as a second, independent CPU answer."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = 1 << logn
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", SEED, n, 1 << 10, d_b.data_ptr())
    d_s = non_uniform_scalars(torch, M, "bn254_fr", n)
    m = M.VariableBaseMSMGpu("bn254_g1")
    got = m.run(d_b, d_s)
    m.close()
    hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
    del d_b, d_s
    assert O.msm_np("bn254_g1", hb, hs) == got
    from tachyon_amd import params as P
    ones = np.tile(np.frombuffer(P.mont(1, P.BN254_FR, 4).to_bytes(32, "little"), np.uint8), n)
    total = O.msm_np("bn254_g1", hb, ones)
    assert O.msm("bn254_g1", total, hs[:32].tobytes())[0] == got


@pytest.mark.timeout(600)
@pytest.mark.parametrize("curve,pb", [("bls12_381_g1", 96), ("bls12_381_g2", 192)])
def test_bls_full_2_24_vs_oracle(curve, pb):
    """BASELINE configs[3] at the size the bench times: the whole 2^24-point
    BLS12-381 G1 / G2 MSM on the bench's own input (one GPU, the bench's plan)
    equals the oracle's kParallelTerm MSM on all host threads
    (variable_base_msm_gpu_unittest.cc:25-78 compares these groups GPU vs CPU)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = 1 << 24
    d_b = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases(curve, SEED, n, 1 << 10, d_b.data_ptr())
    M.gen_scalars("bls12_381_fr", SEED, n, d_s.data_ptr())
    torch.cuda.synchronize()
    m = M.VariableBaseMSMGpu(curve)
    got = m.run(d_b, d_s)
    m.close()
    hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
    del d_b, d_s
    assert O.msm_np(curve, hb, hs) == got


@pytest.mark.timeout(120)
@pytest.mark.parametrize("curve,pb", [("bn254_g1", 64), ("bls12_381_g2", 192)])
def test_gen_bases_any_start(curve, pb):
    """A rank's slice [start, start + n) of the seeded base sequence equals the
    same slice of the whole sequence for any start, not only multiples of the
    chunk (ceil(2^k / N) shards for N = 3, 5, 6, 7 ranks)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import dist as D
    from tachyon_amd import msm as M
    n_total, chunk = 3 * 4096 + 17, 1 << 10
    full = torch.empty(n_total * pb, dtype=torch.uint8, device="cuda")
    M.gen_bases(curve, SEED, n_total, chunk, full.data_ptr())
    for world in (3, 5, 7):
        for rank in range(world):
            start, n = D.shard_range(n_total, rank, world)
            part = torch.empty(max(1, n) * pb, dtype=torch.uint8, device="cuda")
            M.gen_bases(curve, SEED, n, chunk, part.data_ptr(), start=start)
            torch.cuda.synchronize()
            assert torch.equal(part[:n * pb], full[start * pb:(start + n) * pb]), (world, rank, start)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("logn", [20, 22, 24])
def test_ntt_sweep_vs_oracle(logn):
    """Forward and inverse transforms of the bench's input at 2^20..2^24."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    from tachyon_amd.ntt import Radix2EvaluationDomain
    n = 1 << logn
    d = Radix2EvaluationDomain(n)
    x = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_scalars("bn254_fr", SEED + 1, n, x.data_ptr())
    torch.cuda.synchronize()
    coeffs = x.cpu().numpy().view(np.uint64).copy()
    s = torch.cuda.ExternalStream(d.stream)
    d.transform_device(x.data_ptr(), inverse=False)
    s.synchronize()
    evals = x.cpu().numpy().view(np.uint64).copy()
    d.transform_device(x.data_ptr(), inverse=True)
    s.synchronize()
    back = x.cpu().numpy().view(np.uint64)
    d.close()
    expect = coeffs.copy()
    O.fft_np(expect)
    assert np.array_equal(evals, expect)
    O.fft_np(expect, inverse=True)
    assert np.array_equal(back, expect) and np.array_equal(back, coeffs)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("curve,pb", [("bls12_381_g1", 96), ("bls12_381_g2", 192)])
def test_bls_shard_vs_oracle(curve, pb):
    """BASELINE configs[3] (BLS12-381 G1 + G2 MSM 2^24 over 8 GPUs): one
    rank's 2^21-point shard of the bench's input equals the oracle."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = 1 << 21
    d_b = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases(curve, SEED, n, 1 << 10, d_b.data_ptr())
    M.gen_scalars("bls12_381_fr", SEED, n, d_s.data_ptr())
    torch.cuda.synchronize()
    m = M.VariableBaseMSMGpu(curve)
    got = m.run(d_b, d_s)
    m.close()
    assert O.msm_np(curve, d_b.cpu().numpy(), d_s.cpu().numpy()) == got


@pytest.mark.timeout(300)
def test_ntt_halo2_domain_vs_oracle():
    """The halo2 BN254 Fr domain (generator 7, OverrideSubgroupGenerator) at
    2^22: the HIP FFT and IFFT equal the oracle's on that domain."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    from tachyon_amd.ntt import Radix2EvaluationDomain, ScopedSubgroupGeneratorOverrider
    n = 1 << 22
    x = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_scalars("bn254_fr", SEED + 2, n, x.data_ptr())
    torch.cuda.synchronize()
    coeffs = x.cpu().numpy().view(np.uint64).copy()
    with ScopedSubgroupGeneratorOverrider():
        d = Radix2EvaluationDomain(n)
    s = torch.cuda.ExternalStream(d.stream)
    d.transform_device(x.data_ptr(), inverse=False)
    s.synchronize()
    evals = x.cpu().numpy().view(np.uint64).copy()
    d.transform_device(x.data_ptr(), inverse=True)
    s.synchronize()
    back = x.cpu().numpy().view(np.uint64)
    d.close()
    expect = coeffs.copy()
    with O.halo2_domain():
        O.fft_np(expect)
        assert np.array_equal(evals, expect)
        O.fft_np(expect, inverse=True)
    assert np.array_equal(back, coeffs) and np.array_equal(expect, coeffs)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("curve,logn,start", [("bn254_g1", 26, 0), ("bn254_g1", 23, 3 << 23), ("bn254_g2", 22, 0),
                                              ("bls12_381_g1", 24, 0), ("bls12_381_g2", 24, 0),
                                              ("bls12_381_g2", 21, 5 << 21)])
def test_msm_dlog_identity(curve, logn, start):
    """A full-size answer that shares nothing with the Pippenger restatement:
    the bench's bases are known multiples of G (chunk j of 2^10 points starts
    at k_j G and doubles), so the MSM equals (sum_i s_i k_j 2^t mod r) G --
    one inner product over Fr (oracle_dlog_dot) and one scalar multiplication
    in pure Python (oracle/pyref.py).  The whole 2^26 BN254 G1 MSM, the 2^24
    BLS12-381 G1 / G2 MSMs of configs[3], and rank shards that start mid-input
    (ranks 3 of 8 and 5 of 8), all on the device-generated bench inputs."""
    torch = pytest.importorskip("torch")
    from oracle import pyref
    from tachyon_amd import msm as M
    from tachyon_amd._lib import CURVE_INFO
    pb, sf = CURVE_INFO[curve]
    n = 1 << logn
    d_b = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases(curve, SEED, n, 1 << 10, d_b.data_ptr(), start=start)
    M.gen_scalars(sf, SEED, n, d_s.data_ptr(), start=start)
    torch.cuda.synchronize()
    m = M.VariableBaseMSMGpu(curve)
    got = m.run(d_b, d_s)
    m.close()
    hs = d_s.cpu().numpy()
    del d_b, d_s
    C = pyref.Curve(curve)
    assert got == C.to_bytes(C.mul(C.G, O.dlog_dot(sf, SEED, 1 << 10, hs, start=start)))


@pytest.mark.timeout(300)
def test_msm_dlog_identity_non_uniform_2_26():
    """NonUniform(2^26, 1) (every scalar equal) against the discrete-log identity."""
    torch = pytest.importorskip("torch")
    from oracle import pyref
    from tachyon_amd import msm as M
    n = 1 << 26
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", SEED, n, 1 << 10, d_b.data_ptr())
    d_s = non_uniform_scalars(torch, M, "bn254_fr", n)
    m = M.VariableBaseMSMGpu("bn254_g1")
    got = m.run(d_b, d_s)
    m.close()
    hs = d_s.cpu().numpy()
    del d_b, d_s
    C = pyref.Curve("bn254_g1")
    assert got == C.to_bytes(C.mul(C.G, O.dlog_dot("bn254_fr", SEED, 1 << 10, hs)))
