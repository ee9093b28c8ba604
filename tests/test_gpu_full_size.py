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
