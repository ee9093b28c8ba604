"""Radix-2 domains between and above the bench sizes, up to the two-adicity.

The reference's Radix2EvaluationDomain serves every power of two up to
2^kTwoAdicity = 2^28 for BN254 Fr (radix2_evaluation_domain.h:95-97; the
factory only switches to MixedRadix above it,
univariate_evaluation_domain_factory.h:33-43), so the C-ABI accepts those
sizes too.  From 2^25 the pass plan has four passes (k = 6/6/6/7 stages at
2^25, 7/7/7/7 at 2^28) and at 2^23 three uneven ones (7/8/8): each is checked
here bytewise against the oracle's transform (radix2_evaluation_domain.h:213-333)
through the device entry point, and at 2^25 also through the host C-ABI
(tachyon_bn254_univariate_evaluation_domain_fft / _ifft), on the coset, and
through the four-step plans.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
SEED = 0x7AC40001


def _device_input(torch, n, seed):
    from tachyon_amd import msm as M
    x = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_scalars("bn254_fr", seed, n, x.data_ptr())
    torch.cuda.synchronize()
    return x


def _transform(torch, d, x, inverse):
    s = torch.cuda.ExternalStream(d.stream)
    d.transform_device(x.data_ptr(), inverse=inverse)
    s.synchronize()
    return x.cpu().numpy().view(np.uint64).copy()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("logn", [23, 25, 26, 27])
def test_ntt_device_vs_oracle_above_bench_sizes(logn):
    """transform_device forward and inverse bytewise equal to the oracle."""
    torch = pytest.importorskip("torch")
    from tachyon_amd.ntt import Radix2EvaluationDomain
    n = 1 << logn
    d = Radix2EvaluationDomain(n)
    assert d.size == n
    x = _device_input(torch, n, SEED + logn)
    coeffs = x.cpu().numpy().view(np.uint64).copy()
    evals = _transform(torch, d, x, False)
    back = _transform(torch, d, x, True)
    d.close()
    del x
    expect = coeffs.copy()
    O.fft_np(expect)
    assert np.array_equal(evals, expect)
    O.fft_np(expect, inverse=True)
    assert np.array_equal(back, expect) and np.array_equal(back, coeffs)


@pytest.mark.timeout(900)
def test_ntt_two_adicity_2_28():
    """The largest radix-2 domain, 2^28 = 2^kTwoAdicity: the forward transform
    equals the oracle's bytewise and the inverse returns the input (with the
    forward equal to the oracle's bijection, that pins the inverse too)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd.ntt import Radix2EvaluationDomain
    logn = 28
    n = 1 << logn
    d = Radix2EvaluationDomain(n)
    x = _device_input(torch, n, SEED + logn)
    coeffs = x.cpu().numpy().view(np.uint64).copy()
    evals = _transform(torch, d, x, False)
    back = _transform(torch, d, x, True)
    d.close()
    del x
    torch.cuda.empty_cache()
    assert np.array_equal(back, coeffs)
    del back
    O.fft_np(coeffs)
    assert np.array_equal(evals, coeffs)


@pytest.mark.timeout(600)
def test_ntt_2_25_host_abi_and_coset():
    """2^25 through the reference C-ABI (host containers, fft / ifft with the
    degree-aware path for a short polynomial) and on the coset 5<w>, forward
    and inverse, plus transform_host (IcicleNTT::Run semantics) on the coset."""
    from tachyon_amd.ntt import Radix2EvaluationDomain
    logn = 25
    n = 1 << logn
    coeffs = O.gen_scalars("bn254_fr", 4000 + logn, n).tobytes()
    d = Radix2EvaluationDomain(n)
    ev = d.fft(coeffs)
    want = O.fft(coeffs, n)
    assert ev == want
    assert d.ifft(ev) == O.ifft(ev, n)
    short = coeffs[:32 * (n // 5)]
    assert d.fft(short) == O.fft(short, n)
    five = O.field_op("bn254_fr", "to_mont", (5).to_bytes(32, "little"))
    d.set_offset(five)
    evc = d.fft(coeffs)
    assert evc == O.fft(coeffs, n, five)
    assert d.ifft(evc) == O.ifft(evc, n, five)
    arr = np.frombuffer(coeffs, dtype=np.uint64).copy()
    d.transform_host(arr)
    assert arr.tobytes() == evc
    d.transform_host(arr, inverse=True)
    assert arr.tobytes() == coeffs
    d.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 8])
def test_four_step_2_25(world):
    """The distributed four-step plan at 2^25 (R = 2^12, C = 2^13) with
    `world` simulated ranks on one GPU: each rank's slab equals the oracle's
    FFT, and the inverse returns every rank's input."""
    _four_step_full(25, world, None)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [4, 8])
def test_four_step_2_24_split(world):
    """The bench's plan for 2^24 (split_log_r: R = 2^8, C = 2^16 -- packed
    one-pass column NTTs, the precomputed exchange twiddles, the
    transpose-free exchange layout) with `world` simulated ranks on one GPU:
    every slab equals the oracle's FFT, the inverse returns the input."""
    from tachyon_amd.ntt import FourStepNtt
    assert FourStepNtt.split_log_r(24, world) == 8
    _four_step_full(24, world, 8)


def _four_step_full(log_n, world, log_r):
    import torch
    from tachyon_amd.ntt import FourStepNtt
    n = 1 << log_n
    x = O.gen_scalars("bn254_fr", 5100 + log_n + world, n).reshape(n, 4)
    X = x.copy().reshape(-1)
    O.fft_np(X)
    X = X.reshape(n, 4)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    try:
        plans = [FourStepNtt(log_n, world, r, stream, log_r=log_r) for r in range(world)]
        chunk = (n // world // world) * 32

        def run(inputs, inverse):
            sends = [torch.empty_like(t) for t in inputs]
            for r in range(world):
                plans[r].run_stage(1, inverse, inputs[r], sends[r])
            recvs = [torch.cat([sends[h][r * chunk:(r + 1) * chunk] for h in range(world)]) for r in range(world)]
            outs = [torch.empty_like(t) for t in inputs]
            for r in range(world):
                plans[r].run_stage(2, inverse, recvs[r], outs[r])
            torch.cuda.synchronize()
            return outs

        ins = [torch.from_numpy(np.ascontiguousarray(x[FourStepNtt.input_indices(log_n, world, r, log_r)])
                                .view(np.uint8).reshape(-1)).cuda() for r in range(world)]
        outs = run(ins, False)
        for r in range(world):
            want = X[FourStepNtt.output_indices(log_n, world, r, log_r)].tobytes()
            assert outs[r].cpu().numpy().tobytes() == want, r
        back = run(outs, True)
        for r in range(world):
            assert torch.equal(back[r], ins[r]), r
        for p in plans:
            p.close()
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())


@pytest.mark.timeout(600)
def test_multi_device_domain_2_25_logical():
    """set_devices([0, 0, 0, 0]) at 2^25: the one-process four-step inside the
    domain (peer-copy all-to-all) equals the oracle, forward and inverse."""
    torch = pytest.importorskip("torch")
    from tachyon_amd.ntt import Radix2EvaluationDomain
    n = 1 << 25
    x = _device_input(torch, n, SEED + 125)
    coeffs = x.cpu().numpy().view(np.uint64).copy()
    d = Radix2EvaluationDomain(n)
    d.set_devices([0, 0, 0, 0])
    assert d.devices() == [0, 0, 0, 0]
    d.transform_device(x.data_ptr())
    torch.cuda.synchronize()
    evals = x.cpu().numpy().view(np.uint64).copy()
    d.transform_device(x.data_ptr(), inverse=True)
    torch.cuda.synchronize()
    back = x.cpu().numpy().view(np.uint64).copy()
    d.close()
    expect = coeffs.copy()
    O.fft_np(expect)
    assert np.array_equal(evals, expect)
    assert np.array_equal(back, coeffs)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("logn", [24, 26, 28])
def test_ntt_direct_evaluation_samples(logn):
    """Full-size transforms checked without the butterfly network: output i of
    the forward transform equals sum_j c_j w^(ij) (oracle_eval_at_powers, a
    blocked Horner over all n coefficients) at sampled indices, with w the
    pure-Python root of unity (oracle/pyref.py, the arkworks generator); the
    inverse returns the coefficients."""
    torch = pytest.importorskip("torch")
    from oracle import pyref
    from tachyon_amd.ntt import Radix2EvaluationDomain
    n = 1 << logn
    Fr = pyref.Field("bn254_fr")
    d = Radix2EvaluationDomain(n)
    w = Fr.to_bytes(Fr.root_of_unity(n))
    assert d.group_gen == w
    x = _device_input(torch, n, SEED + 100 + logn)
    coeffs = x.cpu().numpy().view(np.uint64).copy()
    evals = _transform(torch, d, x, False)
    back = _transform(torch, d, x, True)
    d.close()
    del x
    assert np.array_equal(back, coeffs)
    rng = np.random.default_rng(logn)
    idx = [0, 1, n - 1, n // 2, n // 3] + rng.integers(0, n, 3).tolist()
    ev = evals.view(np.uint8).reshape(n, 32)
    want = O.eval_at_powers(coeffs, w, idx)
    for q, i in enumerate(idx):
        assert ev[i].tobytes() == want[q], i
