"""Fixed-base folding (MsmGpu::fold_bases / run_folded, the C-ABI
tachyon_mi355x_msm_gpu_fold_bases / _folded_affine): an MSM over a table of
`fold` copies of the bases, copy k = 2^(k c W / fold) P, with W / fold window
sums.  The answer is the same group element as the plain MSM -- checked
bit-exact against the CPU oracle (and the unfolded GPU run) on every curve,
for every fold dividing W, with edge inputs (zero scalars, identity bases,
r - 1, a repeated scalar), and the refusals (a fold not dividing W, host
arrays)."""
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
CURVES = ["bn254_g1", "bn254_g2", "bls12_381_g1", "bls12_381_g2"]


def _dev(torch, b):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()


@pytest.mark.parametrize("curve", CURVES)
def test_msm_folded_vs_oracle(curve):
    torch = pytest.importorskip("torch")
    from tachyon_amd.msm import VariableBaseMSMGpu
    pb, sf = O.CURVE_INFO[curve]
    m = VariableBaseMSMGpu(curve)
    try:
        # c = 16: W = 16 for both scalar widths; c = 13: W = 20 (BN254) / 20 (BLS12-381)
        for n, c in [(1, 16), (300, 16), (1000, 13), (3000, 16)]:
            m.set_window_bits(c)
            W = m.plan_windows(n)
            bases = bytearray(O.gen_bases(curve, 71 + n, n, 64).tobytes())
            scalars = bytearray(O.gen_scalars(sf, 7100 + n, n).tobytes())
            if n > 2:
                bases[pb:2 * pb] = bytes(pb)  # an identity base
                scalars[:32] = bytes(32)  # a zero scalar
            if n > 10:
                r_minus_1 = O.field_op(sf, "neg", O.field_op(sf, "to_mont", (1).to_bytes(32, "little")))
                scalars[32 * 5:32 * 6] = r_minus_1
                scalars[32 * 6:32 * 9] = scalars[32 * 9:32 * 10] * 3  # a repeated scalar
            bases, scalars = bytes(bases), bytes(scalars)
            want = O.msm(curve, bases, scalars)[0]
            d_bases, d_scalars = _dev(torch, bases), _dev(torch, scalars)
            assert m.run(d_bases, d_scalars, n) == want
            for fold in [f for f in (1, 2, 4, 5, 8, 10, 16, 20) if W % f == 0]:
                d_tab = torch.empty(fold * n * pb, dtype=torch.uint8, device="cuda")
                m.fold_bases(d_bases, n, fold, d_tab)
                assert m.run_folded(d_tab, d_scalars, n, fold) == want, (n, c, fold)
        m.set_window_bits(16)
        n = 64
        d_bases = _dev(torch, O.gen_bases(curve, 5, n, 64).tobytes())
        d_scalars = _dev(torch, O.gen_scalars(sf, 55, n).tobytes())
        d_tab = torch.empty(16 * n * pb, dtype=torch.uint8, device="cuda")
        with pytest.raises(ValueError):
            m.fold_bases(d_bases, n, 3, d_tab)  # 3 does not divide W = 16
        with pytest.raises(ValueError):
            m.run_folded(d_tab, d_scalars, n, 3)
        with pytest.raises(ValueError):
            m.run_folded(0, d_scalars, n, 2)  # null table: not device memory
    finally:
        m.close()


def test_msm_folded_default_plan_2_16():
    """The size's default window bits (no forced c) at 2^16 points, BN254 G1
    and G2, folds 2 and 4 where they divide W; the plain MSM after a folded one
    is unaffected (the fold applies to run_folded only)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd.msm import VariableBaseMSMGpu
    n = 1 << 16
    for curve in ("bn254_g1", "bn254_g2"):
        pb, sf = O.CURVE_INFO[curve]
        bases = O.gen_bases(curve, 9, n, 1024).tobytes()
        scalars = O.gen_scalars(sf, 99, n).tobytes()
        want = O.msm(curve, bases, scalars)[0]
        m = VariableBaseMSMGpu(curve)
        try:
            W = m.plan_windows(n)
            d_bases, d_scalars = _dev(torch, bases), _dev(torch, scalars)
            for fold in [f for f in (2, 4) if W % f == 0]:
                d_tab = torch.empty(fold * n * pb, dtype=torch.uint8, device="cuda")
                m.fold_bases(d_bases, n, fold, d_tab)
                assert m.run_folded(d_tab, d_scalars, n, fold) == want, (curve, fold)
            assert m.run(d_bases, d_scalars, n) == want
        finally:
            m.close()


@pytest.mark.parametrize("variant", [4, 8, 12])
def test_msm_folded_under_pipelined_group_variants(variant):
    """set_variant bits 2-3 (pipelined window groups: group = 1 or 2 windows)
    are accepted for every MSM, but a folded run's recode writes its entries
    by scalar window, so the fold keeps one group of all key windows
    (run_windows forces G = W under a fold, as under a batch): the folded MSM
    still equals the oracle's, and so does the plain one under the variant."""
    torch = pytest.importorskip("torch")
    from tachyon_amd.msm import VariableBaseMSMGpu
    curve = "bn254_g1"
    pb, sf = O.CURVE_INFO[curve]
    n = 2000
    bases = O.gen_bases(curve, 404, n, 64).tobytes()
    scalars = O.gen_scalars(sf, 4040, n).tobytes()
    want = O.msm(curve, bases, scalars)[0]
    m = VariableBaseMSMGpu(curve)
    try:
        m.set_window_bits(16)  # W = 16
        m.set_variant(variant)
        d_bases, d_scalars = _dev(torch, bases), _dev(torch, scalars)
        assert m.run(d_bases, d_scalars, n) == want
        for fold in (2, 4, 8):
            d_tab = torch.empty(fold * n * pb, dtype=torch.uint8, device="cuda")
            m.fold_bases(d_bases, n, fold, d_tab)
            assert m.run_folded(d_tab, d_scalars, n, fold) == want, fold
    finally:
        m.close()
