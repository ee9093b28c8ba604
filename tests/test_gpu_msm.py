"""GPU MSM parity through the C-ABI (the reference's variable_base_msm_gpu_unittest.cc,
msm_gpu_unittest.cc and msm_benchmark_gpu.cc --check_results): results must be
bit-exact (affine coordinates) against the CPU oracle on the same inputs."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CURVES = ["bn254_g1", "bn254_g2", "bls12_381_g1", "bls12_381_g2"]
_ctx = {}


def ctx(curve):
    from tachyon_amd.msm import VariableBaseMSMGpu
    if curve not in _ctx:
        _ctx[curve] = VariableBaseMSMGpu(curve)
    return _ctx[curve]


@pytest.mark.parametrize("curve", CURVES)
def test_msm_golden(curve):
    """Golden vectors of the independent Python restatement, incl. edge cases
    (zero scalars, identity bases, P + (-P), r-1) and the Easy KAT."""
    g = json.load(open(os.path.join(GOLDEN, "msm.json")))[curve]
    for c in g["cases"]:
        bases = b"".join(bytes.fromhex(x) for x in c["bases"])
        scalars = b"".join(bytes.fromhex(x) for x in c["scalars"])
        assert ctx(curve).run(bases, scalars).hex() == c["expected"], (c["n"], c.get("label"))


@pytest.mark.parametrize("variant", [4096, 8192, 8192 | 4096, 16384, 131072, 262144, 524288])
def test_msm_golden_bn254_g1_variants(variant):
    """The golden edge cases (zero scalars, identity bases, P + (-P), doubling
    inside a bucket, r - 1, Easy KAT) through the workgroup-tree window
    reduction (bit 12) and the 29-bit-limb accumulation (bit 13), plus a
    NonUniform set whose every bucket takes the doubling / cancellation paths."""
    from tachyon_amd.msm import VariableBaseMSMGpu
    g = json.load(open(os.path.join(GOLDEN, "msm.json")))["bn254_g1"]
    m = VariableBaseMSMGpu("bn254_g1")
    m.set_variant(variant)
    if variant == 524288:  # bit 19 (one-launch segment sums + tree) needs S = B / L <= 256: c = 10
        m.set_window_bits(10)
    for c in g["cases"]:
        bases = b"".join(bytes.fromhex(x) for x in c["bases"])
        scalars = b"".join(bytes.fromhex(x) for x in c["scalars"])
        assert m.run(bases, scalars).hex() == c["expected"], (c["n"], c.get("label"))
    # the same base repeated with equal scalars: every madd after the first is a doubling
    n = 600
    g1 = O.gen_bases("bn254_g1", 3, 1, 1).tobytes()
    s1 = O.gen_scalars("bn254_fr", 3, 1).tobytes()
    assert m.run(g1 * n, s1 * n) == O.msm("bn254_g1", g1 * n, s1 * n)[0]
    # P and -P alternating in one bucket: every other madd cancels to the identity
    neg = O.field_op("bn254_fq", "neg", g1[32:64])
    pm = (g1 + g1[:32] + neg) * (n // 2)
    assert m.run(pm, s1 * n) == bytes(64)
    m.close()


@pytest.mark.parametrize("curve,variant", [("bn254_g2", 0), ("bn254_g2", 32768), ("bn254_g2", 1 << 20),
                                           ("bn254_g2", 1 << 22), ("bls12_381_g2", 1 << 22),
                                           ("bls12_381_g2", 0),
                                           ("bls12_381_g2", 32768), ("bls12_381_g2", 65536 | (1 << 20)),
                                           ("bls12_381_g2", 1 << 20), ("bn254_g2", 1 << 23),
                                           ("bls12_381_g2", 1 << 23), ("bn254_g2", 1 << 24),
                                           ("bls12_381_g2", 1 << 24), ("bls12_381_g2", (1 << 24) | (1 << 22))])
def test_msm_golden_g2_lane_pair(curve, variant):
    """The G2 accumulations and reductions: a lane pair per point over the
    limb fields (the default: BN254 9 x 29-bit, BLS12-381 14 x 28-bit), the
    FIPS pair (bit 20), the FIPS pair reductions (bit 22), the two-level
    window sums instead of the per-segment fix-ups (bit 23, an A/B),
    the one-lane kernel (set_variant bit 15) and, for BLS12-381, the FIPS pair
    with out-of-line 12-limb products (bit 16) -- golden edge cases, a
    random set, a repeated base (doublings inside one bucket) and P, -P
    alternating (cancellations)."""
    from tachyon_amd.msm import VariableBaseMSMGpu
    g = json.load(open(os.path.join(GOLDEN, "msm.json")))[curve]
    m = VariableBaseMSMGpu(curve)
    m.set_variant(variant)
    for c in g["cases"]:
        bases = b"".join(bytes.fromhex(x) for x in c["bases"])
        scalars = b"".join(bytes.fromhex(x) for x in c["scalars"])
        assert m.run(bases, scalars).hex() == c["expected"], (c["n"], c.get("label"))
    pb, sf = O.CURVE_INFO[curve]
    n = 3001
    bases = O.gen_bases(curve, 17, n, 40).tobytes()
    scalars = O.gen_scalars(sf, 17, n).tobytes()
    assert m.run(bases, scalars) == O.msm(curve, bases, scalars)[0]
    g1, s1 = bases[:pb], scalars[:32]
    assert m.run(g1 * 300, s1 * 300) == O.msm(curve, g1 * 300, s1 * 300)[0]
    fq = "bn254_fq" if curve.startswith("bn254") else "bls12_381_fq"
    half = pb // 4  # one Fq
    ny = O.field_op(fq, "neg", g1[2 * half:])  # -y, component-wise
    pm = (g1 + g1[:2 * half] + ny) * 150
    assert m.run(pm, s1 * 300) == bytes(pb)
    m.close()


def test_msm_zkey_points():
    z = json.load(open(os.path.join(GOLDEN, "zkey_multiplier_3.json")))
    for key, curve in (("g1", "bn254_g1"), ("g2", "bn254_g2")):
        bases = b"".join(bytes.fromhex(x) for x in z[f"{key}_points"])
        scalars = b"".join(bytes.fromhex(x) for x in z[f"msm_{key}"]["scalars"])
        assert ctx(curve).run(bases, scalars).hex() == z[f"msm_{key}"]["expected"]


def test_reference_entry_points_bn254():
    """tachyon_bn254_g1_{affine,point2}_msm{,_gpu}: Jacobian result, caller-owned."""
    import ctypes
    from tachyon_amd._lib import lib
    L = lib()
    for n in (32, 2, 5):  # sizes of msm_gpu_unittest.cc:13-66
        bases = O.gen_bases("bn254_g1", 100 + n, n, 3).tobytes()
        scalars = O.gen_scalars("bn254_fr", 100 + n, n).tobytes()
        expect, _ = O.msm("bn254_g1", bases, scalars, method="naive")
        for create, run, destroy in (("tachyon_bn254_g1_create_msm_gpu", "tachyon_bn254_g1_affine_msm_gpu",
                                      "tachyon_bn254_g1_destroy_msm_gpu"),
                                     ("tachyon_bn254_g1_create_msm_gpu", "tachyon_bn254_g1_point2_msm_gpu",
                                      "tachyon_bn254_g1_destroy_msm_gpu"),
                                     ("tachyon_bn254_g1_create_msm", "tachyon_bn254_g1_affine_msm",
                                      "tachyon_bn254_g1_destroy_msm")):
            c = getattr(L, create)(0)
            p = getattr(L, run)(c, bases, scalars, n)
            jac = ctypes.string_at(p, 96)
            L.tachyon_mi355x_jacobian_destroy(0, p)
            getattr(L, destroy)(c)
            from tachyon_amd.msm import jacobian_to_affine
            assert jacobian_to_affine("bn254_g1", jac) == expect, (n, run)


@pytest.mark.parametrize("logn", [10, 13, 16])
def test_msm_random_bn254_vs_oracle(logn):
    n = 1 << logn
    bases = O.gen_bases("bn254_g1", logn, n, 64).tobytes()
    scalars = O.gen_scalars("bn254_fr", logn, n).tobytes()
    expect, _ = O.msm("bn254_g1", bases, scalars)
    assert ctx("bn254_g1").run(bases, scalars) == expect


@pytest.mark.parametrize("curve", ["bn254_g2", "bls12_381_g1", "bls12_381_g2"])
def test_msm_random_other_curves_vs_oracle(curve):
    n = 1 << 10  # variable_base_msm_gpu_unittest.cc:25-78 uses 2^10 on all four groups
    bases = O.gen_bases(curve, 77, n, 32).tobytes()
    scalars = O.gen_scalars(O.CURVE_INFO[curve][1], 77, n).tobytes()
    expect, _ = O.msm(curve, bases, scalars)
    assert ctx(curve).run(bases, scalars) == expect


def test_msm_non_uniform_all_equal_scalars():
    """benchmark --test_set non_uniform = NonUniform(n, 1): every scalar equal, so
    every window puts all n points in ONE bucket (the skew path)."""
    n = 1 << 14
    bases = O.gen_bases("bn254_g1", 9, n, 64).tobytes()
    one = O.gen_scalars("bn254_fr", 9, 1).tobytes()
    scalars = one * n
    expect, _ = O.msm("bn254_g1", bases, scalars)
    assert ctx("bn254_g1").run(bases, scalars) == expect


@pytest.mark.parametrize("logn", [14, 17, 19])
@pytest.mark.parametrize("kind", ["random", "non_uniform", "three_scalars"])
def test_msm_chain_table_modes(logn, kind):
    """The bucket chains' tables are built from the sorted keys before the
    accumulation (2^14 / 2^17: with every join level's offsets from the
    device-side counts; 2^19: tables only) or from the accumulation's flags
    after it (set_variant bit 2: one window per sort group).  Random scalars
    (short chains), NonUniform(n, 1) (one bucket per window: the longest
    chains, the most 4-ary levels) and three repeated scalars (a few long
    chains among short ones) agree with the oracle in both schedules."""
    n = 1 << logn
    bases = O.gen_bases("bn254_g1", 40 + logn, n, 64).tobytes()
    if kind == "random":
        scalars = O.gen_scalars("bn254_fr", 40 + logn, n).tobytes()
    elif kind == "non_uniform":
        scalars = O.gen_scalars("bn254_fr", 40 + logn, 1).tobytes() * n
    else:
        three = O.gen_scalars("bn254_fr", 40 + logn, 3).tobytes()
        scalars = b"".join(three[32 * (i % 3):32 * (i % 3) + 32] for i in range(n))
    expect, _ = O.msm("bn254_g1", bases, scalars)
    m = ctx("bn254_g1")
    try:
        for var in (0, 4):
            m.set_variant(var)
            assert m.run(bases, scalars) == expect, (logn, kind, var)
    finally:
        m.set_variant(0)


def test_msm_window_sizes_agree():
    """Any window size gives the same point (MSMCtx only changes the schedule)."""
    n = 3000
    bases = O.gen_bases("bn254_g1", 4, n, 10).tobytes()
    scalars = O.gen_scalars("bn254_fr", 4, n).tobytes()
    expect, _ = O.msm("bn254_g1", bases, scalars)
    m = ctx("bn254_g1")
    try:
        for var in (0, 4096, 8192, 131072):  # fix-up / workgroup-tree reduction / 29-bit accumulation (+ LDS-DMA)
            m.set_variant(var)
            for c in (4, 7, 11, 16, 21):
                m.set_window_bits(c)
                assert m.run(bases, scalars) == expect, (c, var)
    finally:
        m.set_window_bits(0)
        m.set_variant(0)


def test_msm_empty_and_single():
    m = ctx("bn254_g1")
    assert m.run(b"", b"", n=0) == b"\x00" * 64
    b1 = O.gen_bases("bn254_g1", 1, 1, 1).tobytes()
    s1 = O.gen_scalars("bn254_fr", 1, 1).tobytes()
    assert m.run(b1, s1) == O.msm("bn254_g1", b1, s1)[0]


def test_device_generator_matches_oracle():
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    for curve in CURVES:
        pb, sf = O.CURVE_INFO[curve]
        n, chunk = 300, 7
        d_b = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
        d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        M.gen_bases(curve, 31, n, chunk, d_b.data_ptr())
        M.gen_scalars(sf, 31, n, d_s.data_ptr())
        torch.cuda.synchronize()
        assert d_b.cpu().numpy().tobytes() == O.gen_bases(curve, 31, n, chunk).tobytes(), curve
        assert d_s.cpu().numpy().tobytes() == O.gen_scalars(sf, 31, n).tobytes(), curve
        # a shard [start, start + m) of the same sequence (bench.py's per-rank inputs)
        start, m = 14 * chunk, 100
        d_p = torch.empty(m * pb, dtype=torch.uint8, device="cuda")
        d_q = torch.empty(m * 32, dtype=torch.uint8, device="cuda")
        M.gen_bases(curve, 31, m, chunk, d_p.data_ptr(), start=start)
        M.gen_scalars(sf, 31, m, d_q.data_ptr(), start=start)
        torch.cuda.synchronize()
        assert d_p.cpu().numpy().tobytes() == d_b.cpu().numpy().tobytes()[start * pb:(start + m) * pb], curve
        assert d_q.cpu().numpy().tobytes() == d_s.cpu().numpy().tobytes()[start * 32:(start + m) * 32], curve


def test_device_resident_inputs_and_shard_sum():
    """Device pointers are used in place; MSM(A||B) == MSM(A) + MSM(B) (the
    kParallelTerm / multi-GPU sharding contract, pippenger_adapter_unittest.cc)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = 1 << 18
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", 5, n, 256, d_b.data_ptr())
    M.gen_scalars("bn254_fr", 5, n, d_s.data_ptr())
    torch.cuda.synchronize()
    m = ctx("bn254_g1")
    whole = m.run(d_b, d_s)
    h = n // 2
    a = m.run(d_b[:h * 64], d_s[:h * 32])
    b = m.run(d_b[h * 64:], d_s[h * 32:])
    assert M.affine_sum("bn254_g1", a + b) == whole
    hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
    assert O.msm_np("bn254_g1", hb, hs) == whole


@pytest.mark.parametrize("chunks,mixed", [(3, None), (8, "bases"), (5, "scalars")])
def test_host_pipelined_upload(chunks, mixed, monkeypatch):
    """Host-resident inputs run as chunked MSMs overlapping the per-chunk
    uploads (MsmGpu::run_host_pipelined); the sum must equal the one-shot
    device-resident MSM -- also with only one operand on the host and an
    uneven split (TACHYON_MSM_HOST_CHUNKS forces the chunking at 2^18)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = (1 << 18) + 77
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", 8, n, 512, d_b.data_ptr())
    M.gen_scalars("bn254_fr", 8, n, d_s.data_ptr())
    torch.cuda.synchronize()
    m = ctx("bn254_g1")
    whole = m.run(d_b, d_s)
    hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
    monkeypatch.setenv("TACHYON_MSM_HOST_CHUNKS", str(chunks))
    b = d_b if mixed == "scalars" else hb
    s = d_s if mixed == "bases" else hs
    assert m.run(b, s) == whole
    monkeypatch.setenv("TACHYON_MSM_HOST_CHUNKS", "1")
    assert m.run(hb, hs) == whole


def test_memory_divisions(monkeypatch):
    """DetermineMsmDivisionsForMemory (icicle_msm_utils.cc:10-68): with the free
    device memory capped below the working set of one MSM, the run is split
    into point chunks whose sum equals the undivided result (device- and
    host-resident inputs)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = 1 << 19
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", 12, n, 512, d_b.data_ptr())
    M.gen_scalars("bn254_fr", 12, n, d_s.data_ptr())
    torch.cuda.synchronize()
    from tachyon_amd.msm import VariableBaseMSMGpu
    m = VariableBaseMSMGpu("bn254_g1")  # fresh context: no buffers held yet
    whole = ctx("bn254_g1").run(d_b, d_s)
    # the 2^19 working set is a few hundred MB (MsmGpu::work_bytes); the caps
    # step down until the run is divided (200 MB still fits 2^16-point chunks)
    divided = 0
    for limit_mb in (600, 400, 200):
        monkeypatch.setenv("TACHYON_MSM_MEM_LIMIT", str(limit_mb << 20))
        assert m.run(d_b, d_s) == whole, limit_mb
        divided = max(divided, m.last_divisions())
    assert divided >= 2
    monkeypatch.setenv("TACHYON_MSM_HOST_CHUNKS", "1")
    monkeypatch.setenv("TACHYON_MSM_MEM_LIMIT", str(200 << 20))
    assert m.run(d_b.cpu().numpy(), d_s.cpu().numpy()) == whole
    assert m.last_divisions() >= 2
    # a window-range MSM divides the same way (its chunks keep the whole input's
    # window bits): the ranges of a 2-way window split still add up to the MSM
    from tachyon_amd import dist as D
    c, W = M.plan("bn254_g1", n)
    parts = []
    for w0, w1 in (D.window_range(W, 0, 2), D.window_range(W, 1, 2)):
        parts.append(m.run_window_range(d_b, d_s, w0, w1))
        assert m.last_divisions() >= 2
    assert M.affine_sum("bn254_g1", b"".join(parts)) == whole
    parts = [m.run_window_range(d_b.cpu().numpy(), d_s.cpu().numpy(), w0, w1)
             for w0, w1 in (D.window_range(W, 0, 2), D.window_range(W, 1, 2))]
    assert M.affine_sum("bn254_g1", b"".join(parts)) == whole
    m.close()


@pytest.mark.parametrize("curve", ["bn254_g1", "bn254_g2", "bls12_381_g1"])
def test_window_ranges_tile_the_msm(curve):
    """run_window_range: the partials of window ranges that tile [0, W) add up
    to the MSM (pippenger_base.h:59-77 split by windows); empty and
    out-of-range ranges are the identity; one range covering everything is
    the MSM itself."""
    from tachyon_amd import dist as D
    from tachyon_amd import msm as M
    from tachyon_amd.msm import VariableBaseMSMGpu
    n = 2500
    pb, sf = O.CURVE_INFO[curve]
    bases = O.gen_bases(curve, 9, n, 64).tobytes()
    scalars = O.gen_scalars(sf, 9, n).tobytes()
    want, _ = O.msm(curve, bases, scalars)
    m = VariableBaseMSMGpu(curve)
    for c in (7, 16):
        m.set_window_bits(c)
        W = D._windows_for(curve, c)
        assert m.run_window_range(bases, scalars, 0, W) == want
        assert m.run_window_range(bases, scalars, 0, 10 ** 6) == want
        assert m.run_window_range(bases, scalars, 3, 3) == bytes(pb)
        assert m.run_window_range(bases, scalars, W, W + 4) == bytes(pb)
        for parts in (2, 3, 8):
            ranges = [D.window_range(W, r, parts) for r in range(parts)]
            got = [m.run_window_range(bases, scalars, w0, w1) for w0, w1 in ranges]
            assert M.affine_sum(curve, b"".join(got)) == want, (c, parts)
        assert m.run(bases, scalars) == want  # the range is per call
    m.close()


@pytest.mark.parametrize("curve,logn", [("bn254_g1", 16), ("bn254_g1", 18), ("bls12_381_g1", 16), ("bls12_381_g2", 16)])
def test_msm_schedule_variants_agree(curve, logn):
    """Every accepted set_variant schedule computes the same point: the separate
    recode + full sort (bit 7), rocPRIM's own digit-histogram pass instead of the
    recode's counts (bit 10), 8-byte LDS staging in the recode scatter (bit 11),
    the onesweep tile shapes (bits 4-5) and one window per sort group (bits 2-3);
    the wrong-result bit 6 and bits above 11 are refused.  At 2^16 (one onesweep
    place after the fused low byte) and 2^18 (two places) the default schedule is
    the fused recode feeding the onesweep passes its digit counts, so bits 10
    and 11 really switch schedules -- asserted through last_schedule()."""
    n = 1 << logn
    bases = O.gen_bases(curve, 21, n, 16).tobytes()
    scalars = O.gen_scalars(O.CURVE_INFO[curve][1], 21, n).tobytes()
    expect, _ = O.msm(curve, bases, scalars)
    m = ctx(curve)
    want = {0: (True, True, True), 128: (False, False, False), 1024: (True, False, True),
            2048: (True, True, False), 1024 | 2048: (True, False, False)}
    try:
        for v in (0, 128, 1024, 2048, 1024 | 2048, 16, 32, 48, 4, 256, 4096, 4096 | 128, 8192, 8192 | 4096, 16384,
                  32768, 65536, 131072, 262144, 524288, 1 << 20, (1 << 20) | 65536, 1 << 21, 1 << 22, 1 << 25):
            m.set_variant(v)
            assert m.run(bases, scalars) == expect, hex(v)
            if v in want:
                s = m.last_schedule()
                assert (s["fused_recode"], s["recode_fed_sort"], s["narrow_staging"]) == want[v], (hex(v), s)
            s = m.last_schedule()
            if curve == "bn254_g1":  # the 29-bit field by default; bit 18 the FIPS 32-bit field
                assert s["acc29"] == (v != 262144), (hex(v), s)
                # its entries LDS-staged unless bit 25 (or a base-prefetch mode, bits 13 / 17)
                assert s["entries_staged"] == (s["acc29"] and v not in (1 << 25, 8192, 8192 | 4096, 131072)), (hex(v), s)
            elif curve == "bls12_381_g1":  # the 28-bit field by default; bit 20 the FIPS 32-bit field
                assert s["acc28"] == (not v & (1 << 20)), (hex(v), s)
                assert s["entries_staged"] == (s["acc28"] and v != 1 << 25), (hex(v), s)
            else:  # G2: the lane pair by default; bit 15 the one-lane kernel
                assert s["lane_pair"] == (v != 32768), (hex(v), s)
                limb = v != 32768 and not v & (1 << 20)
                # staged entries for the BLS12-381 pair (BN254 G2 measured faster without)
                assert s["entries_staged"] == (limb and v != 1 << 25 and curve == "bls12_381_g2"), (hex(v), s)
                if curve == "bls12_381_g2":  # the pair over 28-bit limbs; bit 20 the FIPS pair
                    assert s["acc28"] == limb, (hex(v), s)
                else:  # BN254 G2: the pair over 29-bit limbs; bit 20 the FIPS pair
                    assert s["acc29"] == limb, (hex(v), s)
        for bad in (64, 1 << 26):
            with pytest.raises(ValueError):
                m.set_variant(bad)
    finally:
        m.set_variant(0)


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["bn254_g1", "bls12_381_g1", "bn254_g2", "bls12_381_g2"])
def test_msm_entry_reads_odd_sizes(curve):
    """The limb-field accumulations' ways of reading the sorted entries
    (seg_acc_limb_body's kEnt; the G2 lane pairs' kStaged) on sizes that
    stress their edges: odd n (a lane's
    last LDS-staged chunk runs past the entry array's end into its slack; the
    last 16-byte pair is cut at gend), one window per sort group (variant 4:
    groups start at odd entries when n is odd, so the 16-byte pairs take over
    from the staged chunks), accumulation chunks K / 2 and 2 K (variants 3, 1),
    and bit 25 (8-byte loads).  Every schedule equals the oracle."""
    from tachyon_amd import msm as M
    m = ctx(curve)
    try:
        for n in (1, 7, 4097, 12289):
            bases = O.gen_bases(curve, 23, n, 16).tobytes()
            scalars = O.gen_scalars(O.CURVE_INFO[curve][1], 23 + n, n).tobytes()
            expect, _ = O.msm(curve, bases, scalars)
            for v in (0, 4, 3, 1, 4 | 3, 1 << 25, (1 << 25) | 4):
                m.set_variant(v)
                assert m.run(bases, scalars) == expect, (n, hex(v))
    finally:
        m.set_variant(0)


@pytest.mark.gpu
@pytest.mark.parametrize("curve,n", [("bn254_g1", 300000), ("bls12_381_g1", 300000)])
def test_msm_entry_pairs_odd_chunk(curve, n):
    """The plan rounds the accumulation chunk K up to even (here 38 / 42), so
    every lane's first entry is 16-byte aligned and the entries are
    LDS-staged; set_variant bit 0-1 = 3 halves K to an odd 19 / 21, where the
    lanes' alignment alternates and the accumulation reads 16-byte pairs
    (kEnt 1, the pair shift taken per lane); bit 25 the 8-byte loads. All
    three equal the oracle."""
    bases = O.gen_bases(curve, 29, n, 64).tobytes()
    scalars = O.gen_scalars(O.CURVE_INFO[curve][1], 29, n).tobytes()
    expect, _ = O.msm(curve, bases, scalars)
    m = ctx(curve)
    try:
        assert m.run(bases, scalars) == expect
        assert m.last_schedule()["entries_staged"]
        m.set_variant(3)
        assert m.run(bases, scalars) == expect
        assert not m.last_schedule()["entries_staged"]
        m.set_variant(1 << 25)
        assert m.run(bases, scalars) == expect
    finally:
        m.set_variant(0)


@pytest.mark.gpu
def test_madd_ceiling():
    """The bench's VALU ceiling (tachyon_mi355x_msm_madd_ceiling): a positive
    rate for BN254 G1's two field widths, 0 where not provided."""
    from tachyon_amd import msm as M
    g1 = M.VariableBaseMSMGpu("bn254_g1")
    r29, r32 = g1.madd_ceiling(29), g1.madd_ceiling(32)
    assert 1.0 < r29 < 200.0 and 1.0 < r32 < 200.0, (r29, r32)
    assert g1.madd_ceiling(31) == 0.0
    # BLS12-381 G1's 28-bit field and the G2 lane pairs (whole G2 additions): slower than G1's
    bls = M.VariableBaseMSMGpu("bls12_381_g1").madd_ceiling(28)
    g2 = M.VariableBaseMSMGpu("bn254_g2").madd_ceiling(29)
    bls2 = M.VariableBaseMSMGpu("bls12_381_g2").madd_ceiling(28)
    assert 0.5 < bls2 < g2 < r29 and 0.5 < bls2 < bls < r29, (r29, bls, g2, bls2)
    assert M.VariableBaseMSMGpu("bn254_g2").madd_ceiling(28) == 0.0


def _neg_point(curve, p: bytes) -> bytes:
    """-P of an affine point (y -> -y componentwise in the base field)."""
    fq = "bn254_fq" if curve.startswith("bn254") else "bls12_381_fq"
    half = len(p) // 2
    return p[:half] + O.field_op(fq, "neg", p[half:])


@pytest.mark.gpu
@pytest.mark.parametrize("curve,variant", [("bn254_g1", 0), ("bn254_g1", 262144), ("bn254_g2", 0),
                                           ("bn254_g2", 1 << 22), ("bls12_381_g1", 0), ("bls12_381_g1", 1 << 22),
                                           ("bls12_381_g2", 0), ("bls12_381_g2", 1 << 22),
                                           ("bls12_381_g2", 32768), ("bls12_381_g1", 1 << 23),
                                           ("bls12_381_g2", 1 << 23), ("bn254_g2", 1 << 23),
                                           ("bn254_g1", 262144 | (1 << 23)), ("bn254_g2", 1 << 24),
                                           ("bls12_381_g2", 1 << 24)])
def test_msm_reduction_edge_cases(curve, variant):
    """Inputs that drive the chain join and the window sums through their
    special cases: every base the same point (equal bucket pieces and equal
    running sums -> the doubling branch of the reduction additions), bases
    alternating P, -P under one repeated scalar (pieces and bucket sums that
    cancel -> the identity branch), and one repeated base and scalar.
    Default schedule (29-bit reductions on BN254 G1, 28-bit on BLS12-381 G1,
    limb-field lane-pair reductions on G2) and the FIPS / FIPS-pair /
    one-lane ones (bits 18 / 22 / 15)."""
    pb, fr = O.CURVE_INFO[curve]
    n = 1 << 13
    g = O.gen_bases(curve, 31, 1, 1).tobytes()
    m = ctx(curve)
    m.set_variant(variant)
    try:
        same = g * n
        scalars = O.gen_scalars(fr, 31, n).tobytes()
        assert m.run(same, scalars) == O.msm(curve, same, scalars)[0]
        alt = (g + _neg_point(curve, g)) * (n // 2)
        one = O.gen_scalars(fr, 32, 1).tobytes() * n
        expect = O.msm(curve, alt, one)[0]
        assert expect == bytes(pb)  # the identity, (0, 0)
        assert m.run(alt, one) == expect
        assert m.run(same, one) == O.msm(curve, same, one)[0]
    finally:
        m.set_variant(0)


@pytest.mark.parametrize("curve", ["bn254_g1", "bls12_381_g1", "bn254_g2"])
@pytest.mark.parametrize("logn", [14, 16, 17, 19])
def test_chain_flags_pre_derived_match(curve, logn):
    """below 2^21 accumulation threads the chain tables are built
    from chain_flags_kernel's re-derivation of the run flags, not from the
    flags the accumulation writes.  set_variant bit 21 compares the two on the
    device after every accumulation (the run aborts on a mismatch): random,
    NonUniform (one scalar) and digit-0-heavy (small) scalars, all equal to the
    oracle."""
    n = 1 << logn
    pb, sf = O.CURVE_INFO[curve]
    bases = O.gen_bases(curve, 51, n, 64).tobytes()
    sets = {"random": O.gen_scalars(sf, 51, n).tobytes(),
            "non_uniform": O.gen_scalars(sf, 52, 1).tobytes() * n,
            "small": b"".join(O.field_op(sf, "to_mont", (i % 5).to_bytes(32, "little")) for i in range(64)) * (n // 64)}
    m = ctx(curve)
    m.set_variant(1 << 21)
    try:
        for name, sc in sets.items():
            if logn > 16 and name == "small":
                continue  # (the 64-scalar pattern is the same test at every size)
            assert m.run(bases, sc) == O.msm(curve, bases, sc)[0], name
            assert m.last_schedule()["chains_checked"], name
    finally:
        m.set_variant(0)


@pytest.mark.parametrize("curve,length,count", [("bn254_g1", 1, 3), ("bn254_g1", 100, 5), ("bn254_g1", 3001, 17),
                                                ("bn254_g1", 1 << 14, 6), ("bn254_g1", 64, 70), ("bn254_g2", 500, 4),
                                                ("bls12_381_g1", 777, 5), ("bls12_381_g2", 300, 3)])
def test_msm_batch_vs_oracle(curve, length, count):
    """tachyon_mi355x_msm_gpu_batch_affine: `count` MSMs over the same device
    bases in one launch sequence (a block of windows per MSM) -- every result
    equal to the oracle's MSM of its scalar vector; ragged vectors (zero
    padding), an all-zero vector, a NonUniform (one repeated scalar) vector,
    host and device scalars."""
    torch = pytest.importorskip("torch")
    from tachyon_amd.msm import VariableBaseMSMGpu
    pb, sf = O.CURVE_INFO[curve]
    bases = O.gen_bases(curve, 61, length, 64).tobytes()
    d_bases = torch.frombuffer(bytearray(bases), dtype=torch.uint8).cuda()
    vecs = []
    for g in range(count):
        v = O.gen_scalars(sf, 6100 + g, length).tobytes()
        if g % 3 == 1:  # ragged: the tail zero
            keep = max(1, length * (g + 1) // (count + 1))
            v = v[:32 * keep] + bytes(32 * (length - keep))
        if g == 2:
            v = bytes(32 * length)
        if g == 3:
            v = O.gen_scalars(sf, 6200, 1).tobytes() * length
        vecs.append(v)
    scalars = b"".join(vecs)
    m = VariableBaseMSMGpu(curve)
    try:
        got = m.run_batch(d_bases, scalars, length, count)
        want = [O.msm(curve, bases, v)[0] for v in vecs]
        assert got == want
        d_scalars = torch.frombuffer(bytearray(scalars), dtype=torch.uint8).cuda()
        torch.cuda.synchronize()
        assert m.run_batch(d_bases, d_scalars, length, count) == want
        with pytest.raises(ValueError):
            m.run_batch(0, scalars, length, count)  # null bases: not device memory
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("c", [5, 9, 12])
def test_msm_batch_forced_window_bits(c):
    """run_batch under set_window_bits: the forced c is used (any c gives the
    same sums) and survives the batch -- the single MSM after it, and a second
    batch, still match the oracle."""
    torch = pytest.importorskip("torch")
    from tachyon_amd.msm import VariableBaseMSMGpu
    curve, length, count = "bn254_g1", 700, 9
    pb, sf = O.CURVE_INFO[curve]
    bases = O.gen_bases(curve, 71, length, 64).tobytes()
    d_bases = torch.frombuffer(bytearray(bases), dtype=torch.uint8).cuda()
    vecs = [O.gen_scalars(sf, 7100 + g, length).tobytes() for g in range(count)]
    want = [O.msm(curve, bases, v)[0] for v in vecs]
    m = VariableBaseMSMGpu(curve)
    try:
        m.set_window_bits(c)
        assert m.run_batch(d_bases, b"".join(vecs), length, count) == want
        assert m.run(bases, vecs[4]) == want[4]
        m.set_window_bits(0)
        assert m.run_batch(d_bases, b"".join(vecs), length, count) == want
        assert m.run(bases, vecs[7]) == want[7]
    finally:
        m.close()
