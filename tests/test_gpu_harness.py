"""The benchmark/msm and benchmark/fft harnesses re-created on the C-ABI
(tachyon_amd/bin/{msm,fft}_benchmark_gpu; reference:
benchmark/msm/msm_benchmark_gpu.cc, benchmark/fft/fft_benchmark_gpu.cc):
they run with the reference's flags, pass --check_results and print the
reference's table plus one JSON line."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tachyon_amd", "bin")


def run(args):
    out = subprocess.run([os.path.join(BIN, args[0])] + args[1:], check=True, timeout=120, capture_output=True,
                         text=True).stdout
    return out, json.loads(out.strip().splitlines()[-1])


@pytest.mark.parametrize("flags", [[], ["--test_set", "non_uniform"], ["--device_resident"],
                                   ["--curve", "bls12_381"]])
def test_msm_benchmark_gpu(flags):
    out, res = run(["msm_benchmark_gpu", "-k", "12", "-k", "10", "--check_results"] + flags)
    assert "Degree (2^x)" in out
    assert res["check_results"] == "pass"
    assert [r["k"] for r in res["results"]] == [10, 12]


SEED = 0x7AC40001


@pytest.mark.parametrize("curve,ks,flags", [
    ("bn254", [10, 16], []),                          # 2^16 = BASELINE configs[0]'s size
    ("bn254", [12], ["--test_set", "non_uniform"]),
    ("bn254", [11], ["--device_resident"]),
    ("bls12_381", [10], []),
])
def test_msm_benchmark_gpu_vs_cpu_oracle(tmp_path, curve, ks, flags):
    """--check_results as the reference does it (msm_benchmark_gpu.cc:57-70):
    the GPU point of every size equals the CPU MSM (here the oracle's
    kParallelTerm Pippenger on the same inputs, timed beside it)."""
    import time
    from oracle import oracle as O
    g1 = f"{curve}_g1"
    pb, sf = O.CURVE_INFO[g1]
    n_max = 1 << max(ks)
    bases = O.gen_bases(g1, SEED, n_max, 1 << 10).tobytes()
    scalars = O.gen_scalars(sf, SEED, n_max).tobytes()
    if "non_uniform" in flags:
        scalars = scalars[:32] * n_max
    expect, cpu_s = b"", {}
    for k in sorted(ks):
        n = 1 << k
        t0 = time.perf_counter()
        expect += O.msm(g1, bases[:n * pb], scalars[:n * 32])[0]
        cpu_s[k] = time.perf_counter() - t0
    (tmp_path / "expect.bin").write_bytes(expect)
    args = ["msm_benchmark_gpu", "--check_results", "--expect", str(tmp_path / "expect.bin"), "--curve", curve]
    for k in ks:
        args += ["-k", str(k)]
    _, res = run(args + flags)
    assert res["check_results"] == "pass" and res["checked_against"] == "expect_file", res
    gpu_s = {r["k"]: r["seconds"] for r in res["results"]}
    print(json.dumps({"curve": g1, "flags": flags, "cpu_oracle_s": cpu_s, "gpu_s": gpu_s,
                      "cpu_threads": O.max_threads()}))
    # a wrong CPU point fails the check (exit 1, "FAIL")
    bad = bytearray(expect)
    bad[5] ^= 1
    (tmp_path / "bad.bin").write_bytes(bytes(bad))
    p = subprocess.run([os.path.join(BIN, args[0])] + args[1:3] + [str(tmp_path / "bad.bin")] + args[4:] + flags,
                       timeout=120, capture_output=True, text=True)
    assert p.returncode == 1 and json.loads(p.stdout.strip().splitlines()[-1])["check_results"] == "FAIL"


@pytest.mark.parametrize("ks,flags", [([10, 14], []), ([12], ["--run_ifft"]), ([13], ["--device_resident"]),
                                      ([11], ["--run_ifft", "--device_resident"])])
def test_fft_benchmark_gpu_vs_cpu_oracle(tmp_path, ks, flags):
    """--check_results as the reference does it (fft_benchmark_gpu.cc:81-83):
    the timed GPU transform equals the CPU transform of the same input."""
    from oracle import oracle as O
    expect = b""
    for k in sorted(ks):
        n = 1 << k
        x = O.gen_scalars("bn254_fr", SEED + k, n).tobytes()
        y = O.ifft(x, n) if "--run_ifft" in flags else O.fft(x, n)
        expect += y.ljust(32 * n, b"\0")
    (tmp_path / "expect.bin").write_bytes(expect)
    args = ["fft_benchmark_gpu", "--check_results", "--expect", str(tmp_path / "expect.bin")]
    for k in ks:
        args += ["-k", str(k)]
    _, res = run(args + flags)
    assert res["check_results"] == "pass" and res["checked_against"] == "expect_file", res


@pytest.mark.parametrize("flags", [[], ["--run_ifft"], ["--device_resident"]])
def test_fft_benchmark_gpu(flags):
    out, res = run(["fft_benchmark_gpu", "-k", "14", "-k", "10", "--check_results"] + flags)
    assert res["check_results"] == "pass"
    assert [r["k"] for r in res["results"]] == [10, 14]


REPLAY_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
from tachyon_amd.msm import VariableBaseMSMGpu
m = VariableBaseMSMGpu("bn254_g1")
for i, n in enumerate((300, 77)):
    m.run_jacobian(O.gen_bases("bn254_g1", 40 + i, n, 8).tobytes(), O.gen_scalars("bn254_fr", 40 + i, n).tobytes())
"""


def test_msm_dump_and_replay(tmp_path):
    """TACHYON_MSM_GPU_INPUT_DIR dumps (msm_gpu.h:99-119) replayed by
    bin/msm_gpu_replay (msm_gpu_replay.cc) give the oracle's MSM; the dump
    holds canonical limbs after a u64 count; TACHYON_LOG_MSM prints the result."""
    import sys
    from oracle import oracle as O
    from oracle import pyref
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TACHYON_MSM_GPU_INPUT_DIR=str(tmp_path), TACHYON_LOG_MSM="1")
    log = subprocess.run([sys.executable, "-c", REPLAY_CHILD, root], env=env, check=True, timeout=120,
                         capture_output=True, text=True).stdout
    G1 = pyref.Curve("bn254_g1")
    expect = []
    for i, n in enumerate((300, 77)):
        bases = O.gen_bases("bn254_g1", 40 + i, n, 8).tobytes()
        scalars = O.gen_scalars("bn254_fr", 40 + i, n).tobytes()
        dump = open(tmp_path / f"scalars{i}.txt", "rb").read()
        assert int.from_bytes(dump[:8], "little") == n
        assert dump[8:40] == G1.Fr.from_bytes(scalars[:32]).to_bytes(32, "little")
        pt = G1.from_bytes(O.msm("bn254_g1", bases, scalars)[0])
        expect.append(f"({hex(pt[0])}, {hex(pt[1])})")
        assert f"DoMSMGpu(){i}\n{expect[-1]}" in log
    out = subprocess.run([os.path.join(BIN, "msm_gpu_replay"), "--input_dir", str(tmp_path), "--degree", "9",
                          "--idx", "0", "--idx", "1"], check=True, timeout=120, capture_output=True, text=True,
                         env={k: v for k, v in os.environ.items() if k != "TACHYON_MSM_GPU_INPUT_DIR"}).stdout
    got = [l for l in out.splitlines() if l.startswith("(")]
    assert got == expect


@pytest.mark.parametrize("log_n", [1, 10, 16])
def test_ntt_holder_cpp_hook(tmp_path, log_n):
    """include/tachyon_mi355x_ntt_holder.h (the IcicleNTTHolder-shaped C++
    hook): in-place host FFT/IFFT, plain and on the coset 5<w>, from a C++
    client; its outputs equal the CPU oracle's transforms."""
    from oracle import oracle as O
    dump = tmp_path / "ntt.bin"
    _, res = run(["ntt_holder_check", str(log_n), "--dump", str(dump)])
    assert all(res[k] for k in ("fft_matches_capi", "round_trip", "coset_differs", "coset_round_trip")), res
    n = 1 << log_n
    raw = dump.read_bytes()
    inp, fft, coset = raw[:n * 32], raw[n * 32:2 * n * 32], raw[2 * n * 32:]
    five = O.field_op("bn254_fr", "to_mont", (5).to_bytes(32, "little"))
    assert fft == O.fft(inp, n)
    assert coset == O.fft(inp, n, five)


@pytest.mark.parametrize("log_n", [0, 8, 12])
def test_msm_cpp_plugin_boundary(log_n):
    """include/tachyon_mi355x_msm.h -- VariableBaseMSMGpu<Point>::Run
    (ProjectivePoint result; host vectors and device-resident bases) and
    VariableBaseMSM<Point>::Run (XYZZ bucket; containers and iterators) -- for
    the four groups from a C++ client: the results equal the CPU oracle's MSM
    of the same seeded inputs, mismatched sizes return false, an empty MSM is
    the XYZZ identity (1, 1, 0, 0)."""
    from oracle import oracle as O
    from oracle import pyref
    seed = 0x5EED + log_n
    out = subprocess.run([os.path.join(BIN, "msm_plugin_check"), str(log_n), str(seed)], timeout=300,
                         capture_output=True, text=True)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0, res
    n = 1 << log_n
    for gid, curve in enumerate(("bn254_g1", "bn254_g2", "bls12_381_g1", "bls12_381_g2")):
        g = res["groups"][str(gid)]
        assert g["ok"] and g["mismatch_false"], (curve, g)
        C = pyref.Curve(curve)
        cb = C.K.nbytes
        one, zero = C.K.to_bytes(C.K.const(1)), b"\0" * cb
        sf = O.CURVE_INFO[curve][1]
        want = O.msm(curve, O.gen_bases(curve, seed, n, 16).tobytes(), O.gen_scalars(sf, seed, n).tobytes())[0]
        proj, xyzz = bytes.fromhex(g["projective"]), bytes.fromhex(g["xyzz"])
        if want == b"\0" * (2 * cb):
            assert proj == one + one + zero and xyzz == one + one + zero + zero
        else:
            assert proj == want + one
            assert xyzz == want + one + one
        assert bytes.fromhex(g["empty_xyzz"]) == one + one + zero + zero
        # VariableBaseMSM<Projective / Jacobian / XYZZ bases> (the check requires
        # all three to equal this affine-input bucket): the oracle's MSM over the
        # same bases with every 37th point (i % 37 == 3) the identity
        assert g["non_affine_ok"], (curve, g)
        pb = 2 * cb
        bases = bytearray(O.gen_bases(curve, seed, n, 16).tobytes())
        for i in range(3, n, 37):
            bases[i * pb:(i + 1) * pb] = bytes(pb)
        want0 = O.msm(curve, bytes(bases), O.gen_scalars(sf, seed, n).tobytes())[0]
        z0 = bytes.fromhex(g["zeroed_xyzz"])
        assert z0 == (one + one + zero + zero if want0 == bytes(pb) else want0 + one + one), curve
