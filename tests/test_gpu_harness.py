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
