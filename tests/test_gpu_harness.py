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
