"""CPU-side checks of the product library: it was built for gfx950, loads
without a GPU, and exports every symbol include/tachyon_mi355x.h declares
(no compute calls here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tachyon_mi355x.h")
LIB = os.path.join(ROOT, "tachyon_amd", "libtachyon_mi355x.so")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"TACHYON_C_EXPORT[^;(]*?\b(tachyon_\w+)\s*\(", text, re.S)))


@pytest.fixture(scope="module")
def libpath():
    if not os.path.exists(LIB):
        pytest.skip("libtachyon_mi355x.so not built (run __graft_entry__.build())")
    return LIB


def test_header_declares_reference_abi():
    syms = declared_symbols()
    for s in ("tachyon_bn254_g1_create_msm_gpu", "tachyon_bn254_g1_affine_msm_gpu", "tachyon_bn254_g1_point2_msm_gpu",
              "tachyon_bn254_g1_destroy_msm_gpu", "tachyon_bn254_g1_affine_msm", "tachyon_bls12_381_g1_affine_msm_gpu",
              "tachyon_bn254_univariate_evaluation_domain_create", "tachyon_bn254_univariate_evaluation_domain_fft",
              "tachyon_bn254_univariate_evaluation_domain_ifft_inplace", "tachyon_bn254_univariate_evaluations_set_value"):
        assert s in syms


def test_library_exports_every_declared_symbol(libpath):
    out = subprocess.run(["nm", "-D", "--defined-only", libpath], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if " T " in line)
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_library_loads_and_binds_signatures(libpath):
    from tachyon_amd._lib import SIGNATURES, lib
    L = lib()
    names = {n for n, _, _ in SIGNATURES}
    assert set(declared_symbols()) == names
    assert b"gfx950" in L.tachyon_mi355x_version()


def test_code_object_targets_gfx950(libpath):
    # the fat binary carries one code object, for gfx950 only
    data = open(libpath, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx\w+)", data))
    assert targets == {b"gfx950"}, targets


def test_no_oracle_in_product():
    """The product path never imports / links the oracle."""
    bad = re.compile(r"^\s*(import\s+oracle|from\s+oracle)|#\s*include\s*[\"<][^\">]*oracle|liboracle", re.M)
    for dirpath, _, files in os.walk(os.path.join(ROOT, "tachyon_amd")):
        for f in files:
            if f.endswith((".py", ".h", ".hip", ".cc", "Makefile")) and f != "build.py":
                text = open(os.path.join(dirpath, f), errors="ignore").read()
                assert not bad.search(text), f
    out = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True).stdout if os.path.exists(LIB) else ""
    assert "oracle_" not in out


def test_ntt_holder_header_compiles(tmp_path):
    """include/tachyon_mi355x_ntt_holder.h (the IcicleNTTHolder-shaped C++ hook)
    is self-contained C++17 over the C-ABI header, usable with any 32-byte
    Montgomery element type (bn254::Fr in a Tachyon build)."""
    src = tmp_path / "use_holder.cc"
    src.write_text('#include "tachyon_mi355x_ntt_holder.h"\n'
                   "struct Fr { unsigned long long limbs[4]; };\n"
                   "bool f(std::vector<Fr>& v, const Fr* h) {\n"
                   "  auto holder = tachyon_mi355x::NTTHolder::Create(v.size());\n"
                   "  return holder->FFT(v, h) && holder->IFFT(v);\n}\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_circom_prover_device_list_parsing():
    """bin/circom_prover --devices: malformed lists (a non-numeric id, only
    separators) print the usage and exit 1 instead of an uncaught
    std::invalid_argument (no GPU work happens before the parse)."""
    import subprocess
    exe = os.path.join(ROOT, "tachyon_amd", "bin", "circom_prover")
    if not os.path.exists(exe):
        pytest.skip("circom_prover not built")
    for bad in ("0,x", ",", "", "1,-2"):
        r = subprocess.run([exe, "--zkey", "a", "--wtns", "b", "--proof", "c", "--public", "d", "--devices", bad],
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 1 and "usage:" in r.stderr + r.stdout, (bad, r.returncode, r.stderr)


def test_four_step_split_rule_on_the_host(libpath):
    """tachyon_mi355x_ntt4_split_log_r is host logic (no GPU call): the R x C
    split with the fewest pass launches (passes of <= 8 stages), R and C >=
    the world, ties to the larger R up to C -- the rule the bench's four-step
    leg, its projection and the multi-device domain follow."""
    from tachyon_amd._lib import lib

    def passes(k):
        return (k + 7) // 8

    for log_n in range(2, 29):
        for lg in range(0, 4):
            r = lib().tachyon_mi355x_ntt4_split_log_r(log_n, lg)
            if 2 * lg > log_n:
                assert r == log_n // 2  # no valid split: the default, which the plan then refuses
                continue
            c = log_n - r
            assert lg <= r <= c, (log_n, lg, r)
            best = min(passes(x) + passes(log_n - x) for x in range(max(1, lg), log_n) if lg <= log_n - x and x <= log_n - x)
            assert passes(r) + passes(c) == best, (log_n, lg, r)
    assert lib().tachyon_mi355x_ntt4_split_log_r(24, 3) == 8
