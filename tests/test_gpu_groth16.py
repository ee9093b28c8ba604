"""GPU Groth16 parity through the C-ABI: the prover's
witness map and proofs must equal the CPU oracle's (oracle/groth16.py) bit for
bit, on the reference's multiplier_3 fixtures (where the proof must also pass
the pairing check) and on synthetic proving keys (BN254 and BLS12-381, ragged
rows, empty rows, identity query points, zero witnesses, NoZK and ZK)."""
import json
import os

import pytest

from oracle import bn254_pairing as BP
from oracle import circom_format as CF
from oracle import groth16 as OG
from oracle import pyref
from tachyon_amd import params as P

from groth16_synth import synth_zkey

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def fr_bytes(curve, vals):
    Fr = pyref.Field("bn254_fr" if curve == "bn254" else "bls12_381_fr")
    return b"".join(Fr.to_bytes(v) for v in vals)


def test_multiplier_3_matches_golden_and_verifies():
    from tachyon_amd.groth16 import Groth16Prover, wtns_parse
    zbytes = open(os.path.join(GOLDEN, "multiplier_3.zkey"), "rb").read()
    wbytes = open(os.path.join(GOLDEN, "multiplier_3.wtns"), "rb").read()
    zk = CF.parse_zkey(zbytes)
    w = CF.parse_wtns(wbytes, P.BN254_FR)
    full = wtns_parse(wbytes, "bn254")
    assert full == fr_bytes("bn254", w)
    g = json.load(open(os.path.join(GOLDEN, "groth16_multiplier_3.json")))
    prover = Groth16Prover(zbytes)
    assert (prover.num_vars, prover.num_public, prover.domain_size) == (6, 1, 4)
    h = prover.witness_map(full)
    assert [h[i * 32:(i + 1) * 32].hex() for i in range(4)] == g["h_evals"]
    G1, G2 = pyref.Curve("bn254_g1"), pyref.Curve("bn254_g2")
    vk = {k: (G2 if k.endswith("g2") else G1).from_bytes(v) for k, v in zk["vk"].items()}
    ic = [G1.from_bytes(b) for b in zk["ic"]]
    Fr = G1.Fr
    for case in g["cases"]:
        r, s = int(case["r"]), int(case["s"])
        proof = prover.prove(full) if case["label"] == "nozk" else prover.prove(full, Fr.to_bytes(r), Fr.to_bytes(s))
        assert [x.hex() for x in proof] == case["proof"], case["label"]
        A, B, C = proof
        assert BP.groth16_verify(vk, ic, w[1:2], (G1.from_bytes(A), G2.from_bytes(B), G1.from_bytes(C)))
    prover.close()


@pytest.mark.parametrize("curve,log_n,num_public,seed", [
    ("bn254", 3, 1, 1), ("bn254", 6, 2, 2), ("bn254", 9, 0, 3), ("bn254", 11, 5, 4),
    ("bls12_381", 5, 1, 5), ("bls12_381", 8, 3, 6),
])
def test_synthetic_parity(curve, log_n, num_public, seed):
    from tachyon_amd.groth16 import Groth16Prover
    zbytes, full = synth_zkey(curve, log_n=log_n, num_public=num_public, seed=seed)
    zk = CF.parse_zkey(zbytes)
    prover = Groth16Prover(zbytes)
    fb = fr_bytes(curve, full)
    h_gpu = prover.witness_map(fb)
    h = OG.witness_map(zk, full)
    assert h_gpu == fr_bytes(curve, h)
    assert list(prover.prove(fb)) == list(OG.prove(zk, full, h=h))
    Fr = pyref.Field("bn254_fr" if curve == "bn254" else "bls12_381_fr")
    r, s = 0x5EED + seed, Fr.p - 3 - seed
    want_zk = list(OG.prove(zk, full, r, s, h=h))
    assert list(prover.prove(fb, Fr.to_bytes(r), Fr.to_bytes(s))) == want_zk
    # A and the witness + h MSM as two MSMs (variant 1, round 4) instead of the
    # default grouped MSM: the same proofs; then forced window bits
    prover.set_variant(1)
    assert list(prover.prove(fb)) == list(OG.prove(zk, full, h=h))
    # the fixed-base fold tables of the G2 B MSM (variant bits 1-3) and the
    # grouped G1 MSM (bits 4-6): none (18), two copies each (36), B2 eight with
    # the default G1 (8), B2 sixteen and G1 eight (74); the default is B2
    # sixteen, G1 four (groth16.h kB2Fold / kG1Fold, where they divide W)
    for v in (18, 36, 8, 74):
        prover.set_variant(v)
        assert list(prover.prove(fb, Fr.to_bytes(r), Fr.to_bytes(s))) == want_zk, v
    prover.set_variant(0)
    prover.set_msm_window_bits(5, 6, 7)
    assert list(prover.prove(fb, Fr.to_bytes(r), Fr.to_bytes(s))) == want_zk
    prover.close()


def test_adder_fixture_gpu():
    """The reference's second circom fixture (examples/adder.zkey) with the
    witness of adder_data.json: the GPU proof equals the oracle's and passes
    the pairing check, NoZK and ZK."""
    from tachyon_amd.groth16 import Groth16Prover
    from test_groth16_oracle import adder_witness
    zbytes = open(os.path.join(GOLDEN, "adder.zkey"), "rb").read()
    zk = CF.parse_zkey(zbytes)
    w = adder_witness(3, 4)
    prover = Groth16Prover(zbytes)
    fb = fr_bytes("bn254", w)
    G1, G2 = pyref.Curve("bn254_g1"), pyref.Curve("bn254_g2")
    vk = {k: (G2 if k.endswith("g2") else G1).from_bytes(v) for k, v in zk["vk"].items()}
    ic = [G1.from_bytes(b) for b in zk["ic"]]
    Fr = G1.Fr
    for r, s in ((0, 0), (0xC0DE, Fr.p - 77)):
        proof = prover.prove(fb) if r == 0 else prover.prove(fb, Fr.to_bytes(r), Fr.to_bytes(s))
        assert list(proof) == list(OG.prove(zk, w, r, s))
        A, B, C = proof
        assert BP.groth16_verify(vk, ic, [7], (G1.from_bytes(A), G2.from_bytes(B), G1.from_bytes(C)))
    prover.close()


def test_configs4_size_parity():
    """BASELINE configs[4] at its own size: the bench's synthetic 2^20-constraint
    circom key (bench.synth_groth16_zkey); the GPU proof equals the CPU
    oracle's (witness map and MSMs in oracle/, prove_np), NoZK and ZK."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from tachyon_amd.groth16 import Groth16Prover
    zkey, full = bench.synth_groth16_zkey(20)
    prover = Groth16Prover(zkey)
    fb = full.tobytes()
    assert tuple(prover.prove(fb)) == tuple(OG.prove_np(zkey, full))
    Fr = pyref.Field("bn254_fr")
    r, s = 0x1234_5678_9ABC, Fr.p - 2
    assert tuple(prover.prove(fb, Fr.to_bytes(r), Fr.to_bytes(s))) == tuple(OG.prove_np(zkey, full, r, s))
    prover.set_variant(1)  # the round-4 separate A and witness + h MSMs: the same proof
    assert tuple(prover.prove(fb)) == tuple(OG.prove_np(zkey, full))
    for v in (18, 36, 8, 74):  # fold tables off, two copies each, B2 x8, B2 x16 + G1 x8 (default: B2 x16, G1 x4)
        prover.set_variant(v)
        assert tuple(prover.prove(fb)) == tuple(OG.prove_np(zkey, full)), v
    prover.close()


_FALLBACK_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import bench
from tachyon_amd.groth16 import Groth16Prover
zkey, full = bench.synth_groth16_zkey(int(os.environ["LOG_N"]))
p = Groth16Prover(zkey)
bytes_held = p.prepare()
folds = p.folds()
proof = p.prove(full.tobytes())
print(json.dumps({"bytes": bytes_held, "folds": folds, "proof": [x.hex() for x in proof]}))
"""


def _prove_child(log_n, limit):
    """A proof in a child process (an MSM that cannot fit aborts the process,
    like the reference's CHECKs): prepare() + prove() under TACHYON_MSM_MEM_LIMIT."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, REPO=repo, LOG_N=str(log_n))
    env.pop("TACHYON_MSM_MEM_LIMIT", None)
    if limit:
        env["TACHYON_MSM_MEM_LIMIT"] = str(limit)
    r = subprocess.run([sys.executable, "-c", _FALLBACK_CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_fold_tables_memory_fallback():
    """The proving key's fold tables are an explicit setup step (prepare) and
    memory-aware: with the device capped (TACHYON_MSM_MEM_LIMIT = 256 MiB) a
    2^17-constraint key gets no tables (fold 1) and A and the witness + h MSM
    run as separate MSMs instead of the grouped one; without a cap both get
    tables.  Both proofs equal the CPU oracle's."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    log_n = 17
    zkey, full = bench.synth_groth16_zkey(log_n)
    want = [x.hex() for x in OG.prove_np(zkey, full)]
    free = _prove_child(log_n, None)
    capped = _prove_child(log_n, 256 << 20)
    # (at 2^17 the MSMs' c = 10 gives W = 26 windows: the folds that divide it are 2)
    assert free["folds"]["b2"] > 1 and free["folds"]["grouped_g1"] > 1, free["folds"]
    assert capped["folds"]["b2"] == 1 and capped["folds"]["grouped_g1"] == 0, capped["folds"]
    assert capped["bytes"] == 0 < free["bytes"]
    assert free["proof"] == want and capped["proof"] == want


def test_all_public_no_witness():
    """num_vars = num_public + 1: the witness (l / C1) MSM is empty."""
    from tachyon_amd.groth16 import Groth16Prover
    zbytes, full = synth_zkey("bn254", log_n=4, num_vars=4, num_public=3, seed=9)
    zk = CF.parse_zkey(zbytes)
    prover = Groth16Prover(zbytes)
    assert list(prover.prove(fr_bytes("bn254", full))) == list(OG.prove(zk, full))
    prover.close()


def test_device_resident_witness():
    """The witness may be a CUDA tensor (device pointer, no upload)."""
    import numpy as np
    import torch
    from tachyon_amd.groth16 import Groth16Prover
    zbytes, full = synth_zkey("bn254", log_n=7, seed=11)
    zk = CF.parse_zkey(zbytes)
    prover = Groth16Prover(zbytes)
    fb = fr_bytes("bn254", full)
    d = torch.from_numpy(np.frombuffer(fb, dtype=np.uint8).copy()).cuda()
    assert list(prover.prove(d)) == list(OG.prove(zk, full))
    prover.close()


def test_circom_prover_cli(tmp_path):
    """bin/circom_prover (prover_main.cc on the C-ABI): snarkjs-style proof.json
    and public.json; --no_zk reproduces the golden proof, the ZK proof verifies."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tachyon_amd", "bin",
                       "circom_prover")
    zk = CF.parse_zkey(open(os.path.join(GOLDEN, "multiplier_3.zkey"), "rb").read())
    g = json.load(open(os.path.join(GOLDEN, "groth16_multiplier_3.json")))
    G1, G2 = pyref.Curve("bn254_g1"), pyref.Curve("bn254_g2")
    vk = {k: (G2 if k.endswith("g2") else G1).from_bytes(v) for k, v in zk["vk"].items()}
    ic = [G1.from_bytes(b) for b in zk["ic"]]
    for flags in (["--no_zk"], []):
        proof_p, pub_p = tmp_path / "proof.json", tmp_path / "public.json"
        cmd = [exe, "--zkey", os.path.join(GOLDEN, "multiplier_3.zkey"), "--wtns",
               os.path.join(GOLDEN, "multiplier_3.wtns"), "--proof", str(proof_p), "--public", str(pub_p)] + flags
        subprocess.run(cmd, check=True, timeout=120, capture_output=True)
        proof = json.load(open(proof_p))
        assert json.load(open(pub_p)) == ["60"]
        assert proof["protocol"] == "groth16" and proof["curve"] == "bn128"
        assert proof["pi_a"][2] == "1" and proof["pi_b"][2] == ["1", "0"]
        A = tuple(int(x) for x in proof["pi_a"][:2])
        B = tuple(tuple(int(x) for x in c) for c in proof["pi_b"][:2])
        C = tuple(int(x) for x in proof["pi_c"][:2])
        if flags:
            want = g["cases"][0]["proof"]
            assert G1.to_bytes(A).hex() == want[0] and G2.to_bytes(B).hex() == want[1] and G1.to_bytes(C).hex() == want[2]
        assert BP.groth16_verify(vk, ic, [60], (A, B, C))


@pytest.mark.parametrize("curve,log_n,world", [("bn254", 7, 2), ("bn254", 9, 3), ("bn254", 4, 8), ("bls12_381", 6, 3)])
def test_sharded_partials_assemble(curve, log_n, world):
    """The multi-GPU split (prove_partials per rank + assemble) equals prove()
    and the oracle for every world size, NoZK and ZK, with the partials in any
    order -- world 8 on a 16-point domain leaves some ranks with empty shards.
    (A blob set that is not one rank each aborts, like every C-ABI error.)"""
    from tachyon_amd.groth16 import Groth16Prover
    zbytes, full = synth_zkey(curve, log_n=log_n, num_public=2, seed=40 + world)
    zk = CF.parse_zkey(zbytes)
    prover = Groth16Prover(zbytes)
    fb = fr_bytes(curve, full)
    Fr = pyref.Field("bn254_fr" if curve == "bn254" else "bls12_381_fr")
    r_int, s_int = 0xABCDEF + world, Fr.p - 11
    r, s = Fr.to_bytes(r_int), Fr.to_bytes(s_int)
    parts = [prover.prove_partials(fb, k, world, with_b1=True) for k in range(world)]
    assert len(parts[0]) == prover.partials_size()
    blob = b"".join(parts)
    shuffled = b"".join(reversed(parts))
    expect_nozk = list(OG.prove(zk, full))
    expect_zk = list(OG.prove(zk, full, r_int, s_int))
    assert list(prover.assemble(blob)) == expect_nozk == list(prover.prove(fb))
    assert list(prover.assemble(shuffled, r, s)) == expect_zk
    prover.close()


@pytest.mark.parametrize("curve,log_n,devices", [("bn254", 8, [0, 0]), ("bn254", 10, [0, 0, 0]),
                                                  ("bls12_381", 6, [0, 0])])
def test_multi_device_prover(curve, log_n, devices):
    """One-process multi-device proofs (tachyon_mi355x_groth16_set_devices: a
    prover and a host thread per device entry, partials added on the host) on
    logical devices sharing the box's GPU: NoZK and ZK proofs equal the
    oracle's; [] returns to the single-device prover; bad ids are refused."""
    from tachyon_amd.groth16 import Groth16Prover
    zbytes, full = synth_zkey(curve, log_n=log_n, num_public=2, seed=70 + log_n)
    zk = CF.parse_zkey(zbytes)
    prover = Groth16Prover(zbytes)
    fb = fr_bytes(curve, full)
    Fr = pyref.Field("bn254_fr" if curve == "bn254" else "bls12_381_fr")
    r_int, s_int = 0x1234 + log_n, Fr.p - 5
    prover.set_devices(devices)
    assert list(prover.prove(fb)) == list(OG.prove(zk, full))
    assert list(prover.prove(fb, Fr.to_bytes(r_int), Fr.to_bytes(s_int))) == list(OG.prove(zk, full, r_int, s_int))
    with pytest.raises(ValueError):
        prover.set_devices([0, 4096])
    # a device-resident assignment (a CUDA tensor): every device's prover
    # copies it into its own HBM before its kernels read it
    import numpy as np
    import torch
    d_full = torch.from_numpy(np.frombuffer(fb, dtype=np.uint8).copy()).cuda()
    prover.set_profile(True)  # forwarded to the per-device provers
    assert list(prover.prove(d_full)) == list(OG.prove(zk, full))
    assert prover.last_timings()["total"] > 0  # the lead device's phases
    prover.set_profile(False)
    prover.set_devices([])
    assert list(prover.prove(fb)) == list(OG.prove(zk, full))
    prover.close()


def test_circom_prover_cli_devices(tmp_path):
    """bin/circom_prover --devices 0,0 (two logical devices on the box's GPU):
    the NoZK proof equals the golden one."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tachyon_amd", "bin",
                       "circom_prover")
    g = json.load(open(os.path.join(GOLDEN, "groth16_multiplier_3.json")))
    G1, G2 = pyref.Curve("bn254_g1"), pyref.Curve("bn254_g2")
    proof_p, pub_p = tmp_path / "proof.json", tmp_path / "public.json"
    cmd = [exe, "--zkey", os.path.join(GOLDEN, "multiplier_3.zkey"), "--wtns",
           os.path.join(GOLDEN, "multiplier_3.wtns"), "--proof", str(proof_p), "--public", str(pub_p),
           "--no_zk", "--devices", "0,0"]
    subprocess.run(cmd, check=True, timeout=120, capture_output=True)
    proof = json.load(open(proof_p))
    A = tuple(int(x) for x in proof["pi_a"][:2])
    B = tuple(tuple(int(x) for x in c) for c in proof["pi_b"][:2])
    C = tuple(int(x) for x in proof["pi_c"][:2])
    want = g["cases"][0]["proof"]
    assert G1.to_bytes(A).hex() == want[0] and G2.to_bytes(B).hex() == want[1] and G1.to_bytes(C).hex() == want[2]
    bad = subprocess.run(cmd[:-1] + ["0,4096"], timeout=120, capture_output=True)
    assert bad.returncode != 0
