"""GPU NTT over BLS12-381 Fr at the boundary: IcicleNTT<bls12_381::Fr>
(icicle_ntt_bls12_381.cc:31-115) and the reference's GPU domain test
univariate_evaluation_domain_gpu_unittest.cc:20-66 (Radix2EvaluationDomain
FFT / IFFT at 2^5..2^14, plain and on a coset, against the CPU path).  Here the
field-generic C-ABI domain (tachyon_mi355x_ntt_domain_*, field 3) and the C++
FieldNTTHolder hook are compared bytewise with the oracle's CPU restatement
(O.fft / O.ifft with field="bls12_381_fr", pinned by tests/golden/
ntt_bls12_381_fr.json and the arkworks two-adic root), coset offset 7 = the
field's BUILD subgroup generator."""
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
FIELD = "bls12_381_fr"
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tachyon_amd", "bin")


def domain(n):
    from tachyon_amd.ntt import FieldEvaluationDomain
    return FieldEvaluationDomain(FIELD, n)


def seven():
    return O.field_op(FIELD, "to_mont", (7).to_bytes(32, "little"))


def pad(b, n):
    return b + bytes(32 * n - len(b))


def test_bls_ntt_golden():
    g = json.load(open(os.path.join(GOLDEN, "ntt_bls12_381_fr.json")))
    for c in g["cases"]:
        n = 1 << c["log_n"]
        d = domain(n)
        assert d.group_gen.hex() == g["roots_of_unity_mont"][str(c["log_n"])]
        d.set_offset(bytes.fromhex(c["offset_mont"]) if c["offset"] != 1 else None)
        coeffs = b"".join(bytes.fromhex(x) for x in c["coeffs"])
        ev = d.fft(coeffs)
        assert ev.hex() == "".join(c["evals"]), c
        # (the golden IFFT trims trailing zero coefficients like the reference's container API)
        assert d.ifft(ev) == pad(b"".join(bytes.fromhex(x) for x in c["ifft_of_evals"]), n), c
        d.close()


@pytest.mark.parametrize("logn", list(range(5, 15)) + [20])
def test_bls_fft_ifft_coset_vs_oracle(logn):
    n = 1 << logn
    coeffs = O.gen_scalars(FIELD, 3000 + logn, n).tobytes()
    d = domain(n)
    ev = d.fft(coeffs)
    assert ev == O.fft(coeffs, n, field=FIELD)
    assert d.ifft(ev) == coeffs
    assert d.ifft(coeffs) == pad(O.ifft(coeffs, n, field=FIELD), n)
    d.set_offset(seven())
    cev = d.fft(coeffs)
    assert cev == O.fft(coeffs, n, seven(), field=FIELD) and cev != ev
    assert d.ifft(cev) == coeffs
    assert d.ifft(coeffs) == pad(O.ifft(coeffs, n, seven(), field=FIELD), n)
    d.set_offset(None)  # back to the plain domain
    assert d.fft(coeffs) == ev
    d.close()


@pytest.mark.parametrize("logn,batch", [(10, 3), (16, 2)])
def test_bls_device_batched(logn, batch):
    import torch
    n = 1 << logn
    x = O.gen_scalars(FIELD, 77 + logn, n * batch)
    t = torch.from_numpy(x.view(np.uint8).reshape(-1).copy()).cuda()
    d = domain(n)
    torch.cuda.synchronize()
    d.transform_device(t.data_ptr(), batch)
    torch.cuda.ExternalStream(d.stream).synchronize()
    got = t.cpu().numpy().tobytes()
    raw = x.tobytes()
    for b in range(batch):
        assert got[b * n * 32:(b + 1) * n * 32] == O.fft(raw[b * n * 32:(b + 1) * n * 32], n, field=FIELD), b
    d.transform_device(t.data_ptr(), batch, inverse=True)
    torch.cuda.ExternalStream(d.stream).synchronize()
    assert t.cpu().numpy().tobytes() == raw
    d.close()


def test_bls_domain_refuses_other_fields():
    from tachyon_amd._lib import lib
    assert not lib().tachyon_mi355x_ntt_domain_create(0, 16)  # bn254 Fq: no NTT
    assert not lib().tachyon_mi355x_ntt_domain_create(2, 16)


@pytest.mark.parametrize("log_n", [5, 10, 14])
def test_bls_ntt_holder_cpp_hook(tmp_path, log_n):
    """include/tachyon_mi355x_ntt_holder.h FieldNTTHolder<kBls12_381Fr> from a
    C++ client: in-place host FFT / IFFT, plain and on the coset 7<w>; the
    outputs equal the oracle's CPU transforms."""
    dump = tmp_path / "ntt.bin"
    r = subprocess.run([os.path.join(BIN, "ntt_holder_check"), str(log_n), "--field", "bls12_381", "--dump",
                        str(dump)], timeout=120, capture_output=True, text=True)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and res["field"] == FIELD, (r.stderr, res)
    n = 1 << log_n
    raw = dump.read_bytes()
    inp, fft, coset = raw[:n * 32], raw[n * 32:2 * n * 32], raw[2 * n * 32:]
    assert fft == O.fft(inp, n, field=FIELD)
    assert coset == O.fft(inp, n, seven(), field=FIELD)
