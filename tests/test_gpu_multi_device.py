"""One-process multi-device MSM under the reference C-ABI
(tachyon_mi355x_msm_gpu_set_devices / TACHYON_MSM_GPU_DEVICES): the points are
split into one contiguous shard per device entry, every shard runs on its own
device, host thread and stream, and the shard results are added on the host --
the reference's kParallelTerm chunk-and-sum (pippenger_adapter.h:82-113) across
devices.  The one-GPU test box maps N = 2 and 3 logical devices onto device 0
(separate streams); results must equal the oracle bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tachyon_amd", "bin")


@pytest.mark.parametrize("curve", ["bn254_g1", "bls12_381_g2"])
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_logical_devices_host_inputs(curve, devices):
    """Host-resident inputs (the reference's semantics), odd n: each shard
    uploads its own slice; the sum equals the oracle."""
    from tachyon_amd.msm import VariableBaseMSMGpu
    n = 5001
    pb, sf = O.CURVE_INFO[curve]
    bases = O.gen_bases(curve, 31, n, 64).tobytes()
    scalars = O.gen_scalars(sf, 31, n).tobytes()
    want, _ = O.msm(curve, bases, scalars)
    m = VariableBaseMSMGpu(curve)
    m.set_devices(devices)
    assert m.run(bases, scalars) == want
    shards = m.last_shards()
    assert [d for d, _, _ in shards] == devices
    assert sum(p for _, p, _ in shards) == n and all(ms > 0 for _, _, ms in shards)
    # fewer points than shards: empty shards add the identity
    assert m.run(bases[:pb], scalars[:32]) == O.msm(curve, bases[:pb], scalars[:32])[0]
    assert m.run(b"", b"") == bytes(pb)
    m.set_devices([])  # back to one device
    assert m.run(bases, scalars) == want and m.last_shards() == []
    m.close()


def test_logical_devices_device_inputs_and_reference_entry():
    """Device-resident inputs on device 0 (same device: no copy) and the
    reference entry point tachyon_bn254_g1_affine_msm_gpu of a context created
    under TACHYON_MSM_GPU_DEVICES (what msm_benchmark_gpu and the scroll_halo2
    bridge would pick up without source changes)."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = (1 << 18) + 7
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", 5, n, 1 << 10, d_b.data_ptr())
    M.gen_scalars("bn254_fr", 5, n, d_s.data_ptr())
    torch.cuda.synchronize()
    hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
    want = O.msm_np("bn254_g1", hb, hs)
    m = M.VariableBaseMSMGpu("bn254_g1")
    m.set_devices([0, 0, 0])
    assert m.run(d_b, d_s) == want
    m.close()
    os.environ["TACHYON_MSM_GPU_DEVICES"] = "0,0"
    try:
        m2 = M.VariableBaseMSMGpu("bn254_g1")  # tachyon_bn254_g1_create_msm_gpu reads the list
    finally:
        del os.environ["TACHYON_MSM_GPU_DEVICES"]
    assert [p for _, p, _ in m2.last_shards()] == [0, 0]  # two shards, nothing run yet
    jac = m2.run_jacobian(hb, hs)
    assert M.jacobian_to_affine("bn254_g1", jac) == want
    assert [d for d, _, _ in m2.last_shards()] == [0, 0]
    m2.close()


def test_large_host_shards_pipelined():
    """2^25 host-resident points over 2 logical devices: each 2^24 shard takes
    the chunked upload pipeline (MsmGpu::run_host_pipelined) on its own
    stream; equals the single-device MSM of the same input."""
    torch = pytest.importorskip("torch")
    from tachyon_amd import msm as M
    n = 1 << 25
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", 0x7AC40001, n, 1 << 10, d_b.data_ptr())
    M.gen_scalars("bn254_fr", 0x7AC40001, n, d_s.data_ptr())
    torch.cuda.synchronize()
    m = M.VariableBaseMSMGpu("bn254_g1")
    whole = m.run(d_b, d_s)
    hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
    del d_b, d_s
    torch.cuda.empty_cache()
    m.set_devices([0, 0])
    assert m.run(hb, hs) == whole
    m.close()


def test_settings_reach_every_shard():
    """set_variant / set_profile / set_window_bits reach the shards, whether
    they are set before or after set_devices, and last_schedule / last_timings
    report a shard that ran (they used to report the idle
    single-device context)."""
    from tachyon_amd.msm import VariableBaseMSMGpu
    n = 1 << 13
    bases = O.gen_bases("bn254_g1", 41, n, 64).tobytes()
    scalars = O.gen_scalars("bn254_fr", 41, n).tobytes()
    want, _ = O.msm("bn254_g1", bases, scalars)
    m = VariableBaseMSMGpu("bn254_g1")
    m.set_variant(262144)  # bit 18: the FIPS 32-bit field, visible in last_schedule
    m.set_profile(True)
    m.set_devices([0, 0])
    assert m.run(bases, scalars) == want
    s = m.last_schedule()
    assert s["acc29"] is False, s
    t = m.last_timings()
    assert t["acc"] > 0 and t["total"] > 0, t
    m.set_variant(0)  # after set_devices
    assert m.run(bases, scalars) == want
    assert m.last_schedule()["acc29"] is True
    m.set_window_bits(7)
    assert m.run(bases, scalars) == want
    m.set_devices([])
    m.close()


def test_set_devices_refuses_bad_ids():
    from tachyon_amd.msm import VariableBaseMSMGpu
    m = VariableBaseMSMGpu("bn254_g1")
    with pytest.raises(ValueError):
        m.set_devices([0, 4096])
    with pytest.raises(ValueError):
        m.set_devices([-1, 0])
    assert m.last_shards() == []  # refused: nothing changed
    m.close()


def test_msm_benchmark_gpu_with_device_list():
    """benchmark/msm's GPU harness (msm_benchmark_gpu.cc) unchanged, sharded by
    the environment: --check_results still passes against its CPU check."""
    env = dict(os.environ, TACHYON_MSM_GPU_DEVICES="0,0")
    p = subprocess.run([os.path.join(BIN, "msm_benchmark_gpu"), "-k", "12", "-k", "14", "--check_results"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert '"check_results": "pass"' in p.stdout
