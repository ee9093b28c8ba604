#!/usr/bin/env python3
"""Headline benchmark: BN254 G1 MSM scalars/s at 2^26 (BASELINE.json configs[1])
with the BN254 Fr NTT elems/s at 2^24 (configs[2]) reported beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--log-n 26] [--ntt-log-n 24]
  (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

A step is one full MSM over 2^26 points whose bases/scalars are already in
HBM (generated on the device, seeded).  With N GPUs the 2^26 points are split
into N contiguous shards (the reference's kParallelTerm chunking,
pippenger_adapter.h:82-113) of ONE global input (every rank generates its
slice of the same seeded sequence); every rank runs the MI355X MSM on its
shard and the per-rank partial points are combined with one RCCL all-gather
plus a host group sum (EC addition is not an RCCL reduction op).  `value` =
2^26 / the slowest rank's time per step (strong scaling); at N > 1 rank 0
also runs the unsharded MSM once and the line says whether they agree.

The roofline object prices the dominant kernel (bucket accumulation) with
HIP events recorded on the MSM stream around that launch.  `host_resident`
times the reference semantics (pageable host inputs, H2D + kernels + D2H
inside the call, msm_runner.h:54-58 / fft_runner.h:53-58).  The cpu_baseline
object times the oracle's CPU restatement of PippengerAdapter kParallelTerm
and Radix2EvaluationDomain (rank 0, N=1 only) at the headline sizes on the
same inputs, and checks that the GPU results equal the CPU ones.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "BN254 G1 MSM scalars/s @2^26 and Fr NTT elems/s @2^24, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)
MSM_BYTES_PER_POINT = 96  # 64 B affine base + 32 B scalar
NTT_BYTES_PER_ELEM = 64   # 32 B in + 32 B out per transform
SEED = 0x7AC40001
# Measured BN254 Montgomery-multiply ceiling of the chip (tools/microbench/mulmod_rates.hip,
# DESIGN.md section 4): 138.6 G/s with >= 2 independent product chains per lane or >= 4
# waves per SIMD (129.3 G with one chain at one wave): the VALU roofline of both kernels.
MULMOD_PEAK_G = 138.6
MULMOD_PEAK_NOTE = ("measured BN254 FIPS Montgomery-product ceiling of the chip, 138.6 G/s with >= 2 "
                    "independent chains per lane or >= 4 waves/SIMD (tools/microbench/mulmod_rates.hip)")
# The accumulation's VALU roofline: mixed additions (madd-2008-s,
# point_xyzz_impl.h:129-176) per second against the chip's ceiling for the same
# field code in registers with no gathers or run logic, measured live on this
# box (tachyon_mi355x_msm_madd_ceiling; boxes differ by up to ~8 % in clock).
# The fallback constants are one box's figures (profiles/r03c/madd_rates.log):
# the 29-bit-limb field of the BN254 G1 accumulation and the 32-bit FIPS field.
MADD_PEAK_G = {"seg_acc29_kernel": 19.40, "seg_acc_kernel": 13.67}
MADD_PEAK_NOTE = ("mixed additions/s of the same field code in registers, no gathers or run logic, "
                  "whole chip at 3 waves/SIMD (tachyon_mi355x_msm_madd_ceiling, measured in this run)")


def pmc_traffic(kernel):
    """Per-dispatch HBM bytes of `kernel` from the newest committed rocprofv3 PMC
    passes (profiles/<round>/pmc_traffic.json, written by tools/profile_round.sh
    from separate FETCH_SIZE / WRITE_SIZE runs of this bench command); None if absent."""
    import glob
    import re

    def order(f):  # r05z < r05aa < r05ab (spreadsheet-column order of the run suffix)
        m = re.fullmatch(r"r(\d+)([a-z]*)", os.path.basename(os.path.dirname(f)))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, f)

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic.json")), key=order)
    for f in reversed(files):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in t:
            k = t[kernel]
            return k["traffic_bytes"] / 1e9, os.path.relpath(f, ROOT), k.get("fetch_bytes_raw", 0) / 1e9
    return None, None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=26)
    ap.add_argument("--ntt-log-n", type=int, default=24)
    ap.add_argument("--window-bits", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ntt", action="store_true")
    ap.add_argument("--cpu-log-n", type=int, default=0,
                    help="CPU baseline MSM size (0 = the headline --log-n)")
    ap.add_argument("--no-host-resident", action="store_true")
    ap.add_argument("--no-non-uniform", action="store_true",
                    help="skip the NonUniform(n, 1) leg (benchmark/msm --test_set non_uniform)")
    ap.add_argument("--msm-split", choices=("auto", "points", "windows", "hybrid"), default="auto",
                    help="N > 1 MSM partition: point shards (default), or window ranges with every rank holding "
                         "all points (c = 16: W = 16 windows; measured slower per rank, tools/split_probe.py), or "
                         "hybrid: N / Q point groups x Q window groups (--window-groups; c = --window-bits or 19); "
                         "auto (default): the library's plan (tachyon_mi355x_msm_shard_plan), hybrid or points")
    ap.add_argument("--window-groups", type=int, default=2, help="Q of --msm-split hybrid")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the configs[1]/[2] size sweeps (profiling runs: one MSM and one NTT size only)")
    ap.add_argument("--bls-log-n", type=int, default=24,
                    help="BLS12-381 G1 + G2 MSM size (BASELINE configs[3]); 0 = skip")
    ap.add_argument("--groth16-log-n", type=int, default=20,
                    help="Groth16 prove on a synthetic 2^k-constraint circom key (BASELINE configs[4]); 0 = skip")
    return ap.parse_args()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_threads():
    """Host threads this job may use: the box's CPU share (OMP_NUM_THREADS is
    set to it on the GPU pool) or else the affinity mask."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(avail, int(env))) if env and env.isdigit() else avail


def cpu_baseline(args, h_bases, h_scalars, gpu_affine, ntt_in, gpu_ntt_out):
    """The oracle's C restatement of the reference CPU path, timed on the host
    cores at the headline sizes on the SAME inputs as the GPU legs (copied
    from HBM), one run per size as the reference's runners do; it also
    cross-checks the GPU results.  configs[0] (2^16, benchmark/msm's CPU
    path) is timed beside it."""
    from oracle import oracle as O
    threads = cpu_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    n = h_scalars.nbytes // 32
    t0 = time.perf_counter()
    cpu_point = O.msm_np("bn254_g1", h_bases, h_scalars, method="parallel_term", threads=threads)
    dt = time.perf_counter() - t0
    m16 = 1 << 16
    t1 = time.perf_counter()
    O.msm_np("bn254_g1", h_bases[:m16 * 64], h_scalars[:m16 * 32], method="parallel_term", threads=threads)
    dt16 = time.perf_counter() - t1
    out = {"value": n / dt, "unit": "scalars/s", "cores": threads, "kind": "port",
           "sample": f"BN254 G1 MSM 2^{n.bit_length() - 1} points (the headline size, the bench's own inputs), "
                     f"PippengerAdapter kParallelTerm restated in C (oracle/), {threads} OpenMP threads "
                     f"(the job's CPU share; {os.cpu_count()} CPUs visible), {cpu_model()}; portable CIOS "
                     f"field (the reference's x86 ffiasm asm field is unavailable)",
           "seconds": dt, "gpu_equals_cpu": cpu_point == gpu_affine,
           "configs0": {"workload": "BN254 G1 MSM 2^16, CPU path (BASELINE configs[0])", "seconds": dt16,
                        "value": m16 / dt16, "unit": "scalars/s"}}
    if ntt_in is not None:
        import numpy as np
        v = ntt_in.copy()
        m = v.nbytes // 32
        t0 = time.perf_counter()
        O.fft_np(v.view(np.uint64))
        dt2 = time.perf_counter() - t0
        out["ntt"] = {"value": m / dt2, "unit": "elems/s", "seconds": dt2,
                      "sample": f"BN254 Fr FFT 2^{m.bit_length() - 1} (the headline size, the bench's input), "
                                f"Radix2EvaluationDomain restated in C, {threads} threads",
                      "gpu_equals_cpu": gpu_ntt_out is not None and v.tobytes() == gpu_ntt_out.tobytes()}
    return out


def synth_groth16_zkey(log_n, seed=SEED):
    """Synthetic circom zkey v1 (BN254) built with numpy from device-generated
    points: domain n = 2^log_n constraints, num_vars = n, one public input,
    two A and two B terms per constraint (random signals and values).  The
    points are seeded k*G doubling chains (valid curve points, no trapdoor):
    the proof exercises the whole prover but does not verify -- the parity
    tests pin it against the oracle and the pairing check."""
    import struct
    import numpy as np
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd import params as P
    n = 1 << log_n
    m, npub = n, 1
    n1 = 5 + (npub + 1) + 3 * m - npub - 1 + n
    g1 = torch.empty(n1 * 64, dtype=torch.uint8, device="cuda")
    g2 = torch.empty((3 + m) * 128, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", seed, n1, 1 << 10, g1.data_ptr())
    M.gen_bases("bn254_g2", seed + 1, 3 + m, 1 << 10, g2.data_ptr())
    full = torch.empty(m * 32, dtype=torch.uint8, device="cuda")
    M.gen_scalars("bn254_fr", seed + 2, m, full.data_ptr())
    torch.cuda.synchronize()
    g1 = g1.cpu().numpy()
    g2 = g2.cpu().numpy()
    full = full.cpu().numpy()
    full[:32] = np.frombuffer(P.mont(1, P.BN254_FR, 4).to_bytes(32, "little"), np.uint8)  # full[0] = 1
    rng = np.random.default_rng(seed)
    per_row = 2
    nnz = 2 * per_row * n
    coef = np.zeros(nnz, dtype=[("m", "<u4"), ("c", "<u4"), ("s", "<u4"), ("v", "<u8", 4)])
    coef["m"] = np.repeat(np.arange(2, dtype=np.uint32), per_row * n)
    coef["c"] = np.tile(np.repeat(np.arange(n, dtype=np.uint32), per_row), 2)
    coef["s"] = rng.integers(0, m, nnz, dtype=np.uint32)
    v = rng.integers(0, 1 << 63, (nnz, 4), dtype=np.uint64)
    v[:, 3] &= (1 << 60) - 1  # < r
    coef["v"] = v
    q, r = P.BN254_FQ, P.BN254_FR
    g = lambda i, k: g1[i * 64:(i + k) * 64].tobytes()
    vk = g(0, 1) + g(1, 1) + g2[0:128].tobytes() + g2[128:256].tobytes() + g(2, 1) + g2[256:384].tobytes()
    o = 5
    ic = g(o, npub + 1); o += npub + 1
    a1 = g(o, m); o += m
    b1 = g(o, m); o += m
    c1 = g(o, m - npub - 1); o += m - npub - 1
    h1 = g(o, n)
    groth = struct.pack("<I", 32) + q.to_bytes(32, "little") + struct.pack("<I", 32) + r.to_bytes(32, "little") + \
        struct.pack("<III", m, npub, n) + vk
    secs = [(1, struct.pack("<I", 1)), (2, groth), (3, ic), (4, struct.pack("<I", nnz) + coef.tobytes()),
            (5, a1), (6, b1), (7, g2[384:].tobytes()), (8, c1), (9, h1)]
    parts = [b"zkey", struct.pack("<II", 1, len(secs))]
    for t, body in secs:
        parts += [struct.pack("<IQ", t, len(body)), body]
    return b"".join(parts), full


def bench_bls(args, rank, world, barrier, dist, backend, lib_comm=None):
    """BLS12-381 G1 and G2 MSMs at 2^k (BASELINE configs[3]): each rank's share
    of one global input (the library's partition: point shards or the hybrid) + the
    all-gather of partials, device-resident inputs, as the headline."""
    import torch
    from tachyon_amd import dist as D
    from tachyon_amd import msm as M
    out = {}
    n_total = 1 << args.bls_log_n
    parts = {}
    for curve, pb in (("bls12_381_g1", 96), ("bls12_381_g2", 192)):
        split, start, n, wrange, split_c, p_groups, q_groups, shard = msm_partition(args, curve, world, rank, n_total)
        parts[curve] = (split if split != "hybrid" else f"hybrid {p_groups} point groups x {q_groups} window groups, "
                        f"c = {split_c}")
        d_b = torch.empty(max(1, n) * pb, dtype=torch.uint8, device="cuda")
        d_s = torch.empty(max(1, n) * 32, dtype=torch.uint8, device="cuda")
        M.gen_bases(curve, SEED, n, 1 << 10, d_b.data_ptr(), start=start)  # this rank's slice of one input
        M.gen_scalars("bls12_381_fr", SEED, n, d_s.data_ptr(), start=start)
        torch.cuda.synchronize()
        msm = M.VariableBaseMSMGpu(curve)
        if wrange is not None:
            msm.set_window_bits(split_c)

        def local_run():
            if wrange is not None:
                return msm.run_window_range(d_b, d_s, wrange[0], wrange[1], n)
            return msm.run(d_b, d_s, n)

        def step():
            if lib_comm is not None and shard is not None:  # the library's sharded entry (as the headline)
                return msm.run_sharded_plan(lib_comm, shard, d_b, d_s)
            return D.sharded_msm(curve, local_run, device="cuda")

        ref = step()
        reps = max(2, min(args.steps, 3))
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            res = step()
        barrier()
        dt = (time.perf_counter() - t0) / reps
        if dist is not None:
            t = torch.tensor([dt], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        leg = out[curve.split("_")[-1]] = {"ms_per_msm": dt * 1e3, "scalars_per_s": n_total / dt,
                                           "consistent": res == ref, "points_per_gpu": n,
                                           "partition": parts[curve] if world > 1 else "single GPU"}
        if world == 1:
            leg.update(msm_rooflines(msm, curve, d_b, d_s, n, pb))
        if world == 1 and not args.no_sweep:
            # the per-rank shards of this MSM at N = 2, 4, 8 (prefixes of the same input) and the
            # point-shard projection built on them
            sw = {str(args.bls_log_n): {"ms": round(dt * 1e3, 3)}}
            for k in range(args.bls_log_n - 3, args.bls_log_n):
                msm.run(d_b, d_s, 1 << k)
                ts = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    msm.run(d_b, d_s, 1 << k)
                    ts.append(time.perf_counter() - t0)
                sw[str(k)] = {"ms": round(sorted(ts)[1] * 1e3, 3), "scalars_per_s": (1 << k) / sorted(ts)[1]}
            leg["shard_sweep"] = sw
            hybrid = {str(w): hybrid_rank_ms(msm, curve, d_b, d_s, n_total, w)
                      for w in (2, 4, 8) if hybrid_plan(curve, w)}
            leg["projected_scaling"] = project_msm_scaling(curve, args.bls_log_n, sw, hybrid)
        msm.close()
        if world == 1 and not args.no_cpu_baseline:
            # the reference's GPU-vs-CPU check (variable_base_msm_gpu_unittest.cc:25-78) at the timed
            # size: the oracle's kParallelTerm MSM of the same inputs on the host cores
            from oracle import oracle as O
            hb, hs = d_b.cpu().numpy(), d_s.cpu().numpy()
            t0 = time.perf_counter()
            leg["gpu_equals_cpu"] = O.msm_np(curve, hb, hs, method="parallel_term", threads=cpu_threads()) == res
            leg["cpu_seconds"] = round(time.perf_counter() - t0, 2)
            del hb, hs
        del d_b, d_s
        if world > 1:  # the sharded MSM must equal the unsharded one
            out[curve.split("_")[-1]]["consistent_with_1gpu"] = full_msm_equals(curve, n_total, res, rank, dist)
    out["workload"] = (f"BLS12-381 G1 and G2 VariableBaseMSM 2^{args.bls_log_n} (BASELINE configs[3]), "
                       f"device-resident inputs" + (f", {world} ranks (partition per curve) + all-gather of partials"
                                                    if world > 1 else ""))
    return out


# the in-register madd ceiling's field per curve (tachyon_mi355x_msm_madd_ceiling):
# BN254 G1 29-bit limbs, BLS12-381 G1 28-bit, the G2 lane pairs over the same limbs
CEILING_FIELD = {"bn254_g1": 29, "bls12_381_g1": 28, "bn254_g2": 29, "bls12_381_g2": 28}


def acc_kernel_name(curve, schedule):
    """The accumulation kernel the last run launched (rocprofv3's short name)."""
    if schedule["lane_pair"]:  # (G2; the BLS12-381 G2 run also reports the 28-bit field bit)
        return "seg_acc_pair_limb_kernel" if not curve.endswith("g1") else "seg_acc_kernel"
    if schedule["acc29"]:
        return "seg_acc29_kernel"
    if schedule["acc28"]:
        return "seg_acc28_kernel"
    return "seg_acc_kernel"


def msm_rooflines(msm, curve, d_b, d_s, n, point_bytes, reps=3):
    """HBM and VALU rooflines of an MSM's bucket accumulation (the dominant
    kernel), as the headline's: achieved = n x (affine base + 32-B scalar)
    algorithmic bytes / the kernel's HIP-event time; VALU = n x W mixed
    additions / that time against the in-register madd ceiling of the same
    field code measured in this run; traffic from the newest committed PMC
    passes that profiled this kernel (profiles/*/pmc_traffic.json)."""
    from tachyon_amd import msm as M
    msm.set_profile(True)
    prof = []
    for _ in range(reps):
        msm.run(d_b, d_s, n)
        prof.append(msm.last_timings())
    msm.set_profile(False)
    launches = max(1, int(prof[0]["acc_launches"]))
    acc_ms = sorted(p["acc"] for p in prof)[len(prof) // 2] / launches
    kernel = acc_kernel_name(curve, msm.last_schedule())
    c, windows = M.plan(curve, n)
    if msm.window_bits:
        from tachyon_amd import dist as D
        c, windows = msm.window_bits, D._windows_for(curve, msm.window_bits)
    algo = n / launches * (point_bytes + 32)
    gbs = algo / (acc_ms * 1e-3) / 1e9
    traffic, src, raw = pmc_traffic(kernel)
    gmadd = n * windows / launches / (acc_ms * 1e-3) / 1e9
    try:
        peak = msm.madd_ceiling(CEILING_FIELD[curve])
        peak_src = "measured in this run"
    except Exception as e:  # noqa: BLE001 -- a diagnostic
        peak, peak_src = 0.0, f"not measured ({e})"
    return {
        "phase_ms": {k: round(sorted(p[k] for p in prof)[len(prof) // 2], 4) for k in prof[0]},
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_unit": "GB per launch", "traffic_source": src,
                     "traffic_fetch_raw": raw, "kernel": kernel, "kernel_ms": acc_ms,
                     "algorithmic_bytes_per_launch": algo,
                     "note": f"n x ({point_bytes} B affine base + 32 B scalar) per launch / the accumulation's "
                             f"HIP-event time (SURVEY 8(d)'s per-point bytes for this group)"},
        "valu_roofline": {"bound": "valu", "kernel": kernel, "achieved": gmadd, "peak": peak,
                          "peak_source": peak_src, "unit": "G mixed additions/s",
                          "frac": (gmadd / peak) if peak else None, "window_bits": c, "windows": windows,
                          "note": "n x W mixed additions per launch / the launch's time; peak = the same field "
                                  "code's madd chain in registers (no gathers, no run logic), whole chip, this box"},
    }


def stream_copy_gbs(nbytes=1 << 31, reps=5):
    """On-box HBM peak reference: a device-to-device copy of
    nbytes, read + write bytes per second, best of reps (HIP events)."""
    import torch
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    dst.copy_(src)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del src, dst
    torch.cuda.empty_cache()
    return 2 * nbytes / (best * 1e-3) / 1e9


def full_msm_equals(curve, n_total, sharded, rank, dist):
    """Rank 0 runs the unsharded MSM of the same global input once; every rank
    learns whether the sharded result equals it."""
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd._lib import CURVE_INFO
    ok = 1
    if rank == 0:
        pb, sf = CURVE_INFO[curve]
        d_b = torch.empty(n_total * pb, dtype=torch.uint8, device="cuda")
        d_s = torch.empty(n_total * 32, dtype=torch.uint8, device="cuda")
        M.gen_bases(curve, SEED, n_total, 1 << 10, d_b.data_ptr())
        M.gen_scalars(sf, SEED, n_total, d_s.data_ptr())
        torch.cuda.synchronize()
        m = M.VariableBaseMSMGpu(curve)
        ok = int(m.run(d_b, d_s, n_total) == sharded)
        m.close()
        del d_b, d_s
        torch.cuda.empty_cache()
    t = torch.tensor([ok], dtype=torch.int32, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.broadcast(t, 0)
    return bool(t.item())


# xGMI figures for the N-GPU projections (MI355X_MICROARCH.md: 7 links x ~153 GB/s
# per GPU, taken as ~76 GB/s per direction per link) and a small-message RCCL
# all-gather latency; both are ASSUMPTIONS (no multi-GPU box here), every other
# term of a projection is measured in this run.
XGMI_LINK_GBS = 76.0
def hybrid_plan(curve, world):
    """(window groups Q, window bits c) of the hybrid point x window partition
    the LIBRARY runs for (curve, world) -- tachyon_mi355x_msm_shard_plan, the
    table of measured plans in capi.hip (BN254 G1 at 8 ranks, BLS12-381 G2 at
    4 and 8) -- or None where it keeps point shards."""
    from tachyon_amd import msm as M
    s = M.shard_plan(curve, 1 << 20, world, 0)
    return (s.window_groups, s.window_bits) if s.window_groups > 1 else None


def hybrid_plans():
    """{(curve, N): (Q, c)} of hybrid_plan over the curves and N = 2, 4, 8."""
    out = {}
    for curve in ("bn254_g1", "bn254_g2", "bls12_381_g1", "bls12_381_g2"):
        for world in (2, 4, 8):
            h = hybrid_plan(curve, world)
            if h:
                out[(curve, world)] = h
    return out


def msm_partition(args, curve, world, rank, n_total):
    """This rank's share of the MSM: (split, start, count, window range or None,
    c or 0, point groups, window groups, shard) -- auto: the library's plan
    (tachyon_mi355x_msm_shard_plan: point shards or the hybrid); forced point
    shards / hybrid (--window-groups, --window-bits) / window split.  `shard`
    is the tachyon_mi355x_msm_shard the library's sharded entry takes (None for
    the window split, which combines in Python)."""
    from tachyon_amd import dist as D
    from tachyon_amd import msm as M
    from tachyon_amd._lib import MsmShard
    split = args.msm_split
    if world == 1:
        split = "points"
    if split == "auto":
        s = M.shard_plan(curve, n_total, world, rank)
        if s.window_groups > 1:
            return ("hybrid", s.start, s.count, (s.w_begin, s.w_end), s.window_bits, s.point_groups,
                    s.window_groups, s)
        return "points", s.start, s.count, None, 0, world, 1, s
    if split == "points":
        start, n = D.shard_range(n_total, rank, world)
        return split, start, n, None, 0, world, 1, MsmShard(start, n, world, 1, 0, 0, 0)
    if split == "windows":
        c = args.window_bits or 16
        return split, 0, n_total, D.window_range(D._windows_for(curve, c), rank, world), c, 1, world, None
    q, c = args.window_groups, args.window_bits or (hybrid_plan(curve, world) or (0, 19))[1]
    q = max(1, min(q, world))
    p = world // q
    if p * q != world:
        raise SystemExit("--window-groups must divide the world size")
    start, n = D.shard_range(n_total, rank // q, p)
    w0, w1 = D.window_range(D._windows_for(curve, c), rank % q, q)
    return split, start, n, (w0, w1), c, p, q, MsmShard(start, n, p, q, c, w0, w1)


def lib_communicator(world, backend):
    """The library communicator the multi-rank legs exchange through
    (TACHYON_BENCH_COMM): rccl (default with the nccl backend) -- the
    library's own RCCL communicator over xGMI; host (default under gloo) --
    host-staged through this process group's collectives; torch -- none (the
    Python combine, tachyon_amd.dist).  Returns (LibComm or None, label)."""
    from tachyon_amd import dist as D
    if world == 1:
        return None, "single GPU"
    kind = os.environ.get("TACHYON_BENCH_COMM", "rccl" if backend == "nccl" else "host")
    if kind == "torch":
        return None, "torch.distributed (Python combine)"
    if kind == "rccl" and backend == "nccl":
        try:
            return D.LibComm.rccl(), "library rccl communicator"
        except Exception as e:  # noqa: BLE001 -- recorded in the line, the host-staged one stands in
            return D.LibComm.from_process_group(), f"library host-staged communicator (rccl init failed: {e})"
    return D.LibComm.from_process_group(), "library host-staged communicator"


def hybrid_rank_ms(msm, curve, d_bases, d_scalars, n_total, world, reps=3):
    """The slowest rank of hybrid_plan(curve, world) on this GPU: n/P points
    (a prefix of this run's input) over the first ceil(W/Q) c-bit windows."""
    from tachyon_amd import dist as D
    q, c = hybrid_plan(curve, world)
    m = n_total // (world // q)
    w1 = -(-D._windows_for(curve, c) // q)
    prev = getattr(msm, "window_bits", 0)
    msm.set_window_bits(c)
    try:
        msm.run_window_range(d_bases, d_scalars, 0, w1, m)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            msm.run_window_range(d_bases, d_scalars, 0, w1, m)
            ts.append(time.perf_counter() - t0)
    finally:
        msm.set_window_bits(prev)
    return round(sorted(ts)[len(ts) // 2] * 1e3, 3)
RCCL_SMALL_ALLGATHER_MS = 0.03


def combine_cost_ms(curve, world, reps=20):
    """Measured, on this GPU: the host side of D.sharded_msm's combine for
    `world` ranks -- the partial to a device tensor, the gathered N-point buffer
    back to the host, and the host group sum of N affine points (the RCCL
    collective itself is RCCL_SMALL_ALLGATHER_MS, assumed)."""
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd._lib import CURVE_INFO
    pb = CURVE_INFO[curve][0]
    g = torch.empty(world * pb, dtype=torch.uint8, device="cuda")
    M.gen_bases(curve, SEED + 9, world, 1, g.data_ptr())
    torch.cuda.synchronize()
    pts = g.cpu().numpy().tobytes()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        t = torch.frombuffer(bytearray(pts[:pb]), dtype=torch.uint8).to("cuda")
        g[:pb].copy_(t)
        blob = g.cpu().numpy().tobytes()
        M.affine_sum(curve, blob)
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def project_msm_scaling(curve, log_n, sweep, hybrid=None):
    """Projection of the 2^log_n MSM onto N = 2, 4, 8 GPUs from THIS run's
    single-GPU times: point shards (the 2^(log_n - log N) entries of the
    sweep, prefixes of the same input) or, where hybrid_plan has a plan for
    (curve, N), the hybrid partition's slowest rank (`hybrid[N]`, measured
    by hybrid_rank_ms) -- the partition --msm-split auto runs; per rank T +
    the combine (host side measured here + the assumed RCCL all-gather
    latency).  Efficiency = projected value / (N x the 1-GPU value)."""
    t1 = sweep[str(log_n)]["ms"]
    out = {"model": "t(N) = min(t_1gpu(2^log_n / N points), t_1gpu(hybrid rank)) (measured above) + combine "
                    f"(measured host side + {RCCL_SMALL_ALLGATHER_MS} ms assumed RCCL small all-gather)", "t1_ms": t1}
    for lg_world in (1, 2, 3):
        world = 1 << lg_world
        key = str(log_n - lg_world)
        if key not in sweep:
            continue
        comb = combine_cost_ms(curve, world) + RCCL_SMALL_ALLGATHER_MS
        t_points = sweep[key]["ms"]
        t_hybrid = (hybrid or {}).get(str(world))
        plan = hybrid_plan(curve, world)
        use_hybrid = t_hybrid is not None and plan is not None
        t = (t_hybrid if use_hybrid else t_points) + comb
        q, c = plan or (0, 0)
        out[f"n{world}"] = {"shard_log_n": log_n - lg_world, "shard_ms": t_points,
                            "hybrid_rank_ms": t_hybrid,
                            "plan": f"hybrid {world // q} point groups x {q} window groups, c = {c}"
                                    if use_hybrid else "point shards",
                            "combine_ms": round(comb, 4), "ms": round(t, 3),
                            "scalars_per_s": (1 << log_n) / (t * 1e-3), "efficiency": round(t1 / (world * t), 3)}
    return out


def project_ntt_scaling(log_n, t1_ms, reps=20):
    """Four-step projection of the 2^log_n NTT onto N = 2, 4, 8 GPUs: rank 0's
    two local stages of the N-rank plan timed on this GPU (tachyon_mi355x_bn254_ntt4,
    the same kernels the sharded bench runs) + the all-to-all as its per-pair
    bytes over one xGMI link (XGMI_LINK_GBS, assumed; pairs run in parallel on
    the N - 1 links) + RCCL_SMALL_ALLGATHER_MS of latency."""
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd.ntt import FourStepNtt
    out = {"model": f"t(N) = rank 0's local stages (measured) + n/N^2 x 32 B per pair at {XGMI_LINK_GBS} GB/s "
                    f"per xGMI link (assumed) + {RCCL_SMALL_ALLGATHER_MS} ms", "t1_ms": t1_ms}
    for world in (2, 4, 8):
        # the split with the fewest pass launches (2^24: 2^8 x 2^16, one packed
        # pass for the columns) -- local stages 0.282 / 0.545 ms at N = 8 / 4 vs
        # 0.299 / 0.562 for 2^12 x 2^12 (profiles/r05o/ntt4_probe.jsonl)
        plan = FourStepNtt(log_n, world, 0, log_r=FourStepNtt.split_log_r(log_n, world))
        m = plan.local_size
        x = torch.empty(m * 32, dtype=torch.uint8, device="cuda")
        y = torch.empty_like(x)
        M.gen_scalars("bn254_fr", SEED + 1, m, x.data_ptr())
        torch.cuda.synchronize()
        s = plan.torch_stream
        for _ in range(2):
            plan.run_stage(1, False, x, y)
            plan.run_stage(2, False, y, x)
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            plan.run_stage(1, False, x, y)
            plan.run_stage(2, False, y, x)
        s.synchronize()
        local = (time.perf_counter() - t0) / reps * 1e3
        plan.close()
        pair_bytes = (1 << log_n) // (world * world) * 32
        a2a = pair_bytes / (XGMI_LINK_GBS * 1e9) * 1e3 + RCCL_SMALL_ALLGATHER_MS
        t_split = local + a2a
        # the plan the bench (and the library's set_devices) runs: the split
        # where it projects faster than one GPU, else the single device
        split = t_split < t1_ms
        t = t_split if split else t1_ms
        out[f"n{world}"] = {"log_r": plan.log_r, "local_stages_ms": round(local, 4),
                            "all_to_all_ms_model": round(a2a, 4),
                            "split_ms": round(t_split, 4),
                            "plan": "four-step" if split else "single GPU (the split projects slower)",
                            "ms": round(t, 4), "elems_per_s": (1 << log_n) / (t * 1e-3),
                            "efficiency": round(t1_ms / (world * t), 3)}
        del x, y
    return out


def bench_groth16(args, rank=0, world=1, barrier=lambda: None, dist=None, backend=None, lib_comm=None):
    """Groth16 prove (witness map + 4 G1 MSMs + 1 G2 MSM, NoZK) on a synthetic
    2^k-constraint key; the witness is host memory as in prover_main.cc.  With
    N ranks (BASELINE configs[4] "1 and 8 GPUs") every rank runs the witness
    map and 1/N of every MSM, one all-gather exchanges the partials and every
    rank assembles the proof (Groth16Prover.prove_sharded)."""
    import torch
    from tachyon_amd.groth16 import Groth16Prover
    t0 = time.perf_counter()
    zkey, full = synth_groth16_zkey(args.groth16_log_n)
    prover = Groth16Prover(zkey)
    setup_s = time.perf_counter() - t0
    # the proving key's setup step: the fold tables of this rank's shard of the
    # fixed queries (memory-aware, tachyon_mi355x_groth16_prepare), timed apart
    t_fold = time.perf_counter()
    fold_bytes = prover.prepare(rank, world)
    fold_setup_s = time.perf_counter() - t_fold
    folds = prover.folds()

    def step():
        if world == 1:
            return prover.prove(full)
        if lib_comm is not None:  # partials, all-gather and assembly inside the library
            return prover.prove_sharded(full, comm=lib_comm)
        return prover.prove_sharded(full, device="cuda" if backend == "nccl" else None)

    t_first = time.perf_counter()
    ref = step()
    first_ms = (time.perf_counter() - t_first) * 1e3
    step()  # a second untimed proof: the first timed one still ran ~0.7 ms slow after one (profiles/r05k)
    reps = max(2, min(args.steps, 5))
    barrier()
    t0 = time.perf_counter()
    rep_ms = []
    for _ in range(reps):
        t_rep = time.perf_counter()
        proof = step()
        rep_ms.append((time.perf_counter() - t_rep) * 1e3)
    barrier()
    dt = (time.perf_counter() - t0) / reps
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if world == 1:
        prover.set_profile(True)
        prover.prove(full)
    else:  # this rank's phases of one sharded proof (witness map + its MSM shards)
        prover.set_profile(True)
        prover.prove_partials(full, rank, world)
    phases = {k: round(v, 3) for k, v in prover.last_timings().items()}
    if world > 1:  # the sharded proof must equal the single-GPU one
        consistent_1gpu = prover.prove(full) == proof
    equals_oracle = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import groth16 as OG  # checker only: the CPU restatement of the same proof
        equals_oracle = tuple(OG.prove_np(zkey, full)) == tuple(proof)
    out = {"ms_per_proof": dt * 1e3, "proofs_per_s": 1 / dt, "ms_per_proof_reps": [round(x, 3) for x in rep_ms],
           "constraints": 1 << args.groth16_log_n,
           "num_vars": prover.num_vars,
           "mode": "NoZK, host-resident witness, device-resident proving key with fixed-base fold tables "
                   "built in the key's setup step (prepare: up to 16 copies of the G2 B query and 4 of the "
                   "grouped G1 ones, as the device memory allows)",
           "first_proof_ms": round(first_ms, 1),
           "fold_setup_s": round(fold_setup_s, 3), "fold_table_bytes": fold_bytes, "folds": folds,
           "consistent": proof == ref, "equals_cpu_oracle": equals_oracle, "phase_ms": phases,
           "setup_s": round(setup_s, 1),
           "workload": f"synthetic circom zkey, 2^{args.groth16_log_n} constraints, 2+2 A/B terms per row "
                       f"(BASELINE configs[4] shape; seeded points, no trapdoor)"}
    if world == 1:
        out["msm_rooflines"] = groth16_msm_rooflines(prover, phases)
    if world > 1:
        out["consistent_with_1gpu"] = consistent_1gpu
        out["mode"] += f"; witness map on every rank, MSM point shards x{world} + one all-gather of partials"
    prover.close()
    return out


def groth16_msm_rooflines(prover, phases):
    """Per-MSM rooflines of one profiled proof (phase times are whole MSMs:
    recode, sort, accumulation and reduction on the host clock): the B-in-G2
    MSM over num_vars - 1 points (128 B base + 32 B scalar) and the grouped
    G1 MSM (A over num_vars - 1 points + the merged witness + h MSM over
    num_witness + n points, 64 + 32 B each); VALU = points x W mixed
    additions / the phase time against the madd ceilings of the same fields."""
    from tachyon_amd import msm as M
    m, npub, n = prover.num_vars, prover.num_public, prover.domain_size
    q = m - 1
    nlh = (m - npub - 1) + n
    out = {}
    for key, curve, points, pbytes, ms, lg_len in (
            ("b2_g2", "bn254_g2", q, 128, phases.get("msm_b2", 0.0), None),
            ("a_lh_g1_grouped", "bn254_g1", q + nlh, 64, phases.get("msm_a", 0.0), max(q, (nlh + 1) // 2))):
        if not ms or points <= 0:
            continue
        if lg_len is None:
            c, W = M.plan(curve, points)
        else:  # run_groups' window bits (MsmGpu::batch_window_bits) over glen-point groups
            lg = max(1, (lg_len - 1).bit_length())
            c = max(M.plan(curve, lg_len)[0], min(lg + 1, 8) if lg <= 13 else 10)
            W = -(-255 // c)
        gbs = points * (pbytes + 32) / (ms * 1e-3) / 1e9
        gmadd = points * W / (ms * 1e-3) / 1e9
        ctx = M.VariableBaseMSMGpu(curve)
        try:
            peak = ctx.madd_ceiling(CEILING_FIELD[curve])
        finally:
            ctx.close()
        out[key] = {"points": points, "ms": ms, "window_bits": c, "windows": W,
                    "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": gbs / HBM_PEAK_GBS},
                    "valu_roofline": {"bound": "valu", "achieved": gmadd, "peak": peak,
                                      "unit": "G mixed additions/s", "frac": gmadd / peak if peak else None}}
    out["note"] = ("whole-MSM phase times of one profiled proof (host clock; the fold tables cut the window "
                   "sums, not the n x W additions), so these fractions sit below the accumulation kernel's own")
    return out


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    # one process per GPU; TACHYON_DIST_BACKEND=gloo rehearses the multi-rank
    # path with several ranks on one GPU (host-staged collectives)
    backend = os.environ.get("TACHYON_DIST_BACKEND", "nccl")
    device_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device_index)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device_index))
        else:
            dist.init_process_group(backend)

    from tachyon_amd import msm as M
    from tachyon_amd._lib import lib

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- MSM inputs (device-resident, this rank's shard) ----
    from tachyon_amd import dist as D
    n_total = 1 << args.log_n
    # N > 1: point shards of one global input (each rank n/N points, all W
    # windows; default) or the window split (each rank all n points, W/N of
    # W = 16 windows) -- per-rank cost at 2^26 / 8 ranks 14.4 vs 16.2 ms: the
    # split's recode of all n scalars per rank and its 2 x 2^26 additions
    # (vs 15 x 2^23 at the shard's c = 17) outweigh the smaller bucket set.
    # The hybrid (N/Q point groups x Q window groups, hybrid_plan) sits
    # between: 2^24 points over 7 of 14 windows per rank at N = 8, 11.45 vs
    # 12.11 ms for the point shard (profiles/r05c), so auto runs it at 8 GPUs
    split, start, n, wrange, split_c, p_groups, q_groups, shard = msm_partition(args, "bn254_g1", world, rank,
                                                                                   n_total)
    d_bases = torch.empty(max(1, n) * 64, dtype=torch.uint8, device="cuda")
    d_scalars = torch.empty(max(1, n) * 32, dtype=torch.uint8, device="cuda")
    chunk = 1 << 10
    # this rank's slice [start, start + n) of ONE seeded global input
    M.gen_bases("bn254_g1", SEED, n, chunk, d_bases.data_ptr(), start=start)
    M.gen_scalars("bn254_fr", SEED, n, d_scalars.data_ptr(), start=start)
    torch.cuda.synchronize()

    msm = M.VariableBaseMSMGpu("bn254_g1")
    if wrange is not None:
        w_lo, w_hi = wrange
        msm.set_window_bits(split_c)
    elif args.window_bits:
        msm.set_window_bits(args.window_bits)

    def local_run():
        if split in ("windows", "hybrid"):
            return msm.run_window_range(d_bases, d_scalars, w_lo, w_hi, n)
        return msm.run(d_bases, d_scalars, n)

    # N > 1: the library's sharded entry over a library communicator -- this
    # rank's part of the partition (point shard or hybrid point group x window
    # range), the all-gather of the partials and their group sum inside
    # libtachyon_mi355x (tachyon_mi355x_msm_gpu_sharded_plan_affine); RCCL by
    # default (lib_communicator); the window split and TACHYON_BENCH_COMM=torch
    # combine in Python (tachyon_amd.dist)
    lib_comm, comm_label = lib_communicator(world, backend)

    def step():
        if split == "windows":
            return D.window_split_msm("bn254_g1", msm, d_bases, d_scalars, n, split_c, device="cuda")
        if lib_comm is not None:
            return msm.run_sharded_plan(lib_comm, shard, d_bases, d_scalars)
        return D.sharded_msm("bn254_g1", local_run, device="cuda")

    for _ in range(args.warmup):
        ref = step()
    barrier()
    t0 = time.perf_counter()
    results = [step() for _ in range(args.steps)]
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    consistent = all(r == results[0] for r in results) and (args.warmup == 0 or results[0] == ref)
    ms_per_step = elapsed / args.steps * 1e3
    value = n_total / (elapsed / args.steps)
    consistent_1gpu = full_msm_equals("bn254_g1", n_total, results[0], rank, dist) if world > 1 else None

    # ---- dominant-kernel timing (HIP events on the MSM stream) ----
    msm.set_profile(True)
    prof = []
    for _ in range(3):
        local_run()
        prof.append(msm.last_timings())
    msm.set_profile(False)
    phases = {k: round(sorted(p[k] for p in prof)[1], 4) for k in prof[0]}
    launches = max(1, int(prof[0]["acc_launches"]))
    acc_ms = sorted(p["acc"] for p in prof)[1] / launches
    c, windows = M.plan("bn254_g1", n)
    rank_windows = windows
    if split in ("windows", "hybrid"):
        c, windows = split_c, D._windows_for("bn254_g1", split_c)
        rank_windows = w_hi - w_lo
    elif args.window_bits:
        c, windows = args.window_bits, D._windows_for("bn254_g1", args.window_bits)
        rank_windows = windows
    # the algorithmic bytes of the MSM are its inputs read once,
    # 96 B per point (64 B affine base + 32 B scalar); one launch covers all n
    # points of this rank (all windows), so achieved = n x 96 B / launch time.
    # The (point, window) gathers the kernel actually performs (W x 64 B bases
    # + 8 B sorted entries per point) are reported beside it as gather_gbs.
    points_per_launch = n / launches
    acc_gbs = points_per_launch * MSM_BYTES_PER_POINT / (acc_ms * 1e-3) / 1e9
    units = n * rank_windows / launches  # mixed additions (point, window) per launch
    gather_gbs = units * (64 + 8) / (acc_ms * 1e-3) / 1e9
    acc_kernel = "seg_acc29_kernel" if msm.last_schedule()["acc29"] else "seg_acc_kernel"
    acc_traffic, acc_traffic_src, acc_traffic_raw = pmc_traffic(acc_kernel)
    acc_gmadd = units / (acc_ms * 1e-3) / 1e9
    try:
        madd_peak = msm.madd_ceiling(29 if acc_kernel == "seg_acc29_kernel" else 32) or MADD_PEAK_G[acc_kernel]
        madd_peak_src = "measured in this run"
    except Exception:  # noqa: BLE001 -- a diagnostic; the committed figure stands in
        madd_peak, madd_peak_src = MADD_PEAK_G[acc_kernel], "profiles/r03c/madd_rates.log"
    stream_gbs = stream_copy_gbs()

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "scalars/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: seeded splitmix64 scalars (BigInt::Random halving, Montgomery form) and k*G "
                "doubling-chain bases (test/random.h scheme), generated on the device",
        "config": {"workload": f"BN254 G1 VariableBaseMSM 2^{args.log_n} (BASELINE configs[1]), device-resident "
                               f"inputs, result normalised to affine on the host",
                   "msm_log_n": args.log_n, "points_per_gpu": n, "window_bits": c, "windows": windows,
                   "windows_per_gpu": rank_windows,
                   "parallelism": (f"msm window ranges x{world} (every rank all points, {rank_windows} of {windows} "
                                   f"windows) + RCCL all-gather of partial points" if split == "windows" else
                                   f"msm point groups x{p_groups} x window groups x{q_groups} ({rank_windows} of "
                                   f"{windows} windows per rank) + RCCL all-gather of partial points"
                                   if split == "hybrid" else
                                   f"msm point shards x{world} + RCCL all-gather of partial points")
                                  + (f"; exchange: {comm_label}" if world > 1 else ""),
                   "communicator": (lib_comm.backend if lib_comm else comm_label)},
        "consistent_across_steps": consistent,
        "consistent_with_1gpu": consistent_1gpu,
        "roofline": {"bound": "hbm", "achieved": acc_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": acc_gbs / HBM_PEAK_GBS,
                     "traffic": acc_traffic, "traffic_unit": "GB per launch", "traffic_source": acc_traffic_src,
                     "traffic_fetch_raw": acc_traffic_raw,
                     "traffic_correction": "FETCH_SIZE x2 (the guide's factor for wide coalesced streaming reads) "
                                           "+ WRITE_SIZE; the 64-B base gathers are an uncalibrated width, so the "
                                           "uncorrected FETCH_SIZE is given as traffic_fetch_raw",
                     "pmc_gbs": (acc_traffic / (acc_ms * 1e-3)) if acc_traffic else None,
                     "kernel": f"{acc_kernel} (bucket accumulation)", "kernel_ms": acc_ms,
                     "launches_per_msm": launches, "points_per_launch": points_per_launch,
                     "algorithmic_bytes_per_launch": points_per_launch * MSM_BYTES_PER_POINT,
                     "gather_gbs": gather_gbs, "gathers_per_launch": units,
                     "stream_copy_gbs": stream_gbs, "frac_of_stream_copy": acc_gbs / stream_gbs,
                     "note": "algorithmic bytes = SURVEY 8(d)'s 96 B per point (base + scalar read once) x the n "
                             "points one launch covers / the launch's HIP-event time; gather_gbs = the W x (64 B "
                             "base + 8 B entry) per point the kernel gathers; the kernel is VALU-bound "
                             "(valu_roofline), see DESIGN.md; peak = the guide's nominal 8 TB/s, "
                             "stream_copy_gbs = a device-to-device copy measured on this box"},
        "msm_phase_ms": phases,
        "valu_roofline": {"bound": "valu", "kernel": acc_kernel, "achieved": acc_gmadd,
                          "peak": madd_peak, "peak_source": madd_peak_src, "unit": "G mixed additions/s",
                          "frac": acc_gmadd / madd_peak,
                          "note": "n x windows mixed additions per launch / launch time; peak = " + MADD_PEAK_NOTE},
    }

    # ---- configs[1] sweep (2^16, 2^20 .. 2^25: prefixes of the same device-resident input; 2^25 / 2^24 /
    # 2^23 are the per-rank shards of the 2^26 MSM at N = 2 / 4 / 8, priced in projected_scaling) ----
    if world == 1 and args.log_n >= 24 and not args.no_sweep:
        sweep = {}
        for k in (16, 20, 21, 22, 23, 24, 25):
            if k >= args.log_n:
                continue
            m = 1 << k
            msm.run(d_bases, d_scalars, m)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                msm.run(d_bases, d_scalars, m)
                ts.append(time.perf_counter() - t0)
            best = sorted(ts)[2]
            sweep[str(k)] = {"ms": round(best * 1e3, 3), "scalars_per_s": m / best}
        sweep[str(args.log_n)] = {"ms": round(ms_per_step, 3), "scalars_per_s": value}
        out["msm_sweep"] = sweep
        # the hybrid partition's slowest rank where auto runs it (the library's
        # plan: N = 8, 4 point groups x 2 window groups at c = 19)
        hybrid = {str(w): hybrid_rank_ms(msm, "bn254_g1", d_bases, d_scalars, 1 << args.log_n, w)
                  for w in (2, 4, 8) if hybrid_plan("bn254_g1", w)}
        out["projected_scaling"] = {"msm": project_msm_scaling("bn254_g1", args.log_n, sweep, hybrid)}

    # ---- NonUniform(n, 1) test set (variable_base_msm_test_set.h:43-53), the set of the reference's
    # published GPU table (benchmark/msm/README.md:97-111): every scalar equal, so every window puts
    # all of this rank's points into ONE bucket (the skew path of the load-balanced accumulation) ----
    if not args.no_non_uniform:
        one = torch.empty(32, dtype=torch.uint8, device="cuda")
        M.gen_scalars("bn254_fr", SEED + 3, 1, one.data_ptr())
        d_nu = one.repeat(max(1, n))
        torch.cuda.synchronize()

        def nu_step():  # the same partition and exchange as the headline step
            if split == "windows":
                return D.window_split_msm("bn254_g1", msm, d_bases, d_nu, n, split_c, device="cuda")
            if lib_comm is not None:
                return msm.run_sharded_plan(lib_comm, shard, d_bases, d_nu)
            if split == "hybrid":
                return D.sharded_msm("bn254_g1", lambda: msm.run_window_range(d_bases, d_nu, w_lo, w_hi, n),
                                     device="cuda")
            return D.sharded_msm("bn254_g1", lambda: msm.run(d_bases, d_nu, n), device="cuda")

        nu_ref = nu_step()
        reps = max(2, min(args.steps, 3))
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            nu_res = nu_step()
        barrier()
        dt = (time.perf_counter() - t0) / reps
        if dist is not None:
            t = torch.tensor([dt], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out["non_uniform"] = {"ms_per_msm": dt * 1e3, "scalars_per_s": n_total / dt,
                              "vs_random_set": dt * 1e3 / ms_per_step, "consistent": nu_res == nu_ref,
                              "workload": f"BN254 G1 MSM 2^{args.log_n}, NonUniform(n, 1): one seeded scalar "
                                          f"repeated (benchmark/msm --test_set non_uniform), device-resident"}
        msm.set_profile(True)
        msm.run(d_bases, d_nu, n)
        out["non_uniform"]["phase_ms"] = {k: round(v, 4) for k, v in msm.last_timings().items()}
        msm.set_profile(False)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle import oracle as O
            t0 = time.perf_counter()
            out["non_uniform"]["gpu_equals_cpu"] = O.msm_np(
                "bn254_g1", d_bases.cpu().numpy(), d_nu.cpu().numpy(), method="parallel_term",
                threads=cpu_threads()) == nu_res
            out["non_uniform"]["cpu_seconds"] = round(time.perf_counter() - t0, 2)
        del d_nu

    # ---- NTT 2^24: one GPU, or the four-step sharded transform (one RCCL all-to-all) ----
    # Two ranks: the four-step exchanges n/4 elements over ONE xGMI link (134 MB
    # at 2^24), which costs more than the whole transform on one GPU
    # (projected_scaling.ntt; the library's set_devices applies the same rule),
    # so the transform runs on rank 0 alone; from four ranks the exchange
    # spreads over several links and the split pays.
    if not args.no_ntt and world == 2:
        from tachyon_amd.ntt import Radix2EvaluationDomain
        nn = 1 << args.ntt_log_n
        reps = max(2, args.steps)
        dt_local, ok_local = 0.0, 1
        if rank == 0:
            dom = Radix2EvaluationDomain(nn)
            x = torch.empty(nn * 32, dtype=torch.uint8, device="cuda")
            M.gen_scalars("bn254_fr", SEED + 1, nn, x.data_ptr())
            torch.cuda.synchronize()
            orig = x.clone()
            for _ in range(2):
                dom.transform_device(x.data_ptr(), inverse=False)
                dom.transform_device(x.data_ptr(), inverse=True)
            torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        if rank == 0:
            for _ in range(reps):
                dom.transform_device(x.data_ptr(), inverse=False)
                dom.transform_device(x.data_ptr(), inverse=True)
            torch.cuda.synchronize()
        barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item()) / (2 * reps)
        if rank == 0:
            ok_local = 1 if torch.equal(x, orig) else 0
            dom.close()
        ok = torch.tensor([ok_local], dtype=torch.int32, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        out["ntt"] = {"value": nn / dt, "unit": "elems/s", "log_n": args.ntt_log_n, "ms_per_transform": dt * 1e3,
                      "round_trip_ok": bool(ok.item()), "scaling": "strong",
                      "mode": "single GPU (rank 0): a 2-rank four-step would exchange "
                              f"{nn * 32 // 4} B over one xGMI link, projected slower than one GPU"}
    if not args.no_ntt and world > 2:
        from tachyon_amd.ntt import FourStepNtt
        # its own stream (sharded_ntt orders on it); the split with the fewest passes
        plan = FourStepNtt(args.ntt_log_n, world, rank, log_r=FourStepNtt.split_log_r(args.ntt_log_n, world))
        m = plan.local_size
        x = torch.empty(m * 32, dtype=torch.uint8, device="cuda")
        M.gen_scalars("bn254_fr", SEED + 1, m, x.data_ptr(), start=rank * m)
        torch.cuda.synchronize()
        orig = x.clone()
        y = torch.empty_like(x)

        def round_trip(x):
            if lib_comm is not None:  # stage 1, the all-to-all, stage 2 inside the library (tachyon_mi355x_bn254_ntt4_run)
                plan.run(lib_comm, x, y)
                plan.run(lib_comm, y, x, inverse=True)
                return x
            return D.sharded_ntt(plan, D.sharded_ntt(plan, x), inverse=True)

        for _ in range(2):
            x = round_trip(x)
        reps = max(2, args.steps)
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            x = round_trip(x)
        barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                         device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item()) / (2 * reps)
        ok = torch.tensor([1 if torch.equal(x, orig) else 0], dtype=torch.int32,
                          device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        nn = 1 << args.ntt_log_n
        out["ntt"] = {"value": nn / dt, "unit": "elems/s", "log_n": args.ntt_log_n, "ms_per_transform": dt * 1e3,
                      "round_trip_ok": bool(ok.item()), "scaling": "strong",
                      "mode": f"four-step sharded x{world}: local R/C-point NTTs (R = 2^{plan.log_r}) + one "
                              f"all-to-all ({nn * 32 // world // world} B per rank pair); exchange: {comm_label}"}
        plan.close()

    if not args.no_ntt and world == 1:
        from tachyon_amd.ntt import Radix2EvaluationDomain
        nn = 1 << args.ntt_log_n
        dom = Radix2EvaluationDomain(nn)
        x = torch.empty(nn * 32, dtype=torch.uint8, device="cuda")
        M.gen_scalars("bn254_fr", SEED + 1, nn, x.data_ptr())
        torch.cuda.synchronize()
        orig = x.clone()
        s = torch.cuda.ExternalStream(dom.stream)
        for _ in range(2):
            dom.transform_device(x.data_ptr(), inverse=False)
            dom.transform_device(x.data_ptr(), inverse=True)
        torch.cuda.synchronize()
        reps = max(2, args.steps)
        t0 = time.perf_counter()
        for _ in range(reps):
            dom.transform_device(x.data_ptr(), inverse=False)
            dom.transform_device(x.data_ptr(), inverse=True)
        s.synchronize()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (2 * reps)
        round_trip_ok = bool(torch.equal(x, orig))
        # forward-only and inverse-only loops (back to back on the domain's
        # stream, wall time / transform): the rooflines' denominator is the
        # forward loop's time, not the profile-mode events (which add an event
        # record between passes)
        y = x.clone()
        torch.cuda.synchronize()
        dir_ms = {}
        dir_reps = max(10, args.steps)
        for inv in (False, True):
            for _ in range(2):  # untimed: the first launches after the idle host sync run slow
                dom.transform_device(y.data_ptr(), inverse=inv)
            s.synchronize()
            t0 = time.perf_counter()
            for _ in range(dir_reps):
                dom.transform_device(y.data_ptr(), inverse=inv)
            s.synchronize()
            dir_ms["inverse" if inv else "forward"] = (time.perf_counter() - t0) / dir_reps * 1e3
        del y
        dom.set_profile(True)
        dom.transform_device(x.data_ptr(), inverse=False)
        s.synchronize()
        tot, passes = dom.last_timings()
        dom.set_profile(False)
        dom.transform_device(x.data_ptr(), inverse=True)  # back to orig
        s.synchronize()
        ntt_in = orig.cpu().numpy()
        dom.transform_device(x.data_ptr(), inverse=False)
        s.synchronize()
        ntt_gpu_out = x.cpu().numpy()  # FFT of the input
        fwd_ms = dir_ms["forward"]
        # 64 B per element per TRANSFORM (read + write the array
        # once), over the timed forward transform (all passes + launch gaps)
        xform_gbs = nn * NTT_BYTES_PER_ELEM / (fwd_ms * 1e-3) / 1e9
        # pass shares from the profile events, applied to the timed transform
        share = [p / sum(passes) for p in passes]
        pass_ms_timed = [round(fwd_ms * f, 4) for f in share]
        avg_pass = fwd_ms / len(passes)
        pass_gbs = nn * NTT_BYTES_PER_ELEM / (avg_pass * 1e-3) / 1e9
        ntt_traffic, ntt_traffic_src, _ = pmc_traffic("dif_pass_kernel")
        # algorithmic butterflies (one product each) per transform: n/2 x log n
        ntt_gmulmod = nn // 2 * args.ntt_log_n / (fwd_ms * 1e-3) / 1e9
        out["ntt"] = {"value": nn / dt, "unit": "elems/s", "log_n": args.ntt_log_n, "ms_per_transform": dt * 1e3,
                      "ms_forward": round(fwd_ms, 4), "ms_inverse": round(dir_ms["inverse"], 4),
                      "round_trip_ok": round_trip_ok, "pass_ms_events": passes, "pass_ms": pass_ms_timed,
                      "mode": "single GPU",
                      "roofline": {"bound": "hbm", "achieved": xform_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": xform_gbs / HBM_PEAK_GBS, "traffic": ntt_traffic,
                                   "traffic_unit": "GB per dif_pass_kernel launch",
                                   "traffic_source": ntt_traffic_src,
                                   "kernel": "dif_pass_kernel (all passes of one forward transform)",
                                   "transform_ms": fwd_ms, "passes": len(passes), "kernel_ms": avg_pass,
                                   "per_pass_gbs": pass_gbs,
                                   "note": "algorithmic bytes = SURVEY 8(d)'s 64 B per element per transform / the "
                                           "timed forward transform (back-to-back loop, wall / transform); "
                                           "per_pass_gbs prices one pass's own read + write at the average pass",
                                   "stream_copy_gbs": stream_gbs, "frac_of_stream_copy": xform_gbs / stream_gbs},
                      "valu_roofline": {"bound": "valu", "kernel": "dif_pass_kernel", "achieved": ntt_gmulmod,
                                        "peak": MULMOD_PEAK_G, "unit": "G mulmod/s",
                                        "frac": ntt_gmulmod / MULMOD_PEAK_G,
                                        "note": "n/2 x log n butterflies per forward transform / its timed ms, "
                                                "one product each (the add/sub of a butterfly are not counted); "
                                                "peak = " + MULMOD_PEAK_NOTE}}
        if not args.no_sweep and "projected_scaling" in out:
            out["projected_scaling"]["ntt"] = project_ntt_scaling(args.ntt_log_n, dt * 1e3)
        if not args.no_host_resident:
            # reference semantics (fft_runner.h:53-58): host vector in, H2D + transform + D2H
            hv = ntt_in.copy()
            dom.transform_host(hv)
            same = hv.tobytes() == ntt_gpu_out.tobytes()
            ts = []
            for _ in range(3):
                hv[:] = ntt_in
                t0 = time.perf_counter()
                dom.transform_host(hv)
                ts.append(time.perf_counter() - t0)
            out["ntt"]["host_resident"] = {"value": nn / min(ts), "unit": "elems/s", "ms": min(ts) * 1e3,
                                           "ms_median": sorted(ts)[1] * 1e3, "equals_device_path": same,
                                           "path": "IcicleNTT::Run semantics on a pageable host vector "
                                                   "(..._evaluation_domain_transform_host)"}
        dom.close()
        # configs[2] sweep: 2^20 and 2^22 on prefixes of the same input (forward + inverse per rep)
        nsweep = {}
        for k in (20, 22):
            if k >= args.ntt_log_n or args.no_sweep:
                continue
            m = 1 << k
            dk = Radix2EvaluationDomain(m)
            sk = torch.cuda.ExternalStream(dk.stream)
            y = x[:m * 32].clone()
            torch.cuda.synchronize()
            dk.transform_device(y.data_ptr(), inverse=False)
            dk.transform_device(y.data_ptr(), inverse=True)
            sk.synchronize()
            reps_k = 10
            t0 = time.perf_counter()
            for _ in range(reps_k):
                dk.transform_device(y.data_ptr(), inverse=False)
                dk.transform_device(y.data_ptr(), inverse=True)
            sk.synchronize()
            dtk = (time.perf_counter() - t0) / (2 * reps_k)
            nsweep[str(k)] = {"ms": round(dtk * 1e3, 4), "elems_per_s": m / dtk,
                              "round_trip_ok": bool(torch.equal(y, x[:m * 32]))}
            dk.close()
        nsweep[str(args.ntt_log_n)] = {"ms": round(dt * 1e3, 4), "elems_per_s": nn / dt}
        out["ntt"]["sweep"] = nsweep

    if args.bls_log_n:
        out["bls12_381"] = bench_bls(args, rank, world, barrier, dist, backend, lib_comm)

    if args.groth16_log_n:
        out["groth16"] = bench_groth16(args, rank, world, barrier, dist, backend, lib_comm)

    h_bases = h_scalars = None
    if world == 1 and not (args.no_host_resident and args.no_cpu_baseline):
        h_bases, h_scalars = d_bases.cpu().numpy(), d_scalars.cpu().numpy()
    if world == 1 and not args.no_host_resident:
        # reference semantics (msm_runner.h:54-58): pageable host vectors through
        # tachyon_bn254_g1_affine_msm_gpu, H2D + kernels + D2H inside the call
        jac = msm.run_jacobian(h_bases, h_scalars, n)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            msm.run_jacobian(h_bases, h_scalars, n)
            ts.append(time.perf_counter() - t0)
        out["host_resident"] = {"value": n_total / min(ts), "unit": "scalars/s", "ms": min(ts) * 1e3,
                                "ms_median": sorted(ts)[1] * 1e3,
                                "equals_device_path": M.jacobian_to_affine("bn254_g1", jac) == results[0],
                                "path": "tachyon_bn254_g1_affine_msm_gpu on pageable host vectors "
                                        "(reference C-ABI, H2D inside the timed call)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        nb, ns = h_bases, h_scalars
        if args.cpu_log_n and args.cpu_log_n < args.log_n:
            nb, ns = h_bases[:(1 << args.cpu_log_n) * 64], h_scalars[:(1 << args.cpu_log_n) * 32]
        gpu_point = results[0] if nb is h_bases else msm.run(nb, ns)
        nin = ntt_in if not args.no_ntt else None
        nout = ntt_gpu_out if not args.no_ntt else None
        out["cpu_baseline"] = cpu_baseline(args, nb, ns, gpu_point, nin, nout)

    if rank == 0:
        print(json.dumps(out), flush=True)
    msm.close()
    if lib_comm is not None:
        lib_comm.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
