#!/usr/bin/env python3
"""A/B probe of the BN254 Fr NTT pass kernels in one process: forward (and
inverse) transforms of 2^log_n device-resident elements per domain variant
(0 = the 9 x 29-bit-limb passes, 1 = the 8 x 32-bit ones), wall ms per
transform and the profile-event pass times; every variant's output checked
against the first one.  Used under rocprofv3 for the kernel trace and PMC passes.

  python tools/ntt_probe.py [--log-n 24] [--reps 10] [--variants 0,1] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0,1,3")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd.ntt import Radix2EvaluationDomain
    n = 1 << args.log_n
    x0 = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_scalars("bn254_fr", 0x5EED, n, x0.data_ptr())
    torch.cuda.synchronize()
    variants = [int(v) for v in args.variants.split(",")]
    doms = {}
    for v in variants:
        d = Radix2EvaluationDomain(n)
        d.set_variant(v)
        doms[v] = d
    ref = None
    for rnd in range(args.rounds):
        for v in variants:
            d = doms[v]
            s = torch.cuda.ExternalStream(d.stream)
            x = x0.clone()
            torch.cuda.synchronize()
            d.transform_device(x.data_ptr(), inverse=False)
            s.synchronize()
            out = x.clone()
            if ref is None:
                ref = out
            same = bool(torch.equal(out, ref))
            res = {"variant": v, "round": rnd, "log_n": args.log_n, "equal": same}
            for inv in (False, True):
                t0 = time.perf_counter()
                for _ in range(args.reps):
                    d.transform_device(x.data_ptr(), inverse=inv)
                s.synchronize()
                res["inverse_ms" if inv else "forward_ms"] = round((time.perf_counter() - t0) / args.reps * 1e3, 4)
            d.set_profile(True)
            d.transform_device(x.data_ptr(), inverse=False)
            s.synchronize()
            _, passes = d.last_timings()
            d.set_profile(False)
            res["pass_ms"] = [round(p, 4) for p in passes]
            print(json.dumps(res), flush=True)
    for d in doms.values():
        d.close()


if __name__ == "__main__":
    main()
