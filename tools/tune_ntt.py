#!/usr/bin/env python3
"""NTT pass timing (device-resident, HIP events per pass) for A/B runs.

  TACHYON_NTT_RADIX_LOG=3 python tools/tune_ntt.py --log-n 20 24
(the TACHYON_NTT_* overrides exist only in a tuning build of the library:
 make -C tachyon_amd/csrc EXTRA_CXXFLAGS=-DTACHYON_TUNING_KNOBS)
Prints per-pass device ms and the per-transform wall time; checks the round trip.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, nargs="+", default=[24])
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd.ntt import Radix2EvaluationDomain
    for lg in args.log_n:
        n = 1 << lg
        dom = Radix2EvaluationDomain(n)
        x = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        M.gen_scalars("bn254_fr", 5, n, x.data_ptr())
        torch.cuda.synchronize()
        orig = x.clone()
        s = torch.cuda.ExternalStream(dom.stream)
        for _ in range(2):
            dom.transform_device(x.data_ptr(), inverse=False)
            dom.transform_device(x.data_ptr(), inverse=True)
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            dom.transform_device(x.data_ptr(), inverse=False)
            dom.transform_device(x.data_ptr(), inverse=True)
        s.synchronize()
        dt = (time.perf_counter() - t0) / (2 * args.reps)
        ok = bool(torch.equal(x, orig))
        dom.set_profile(True)
        dom.transform_device(x.data_ptr(), inverse=False)
        _, passes = dom.last_timings()
        dom.set_profile(False)
        print(json.dumps({"log_n": lg, "radix_log": os.environ.get("TACHYON_NTT_RADIX_LOG", "default"),
                          "pass_stages": os.environ.get("TACHYON_NTT_PASS_STAGES", "default"),
                          "lds_elems": os.environ.get("TACHYON_NTT_LDS_ELEMS", "default"),
                          "ms_per_transform": round(dt * 1e3, 4), "pass_ms": [round(p, 4) for p in passes],
                          "round_trip_ok": ok}), flush=True)
        dom.close()


if __name__ == "__main__":
    main()
