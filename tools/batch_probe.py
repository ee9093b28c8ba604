#!/usr/bin/env python3
"""Batched MSM (tachyon_mi355x_msm_gpu_batch_affine) against the same MSMs one
by one: `count` MSMs of 2^log_len points over shared device bases, wall ms of
each way (the KZG batch-commitment shape).

  python tools/batch_probe.py [--log-len 12 14 16] [--count 8 32] [--reps 5] [--c 0 9 11]

--c: the batch's window bits to time (0 = run_batch's own choice), one
"batch_ms_c" entry each; the separate MSMs always take their default.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-len", type=int, nargs="+", default=[12, 14, 16])
    ap.add_argument("--count", type=int, nargs="+", default=[8, 32])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--curve", default="bn254_g1")
    ap.add_argument("--c", type=int, nargs="+", default=[0])
    args = ap.parse_args()
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd._lib import CURVE_INFO
    pb, sf = CURVE_INFO[args.curve]
    m = M.VariableBaseMSMGpu(args.curve)
    for lg in args.log_len:
        n = 1 << lg
        d_b = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
        M.gen_bases(args.curve, 1, n, 1024, d_b.data_ptr())
        for count in args.count:
            d_s = torch.empty(n * count * 32, dtype=torch.uint8, device="cuda")
            M.gen_scalars(sf, 2, n * count, d_s.data_ptr())
            torch.cuda.synchronize()
            batch = m.run_batch(d_b, d_s, n, count)  # warm
            one = [m.run(d_b, d_s[g * n * 32:(g + 1) * n * 32], n) for g in range(count)]
            tbc = {}
            for c in args.c:
                m.set_window_bits(c)
                ok = m.run_batch(d_b, d_s, n, count) == one
                t0 = time.perf_counter()
                for _ in range(args.reps):
                    m.run_batch(d_b, d_s, n, count)
                tbc[c] = (round((time.perf_counter() - t0) / args.reps * 1e3, 3), ok)
            m.set_window_bits(0)
            tb = tbc[args.c[0]][0]
            t0 = time.perf_counter()
            for _ in range(args.reps):
                for g in range(count):
                    m.run(d_b, d_s[g * n * 32:(g + 1) * n * 32], n)
            ts = (time.perf_counter() - t0) / args.reps * 1e3
            print(json.dumps({"curve": args.curve, "log_len": lg, "count": count, "batch_ms": round(tb, 3),
                              "separate_ms": round(ts, 3), "equal": batch == one,
                              "batch_ms_c": tbc}), flush=True)
    m.close()


if __name__ == "__main__":
    main()
