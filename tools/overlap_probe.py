#!/usr/bin/env python3
"""Probe: does one MSM's sort overlap another MSM's accumulation for free?

Two point halves of a 2^L MSM on two contexts (two HIP streams): run one
after the other, then concurrently from two host threads with the second
started `--delay-ms` later (so its recode/sort lands on the first one's
accumulation).  Prints wall times; the sum of the two half results must equal
the whole MSM either way.
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=26)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--delay-ms", type=float, nargs="+", default=[0.0, 5.0, 10.0])
    args = ap.parse_args()
    import torch
    from tachyon_amd import msm as M
    n = 1 << args.log_n
    h = n // 2
    d_b = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases("bn254_g1", 1, n, 1024, d_b.data_ptr())
    M.gen_scalars("bn254_fr", 1, n, d_s.data_ptr())
    torch.cuda.synchronize()
    whole = M.VariableBaseMSMGpu("bn254_g1")
    ref = whole.run(d_b, d_s)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        whole.run(d_b, d_s)
    t_whole = (time.perf_counter() - t0) / args.reps * 1e3
    whole.close()
    ma, mb = M.VariableBaseMSMGpu("bn254_g1"), M.VariableBaseMSMGpu("bn254_g1")
    halves = [(d_b[: h * 64], d_s[: h * 32]), (d_b[h * 64:], d_s[h * 32:])]
    out = {}
    ra = ma.run(*halves[0])
    rb = mb.run(*halves[1])
    ok = M.affine_sum("bn254_g1", ra + rb) == ref
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ma.run(*halves[0])
        mb.run(*halves[1])
    t_seq = (time.perf_counter() - t0) / args.reps * 1e3
    res = {}
    for delay in args.delay_ms:
        walls = []
        for _ in range(args.reps):
            def second():
                time.sleep(delay / 1e3)
                res["b"] = mb.run(*halves[1])
            th = threading.Thread(target=second)
            t0 = time.perf_counter()
            th.start()
            res["a"] = ma.run(*halves[0])
            th.join()
            walls.append((time.perf_counter() - t0) * 1e3)
            ok = ok and M.affine_sum("bn254_g1", res["a"] + res["b"]) == ref
        out[f"concurrent_delay_{delay}"] = round(min(walls), 3)
    print(json.dumps({"log_n": args.log_n, "whole_ms": round(t_whole, 3), "two_halves_sequential_ms": round(t_seq, 3),
                      **out, "sum_equals_whole": ok}), flush=True)


if __name__ == "__main__":
    main()
