#!/usr/bin/env python3
"""Per-rank cost of the two multi-GPU MSM partitions, measured on one GPU.

For N ranks over a 2^L MSM: the point split runs an n/N-point MSM (all
windows, the size's default c); the window split runs all n points over
W/N windows of c-bit windows (run_window_range).  The slower rank sets the
N-GPU step time, so these per-rank times are the scaling model the bench's
--msm-split auto rule follows.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def best_ms(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=26)
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--c", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--hybrid", action="store_true",
                    help="N = P point groups x Q window groups: the slowest rank runs n/P points over the first "
                         "ceil(W/Q) windows, for Q in 1, 2, 4 and the window bits of --hybrid-c")
    ap.add_argument("--hybrid-c", type=int, nargs="+", default=[17, 19, 20])
    ap.add_argument("--curve", default="bn254_g1", help="bn254_g1, bls12_381_g1 or bls12_381_g2")
    args = ap.parse_args()
    import torch
    from tachyon_amd import dist as D
    from tachyon_amd import msm as M
    from tachyon_amd._lib import CURVE_INFO
    n = 1 << args.log_n
    curve = args.curve
    pb, sf = CURVE_INFO[curve]
    d_b = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    M.gen_bases(curve, 1, n, 1024, d_b.data_ptr())
    M.gen_scalars(sf, 1, n, d_s.data_ptr())
    torch.cuda.synchronize()
    m = M.VariableBaseMSMGpu(curve)
    whole = best_ms(lambda: m.run(d_b, d_s, n), args.reps)
    if args.hybrid:
        for world in args.worlds:
            for q in (1, 2, 4):
                if q > world:
                    continue
                shard = n // (world // q)
                for c in args.hybrid_c:
                    W = D._windows_for(curve, c)
                    w1 = -(-W // q)
                    m.set_window_bits(c)
                    t = best_ms(lambda: m.run_window_range(d_b, d_s, 0, w1, shard), args.reps)
                    m.set_profile(True)
                    m.run_window_range(d_b, d_s, 0, w1, shard)
                    ph = {k: round(v, 3) for k, v in m.last_timings().items()}
                    m.set_profile(False)
                    m.set_window_bits(0)
                    print(json.dumps({"curve": curve, "log_n": args.log_n, "world": world, "point_groups": world // q,
                                      "window_groups": q, "c": c, "windows_slowest_rank": w1, "points_per_rank": shard,
                                      "whole_ms": round(whole, 3), "rank_ms": round(t, 3),
                                      "efficiency": round(whole / (world * t), 3), "phases": ph}), flush=True)
        m.close()
        return
    W = D._windows_for(curve, args.c)
    for world in args.worlds:
        shard = n // world
        pts = best_ms(lambda: m.run(d_b, d_s, shard), args.reps)
        m.set_window_bits(args.c)
        w0, w1 = D.window_range(W, 0, world)
        win = best_ms(lambda: m.run_window_range(d_b, d_s, w0, w1, n), args.reps)
        m.set_profile(True)
        m.run_window_range(d_b, d_s, w0, w1, n)
        win_phases = {k: round(v, 3) for k, v in m.last_timings().items()}
        m.set_window_bits(0)
        m.run(d_b, d_s, shard)
        pts_phases = {k: round(v, 3) for k, v in m.last_timings().items()}
        m.set_profile(False)
        print(json.dumps({"log_n": args.log_n, "world": world, "whole_ms": round(whole, 3),
                          "point_split_rank_ms": round(pts, 3), "window_split_rank_ms": round(win, 3),
                          "c": args.c, "windows_per_rank": w1 - w0,
                          "eff_points": round(whole / (world * pts), 3),
                          "eff_windows": round(whole / (world * win), 3),
                          "window_phases": win_phases, "point_phases": pts_phases}), flush=True)
    m.close()


if __name__ == "__main__":
    main()
