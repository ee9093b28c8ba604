#!/usr/bin/env python3
"""Window-size sweep for the MSM (device-resident BN254 G1 inputs).

  python tools/tune_msm.py --log-n 26 --c 16 18 20 21 22
Prints per-phase device time (HIP events) for each window size.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, nargs="+", default=[26])
    ap.add_argument("--c", type=int, nargs="+", default=[0])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--non-uniform", action="store_true")
    ap.add_argument("--variants", type=int, nargs="+", default=[0])
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--curve", default="bn254_g1")
    args = ap.parse_args()
    import torch
    from tachyon_amd import msm as M
    for lg in args.log_n:
        n = 1 << lg
        from tachyon_amd._lib import CURVE_INFO
        pb, sf = CURVE_INFO[args.curve]
        d_b = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
        d_s = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        M.gen_bases(args.curve, 1, n, 1024, d_b.data_ptr())
        if args.non_uniform:
            M.gen_scalars(sf, 1, 1, d_s.data_ptr())
            d_s.view(n, 32)[:] = d_s[:32]
        else:
            M.gen_scalars(sf, 1, n, d_s.data_ptr())
        torch.cuda.synchronize()
        m = M.VariableBaseMSMGpu(args.curve)
        ref = None
        for c, var in [(c, v) for _ in range(args.rounds) for c in args.c for v in args.variants]:
            m.set_window_bits(c)
            m.set_variant(var)
            m.set_profile(True)
            res = m.run(d_b, d_s)
            ref = ref or res
            times, walls = [], []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                r = m.run(d_b, d_s)
                walls.append((time.perf_counter() - t0) * 1e3)
                times.append(m.last_timings())
                assert r == ref or (var & 64), "result changed"
            best = min(range(args.reps), key=lambda i: walls[i])
            print(json.dumps({"curve": args.curve, "log_n": lg, "c": c or M.plan(args.curve, n)[0], "variant": var, "wall_ms": round(walls[best], 3),
                              **{k: round(v, 3) for k, v in times[best].items()}}), flush=True)
        m.close()


if __name__ == "__main__":
    main()
