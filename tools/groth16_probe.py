#!/usr/bin/env python3
"""A/B of the Groth16 proof's MSM window bits (Groth16Prover.set_msm_window_bits)
on bench.py's synthetic 2^k-constraint key: wall ms per NoZK proof (host
witness, as the bench), rounds alternating the configurations, the proof
checked equal across configurations.

  python tools/groth16_probe.py --log-n 20 --configs 0,0,0 0,0,17 16,17,17 --rounds 3
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--configs", nargs="+", default=["0,0,0"],
                    help="c_a,c_lh,c_b2[,variant] (0 = default; variant 1 = separate A and witness + h MSMs)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    import bench
    from tachyon_amd.groth16 import Groth16Prover
    zkey, full = bench.synth_groth16_zkey(args.log_n)
    p = Groth16Prover(zkey)
    ref = p.prove(full)
    for rnd in range(args.rounds):
        for cfg in args.configs:
            vals = [int(x) for x in cfg.split(",")]
            ca, clh, cb2 = vals[:3]
            var = vals[3] if len(vals) > 3 else 0
            p.set_variant(var)
            p.set_msm_window_bits(ca, clh, cb2)
            assert p.prove(full) == ref, cfg
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                p.prove(full)
                ts.append((time.perf_counter() - t0) * 1e3)
            p.set_profile(True)
            p.prove(full)
            ph = p.last_timings()
            p.set_profile(False)
            print(json.dumps({"log_n": args.log_n, "c_a": ca, "c_lh": clh, "c_b2": cb2, "variant": var, "round": rnd,
                              "median_ms": round(sorted(ts)[len(ts) // 2], 3), "min_ms": round(min(ts), 3),
                              "mean_ms": round(sum(ts) / len(ts), 3), "reps_ms": [round(t, 3) for t in ts],
                              "phases": {k: round(v, 3) for k, v in ph.items()}}), flush=True)
    p.close()


if __name__ == "__main__":
    main()
