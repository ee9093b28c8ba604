#!/usr/bin/env python3
"""A/B of the four-step NTT's local stages (rank 0 of an N-rank plan, the
stages bench.py's project_ntt_scaling times) over the plan variants:
bit 0 = the round-4 stages (input copy + passes + separate twiddle kernel),
bit 1 = 32-bit-limb sub-transform passes, bit 2 = no packing of one-pass
sub-transforms; --splits: log R of the plan (0 = floor(L/2), -1 =
split_log_r's choice).  Rounds alternate the variants.

  python tools/ntt4_probe.py --log-n 24 --worlds 2 4 8 --variants 0 1 2 3 --rounds 3 --splits 0 -1
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
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--splits", type=int, nargs="+", default=[0])
    args = ap.parse_args()
    import torch
    from tachyon_amd import msm as M
    from tachyon_amd.ntt import FourStepNtt
    for world, split in [(w, sp) for w in args.worlds for sp in args.splits]:
        log_r = FourStepNtt.split_log_r(args.log_n, world) if split < 0 else split or None
        plan = FourStepNtt(args.log_n, world, 0, log_r=log_r)
        m = plan.local_size
        x = torch.empty(m * 32, dtype=torch.uint8, device="cuda")
        y = torch.empty_like(x)
        M.gen_scalars("bn254_fr", 99, m, x.data_ptr())
        torch.cuda.synchronize()
        s = plan.torch_stream
        ref = None
        for rnd in range(args.rounds):
            for v in args.variants:
                plan.set_variant(v)
                x0 = x.clone()
                torch.cuda.synchronize()  # the clone (current stream) before the plan's stream reads x0
                # both stages (the round-4 stage 1 leaves lazy [0, 2p) values in the send buffer, the fused
                # one canonical ones, so the variants agree on the transform, not on the packed bytes)
                plan.run_stage(1, False, x0, y)
                plan.run_stage(2, False, y, x0)
                s.synchronize()
                out = x0.clone()
                torch.cuda.synchronize()
                if ref is None:
                    ref = out
                assert torch.equal(out, ref), (world, v)
                for _ in range(2):
                    plan.run_stage(1, False, x, y)
                    plan.run_stage(2, False, y, x0)
                s.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.reps):
                    plan.run_stage(1, False, x, y)
                    plan.run_stage(2, False, y, x0)
                s.synchronize()
                ms = (time.perf_counter() - t0) / args.reps * 1e3
                print(json.dumps({"log_n": args.log_n, "world": world, "log_r": plan.log_r, "variant": v,
                                  "round": rnd, "local_stages_ms": round(ms, 4)}), flush=True)
        plan.close()


if __name__ == "__main__":
    main()
