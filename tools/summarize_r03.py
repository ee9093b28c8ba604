#!/usr/bin/env python3
"""Summarise tools/profile_r03.sh output: kernel-trace stats and, per PMC pass
directory, per-kernel averages of every counter (per dispatch), plus the
derived figures DESIGN.md quotes: VALU instructions per dispatch, INT64 share,
VALU-active fraction of the wave cycles, resident waves per SIMD
(MeanOccupancyPerCU / 4), the effective clock (GRBM_GUI_ACTIVE is summed over
the 8 XCDs: / 8 / dispatch time from the kernel trace) and the per-SIMD VALU
issue utilisation 4 x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): a
wave64 VALU instruction holds its SIMD for 4 cycles (profiles/r03c: the
in-register madd microbenchmark issues at 99 % of that at 2.36 GHz)."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import short  # noqa: E402


def stats(d, sub):
    p = os.path.join(d, sub, "run_kernel_stats.csv")
    if not os.path.exists(p):
        return
    rows = list(csv.DictReader(open(p)))
    print(f"## {sub}: kernel trace (--kernel-trace --stats)\n")
    print("| kernel | calls | total ms | avg ms | % |")
    print("|---|---|---|---|---|")
    for r in rows[:16]:
        print(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
              f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} |")
    print()


def trace_ms(d):
    """average dispatch ms per short kernel name over the trace passes"""
    ms = {}
    for sub in ("trace", "g2_trace"):
        p = os.path.join(d, sub, "run_kernel_stats.csv")
        if os.path.exists(p):
            for r in csv.DictReader(open(p)):
                ms.setdefault(short(r["Name"]), float(r["AverageNs"]) / 1e6)
    return ms


def pmc(d, sub, want=("seg_acc_kernel", "seg_acc29_kernel", "seg_acc_pair_kernel", "dif_pass_kernel",
                      "rocprim::onesweep_iteration", "recode_scatter_kernel", "recode_hist_kernel",
                      "window_segment", "seg_reduce", "k29", "k32")):
    p = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[k] = {"vgpr": r.get("VGPR_Count"), "scratch": r.get("Scratch_Size"), "lds": r.get("LDS_Block_Size")}
    out = {}
    for k, cs in agg.items():
        if not any(w in k for w in want):
            continue
        # one value per dispatch after summing the per-SE / per-XCD rows of that dispatch is what
        # rocprofv3 writes per row already; average over dispatches
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k].update(meta[k])
    return out


def derived(c):
    r = {}
    if "SQ_INSTS_VALU" in c and "SQ_INSTS_VALU_INT64" in c:
        r["int64_share"] = c["SQ_INSTS_VALU_INT64"] / max(1.0, c["SQ_INSTS_VALU"])
    if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
        r["valu_active_per_wave_cycle"] = c["SQ_ACTIVE_INST_VALU"] / max(1.0, c["SQ_WAVE_CYCLES"])
    if "GRBM_GUI_ACTIVE" in c and "SQ_INSTS_VALU" in c:
        gui = c["GRBM_GUI_ACTIVE"] / 8  # per-XCD cycles of the dispatch (rocprofv3 sums the 8 XCDs)
        r["simd_valu_issue_util"] = 4 * c["SQ_INSTS_VALU"] / max(1.0, gui * 1024)
        if c.get("avg_ms"):
            r["clock_ghz"] = gui / (c["avg_ms"] * 1e6)
    if "MeanOccupancyPerCU" in c:
        r["waves_per_simd"] = c["MeanOccupancyPerCU"] / 4
    return r


def main(d):
    print(f"# rocprofv3 summary (round 3): {d}\n")
    for sub in ("trace", "g2_trace"):
        stats(d, sub)
    res = {}
    ms = trace_ms(d)
    for sub in ("fetch", "write", "valu", "occ", "g2_fetch", "g2_write", "g2_valu", "ab_valu", "ab_occ",
                "micro_valu"):
        res[sub] = pmc(d, sub)
        for k, c in res[sub].items():
            if k in ms and not sub.startswith("micro"):
                c["avg_ms"] = ms[k]
    print("## PMC per dispatch (averages)\n")
    for sub, ks in res.items():
        if not ks:
            continue
        print(f"### {sub}\n")
        for k, c in sorted(ks.items()):
            dv = derived(c)
            print(f"- **{k}**: " + ", ".join(f"{n} = {v:.4g}" if isinstance(v, float) else f"{n} = {v}"
                                             for n, v in sorted(c.items())) +
                  ("; derived: " + ", ".join(f"{n} = {v:.4g}" for n, v in dv.items()) if dv else ""))
        print()
    json.dump(res, open(os.path.join(d, "pmc_r03.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
