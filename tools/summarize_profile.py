#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into markdown:
kernel-trace stats (top kernels) and per-kernel PMC averages with the gfx950
FETCH_SIZE correction (x2 for wide coalesced streams, MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import json
import os
import sys


def short(name):
    """Kernel function name without namespaces, template arguments or parameters."""
    if "rocprim" in name:
        for key in ("onesweep_histograms", "onesweep_iteration", "radix_sort", "lookback_scan", "scan"):
            if key in name:
                return "rocprim::" + key
        return "rocprim::other"
    base = name.replace("(anonymous namespace)", "anon")
    depth, out = 0, []
    for ch in base:  # drop <...> template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth = max(0, depth - 1)
        elif depth == 0:
            out.append(ch)
    base = "".join(out).split("(")[0].strip()
    return base.split("::")[-1].split()[-1][:60] if base else name[:60]


def main(d):
    print(f"# rocprofv3 summary: {d}\n")
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        rows = list(csv.DictReader(open(stats)))
        print("## Kernel trace (--kernel-trace --stats)\n")
        print("| kernel | calls | total ms | avg ms | % |")
        print("|---|---|---|---|---|")
        for r in rows[:20]:
            print(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                  f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} |")
        print()
    # average dispatch duration per short kernel name (instantiations merged)
    dur = collections.defaultdict(lambda: [0.0, 0])
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            acc = dur[short(r["Name"])]
            acc[0] += float(r["TotalDurationNs"])
            acc[1] += int(r["Calls"])
    agg = collections.defaultdict(list)
    meta = {}
    for sub in ("fetch", "write", "valu"):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
            meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["Scratch_Size"], r["LDS_Block_Size"])
    if agg:
        print("## PMC (per dispatch averages; separate passes)\n")
        print("| kernel | VGPR | scratch | LDS | FETCH_SIZE KB (x2 corr.) | WRITE_SIZE KB | SQ_INSTS_VALU | "
              "VALU busy % | eff. clock GHz |")
        print("|---|---|---|---|---|---|---|---|---|")
        for k in sorted({k for k, _ in agg}):
            def avg(c):
                v = agg.get((k, c))
                return sum(v) / len(v) if v else None
            fetch, write, insts = avg("FETCH_SIZE"), avg("WRITE_SIZE"), avg("SQ_INSTS_VALU")
            act, busy, grbm = avg("SQ_ACTIVE_INST_VALU"), avg("SQ_BUSY_CYCLES"), avg("GRBM_GUI_ACTIVE")
            wave = avg("SQ_WAVE_CYCLES")
            valu = f"{100.0 * act / wave:.1f}" if act and wave else "-"
            fmt = (lambda x: f"{x:.4g}" if x is not None else "-")
            v, s, sc, l = meta[k]
            clock = "-"
            if grbm and dur[k][1]:  # GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / the dispatch's duration
                clock = f"{grbm / 8 / (dur[k][0] / dur[k][1]):.2f}"
            print(f"| {k} | {v} | {sc} | {l} | {fmt(fetch * 2 if fetch else None)} | {fmt(write)} | {fmt(insts)} | "
                  f"{valu} | {clock} |")
        print("\nVALU busy % = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave-cycles issuing VALU); eff. clock "
              "= GRBM_GUI_ACTIVE / 8 XCDs / the kernel's average trace duration.")
        # per-dispatch HBM traffic for bench.py's roofline "traffic" field
        # (FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE counts half of a
        # wide streaming read -- MI355X_MICROARCH.md, HBM/rocprofv3 -- so the x2
        # value is the corrected one; other access widths are uncalibrated)
        traffic = {}
        for k in sorted({k for k, _ in agg}):
            f = agg.get((k, "FETCH_SIZE"))
            w = agg.get((k, "WRITE_SIZE"))
            if not f or not w:
                continue
            fb = sum(f) / len(f) * 1024
            wb = sum(w) / len(w) * 1024
            traffic[k] = {"dispatches": len(f), "fetch_bytes_raw": fb, "fetch_bytes_x2": 2 * fb, "write_bytes": wb,
                          "traffic_bytes": 2 * fb + wb}
        with open(os.path.join(d, "pmc_traffic.json"), "w") as fh:
            json.dump(traffic, fh, indent=1)
        if os.environ.get("PROFILE_UNITS"):
            derived_units(agg, traffic, os.environ["PROFILE_UNITS"])
        else:
            derived(agg, traffic)


def derived_units(agg, traffic, spec):
    """PROFILE_UNITS='kernel=units[:lanes],...': VALU instructions per unit
    (SQ_INSTS_VALU x 64 / (units x lanes)) and HBM bytes per unit of those
    kernels (e.g. the BLS12-381 accumulations: units = n x W additions,
    lanes = 2 for the G2 lane pairs)."""
    print("\n## Per-unit figures (PROFILE_UNITS)\n")
    for item in spec.split(","):
        k, _, u = item.partition("=")
        units, _, lanes = u.partition(":")
        units, lanes = float(units), float(lanes or 1)
        v = agg.get((k, "SQ_INSTS_VALU"))
        t = traffic.get(k)
        if v:
            print(f"* `{k}`: {sum(v) / len(v) * 64 / (units * lanes):.0f} VALU instructions per unit per lane "
                  f"({units:.4g} units x {lanes:g} lanes per dispatch)")
        if t:
            print(f"* `{k}`: {t['traffic_bytes'] / units:.1f} HBM B per unit ({t['fetch_bytes_raw'] / units:.1f} raw "
                  f"FETCH + {t['write_bytes'] / units:.1f} written)")


def derived(agg, traffic, msm_log_n=26, windows=13, ntt_log_n=24):
    """Per-unit figures of the default bench command: VALU instructions per NTT
    butterfly (a 2^24 pass = 8 stages x 2^23 butterflies) and HBM bytes per
    sorted MSM entry (13 x 2^26 entries of 8 B at the default plan)."""
    lines = []
    v = agg.get(("dif_pass_kernel", "SQ_INSTS_VALU"))
    if v:
        bfly = 8 * (1 << (ntt_log_n - 1))
        lines.append(f"* `dif_pass_kernel`: {sum(v) / len(v) * 64 / bfly:.0f} VALU instructions per butterfly "
                     f"(per-dispatch SQ_INSTS_VALU x 64 / (8 stages x 2^{ntt_log_n - 1} butterflies), "
                     f"{len(v)} dispatches of 2^{ntt_log_n} passes)")
    entries = windows * (1 << msm_log_n)
    for k, what in (("onesweep_iteration", "rocprim::onesweep_iteration"), ("recode_scatter_kernel", None),
                    ("recode_hist_kernel", None), ("seg_acc29_kernel", None)):
        t = traffic.get(what or k)
        if t:
            lines.append(f"* `{what or k}`: {t['traffic_bytes'] / entries:.2f} HBM B per entry "
                         f"({t['fetch_bytes_x2'] / entries:.2f} read x2-corrected + {t['write_bytes'] / entries:.2f} "
                         f"written; {windows} x 2^{msm_log_n} entries of 8 B)")
    if lines:
        print("\n## Per-unit figures (default bench plan: MSM 2^26, c = 20, 13 windows; NTT 2^24)\n")
        print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1])
