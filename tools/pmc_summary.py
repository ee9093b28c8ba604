#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 PMC passes (run_counter_collection.csv of
each pass directory): counter values per dispatch, the dispatch duration, and
a few derived ratios (VALU instructions per wave, LDS bank-conflict share,
issue-stall shares, HBM bytes).
  python tools/pmc_summary.py <dir with p1 p2 ... subdirs> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    n = re.sub(r"tachyon_amd::|\(anonymous namespace\)::|consts::|ntt::|msm::|detail::|fr29::", "", name)
    n = n.split("(")[0] if "(" in n and "<" not in n.split("(")[0][-3:] else n
    return n[:110]


def main():
    root = sys.argv[1]
    pats = sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if pats and not any(p in k for p in pats):
                continue
            key = (short(k), r["Grid_Size"], r["VGPR_Count"], r["LDS_Block_Size"])
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for key, cs in agg.items():
        name, grid, vgpr, lds = key
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {name}  grid={grid} vgpr={vgpr} lds={lds}  dur~{sorted(dur[key])[len(dur[key]) // 2]:.3f} ms")
        for c in sorted(avg):
            print(f"   {c:28s} {avg[c]:.4g}")
        w = avg.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in avg:
                    print(f"   {c + ' / wave':28s} {avg[c] / w:.1f}")
        if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   {'LDS conflict share':28s} {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f}")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if c in avg:
                    print(f"   {c + ' / WAVE_CYCLES':28s} {avg[c] / wc:.3f}")
        if "GRBM_GUI_ACTIVE" in avg and "SQ_INSTS_VALU" in avg:
            clk = avg["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
            print(f"   {'VALU issue share (4 cyc)':28s} {4 * avg['SQ_INSTS_VALU'] / (1024 * clk):.3f}")


if __name__ == "__main__":
    main()
