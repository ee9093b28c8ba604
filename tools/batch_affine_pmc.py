"""Summarise the PMC pass of bin/batch_affine_probe (tools/gpu_r05h.sh): VALU
and LDS wave-instructions per addition for every kernel of the probe, from the
timed dispatch (the largest of a kernel's launches), with the additions that
dispatch performed at `batch_affine_probe 1` (the pass's argument).

    python tools/batch_affine_pmc.py gpurun_out/r05h/pmc/run_counter_collection.csv
"""
import csv
import json
import re
import sys
from collections import defaultdict

LANES = 256 * 12 * 256  # kBlocks x kBlock of the probe (every row covers the same lanes)


def additions(name: str) -> tuple[str, int] | None:
    """(row label, additions of the timed dispatch) at base_rounds = 1."""
    if "madd_reg_kernel" in name:
        return "madd_reg", LANES * 100
    if "madd_tab_kernel" in name:
        return "madd_tab", LANES * 100
    m = re.search(r"batch_affine_(lds_)?kernel<(\d+), (true|false)", name)
    if not m:
        return None
    lds, g, fermat = m.group(1) is not None, int(m.group(2)), m.group(3) == "true"
    rounds = max(1, 100 // g) if lds else 25
    if fermat:
        rounds = max(1, rounds // 4)
    label = f"batch_{'lds' if lds else 'vgpr'} g={g} inv={'fermat' if fermat else 'free'}"
    return label, LANES * rounds * g


def main(path: str):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for row in csv.DictReader(open(path)):
        per[(row["Kernel_Name"], int(row["Dispatch_Id"]))][row["Counter_Name"]] += float(row["Counter_Value"])
    best = {}
    for (kern, _), c in per.items():
        if additions(kern) is None:
            continue
        if kern not in best or c.get("SQ_INSTS_VALU", 0) > best[kern].get("SQ_INSTS_VALU", 0):
            best[kern] = c
    for kern, c in best.items():
        label, adds = additions(kern)
        print(json.dumps({"row": label, "additions": adds,
                          "valu_per_addition": round(c["SQ_INSTS_VALU"] * 64 / adds, 1),
                          "lds_per_addition": round(c.get("SQ_INSTS_LDS", 0) * 64 / adds, 2)}))


if __name__ == "__main__":
    main(sys.argv[1])
