#!/usr/bin/env python3
"""Kernel timeline of the last MSM in a rocprofv3 kernel trace.

  python tools/timeline.py <run_kernel_trace.csv> [--last-from recode_hist]

Prints every kernel dispatch from the last occurrence of the marker kernel on:
start offset (us), duration (us) and the idle gap before it -- where the
small MSMs' wall time goes (launch gaps, the chain read-back, serial levels).
"""
import argparse
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"[\w:]*?(\w+)\s*[<(]", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-from", default="recode_hist_kernel")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    idx = max(i for i, r in enumerate(rows) if r[2] == a.last_from)
    t0 = rows[idx][0]
    prev_end = t0
    busy = 0
    for s, e, n in rows[idx:]:
        if n == "madd_ceiling29_kernel":
            break
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:7.1f}  {n}")
        busy += e - s
        prev_end = max(prev_end, e)
    print(f"span {(prev_end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
