"""Instruction mix of one kernel in a hipcc -S (gfx950) assembly dump.

usage: python tools/isa_stats.py file.s <kernel-name-substring> [--blocks]
Prints VGPR/SGPR/scratch usage and mnemonic counts (whole kernel, and per basic
block with --blocks) -- used to count the VALU cost of a madd / butterfly.
"""
import collections
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    show_blocks = "--blocks" in sys.argv
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l) and pat in l.split(":")[0]:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    name = lines[start].split(":")[0]
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end") or re.match(r"^\s*\.size", l):
            break
        body.append(l)
    tot = collections.Counter()
    blocks = []
    cur = ("entry", collections.Counter())
    for l in body:
        s = l.strip()
        if re.match(r"^\.LBB\S*:", s):
            blocks.append(cur)
            cur = (s.rstrip(":"), collections.Counter())
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        m = s.split()[0]
        tot[m] += 1
        cur[1][m] += 1
    blocks.append(cur)
    print(name)
    for key in ("vgpr_count", "sgpr_count", "private_segment_fixed_size", "vgpr_spill_count"):
        for l in lines:
            if key in l and name in l:
                print(" ", l.strip())
    meta = "\n".join(lines)
    m = re.search(r"\.name:\s+" + re.escape(name) + r"(.*?)\.vgpr_spill_count:\s+(\d+)", meta, re.S)
    for key in (r"\.vgpr_count:\s+(\d+)", r"\.sgpr_count:\s+(\d+)", r"\.private_segment_fixed_size:\s+(\d+)"):
        mm = re.search(r"\.name:\s+" + re.escape(name) + r".*?" + key, meta, re.S) if False else None
    total = sum(tot.values())
    print(f"  total instructions {total}")
    for k, v in tot.most_common(25):
        print(f"  {k:28s} {v}")
    if show_blocks:
        for lab, c in blocks:
            n = sum(c.values())
            if n > int(__import__("os").environ.get("MINB", "50")):
                print(f"block {lab}: {n} instrs; " + ", ".join(f"{k}:{v}" for k, v in c.most_common(8)))


if __name__ == "__main__":
    main()
