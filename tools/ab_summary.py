"""Summarise gpurun_out/ab.log (tools/ab_libs.sh): per build and MSM size,
the phase times (ms) of every run."""
import json
import sys

tag = None
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    if line.startswith("=="):
        tag = line.split()[1]
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    print(tag, d["curve"], d["log_n"], "total", d.get("total"), "acc", d.get("acc"), "reduce", d.get("reduce"),
          "wall", d["wall_ms"])
