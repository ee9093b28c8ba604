"""The bench.py output contract, checked on the newest committed bench line
(profiles/<round>/bench_line*.json, written on the GPU box): the keys the
driver and the judge read, a roofline object with its fraction consistent,
and the CPU baseline beside it.  No GPU needed."""
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def newest_bench_line():
    # newest round tag first (file mtimes are the checkout's); the 1-GPU
    # default-run lines only (multi-rank rehearsals carry no CPU baseline)
    import re

    def order(f):  # run order: r05z < r05aa < r05ab (as bench.pmc_traffic)
        m = re.fullmatch(r"r(\d+)([a-z]*)", os.path.basename(os.path.dirname(f)))
        return (int(m.group(1)), len(m.group(2)), m.group(2), f) if m else (-1, 0, "", f)

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "bench_line*.json")), key=order)
    if not files:
        pytest.skip("no committed bench line")
    for path in reversed(files):
        if "rehearsal" in os.path.basename(path):
            continue
        text = open(path).read().strip()
        if text.startswith("{"):
            d = json.loads(text.splitlines()[-1])
            if d.get("n_gpus") == 1:
                return path, d
    pytest.skip("no parsable bench line")


def test_bench_line_contract():
    path, d = newest_bench_line()
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, (path, k)
    assert d["higher_is_better"] is True and d["unit"] == "scalars/s"
    assert d["scaling"] in ("weak", "strong")
    # value = the 2^msm_log_n scalars of one step / the step time
    n = 1 << d["config"]["msm_log_n"]
    assert abs(d["value"] - n / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-6
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma") and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("reference", "port") and c["cores"] >= 1


def test_bench_cli_parses_without_gpu():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0 and "--gpus" in out.stdout and "--steps" in out.stdout


def test_pmc_traffic_takes_the_newest_run(tmp_path, monkeypatch):
    """bench.pmc_traffic reads the newest committed profile in run order
    (r05z < r05aa < r05ab: spreadsheet-column suffixes), not the
    lexicographically last directory."""
    import json
    import bench
    for run, gb in (("r05y", 1.0), ("r05z", 2.0), ("r05ab", 3.0), ("r04zz", 9.0)):
        d = tmp_path / "profiles" / run
        d.mkdir(parents=True)
        (d / "pmc_traffic.json").write_text(json.dumps({"k": {"traffic_bytes": gb * 1e9}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    traffic, src, _ = bench.pmc_traffic("k")
    assert traffic == 3.0 and src.endswith("r05ab/pmc_traffic.json")
