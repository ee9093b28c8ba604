"""Product-path hygiene (CPU): every environment variable the release library
reads is either compiled out of it (inside #ifdef TACHYON_TUNING_KNOBS, for
tuning builds only) or exercised by a test, so no untested override can change
a kernel schedule in a process that happens to set it."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def release_getenvs():
    found = {}
    for path in glob.glob(os.path.join(ROOT, "tachyon_amd", "csrc", "**", "*.*"), recursive=True):
        if not path.endswith((".h", ".hip", ".cc")):
            continue
        depth = 0
        for line in open(path):
            s = line.strip()
            if s.startswith("#ifdef TACHYON_TUNING_KNOBS"):
                depth += 1
            elif s.startswith("#if") and depth:
                depth += 1
            elif s.startswith("#endif") and depth:
                depth -= 1
            if depth:
                continue
            for name in re.findall(r'getenv\("([A-Z0-9_]+)"\)', line):
                found.setdefault(name, []).append(os.path.relpath(path, ROOT))
    return found


def test_every_release_env_knob_is_tested():
    tests = "".join(open(p).read() for p in glob.glob(os.path.join(ROOT, "tests", "*.py"))
                    if not p.endswith("test_no_untested_knobs.py"))
    knobs = release_getenvs()
    assert knobs, "expected the documented hooks (TACHYON_MSM_GPU_INPUT_DIR, ...)"
    untested = {k: v for k, v in knobs.items() if k not in tests}
    assert not untested, f"environment overrides in the release library with no test: {untested}"


def test_tuning_knobs_are_compiled_out():
    knobs = release_getenvs()
    for name in ("TACHYON_NTT_LDS_ELEMS", "TACHYON_NTT_RADIX_LOG", "TACHYON_NTT_SHOUP", "TACHYON_NTT_VARIANT",
                 "TACHYON_MSM_SEG"):
        assert name not in knobs, name
    ff = open(os.path.join(ROOT, "tachyon_amd", "csrc", "field", "ff.h")).read()
    assert "TA_CALL_FUSED_MUL" not in ff and "TA_CALL_MULSUB" not in ff
