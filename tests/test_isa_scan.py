"""The shipped gfx950 code objects never multiply by a carry mask.

The generated field products are multi-instruction inline-asm statements whose
v_mad_u64_u32 carry-outs go to an SGPR-pair output; without early-clobber the
register allocator may place that output on an SGPR input (a modulus limb) that
a later mad of the same statement reads (round-3 VERDICT Weak 1,
tools/gen_f29_asm.py).  tools/isa_scan.py extracts every gfx950 code object
from libtachyon_mi355x.so, disassembles it and flags any multiply whose SGPR
source was last written as a mad carry-out.  CPU only (llvm-objdump).
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_scan  # noqa: E402

LIB = os.path.join(ROOT, "tachyon_amd", "libtachyon_mi355x.so")


def test_scanner_flags_a_carry_mask_multiplicand():
    bad = """<k>:
  v_mad_u64_u32 v[0:1], s[4:5], v2, s8, v[0:1]
  v_mad_u64_u32 v[0:1], s[6:7], v3, s5, v[0:1]
"""
    assert len(isa_scan.scan_text(bad)) == 1
    # the same SGPR rewritten by a scalar move, or read after a label, is fine
    ok = """<k>:
  v_mad_u64_u32 v[0:1], s[4:5], v2, s8, v[0:1]
  s_mov_b32 s5, 0x1234
  v_mad_u64_u32 v[0:1], s[6:7], v3, s5, v[0:1]
  v_mad_u64_u32 v[0:1], s[4:5], v2, s8, v[0:1]
.LBB0_1:
  v_mad_u64_u32 v[0:1], s[6:7], v3, s4, v[0:1]
  v_addc_co_u32 v9, s[4:5], v9, 0, s[4:5]
"""
    assert isa_scan.scan_text(ok) == []


def test_generated_asm_outputs_are_early_clobber():
    for name in ("f29_asm.h", "mont_asm.h", "f28_asm.h", "fr29_gen.h"):
        text = open(os.path.join(ROOT, "tachyon_amd", "csrc", "field", name)).read()
        assert '"=&s"' in text, name  # the carry-out SGPR pairs are declared early-clobber
        assert not re.search(r'"=s"\(', text), name
        assert not re.search(r'"\+v"\(acc\)', text), name


@pytest.mark.skipif(not os.path.exists(isa_scan.OBJDUMP) or not os.path.exists(LIB), reason="needs llvm-objdump and the built library")
def test_shipped_library_has_no_carry_mask_multiplies():
    nobj, nmads, hits = isa_scan.scan_lib(LIB)
    assert nobj >= 8 and nmads > 100000
    assert hits == [], hits[:10]
