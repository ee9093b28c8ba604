#!/usr/bin/env python3
"""Scan the gfx950 code objects of a built HIP library for a multiply that
reads a carry mask.

Why: the generated field products (field/f29_asm.h, field/mont_asm.h) are
multi-instruction inline-asm statements whose v_mad_u64_u32 carry-outs go to an
SGPR pair output.  If that output is not early-clobber, the register allocator
may give it the SGPRs of an input that a LATER mad of the same statement reads
(a kP29 / modulus limb), which then multiplies by the carry mask instead of the
limb.  Whether a build is hit depends on register allocation alone, so the
shipped binary is checked directly: in straight-line code (state reset at every
label and branch), a v_mad_u64_u32 / v_mad_i64_i32 / v_mul_* source SGPR whose
last writer was a mad's carry-out is reported.  Legitimate carry consumers
(v_addc_co_u32 / v_subb_co_u32 carry-ins, v_cndmask) are not multiplies.

usage: python tools/isa_scan.py [lib.so]   (default tachyon_amd/libtachyon_mi355x.so)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path, arch="gfx950"):
    """The device code objects of every clang offload bundle in a host ELF
    (uncompressed bundles: magic, u64 count, then per entry u64 offset, u64
    size, u64 triple length, triple)."""
    data = open(path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if arch in triple and size:
                out.append((triple, data[pos + off:pos + off + size]))
        pos = data.find(MAGIC, pos + 1)
    return out


def _sgprs(tok):
    tok = tok.strip().rstrip(",")
    m = re.fullmatch(r"s(\d+)", tok)
    if m:
        return [int(m.group(1))]
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    if tok == "vcc":
        return ["vcc_lo", "vcc_hi"]
    if tok in ("vcc_lo", "vcc_hi"):
        return [tok]
    return []


_MULS = ("v_mad_u64_u32", "v_mad_i64_i32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_mul_u32_u24")
# SALU ops whose first operand is a source, not a destination.
_SALU_NO_DST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_endpgm",
                "s_setprio", "s_sleep", "s_setpc", "s_store", "s_buffer_store", "s_dcache", "s_sendmsg",
                "s_set_gpr_idx", "s_trap", "s_ttracedata", "s_cmpk", "s_setreg", "s_setvskip")


def scan_text(text):
    """Hits in llvm-objdump -d text: (function, line) of every multiply whose
    SGPR source was last written as a v_mad_*64 carry-out."""
    hits = []
    func = "?"
    last = {}  # sgpr -> True if last writer was a mad carry-out
    for line in text.splitlines():
        s = line.strip()
        mf = re.match(r"^(?:[0-9a-f]+ )?<(.+)>:$", s)
        if mf:
            func, last = mf.group(1), {}
            continue
        if not s or s.endswith(":"):
            last = {}
            continue
        s = re.sub(r"\s*//.*$", "", s)
        parts = s.split(None, 1)
        if not parts or not re.match(r"^[sv]_", parts[0]):
            continue
        mn = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        if mn.startswith("s_cbranch") or mn.startswith("s_branch") or mn.startswith("s_setpc") or mn.startswith("s_swappc"):
            last = {}
            continue
        if mn.startswith(_MULS):
            srcs = ops[2:] if mn.startswith(("v_mad_u64_u32", "v_mad_i64_i32")) else ops[1:]
            for o in srcs:
                if any(last.get(r) for r in _sgprs(o)):
                    hits.append((func, s))
                    break
        # writes
        if mn.startswith(("v_mad_u64_u32", "v_mad_i64_i32")) and len(ops) > 1:
            for r in _sgprs(ops[1]):
                last[r] = True
        elif mn.startswith("s_") and ops and not mn.startswith(_SALU_NO_DST):
            for r in _sgprs(ops[0]):
                last[r] = False
        elif mn.startswith("v_") and len(ops) > 1:
            # VALU with an SGPR destination (v_cmp sdst, v_add_co carry-out,
            # v_readlane / v_readfirstlane): any SGPR among its first two operands
            for o in ops[:2] if ("_co_" in mn or mn.startswith("v_cmp")) else ops[:1]:
                for r in _sgprs(o):
                    last[r] = False
    return hits


def scan_lib(path):
    hits, nobj, nmads = [], 0, 0
    for i, (triple, blob) in enumerate(code_objects(path)):
        nobj += 1
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(blob)
            f.flush()
            text = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--no-leading-addr", f.name],
                                  capture_output=True, text=True, check=True).stdout
        nmads += text.count("v_mad_u64_u32")
        hits += scan_text(text)
    return nobj, nmads, hits


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tachyon_amd", "libtachyon_mi355x.so")
    nobj, nmads, hits = scan_lib(path)
    print(f"{path}: {nobj} gfx950 code objects, {nmads} v_mad_u64_u32, {len(hits)} carry-mask multiplies")
    for f, s in hits[:50]:
        print(f"  {f}: {s}")
    sys.exit(1 if hits else 0)


if __name__ == "__main__":
    main()
