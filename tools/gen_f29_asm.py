#!/usr/bin/env python3
"""Generate tachyon_amd/csrc/field/f29_asm.h: the 9 x 29-bit carry-free
Montgomery products of field/f29.h as hand-chained v_mad_u64_u32 columns.

Why: seg_acc_kernel runs at one VALU wave-instruction per 4 cycles per SIMD
(profiles/r03a: SQ_INSTS_VALU x 4 / 1024 SIMDs / clock = the kernel time within
1 %), so every instruction costs the same and the product that issues the
fewest wins.  The 32-bit FIPS product issues ~279 (128 v_mad_u64_u32 + 128
v_addc_co_u32 + digits + moves); the compiler's code for f29.h's C++ columns
~274 (164 mads plus the 64-bit partial-sum combines it adds for ILP).  Chained
by hand, a 29-bit column is only its mads on ONE 64-bit accumulator -- a
column of <= 18 products of < 2^58 cannot carry out -- then the digit
(v_mul_lo_u32 + v_and_b32), one more mad, a mask and one 64-bit shift:
162 mads + ~52 others = ~214 instructions per product.

Each column's mads are one asm statement (the digit, mask and shift stay C++,
so the compiler still interleaves independent products between statements).
The mads' carry-outs go to a dummy SGPR pair nobody reads; it is an
early-clobber output ("=&s"), because a multi-mad statement writes it with its
first mad and reads SGPR inputs (kP29 limbs) in later ones (round 3 emitted
"=s", which let the allocator place sc on a kP29 limb; tests/test_isa_scan.py
checks the shipped code objects for that pattern).
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tachyon_amd", "csrc", "field", "f29_asm.h")
N = 9
# the field's limb shape and names (tools/gen_f28.py reuses these generators
# for BLS12-381 Fq in 14 x 28-bit limbs)
SPEC29 = {"N": N, "W": 29, "T": "F29", "mask": "kM29", "pinv": "kPinv29", "p": "kP29"}


def stmt(pairs, indent="  ", operand=None, spec=SPEC29):
    """One column: v_mad_u64_u32 acc += x * y for each (x, y) operand name
    (operand: name -> constraint text; default the Fq field's operands)."""
    if not pairs:
        return []
    names = []
    for x, y in pairs:
        for v in (x, y):
            if v not in names:
                names.append(v)
    lines = [f"v_mad_u64_u32 %[acc], %[sc], %[{x}], %[{y}], %[acc]" for x, y in pairs]
    text = "\\n\\t".join(lines)

    def default_operand(v):
        kind, idx = v[0], v[1:]
        src = {"a": f"a.l[{idx}]", "b": f"b.l[{idx}]", "c": f"c.l[{idx}]", "d": f"d.l[{idx}]",
               "m": f"m[{idx}]", "t": f"dd[{idx}]"}
        if kind == "p":
            return f'[{v}] "s"({spec["p"]}[{idx}])'
        return f'[{v}] "v"({src[kind]})'
    operand = operand or default_operand
    ins = ", ".join(operand(v) for v in names)
    # Early-clobber on both outputs: the FIRST mad writes sc (and acc) while
    # later mads of the same statement still read the "s" / "v" inputs, so
    # neither output may share a register with an input.
    return [f'{indent}asm("{text}" : [acc] "+&v"(acc), [sc] "=&s"(sc) : {ins});']


def column_pairs(k, mode, N=N):
    """Products of column k (without the digit's m_k p_0)."""
    pairs = []
    if mode in ("mul", "mul2"):
        for i in range(N):
            j = k - i
            if 0 <= j < N:
                pairs.append((f"a{i}", f"b{j}"))
        if mode == "mul2":
            for i in range(N):
                j = k - i
                if 0 <= j < N:
                    pairs.append((f"c{i}", f"d{j}"))
    else:  # sqr: a_i * 2 a_j for i < j, a_i^2 on the diagonal
        for i in range(N):
            j = k - i
            if i < j < N:
                pairs.append((f"a{i}", f"t{j}"))
        if k % 2 == 0 and k // 2 < N:
            pairs.append((f"a{k // 2}", f"a{k // 2}"))
    for i in range(N):  # reduction products of earlier digits
        j = k - i
        if i < k and 0 < j < N:
            pairs.append((f"m{i}", f"p{j}"))
    return pairs


def gen(name, mode, add, spec=SPEC29):
    T, N, W = spec["T"], spec["N"], spec["W"]
    args = {"mul": f"const {T}& a, const {T}& b", "mul2": f"const {T}& a, const {T}& b, const {T}& c, const {T}& d",
            "sqr": f"const {T}& a"}[mode]
    if add:
        args += f", const {T}& e"
    L = [f"__device__ __forceinline__ {T} {name}({args}) {{",
         "  uint64_t acc = 0, sc;",
         f"  uint32_t m[{N}];",
         f"  {T} r;"]
    if mode == "sqr":
        L.append(f"  uint32_t dd[{N}];")
        L.append(f"  for (int i = 0; i < {N}; ++i) dd[i] = a.l[i] << 1;")
    for k in range(2 * N - 1):
        L.append(f"  // column {k}")
        L += stmt(column_pairs(k, mode, N), spec=spec)
        if k < N:
            L.append(f"  m[{k}] = ((uint32_t)acc * {spec['pinv']}) & {spec['mask']};")
            L += stmt([(f"m{k}", "p0")], spec=spec)
        else:
            if add:
                L.append(f"  acc += e.l[{k - N}];")
            L.append(f"  r.l[{k - N}] = (uint32_t)acc & {spec['mask']};")
        L.append(f"  acc >>= {W};")
    if add:
        L.append(f"  acc += e.l[{N - 1}];")
    L.append(f"  r.l[{N - 1}] = (uint32_t)acc;")
    L.append("  return r;")
    L.append("}")
    return "\n".join(L) + "\n"


def render():
    head = ['// GENERATED by tools/gen_f29_asm.py -- do not edit.',
            '// Device products of field/f29.h (9 x 29-bit limbs, R\' = 2^261) as hand-chained',
            '// v_mad_u64_u32 columns; see the generator for the instruction budget.',
            '#pragma once',
            '#if defined(__HIP_DEVICE_COMPILE__)',
            'namespace tachyon_amd::f29::asm29 {',
            '']
    body = [gen("mul", "mul", False), gen("mul_add", "mul", True), gen("mul2", "mul2", False),
            gen("mul2_add", "mul2", True), gen("sqr", "sqr", False), gen("sqr_add", "sqr", True)]
    tail = ['}  // namespace tachyon_amd::f29::asm29', '#endif', '']
    return "\n".join(head) + "\n".join(body) + "\n".join(tail)


def main():
    text = render()
    open(OUT, "w").write(text)
    print(f"wrote {OUT}: {text.count('v_mad_u64_u32')} v_mad_u64_u32")


if __name__ == "__main__":
    main()
