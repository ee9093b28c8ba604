#!/usr/bin/env python3
"""Generate tachyon_amd/csrc/field/mont_asm.h: CDNA4 Montgomery multiplication
by Finely Integrated Product Scanning (FIPS) with hand-written v_mad_u64_u32
carry chains.

Why: gfx950's only wide multiplier is v_mad_u64_u32 (32x32 + 64 -> 64 with a
carry-out SGPR, no carry-in), and 64-bit VGPR operands must sit in even-aligned
register pairs.  Compiled from C, the CIOS loop spends ~2.8 v_mov per product
re-pairing registers (measured: 6738 v_mov for 2435 v_mad_u64_u32 in the MSM
accumulation kernel).  Column-wise (product scanning) accumulation keeps ONE
aligned 64-bit accumulator per column: every product is exactly
    v_mad_u64_u32 acc, vcc, x, y, acc      (half-rate)
    v_addc_co_u32 acc2, vcc, 0, acc2, vcc   (collect the carry-out)
and the Montgomery quotient digit m_k = acc.lo * (-p^-1) is folded in as the
column ends (FIPS), so there is no separate reduction pass.

Each column's products are one asm statement (hipcc pads one s_nop after every
statement boundary, so per-product statements cost a nop each).  The statements
are not volatile: they are pure functions of their operands, and letting the
scheduler interleave independent products (the several muls of one point
addition) cut the latency-bound bucket/window reduction by ~20% on MI355X.
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tachyon_amd", "csrc", "field", "mont_asm.h")


# Carry-out SGPR pairs rotate over three registers and each v_addc_co_u32 that
# collects a carry trails its v_mad_u64_u32 by two instructions: gfx940-family
# parts need two wait states between a VALU write of an SGPR (the carry mask)
# and a VALU read of it (hipcc pads its own carry chains with s_nop 1), and the
# rotation meets that without nops wherever a statement has >= 3 products.
NCARRY = 3


def mac_lines(pairs, fresh_c2, carries=True):
    """pairs: list of (x_operand, y_operand) names -> asm text lines.
    fresh_c2: the first collected carry defines c2 (v_addc_co_u32 c2, .., 0, zero)
    instead of a separate zeroing move.  carries=False: a column whose carry
    out is discarded (only the low word is kept) -- mads only."""
    out = []
    if not carries:
        return [f"v_mad_u64_u32 %[acc], %[s{k % NCARRY}], %[{x}], %[{y}], %[acc]" for k, (x, y) in enumerate(pairs)]
    pos = {}  # product index -> position of its mad in `out`

    def collect(j):
        dist = len(out) - pos[j] - 1  # instructions between the mad and this addc
        if dist < 2:
            out.append(f"s_nop {1 - dist}")
        src = "%[z]" if (fresh_c2 and j == 0) else "%[c2]"
        out.append(f"v_addc_co_u32 %[c2], vcc, 0, {src}, %[s{j % NCARRY}]")

    for k, (x, y) in enumerate(pairs):
        pos[k] = len(out)
        out.append(f"v_mad_u64_u32 %[acc], %[s{k % NCARRY}], %[{x}], %[{y}], %[acc]")
        if k >= 2:
            collect(k - 2)
    for j in range(max(0, len(pairs) - 2), len(pairs)):
        collect(j)
    return out


def asm_operand(v):
    """asm input for operand name v = kind + limb index: a, b, m, wq limbs in
    VGPRs, modulus limbs p in SGPRs."""
    kind, idx = v[0], int(v[1:])
    src = {"a": f"a[{idx}]", "b": f"b[{idx}]", "m": f"m[{idx}]", "w": f"wq[{idx}]",
           "d": f"d[{idx}]", "e": f"e[{idx}]", "x": f"x[{idx}]", "y": f"y[{idx}]"}
    if kind == "p":
        return f'[{v}] "s"(Cfg::kP32[{idx}])'
    return f'[{v}] "v"({src[kind]})'


def asm_stmt(pairs, fresh_c2=False, carries=True):
    names = []
    for x, y in pairs:
        for v in (x, y):
            if v not in names:
                names.append(v)
    lines = mac_lines(pairs, fresh_c2, carries)
    text = "\\n\\t".join(lines)
    ins = [asm_operand(v) for v in names]
    if fresh_c2 and carries:
        ins.append('[z] "v"(0u)')
    c2 = '[c2] "=&v"(c2)' if fresh_c2 else '[c2] "+&v"(c2)'
    nsg = min(NCARRY, len(pairs))
    sg = ", ".join(f'[s{i}] "=&s"(sc[{i}])' for i in range(nsg))
    outs = f'[acc] "+&v"(acc), {c2}, {sg}' if carries else f'[acc] "+&v"(acc), {sg}'
    return (f'    asm("{text}"\n'
            f'                 : {outs}\n'
            f'                 : {", ".join(ins)}\n'
            f'                 : "vcc");\n')


def gen(N):
    lines = [f"// N = {N} limbs (32-bit): {2 * N * N} v_mad_u64_u32 + {2 * N * N} v_addc_co_u32",
             "template <class Cfg>",
             f"__device__ __forceinline__ void mont_mul_fips_{N}(uint32_t* __restrict__ r, const uint32_t* __restrict__ a,",
             f"                                                  const uint32_t* __restrict__ b) {{",
             f"  uint32_t m[{N}];",
             "  uint64_t acc = 0;",
             f"  uint64_t sc[{NCARRY}];  // carry-out lane masks (SGPR pairs)",
             "  uint32_t c2;"]
    for k in range(N):
        pairs = []
        for j in range(k):
            pairs.append((f"a{j}", f"b{k - j}"))
            pairs.append((f"m{j}", f"p{k - j}"))
        pairs.append((f"a{k}", "b0"))
        lines.append(f"  {{  // column {k}")
        if k == 0:  # a0*b0 + 0 cannot carry out
            lines.append('    asm("v_mad_u64_u32 %[acc], %[s0], %[a0], %[b0], %[acc]"\n'
                         '                 : [acc] "+&v"(acc), [s0] "=&s"(sc[0])\n'
                         '                 : [a0] "v"(a[0]), [b0] "v"(b[0]));')
            lines.append("    c2 = 0;")
        else:
            lines.append(asm_stmt(pairs, fresh_c2=True).rstrip("\n"))
        lines.append(f"    m[{k}] = (uint32_t)acc * Cfg::kInv32;")
        lines.append(asm_stmt([(f"m{k}", "p0")]).rstrip("\n"))
        lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
        lines.append("  }")
    for k in range(N, 2 * N - 1):
        pairs = []
        for j in range(k - N + 1, N):
            pairs.append((f"a{j}", f"b{k - j}"))
            pairs.append((f"m{j}", f"p{k - j}"))
        lines.append(f"  {{  // column {k}")
        lines.append(asm_stmt(pairs, fresh_c2=True).rstrip("\n"))
        lines.append(f"    r[{k - N}] = (uint32_t)acc;")
        lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
        lines.append("  }")
    lines.append(f"  r[{N - 1}] = (uint32_t)acc;  // < 2p < 2^{32 * N}: the top word is the last one")
    lines.append("}")
    return "\n".join(lines) + "\n"


def gen_sqr(N):
    """Montgomery square by FIPS with the cross products counted once:
    a^2 = sum_i a_i^2 2^(64i) + sum_i a_i 2^(32i) * 2 sum_{j>i} a_j 2^(32j), and
    2 sum_{j>i} a_j 2^(32j) has the limbs of 2a (d_j = a_j << 1 | a_(j-1) >> 31)
    except at j = i + 1, where the bit shifted in from a_i is not part of the
    sum (e_j = a_j << 1), and no limb N when a < 2^(32N-1) (the caller's
    precondition: lazy values < 2p of the 254-bit fields, 381-bit values <
    2p, canonical 255-bit values).  N(N+1)/2 + N^2 products instead of 2N^2:
    100 instead of 128 for N = 8, 222 instead of 288 for N = 12."""
    nprod = N * (N + 1) // 2 + N * N
    lines = [f"// N = {N}: r = a^2 R^-1 < 2p ({nprod} v_mad_u64_u32); a < 2^{32 * N - 1}; see gen_sqr",
             "template <class Cfg>",
             f"__device__ __forceinline__ void mont_sqr_fips_{N}(uint32_t* __restrict__ r, const uint32_t* __restrict__ a) {{",
             f"  uint32_t m[{N}], d[{N}], e[{N}];",
             f"  for (int j = 1; j < {N}; ++j) {{",
             "    d[j] = __builtin_amdgcn_alignbit(a[j], a[j - 1], 31);",
             "    e[j] = a[j] << 1;",
             "  }",
             "  uint64_t acc = 0;",
             f"  uint64_t sc[{NCARRY}];  // carry-out lane masks (SGPR pairs)",
             "  uint32_t c2;"]

    def sq_pairs(k):
        pairs = []
        for i in range(0, (k + 1) // 2):
            j = k - i
            if j >= N or j <= i:
                continue
            pairs.append((f"a{i}", f"e{j}" if j == i + 1 else f"d{j}"))
        if k % 2 == 0 and k // 2 < N:
            pairs.append((f"a{k // 2}", f"a{k // 2}"))
        return pairs

    for k in range(N):
        pairs = []
        sq = sq_pairs(k)
        for j in range(k):
            pairs.append((f"m{j}", f"p{k - j}"))
        # interleave the square's products with the reduction's
        mixed = []
        for t in range(max(len(sq), len(pairs))):
            if t < len(sq):
                mixed.append(sq[t])
            if t < len(pairs):
                mixed.append(pairs[t])
        lines.append(f"  {{  // column {k}")
        if k == 0:  # a0*a0 + 0 cannot carry out
            lines.append('    asm("v_mad_u64_u32 %[acc], %[s0], %[a0], %[a0], %[acc]"\n'
                         '                 : [acc] "+&v"(acc), [s0] "=&s"(sc[0])\n'
                         '                 : [a0] "v"(a[0]));')
            lines.append("    c2 = 0;")
        else:
            lines.append(asm_stmt(mixed, fresh_c2=True).rstrip("\n"))
        lines.append(f"    m[{k}] = (uint32_t)acc * Cfg::kInv32;")
        lines.append(asm_stmt([(f"m{k}", "p0")]).rstrip("\n"))
        lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
        lines.append("  }")
    for k in range(N, 2 * N - 1):
        sq = sq_pairs(k)
        pairs = [(f"m{j}", f"p{k - j}") for j in range(k - N + 1, N)]
        mixed = []
        for t in range(max(len(sq), len(pairs))):
            if t < len(sq):
                mixed.append(sq[t])
            if t < len(pairs):
                mixed.append(pairs[t])
        lines.append(f"  {{  // column {k}")
        lines.append(asm_stmt(mixed, fresh_c2=True).rstrip("\n"))
        lines.append(f"    r[{k - N}] = (uint32_t)acc;")
        lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
        lines.append("  }")
    lines.append(f"  r[{N - 1}] = (uint32_t)acc;")
    lines.append("}")
    return "\n".join(lines) + "\n"


def gen_muladd(N):
    """r = (a*b + c*d) R^-1 mod p with one Montgomery reduction (the Fq2
    product's imaginary part a0 b1 + a1 b0): gen_mulsub's columns with x = c."""
    text = gen_mulsub(N)
    head, body = text.split("  uint64_t acc = 0;", 1)
    head = head.replace(f"mont_mul_sub_fips_{N}", f"mont_mul_add_fips_{N}")
    head = head.replace("r = (a b - c d) R^-1", "r = (a b + c d) R^-1").replace("see gen_mulsub", "see gen_muladd")
    head = head.split(f"  uint32_t m[{N}], x[{N}];")[0] + f"  uint32_t m[{N}];\n  const uint32_t* __restrict__ x = c;\n"
    return head + "  uint64_t acc = 0;" + body


def gen_mulsub(N):
    """r = (a*b - c*d) R^-1 mod p with ONE Montgomery reduction: the columns
    accumulate a*b + x*y + m*p where x = 2p - c (c < 2p, so x in (0, 2p], no
    borrow out) and y = d.  T = a*b + x*y < 8p^2, so the REDC output is
    < 8p^2/R + p: below 2p when p < 2^(32N-3) (BLS12-381 Fq), below 3p when p <
    2^(32N-2) (BN254), where one conditional subtraction of 2p follows (the
    caller's).  2N^2 + N^2 products + N digits instead of two full products
    and a modular subtraction (the y coordinate of every XYZZ addition)."""
    lines = [f"// N = {N}: r = (a b - c d) R^-1 < 8p^2/R + p ({3 * N * N} v_mad_u64_u32); see gen_mulsub",
             "template <class Cfg>",
             f"__device__ __forceinline__ void mont_mul_sub_fips_{N}(uint32_t* __restrict__ r, const uint32_t* __restrict__ a,",
             f"    const uint32_t* __restrict__ b, const uint32_t* __restrict__ c, const uint32_t* __restrict__ y) {{",
             f"  uint32_t m[{N}], x[{N}];"]
    # (a literal and the VCC carry-in would be two constant-bus reads: the
    # modulus limbs move into x first)
    L = [f"v_mov_b32 %[x{i}], %[k{i}]" for i in range(1, N)]
    L += ["v_sub_co_u32 %[x0], vcc, %[k0], %[q0]"]
    for i in range(1, N):
        L += ["s_nop 1", f"v_subb_co_u32 %[x{i}], vcc, %[x{i}], %[q{i}], vcc"]
    lines.append(asm_block(L, [f'[x{i}] "=&v"(x[{i}])' for i in range(N)],
                           [f'[k{i}] "i"(Cfg::kP232[{i}])' for i in range(N)] +
                           [f'[q{i}] "v"(c[{i}])' for i in range(N)]).rstrip("\n"))
    lines += ["  uint64_t acc = 0;", f"  uint64_t sc[{NCARRY}];", "  uint32_t c2;"]
    for k in range(N):
        pairs = []
        for j in range(k + 1):
            pairs.append((f"a{j}", f"b{k - j}"))
            pairs.append((f"x{j}", f"y{k - j}"))
            if j < k:
                pairs.append((f"m{j}", f"p{k - j}"))
        lines.append(f"  {{  // column {k}")
        lines.append(asm_stmt(pairs, fresh_c2=True).rstrip("\n"))
        lines.append(f"    m[{k}] = (uint32_t)acc * Cfg::kInv32;")
        lines.append(asm_stmt([(f"m{k}", "p0")]).rstrip("\n"))
        lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
        lines.append("  }")
    for k in range(N, 2 * N - 1):
        pairs = []
        for j in range(k - N + 1, N):
            pairs.append((f"a{j}", f"b{k - j}"))
            pairs.append((f"x{j}", f"y{k - j}"))
            pairs.append((f"m{j}", f"p{k - j}"))
        lines.append(f"  {{  // column {k}")
        lines.append(asm_stmt(pairs, fresh_c2=True).rstrip("\n"))
        lines.append(f"    r[{k - N}] = (uint32_t)acc;")
        lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
        lines.append("  }")
    lines.append(f"  r[{N - 1}] = (uint32_t)acc;")
    lines.append("}")
    return "\n".join(lines) + "\n"


SHOUP_DROP = 6  # low columns of a*wq left out of the quotient estimate


def gen_shoup(N):
    """Shoup product by a precomputed constant: r = a*w - q*p with
    q = floor(a * wq / 2^(32N)), wq = floor(w * 2^(32N) / p), w < p, any
    a < 2^(32N).  The quotient's low SHOUP_DROP columns are left out (the
    estimate is q or q - 1), and r = lo(a*w) - lo(q*p) in [0, 3p):
    2N^2 - D(D+1)/2 + N(N+1) products and no Montgomery digits."""
    D = SHOUP_DROP
    nprod = sum(min(k, N - 1) - max(0, k - N + 1) + 1 for k in range(D, 2 * N - 1)) + N * (N + 1)
    lines = [f"// N = {N}: r = a*w mod p in [0, 3p) (Shoup; {nprod} v_mad_u64_u32); see gen_shoup",
             "template <class Cfg>",
             f"__device__ __forceinline__ void shoup_mul_{N}(uint32_t* __restrict__ r, const uint32_t* __restrict__ a,",
             f"                                             const uint32_t* __restrict__ b, const uint32_t* __restrict__ wq) {{",
             f"  uint32_t m[{N}];  // quotient estimate",
             "  uint64_t acc = 0;",
             f"  uint64_t sc[{NCARRY}];",
             "  uint32_t c2;"]
    for k in range(D, 2 * N - 1):
        pairs = [(f"a{i}", f"w{k - i}") for i in range(max(0, k - N + 1), min(k, N - 1) + 1)]
        lines.append(f"  {{  // quotient column {k}")
        lines.append(asm_stmt(pairs, fresh_c2=True).rstrip("\n"))
        if k >= N:
            lines.append(f"    m[{k - N}] = (uint32_t)acc;")
        lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
        lines.append("  }")
    lines.append(f"  m[{N - 1}] = (uint32_t)acc;  // a*wq < 2^{64 * N}: the top word")
    # r = lo(a*w) - lo(q*p): two low-half products (the modulus stays in the
    # SGPRs the kernel's Montgomery products already hold) and one borrow chain
    lines.append(f"  uint32_t t[{N}];")
    for name, x, y in (("r", "a", "b"), ("t", "m", "p")):
        lines.append("  acc = 0;")
        for k in range(N):
            pairs = [(f"{x}{i}", f"{y}{k - i}") for i in range(k + 1)]
            last = k == N - 1
            lines.append(f"  {{  // {name}: column {k}")
            if k == 0:
                lines.append(f'    asm("v_mad_u64_u32 %[acc], %[s0], %[{x}0], %[{y}0], %[acc]"\n'
                             f'                 : [acc] "+&v"(acc), [s0] "=&s"(sc[0])\n'
                             f'                 : {asm_operand(x + "0")}, {asm_operand(y + "0")});')
                lines.append("    c2 = 0;")
            else:
                lines.append(asm_stmt(pairs, fresh_c2=True, carries=not last).rstrip("\n"))
            lines.append(f"    {name}[{k}] = (uint32_t)acc;")
            if not last:
                lines.append("    acc = (acc >> 32) | ((uint64_t)c2 << 32);")
            lines.append("  }")
    L = ["v_sub_co_u32 %[r0], vcc, %[r0], %[t0]"]
    for i in range(1, N):
        L += ["s_nop 1", f"v_subb_co_u32 %[r{i}], vcc, %[r{i}], %[t{i}], vcc"]
    lines.append(asm_block(L, [f'[r{i}] "+v"(r[{i}])' for i in range(N)],
                           [f'[t{i}] "v"(t[{i}])' for i in range(N)]).rstrip("\n"))
    lines.append("}")
    return "\n".join(lines) + "\n"


def operand_list(spec):
    return ", ".join(spec)


def asm_block(lines, outs, ins, volatile=False):
    text = "\\n\\t".join(x for x in lines if x)
    kw = "asm volatile" if volatile else "asm"
    return (f'  {kw}("{text}"\n'
            f'      : {operand_list(outs)}\n'
            f'      : {operand_list(ins)}\n'
            f'      : "vcc");\n')


def interleave_select(N, chain_a, chain_b_name, out_sel):
    """Two dependent carry chains, hazard-free without nops: chain A (VCC)
    produces limb i, chain B (SGPR pair %[sb], e64 forms) consumes it one step
    behind, and the N moves of the modulus limbs fill the remaining slot, so
    consecutive links of either chain are two instructions apart.  Finally
    out_sel selects limbwise on B's (or A's) last carry."""
    L = ["v_mov_b32 %[t0], %[m0]"]
    L.append(chain_a(0))
    L.append("v_mov_b32 %[t1], %[m1]")
    for i in range(1, N):
        L.append(chain_b_name(i - 1))
        L.append(chain_a(i))
        if i + 1 < N:
            L.append(f"v_mov_b32 %[t{i + 1}], %[m{i + 1}]")
        else:
            L.append("s_nop 0")
    L.append(chain_b_name(N - 1))
    L.append("s_nop 1")
    L += out_sel
    return L


def gen_addsub(N):
    """add_mod / sub_mod / cond_sub for N 32-bit limbs with the modulus M
    (p or 2p) as 32-bit literals ("i" operands): VCC carry chains instead of
    hipcc's 64-bit emulation (v_lshl_add_u64 + v_ashrrev per limb)."""
    m_in = [f'[m{i}] "i"(ModLimb<Cfg, k2p>::get({i}))' for i in range(N)]
    a_in = [f'[a{i}] "v"(a[{i}])' for i in range(N)]
    b_in = [f'[b{i}] "v"(b[{i}])' for i in range(N)]
    r_out = [f'[r{i}] "=&v"(r[{i}])' for i in range(N)]
    t_out = [f'[t{i}] "=&v"(t[{i}])' for i in range(N)]
    sb_out = ['[sb] "=&s"(sb)']
    out = []

    # ---- add: r = a + b (VCC chain); t = r - M (sb chain); r = borrow(sb) ? r : t
    def add_a(i):
        return ("v_add_co_u32 %[r0], vcc, %[a0], %[b0]" if i == 0
                else f"v_addc_co_u32 %[r{i}], vcc, %[a{i}], %[b{i}], vcc")

    def add_b(i):
        return ("v_sub_co_u32_e64 %[t0], %[sb], %[r0], %[t0]" if i == 0
                else f"v_subb_co_u32_e64 %[t{i}], %[sb], %[r{i}], %[t{i}], %[sb]")
    L = interleave_select(N, add_a, add_b,
                          [f"v_cndmask_b32_e64 %[r{i}], %[t{i}], %[r{i}], %[sb]" for i in range(N)])
    # single-chain form: one VCC chain at a time, s_nop 1 between links
    L1 = [add_a(0)]
    for i in range(1, N):
        L1 += ["s_nop 1", add_a(i)]
    L1 += [f"v_mov_b32 %[t{i}], %[m{i}]" for i in range(1, N)]
    L1 += ["v_subrev_co_u32 %[t0], vcc, %[m0], %[r0]"]
    for i in range(1, N):
        L1 += ["s_nop 1", f"v_subb_co_u32 %[t{i}], vcc, %[r{i}], %[t{i}], vcc"]
    L1 += ["s_nop 1"] + [f"v_cndmask_b32 %[r{i}], %[t{i}], %[r{i}], vcc" for i in range(N)]
    out.append(f"// r = a + b mod M, M = k2p ? 2p : p; a, b < M and 2M < 2^{32 * N}\n"
               f"template <class Cfg, bool k2p>\n"
               f"__device__ __forceinline__ void add_mod_{N}(uint32_t* r, const uint32_t* a, const uint32_t* b) {{\n"
               f"  uint32_t t[{N}];\n  uint64_t sb;\n#if TA_ADDSUB_INTERLEAVE\n"
               + asm_block(L, r_out + t_out + sb_out, a_in + b_in + m_in) + "#else\n  (void)sb;\n"
               + asm_block(L1, r_out + t_out, a_in + b_in + m_in) + "#endif\n}\n")

    # ---- sub: r = a - b (VCC chain); t = r + M (sb chain); r = borrow(vcc) ? t : r
    def sub_a(i):
        return ("v_sub_co_u32 %[r0], vcc, %[a0], %[b0]" if i == 0
                else f"v_subb_co_u32 %[r{i}], vcc, %[a{i}], %[b{i}], vcc")

    def sub_b(i):
        return ("v_add_co_u32_e64 %[t0], %[sb], %[r0], %[t0]" if i == 0
                else f"v_addc_co_u32_e64 %[t{i}], %[sb], %[r{i}], %[t{i}], %[sb]")
    L = interleave_select(N, sub_a, sub_b,
                          [f"v_cndmask_b32 %[r{i}], %[r{i}], %[t{i}], vcc" for i in range(N)])
    L1 = [sub_a(0)]
    for i in range(1, N):
        L1 += ["s_nop 1", sub_a(i)]
    L1 += ["s_nop 1", f"v_subb_co_u32 %[t0], vcc, %[r{N - 1}], %[r{N - 1}], vcc"]  # t0 = -borrow
    L1 += [f"v_and_b32 %[t{i}], %[m{i}], %[t0]" for i in range(N - 1, -1, -1)]
    L1 += ["v_add_co_u32 %[r0], vcc, %[r0], %[t0]"]
    for i in range(1, N):
        L1 += ["s_nop 1", f"v_addc_co_u32 %[r{i}], vcc, %[r{i}], %[t{i}], vcc"]
    out.append(f"// r = a - b mod M (a - b + M selected on borrow)\n"
               f"template <class Cfg, bool k2p>\n"
               f"__device__ __forceinline__ void sub_mod_{N}(uint32_t* r, const uint32_t* a, const uint32_t* b) {{\n"
               f"  uint32_t t[{N}];\n  uint64_t sb;\n#if TA_ADDSUB_INTERLEAVE\n"
               + asm_block(L, r_out + t_out + sb_out, a_in + b_in + m_in) + "#else\n  (void)sb;\n"
               + asm_block(L1, r_out + t_out, a_in + b_in + m_in) + "#endif\n}\n")

    # ---- sub_unreduced: r = a - b + M (mod 2^32N), no borrow test: the a - b
    # chain on VCC, + M one step behind on %[sb]; the final borrow and carry
    # cancel.  ff.h's Fp::sub_unreduced (M = 2p, lazy a, b < 2p, so r < 4p)
    # feeds the result straight into a product with a canonical factor
    def unr_b(i):
        return ("v_add_co_u32_e64 %[r0], %[sb], %[r0], %[t0]" if i == 0
                else f"v_addc_co_u32_e64 %[r{i}], %[sb], %[r{i}], %[t{i}], %[sb]")
    L = interleave_select(N, sub_a, unr_b, [])
    assert L[-1] == "s_nop 1"
    L = L[:-1]  # nothing reads the last carry
    out.append(f"// r = a - b + M (mod 2^{32 * N}) without the borrow test\n"
               f"template <class Cfg, bool k2p>\n"
               f"__device__ __forceinline__ void sub_unreduced_{N}(uint32_t* r, const uint32_t* a, const uint32_t* b) {{\n"
               f"  uint32_t t[{N}];\n  uint64_t sb;\n"
               + asm_block(L, r_out + t_out + sb_out, a_in + b_in + m_in) + "}\n")

    # ---- cond_sub: r = r >= M ? r - M : r  (in place; off the hot path)
    rio = [f'[r{i}] "+v"(r[{i}])' for i in range(N)]
    L = [f"v_mov_b32 %[t{i}], %[m{i}]" for i in range(1, N)]
    L += ["v_subrev_co_u32 %[t0], vcc, %[m0], %[r0]"]
    for i in range(1, N):
        L += ["s_nop 1", f"v_subb_co_u32 %[t{i}], vcc, %[r{i}], %[t{i}], vcc"]
    L += ["s_nop 1"]
    L += [f"v_cndmask_b32 %[r{i}], %[t{i}], %[r{i}], vcc" for i in range(N)]
    out.append(f"// r = r - M if r >= M  (r < 2^{32 * N})\n"
               f"template <class Cfg, bool k2p>\n"
               f"__device__ __forceinline__ void cond_sub_{N}(uint32_t* r) {{\n"
               f"  uint32_t t[{N}];\n" + asm_block(L, rio + t_out, m_in) + "}\n")
    return "\n".join(out)


def render():
    """The text of mont_asm.h (tests/test_generated_asm.py checks the committed
    header against it)."""
    text = ["// GENERATED by tools/gen_mont_asm.py -- do not edit.",
            "// FIPS Montgomery product for gfx950 (see the generator for the rationale).",
            "// Output is < 2p (the caller applies the final conditional subtraction).",
            "#pragma once", "#include <cstdint>", "",
            "// add/sub: 1 = two interleaved carry chains (no nops), 0 = one chain with s_nop 1 per link\n// (0 measured ~1% faster in the MSM accumulation: fewer VGPRs, shorter encodings)",
            "#ifndef TA_ADDSUB_INTERLEAVE", "#define TA_ADDSUB_INTERLEAVE 0", "#endif", "",
            "namespace tachyon_amd::detail {", ""]
    text.append("template <class Cfg, bool k2p>\nstruct ModLimb {\n"
                "  static constexpr uint32_t get(int i) { return k2p ? Cfg::kP232[i] : Cfg::kP32[i]; }\n};\n")
    for N in (8, 12):
        text.append(gen(N))
        text.append(gen_sqr(N))
        text.append(gen_addsub(N))
    text.append(gen_mulsub(8))
    text.append(gen_mulsub(12))
    text.append(gen_muladd(8))
    text.append(gen_muladd(12))
    text.append(gen_shoup(8))
    text.append("}  // namespace tachyon_amd::detail")
    return "\n".join(text) + "\n"


def main():
    with open(OUT, "w") as f:
        f.write(render())
    print("wrote", os.path.relpath(OUT, ROOT))


if __name__ == "__main__":
    main()
