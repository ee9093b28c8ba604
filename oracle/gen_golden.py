#!/usr/bin/env python3
"""ORACLE (test infrastructure only): write the golden fixtures in tests/golden/.

Run from the repo root:  python -m oracle.gen_golden  [--reference /root/reference]

Everything is computed by oracle/pyref.py (independent pure-Python big-int
restatement).  The only reference *data* read is
vendors/circom/examples/multiplier_3.zkey (a binary fixture the reference's own
zkey_unittest.cc parses); its points are extracted as data and cross-checked
against the decimal coordinates that zkey_unittest.cc:71-140 states.
Outputs are JSON with hex strings of the reference's in-memory layout
(Montgomery form, little-endian 64-bit limbs).
"""
import argparse
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyref  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
SEED = 0x7AC40001


def hx(b: bytes) -> str:
    return b.hex()


def field_ops():
    out = {}
    for name in ("bn254_fq", "bn254_fr", "bls12_381_fq", "bls12_381_fr"):
        F = pyref.Field(name)
        cases = []
        vals = [0, 1, 2, F.p - 1, F.p - 2, (F.p - 1) // 2]
        vals += [pyref.rand_scalar(SEED ^ 0xF1E1D, i, F.p) if F.n64 == 4 else
                 sum(pyref.rand_u64(SEED ^ 0xF1E1D, 6 * i + k) << (64 * k) for k in range(6)) % F.p
                 for i in range(26)]
        for i in range(len(vals)):
            a = vals[i]
            b = vals[(i * 7 + 3) % len(vals)]
            cases.append(dict(
                a=hx(F.to_bytes(a)), b=hx(F.to_bytes(b)),
                a_canonical=hx(a.to_bytes(F.nbytes, "little")),
                add=hx(F.to_bytes(a + b)), sub=hx(F.to_bytes(a - b)), mul=hx(F.to_bytes(a * b)),
                sqr=hx(F.to_bytes(a * a)), neg=hx(F.to_bytes(-a)), dbl=hx(F.to_bytes(2 * a)),
                inv=hx(F.to_bytes(F.inv(a))) if a else None,
            ))
        out[name] = cases
    return out


def msm_cases():
    out = {}
    plan = {
        "bn254_g1": [(1, 1), (2, 2), (5, 2), (32, 8), (40, 7), (64, 64)],
        "bn254_g2": [(2, 2), (5, 3), (16, 4)],
        "bls12_381_g1": [(2, 2), (5, 5), (32, 8)],
        "bls12_381_g2": [(2, 2), (5, 3), (12, 4)],
    }
    for cname, sizes in plan.items():
        C = pyref.Curve(cname)
        cases = []
        for n, chunk in sizes:
            seed = SEED + n
            bases = pyref.gen_bases(C, seed, n, chunk)
            scalars = pyref.gen_scalars(C.Fr, seed, n)
            assert all(C.on_curve(b) for b in bases)
            res = pyref.msm(C, bases, scalars)
            cases.append(dict(
                n=n, seed=seed, chunk=chunk,
                bases=[hx(C.to_bytes(b)) for b in bases],
                scalars=[hx(C.Fr.to_bytes(s)) for s in scalars],
                expected=hx(C.to_bytes(res)),
            ))
        # edge cases: zero scalars, identity bases, all-equal scalars, P + (-P)
        n = 9
        bases = pyref.gen_bases(C, SEED, n, 3)
        bases[2] = None
        bases[5] = C.neg(bases[4])
        scalars = pyref.gen_scalars(C.Fr, SEED, n)
        scalars[0] = 0
        scalars[5] = scalars[4]
        scalars[7] = C.Fr.p - 1
        cases.append(dict(n=n, seed=None, chunk=None, label="edge",
                          bases=[hx(C.to_bytes(b)) for b in bases],
                          scalars=[hx(C.Fr.to_bytes(s)) for s in scalars],
                          expected=hx(C.to_bytes(pyref.msm(C, bases, scalars)))))
        # Easy KAT (variable_base_msm_test_set.h:55-68): bases = G, scalars 1..n
        for n in (1, 7, 40):
            cases.append(dict(n=n, seed=None, chunk=None, label="easy",
                              bases=[hx(C.to_bytes(C.G))] * n,
                              scalars=[hx(C.Fr.to_bytes(i + 1)) for i in range(n)],
                              expected=hx(C.to_bytes(C.mul(C.G, n * (n + 1) // 2)))))
        out[cname] = dict(point_bytes=C.point_bytes, scalar_bytes=C.Fr.nbytes, cases=cases)
    return out


def ntt_cases(field="bn254_fr", coset=5, two_adicity=28):
    """Radix-2 FFT / IFFT golden vectors by pyref's O(n^2) DFT: plain and on
    the coset `coset` * <w> (5 for BN254 Fr as the reference's GPU unittest,
    7 = BLS12-381 Fr's BUILD subgroup generator)."""
    F = pyref.Field(field)
    cases = []
    for logn in range(0, 8):
        n = 1 << logn
        for num_coeffs in sorted({n, max(1, n // 2 + 1), max(1, n // 4)}):
            if num_coeffs > n:
                continue
            seed = SEED + 1000 * logn + num_coeffs
            coeffs = pyref.gen_scalars(F, seed, num_coeffs)
            for offset in (1, coset):
                ev = pyref.fft(F, coeffs, n, offset)
                back = pyref.ifft(F, ev, n, offset)
                assert back == coeffs + [] or back == list(coeffs[:len(back)])
                cases.append(dict(
                    log_n=logn, num_coeffs=num_coeffs, offset=offset,
                    offset_mont=hx(F.to_bytes(offset)),
                    coeffs=[hx(F.to_bytes(c)) for c in coeffs],
                    evals=[hx(F.to_bytes(e)) for e in ev],
                    ifft_of_evals=[hx(F.to_bytes(c)) for c in back],
                ))
    roots = {str(k): hx(F.to_bytes(F.root_of_unity(1 << k))) for k in range(0, two_adicity + 1)}
    return dict(field=field, two_adic_root_of_unity=str(F.root_of_unity(1 << two_adicity)),
                roots_of_unity_mont=roots, cases=cases)


# ---- multiplier_3.zkey (binary fixture of the reference) ------------------
# Decimal coordinates stated by vendors/circom/circomlib/zkey/zkey_unittest.cc:71-215.
ZKEY_EXPECTED = {
    "alpha_g1": ["5700502584084766622350343367608487274977128430049880895783423261700075212785",
                 "9143870410831450591509938003078256759736333300521257694515214164265805259830"],
    "beta_g1": ["12699714711422499622362310820475830692566951228171954587615996781136226772367",
                "2601999511749500018822665665362525344184434745926911293241192574303473253831"],
    "delta_g1": ["18121096455458648748006856505340317178704791872899059396361359566439114201168",
                 "1584219057669659447306711278235088033786171030532185363250775914928871374123"],
    "beta_g2": [["11780196173848324687642894328871430898972567583635494711927265792805257024861",
                 "3029614260803671687015271480824975868088527303860361358764452805565479529001"],
                ["17817615377642575824268866714659516420384007262298492272608472268977629075434",
                 "10565581580493997556536063930500447170628763955833078597453719665182760199848"]],
    "points_a1": [["8858563469144920540528478490224638442973773873152551307670564100347093499191",
                   "7888214391937843930525848128254405915157714572978190674521564636068162216311"],
                  ["14537214592124271965353533016257772100455033778428577041971202446686849252644",
                   "2198766467867023896703420308951432042782623727887618971273865174145643356495"],
                  ["8437302598248383817148383036741547214048558400312301295747047351838256772123",
                   "4253086419746464003785043685439509391398040483296248505707498714848332192725"],
                  ["0", "0"], ["0", "0"],
                  ["18141870587741836486360437684811661514896911334995841933942081072546739652377",
                   "11898889550822544273094627075076607374273361105699305622414170117806818640166"]],
}


def parse_zkey(path):
    data = open(path, "rb").read()
    assert data[:4] == b"zkey"
    version, nsec = struct.unpack_from("<II", data, 4)
    off = 12
    sections = {}
    for _ in range(nsec):
        typ, size = struct.unpack_from("<IQ", data, off)
        off += 12
        sections[typ] = data[off:off + size]
        off += size
    g = sections[2]
    n8q = struct.unpack_from("<I", g, 0)[0]
    o = 4 + n8q
    n8r = struct.unpack_from("<I", g, o)[0]
    o += 4 + n8r
    nvars, npub, dsize = struct.unpack_from("<III", g, o)
    o += 12
    g1, g2 = 2 * n8q, 4 * n8q
    hdr = {}
    for name, sz in (("alpha_g1", g1), ("beta_g1", g1), ("beta_g2", g2), ("gamma_g2", g2),
                     ("delta_g1", g1), ("delta_g2", g2)):
        hdr[name] = g[o:o + sz]
        o += sz

    def split(sec, sz):
        return [sec[i:i + sz] for i in range(0, len(sec), sz)]

    return dict(version=version, n_vars=nvars, n_public=npub, domain_size=dsize, header=hdr,
                ic=split(sections[3], g1), a1=split(sections[5], g1), b1=split(sections[6], g1),
                b2=split(sections[7], g2), c1=split(sections[8], g1), h1=split(sections[9], g1))


def zkey_fixture(ref_root):
    path = os.path.join(ref_root, "vendors/circom/examples/multiplier_3.zkey")
    z = parse_zkey(path)
    G1 = pyref.Curve("bn254_g1")
    G2 = pyref.Curve("bn254_g2")
    # zkey stores Montgomery-form LE coordinates (the reference reads them
    # straight into its Montgomery PrimeField).  Check against the decimals.
    def dec_g1(b):
        p = G1.from_bytes(b)
        return ["0", "0"] if p is None else [str(p[0]), str(p[1])]

    def dec_g2(b):
        p = G2.from_bytes(b)
        return [["0", "0"], ["0", "0"]] if p is None else [[str(p[0][0]), str(p[0][1])],
                                                          [str(p[1][0]), str(p[1][1])]]
    assert dec_g1(z["header"]["alpha_g1"]) == ZKEY_EXPECTED["alpha_g1"]
    assert dec_g1(z["header"]["beta_g1"]) == ZKEY_EXPECTED["beta_g1"]
    assert dec_g1(z["header"]["delta_g1"]) == ZKEY_EXPECTED["delta_g1"]
    assert dec_g2(z["header"]["beta_g2"]) == ZKEY_EXPECTED["beta_g2"]
    assert [dec_g1(b) for b in z["a1"]] == ZKEY_EXPECTED["points_a1"]
    g1_points = [z["header"]["alpha_g1"], z["header"]["beta_g1"], z["header"]["delta_g1"]] + \
        z["ic"] + z["a1"] + z["b1"] + z["c1"] + z["h1"]
    g2_points = [z["header"]["beta_g2"], z["header"]["gamma_g2"], z["header"]["delta_g2"]] + z["b2"]
    assert all(G1.on_curve(G1.from_bytes(b)) for b in g1_points)
    assert all(G2.on_curve(G2.from_bytes(b)) for b in g2_points)
    out = dict(source="vendors/circom/examples/multiplier_3.zkey",
               expected_decimal=ZKEY_EXPECTED,
               g1_points=[hx(b) for b in g1_points], g2_points=[hx(b) for b in g2_points])
    # MSMs over the real points, answers by pyref
    for key, C, pts in (("g1", G1, g1_points), ("g2", G2, g2_points)):
        bases = [C.from_bytes(b) for b in pts]
        scalars = pyref.gen_scalars(C.Fr, SEED ^ 0x2EE, len(bases))
        out[f"msm_{key}"] = dict(scalars=[hx(C.Fr.to_bytes(s)) for s in scalars],
                                 expected=hx(C.to_bytes(pyref.msm(C, bases, scalars))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", default=None, help="write only this golden file (e.g. ntt_bls12_381_fr.json)")
    args = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    outputs = {
        "field_ops.json": field_ops,
        "msm.json": msm_cases,
        "ntt_bn254_fr.json": ntt_cases,
        "ntt_bls12_381_fr.json": lambda: ntt_cases("bls12_381_fr", coset=7, two_adicity=32),
    }
    if args.only:
        outputs = {args.only: outputs[args.only]}
    outputs = {k: f() for k, f in outputs.items()}
    if os.path.isdir(args.reference) and not args.only:
        outputs["zkey_multiplier_3.json"] = zkey_fixture(args.reference)
    for name, obj in outputs.items():
        with open(os.path.join(GOLDEN, name), "w") as f:
            json.dump(obj, f, indent=0)
        print("wrote tests/golden/" + name)


if __name__ == "__main__":
    main()
