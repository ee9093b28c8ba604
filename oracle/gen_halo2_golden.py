"""ORACLE (test infrastructure only): extract the reference's own halo2 NTT and
KZG outputs into tests/golden/halo2_circuits.json.

The reference's PLONK example tests hold, per circuit, values that its own
CPU path computed on the halo2 BN254 Fr domain (generator 7, installed by
math::halo2::OverrideSubgroupGenerator(), bn/bn254/halo2/bn254.cc:7-30, in
CircuitTest::SetUpTestSuite, zk/plonk/examples/circuit_test.h:43-46):

* kFixedColumns -> kFixedPolys             fixed_polys_ = domain->IFFT(columns)
                                            (zk/plonk/keys/proving_key.h:97-100)
* kPermutationsColumns -> kPermutationsPolys  the permutation proving key's polys
                                            (IFFT of the permutation columns)
* kLFirst / kLLast / kLActiveRow            IFFT of the l_first / l_last /
                                            l_active_row indicator columns
                                            (proving_key.h:114-166; kScroll vendor:
                                            coefficient form, n entries)
* PinnedVerifyingKey `omega`                the domain generator w_n
* PinnedVerifyingKey `fixed_commitments`    pcs.CommitLagrange(fixed column)
  and `permutation ... commitments`         (zk/plonk/keys/verifying_key.h:94-100),
                                            KZG UnsafeSetup(kN, tau = 2)
                                            (circuit_test.h:66; kzg.h:173-207)

Run here (it reads /root/reference, which the GPU box does not have):
    python oracle/gen_halo2_golden.py
The output is data only: circuit name, n, and canonical hex values (the
reference's own strings, `F::FromHexString` / Rust debug form).
"""
import json
import os
import re
import sys

REF = "/root/reference/tachyon/zk/plonk/examples"
FILES = [
    "simple_circuit_test_data.h",
    "simple_lookup_circuit_test_data.h",
    "shuffle_circuit_test_data.h",
    "shuffle_api_circuit_test_data.h",
    "multi_lookup_circuit_test_data.h",
    "fibonacci/fibonacci1_circuit_test_data.h",
    "fibonacci/fibonacci2_circuit_test_data.h",
    "fibonacci/fibonacci3_circuit_test_data.h",
]
ARRAYS = {
    "kFixedColumns": "fixed_columns",
    "kFixedPolys": "fixed_polys",
    "kPermutationsColumns": "permutations_columns",
    "kPermutationsPolys": "permutations_polys",
    "kLFirst": "l_first",
    "kLLast": "l_last",
    "kLActiveRow": "l_active_row",
}
HEX = re.compile(r'"(0x[0-9a-fA-F]+)"')


def _array_body(seg, start):
    """Text of the brace-balanced initializer that opens at seg[start] == '{'."""
    depth = 0
    for i in range(start, len(seg)):
        c = seg[i]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return seg[start:i + 1]
    raise ValueError("unbalanced initializer")


def _parse_array(body):
    """1-D list of hex strings, or 2-D list (one list per inner {...})."""
    inner = body[1:-1]
    if "{" not in inner:
        return HEX.findall(inner)
    rows, depth, cur = [], 0, []
    for tok in re.finditer(r'\{|\}|"0x[0-9a-fA-F]+"', inner):
        t = tok.group(0)
        if t == "{":
            depth += 1
            cur = []
        elif t == "}":
            depth -= 1
            rows.append(cur)
        else:
            cur.append(t.strip('"'))
    return rows


def _pinned_vk(seg):
    m = re.search(r"kPinnedVerifyingKey\s*=\s*((?:\s*\"(?:[^\"\\]|\\.)*\")+)\s*;", seg)
    if not m:
        return None
    text = "".join(re.findall(r"\"((?:[^\"\\]|\\.)*)\"", m.group(1))).replace('\\"', '"')
    out = {}
    om = re.search(r"omega: (0x[0-9a-f]+)", text)
    k = re.search(r"\bk: (\d+)", text)
    out["k"] = int(k.group(1)) if k else None
    out["omega"] = om.group(1) if om else None

    def points(s):
        return [[a, b] for a, b in re.findall(r"\((0x[0-9a-f]+), (0x[0-9a-f]+)\)", s)]

    fc = re.search(r"fixed_commitments: \[(.*?)\]", text)
    out["fixed_commitments"] = points(fc.group(1)) if fc else []
    pc = re.search(r"permutation: VerifyingKey \{ commitments: \[(.*?)\]", text)
    out["permutation_commitments"] = points(pc.group(1)) if pc else []
    return out


def extract(path):
    text = open(path).read()
    starts = [m.start() for m in re.finditer(r"^class \w+", text, re.M)] + [len(text)]
    cases = []
    for a, b in zip(starts, starts[1:]):
        seg = text[a:b]
        kn = re.search(r"constexpr static size_t kN = (\d+);", seg)
        if not kn:
            continue
        head = seg.split("{", 1)[0]
        case = {"n": int(kn.group(1)), "class": " ".join(head.split())}
        for cname, key in ARRAYS.items():
            m = re.search(r"constexpr static std::string_view " + cname + r"\[\](?:\[kN\])?\s*=\s*", seg)
            if m:
                v = _parse_array(_array_body(seg, seg.index("{", m.end() - 1)))
                if v:
                    case[key] = v
        vk = _pinned_vk(seg)
        if vk:
            case.update({k: v for k, v in vk.items() if v})
        if len(case) > 2:  # some classes leave every value empty (kPinnedVerifyingKey = "")
            cases.append(case)
    return cases


def main():
    out_path = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "halo2_circuits.json")
    result = {
        "source": "reference tachyon/zk/plonk/examples/*_test_data.h (values the reference computed)",
        "domain": "halo2 BN254 Fr (generator 7), bn/bn254/halo2/bn254.cc:7-30",
        "kzg_tau": 2,
        "circuits": [],
    }
    for f in FILES:
        p = os.path.join(REF, f)
        for i, c in enumerate(extract(p)):
            c["file"] = f
            c["index"] = i
            result["circuits"].append(c)
    with open(out_path, "w") as fh:
        json.dump(result, fh, indent=1)
    summary = [(c["file"], c["index"], c["n"], sorted(k for k in c if k in ARRAYS.values() or k.endswith("commitments")))
               for c in result["circuits"]]
    for s in summary:
        print(s)
    return 0


if __name__ == "__main__":
    sys.exit(main())
