"""Curve and field parameters for the MSM/NTT hot path (single source of truth).

Every number here is copied from the reference's bazel rule arguments, which
are the only place the reference states them (its C++ constants are generated
at build time by the prime_field_generator genrule):

* BN254       -- tachyon/math/elliptic_curves/bn/bn254/BUILD.bazel:27-200
* BLS12-381   -- tachyon/math/elliptic_curves/bls12/bls12_381/BUILD.bazel:36-199

`tools/gen_constants.py` turns these into the Montgomery-form C headers that
the HIP kernels (tachyon_amd/csrc/field/constants.h) and the oracle
(oracle/oracle_constants.h) compile against.
"""

# --- BN254 ------------------------------------------------------------------
BN254_FQ = 21888242871839275222246405745257275088696311157297823662689037894645226208583
BN254_FR = 21888242871839275222246405745257275088548364400416034343698204186575808495617
BN254_FR_SUBGROUP_GENERATOR = 5          # BUILD.bazel:46-50 (fr_subgroup_generator)
BN254_FQ_SUBGROUP_GENERATOR = 3          # BUILD.bazel:20-23

BN254_G1 = dict(a=[0], b=[3], x=[1], y=[2])                      # BUILD.bazel:127-147
BN254_G2 = dict(                                                   # BUILD.bazel:149-200
    a=[0, 0],
    b=[19485874751759354771024239261021720505790618469301721065564631296452457478373,
       266929791119991161246907387137283842545076965332900288569378510910307636690],
    x=[10857046999023057135944570762232829481370756359578518086990519993285655852781,
       11559732032986387107991004021392285783925812861821192530917403151452391805634],
    y=[8495653923123431417604973247489272438418190587263600148770280649306958101930,
       4082367875863433681332203403145435568316851327593401208105741076214120093531],
)
BN254_FQ2_NON_RESIDUE = -1                                         # BUILD.bazel:62-71

# --- BLS12-381 --------------------------------------------------------------
BLS12_381_FQ = int(
    "4002409555221667393417789825735904156556882819939007885332058136124031650490837864442687629129015664037894272559787")
BLS12_381_FR = 52435875175126190479447740508185965837690552500527637822603658699938581184513
BLS12_381_FR_SUBGROUP_GENERATOR = 7      # BUILD.bazel (fr_subgroup_generator = 7)
BLS12_381_G1 = dict(                                               # BUILD.bazel:128-150
    a=[0], b=[4],
    x=[int("3685416753713387016781088315183077757961620795782546409894578378688607592378376318836054947676345821548104185464507")],
    y=[int("1339506544944476473020471379941921221584933875938349620426543736416511423956333506472724655353366534992391756441569")],
)
BLS12_381_G2 = dict(                                               # BUILD.bazel:152-199
    a=[0, 0], b=[4, 4],
    x=[int("352701069587466618187139116011060144890029952792775240219908644239793785735715026873347600343865175952761926303160"),
       int("3059144344244213709971259814753781636986470325476647558659373206291635324768958432433509563104347017837885763365758")],
    y=[int("1985150602287291935568054521177171638300868978215655730859378665066344726373823718423869104263333984641494340347905"),
       int("927553665492332455747201965776037880757740193453592970025027978793976877002675564980949289727957565575433344219582")],
)
BLS12_381_FQ2_NON_RESIDUE = -1

# name -> (modulus, 64-bit limb count, multiplicative generator or None)
FIELDS = {
    "bn254_fq": (BN254_FQ, 4, BN254_FQ_SUBGROUP_GENERATOR),
    "bn254_fr": (BN254_FR, 4, BN254_FR_SUBGROUP_GENERATOR),
    "bls12_381_fq": (BLS12_381_FQ, 6, None),
    "bls12_381_fr": (BLS12_381_FR, 4, BLS12_381_FR_SUBGROUP_GENERATOR),
}

# name -> (base field, degree, scalar field, params)
CURVES = {
    "bn254_g1": ("bn254_fq", 1, "bn254_fr", BN254_G1),
    "bn254_g2": ("bn254_fq", 2, "bn254_fr", BN254_G2),
    "bls12_381_g1": ("bls12_381_fq", 1, "bls12_381_fr", BLS12_381_G1),
    "bls12_381_g2": ("bls12_381_fq", 2, "bls12_381_fr", BLS12_381_G2),
}


def two_adicity(p: int) -> int:
    s, t = 0, p - 1
    while t % 2 == 0:
        s, t = s + 1, t // 2
    return s


def mont(x: int, p: int, n64: int) -> int:
    """Montgomery form x*R mod p with R = 2^(64*n64) (prime_field_fallback.h)."""
    return (x % p) * (1 << (64 * n64)) % p


def to_limbs64(x: int, n64: int):
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n64)]


def from_limbs64(limbs) -> int:
    return sum(int(v) << (64 * i) for i, v in enumerate(limbs))
