#!/usr/bin/env python3
"""Constants of the 9 x 29-bit redundant Montgomery field (tachyon_amd/csrc/field/f29.h)
for BN254 Fq: R' = 2^261; p and multiples k p in 29-bit limbs with every low limb
raised by D = m 2^29 (borrowed from the limb above) so that K - x stays limb-wise
non-negative for any x whose limbs are below the raised ones.  Prints C++."""
P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
M29 = (1 << 29) - 1


def limbs(v, n=9):
    return [(v >> (29 * i)) & M29 if i < n - 1 else v >> (29 * i) for i in range(n)]


def raised(k, m):
    s = limbs(k * P)
    out = [s[0] + m * (1 << 29)] + [s[i] + m * (1 << 29) - m for i in range(1, 8)] + [s[8] - m]
    assert sum(x << (29 * i) for i, x in enumerate(out)) == k * P
    assert all(0 <= x < (1 << 32) for x in out)
    return out


def fmt(name, v, comment):
    return f"// {comment}\nconstexpr uint32_t {name}[9] = {{" + ", ".join(f"0x{x:08x}u" for x in v) + "};"


def main():
    print(fmt("kP29", limbs(P), "p"))
    print(f"constexpr uint32_t kPinv29 = 0x{(-pow(P, -1, 1 << 29)) % (1 << 29):08x}u;  // -p^-1 mod 2^29")
    print(f"constexpr uint32_t kPinv32 = 0x{pow(P, -1, 1 << 32):08x}u;  // p^-1 mod 2^32 (zero test)")
    print(fmt("kK4", raised(4, 1), "4p, low limbs raised by 2^29 (>= 2^29 - 1)"))
    print(fmt("kK8", raised(8, 4), "8p, low limbs raised by 2^31 (>= 2^31 - 4)"))
    print(fmt("kK16", raised(16, 1), "16p, low limbs raised by 2^29"))
    print(fmt("kK33", raised(33, 1), "33p, low limbs raised by 2^29 (minus a normalized value < 32p)"))
    print(fmt("kK32r3", raised(32, 3), "32p, low limbs raised by 3 2^29"))
    one = (1 << 261) % P
    print(fmt("kOne29", limbs(one), "1 in R' = 2^261 form"))
    print(fmt("kTo256", limbs(1 << 256), "2^256 as an integer: mont29(x, kTo256) = x 2^-5 (R' -> R form)"))


if __name__ == "__main__":
    main()
