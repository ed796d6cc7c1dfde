"""CPU checks of the arithmetic identities the HIP kernels rely on to stay bit-exact
(uecraytracing_amd/csrc/yk_device.hpp), independent of the GPU:

* mt19937's twist and tempering written with gfx950's three-input bitwise op (v_bitop3_b32,
  truth tables 0x78 = a ^ (b & c) and 0xE4 = (a & c) | (b & ~c)) equal the reference's
  expressions (random.hpp:98-131), emulated bit by bit;
* generate_canonical<double, 53> (random.hpp:161-183; libstdc++: sum = u0 + u1*2^32 rounded once,
  then / 2^64) equals ONE fused multiply-add of the exactly scaled words,
  fma(u1, 2^-32, u0 * 2^-64), over edge and random words (the fma is evaluated exactly with
  fractions and rounded once, as the hardware does);
* uniform_real_distribution(-1, 1) on a canonical c, c*(1 - -1) + -1, equals fma(c, 2, -1).
"""
import random
from fractions import Fraction

import numpy as np

M32 = 0xFFFFFFFF


def bitop3(a, b, c, table):
    """v_bitop3_b32: bit i of the result is bit (a_i << 2 | b_i << 1 | c_i) of the table."""
    r = 0
    for i in range(32):
        idx = (((a >> i) & 1) << 2) | (((b >> i) & 1) << 1) | ((c >> i) & 1)
        r |= ((table >> idx) & 1) << i
    return r


def mix_ref(hi_src, lo_src):  # random.hpp: y = upper bit of hi, lower 31 of lo; (y>>1) ^ (odd ? K : 0)
    y = (hi_src & 0x80000000) | (lo_src & 0x7FFFFFFF)
    return (y >> 1) ^ (0x9908B0DF if y & 1 else 0)


def mix_dev(hi_src, lo_src):  # yk_device.hpp mt_mix
    y = bitop3(hi_src, lo_src, 0x80000000, 0xE4)
    odd = (0 - (lo_src & 1)) & M32
    return bitop3(y >> 1, odd, 0x9908B0DF, 0x78)


def temper_ref(z):
    z ^= z >> 11
    z ^= (z << 7) & 0x9D2C5680
    z ^= (z << 15) & 0xEFC60000
    z ^= z >> 18
    return z & M32


def temper_dev(z):  # yk_device.hpp mt_temper
    z ^= z >> 11
    z = bitop3(z, (z << 7) & M32, 0x9D2C5680, 0x78)
    z = bitop3(z, (z << 15) & M32, 0xEFC60000, 0x78)
    z ^= z >> 18
    return z


def test_bitop3_tables():
    rng = random.Random(3)
    for _ in range(2000):
        a, b, c = (rng.getrandbits(32) for _ in range(3))
        assert bitop3(a, b, c, 0x78) == a ^ (b & c)
        assert bitop3(a, b, c, 0xE4) == (a & c) | (b & ~c & M32)


def test_mt_twist_and_tempering_with_bitop3():
    rng = random.Random(5)
    words = [0, 1, 2, 0x7FFFFFFF, 0x80000000, 0x80000001, M32] + [rng.getrandbits(32) for _ in range(3000)]
    for i, a in enumerate(words):
        b = words[(i * 7 + 3) % len(words)]
        assert mix_dev(a, b) == mix_ref(a, b)
        assert temper_dev(a) == temper_ref(a)


def canonical_ref(u0, u1):  # libstdc++ generate_canonical<double, 53> with a 32-bit engine
    s = 0.0
    s += float(u0) * 1.0
    s += float(u1) * 4294967296.0
    r = s / 18446744073709551616.0
    return r if r < 1.0 else 1.0 - 2.0 ** -53


def canonical_dev(u0, u1):  # yk_device.hpp canonical: fma(u1, 2^-32, u0 * 2^-64), then the clamp
    r = float(Fraction(u1) * Fraction(1, 2 ** 32) + Fraction(u0) * Fraction(1, 2 ** 64))
    return r if r < 1.0 else 1.0 - 2.0 ** -53


def test_canonical_as_one_fma():
    rng = random.Random(11)
    edge = [0, 1, 2, 1023, 1024, 1025, 2047, 2048, 2049, 0x7FFFFFFF, 0x80000000, M32 - 1024, M32 - 1, M32]
    pairs = [(a, b) for a in edge for b in edge]
    pairs += [(rng.getrandbits(32), rng.getrandbits(32)) for _ in range(20000)]
    # u1 >= 2^21 leaves 11 bits of u0 below the rounding point: ties and near-ties of the sum
    pairs += [(rng.getrandbits(11) | (rng.getrandbits(21) << 11), rng.getrandbits(32)) for _ in range(5000)]
    # exact ties: 11 bits dropped when u1 >= 2^31 (halfway = 0x400), 10 when u1 is in [2^30, 2^31)
    pairs += [(((k << 11) | 0x400) & M32, rng.getrandbits(32) | 0x80000000) for k in range(2000)]
    pairs += [(((k << 10) | 0x200) & M32, (rng.getrandbits(30) | 0x40000000)) for k in range(2000)]
    for u0, u1 in pairs:
        assert canonical_dev(u0, u1) == canonical_ref(u0, u1), (u0, u1)


def test_uniform_minus1_1_as_one_fma():
    rng = np.random.default_rng(2)
    cs = np.concatenate([rng.random(20000), [0.0, 2.0 ** -53, 0.25, 0.5, 0.75, 1.0 - 2.0 ** -53]])
    for c in cs:
        c = float(c)
        ref = (c * (1.0 - -1.0)) + -1.0
        dev = float(Fraction(c) * 2 - 1)  # fma(c, 2, -1): exact, rounded once
        assert dev == ref
