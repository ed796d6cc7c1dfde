"""The scratch engine's seed recovery (uecraytracing_amd/csrc/yk_device.hpp mt_seed_from): a lane
does not carry its sample's seed; at its 227th draw cursor A holds x_227 of the seeding sequence
(random.hpp:69-81, x_i = 1812433253 (x_{i-1} ^ x_{i-1} >> 30) + i) and the seed x_0 is recovered
by inverting the steps.  Checked here on the CPU with the header's own constant, against the
forward recurrence, at the seeds' extremes and random ones; the device path is covered by the GPU
parity tests whose samples reach the scratch engine (config 5 rows, mt_fallbacks > 0)."""
import os
import random
import re

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "uecraytracing_amd",
                   "csrc", "yk_device.hpp")
C = 1812433253
M = 1 << 32


def header_constant():
    m = re.search(r"kMtSeedMulInv\s*=\s*(0x[0-9a-fA-F]+)u", open(HDR).read())
    assert m, "kMtSeedMulInv not found in yk_device.hpp"
    return int(m.group(1), 16)


def forward(seed, n):
    x = seed
    for i in range(1, n + 1):
        x = (C * (x ^ (x >> 30)) + i) % M
    return x


def inverse(x, i, cinv):
    # the device loop, restated: t = (x_i - i) C^-1 = u ^ u >> 30, u = t ^ t >> 30
    for k in range(i, 0, -1):
        t = ((x - k) * cinv) % M
        x = t ^ (t >> 30)
    return x


def test_constant_is_the_multiplicative_inverse():
    cinv = header_constant()
    assert (C * cinv) % M == 1


def test_seed_recovered_from_x227():
    cinv = header_constant()
    rng = random.Random(11)
    seeds = [0, 1, 2, 5489, 0x7fffffff, 0x80000000, 0xfffffffe, 0xffffffff] + [rng.getrandbits(32) for _ in range(300)]
    for s in seeds:
        assert inverse(forward(s, 227), 227, cinv) == s, s


def test_each_step_inverts():
    cinv = header_constant()
    rng = random.Random(12)
    for _ in range(2000):
        u, i = rng.getrandbits(32), rng.randrange(1, 624)
        x = (C * (u ^ (u >> 30)) + i) % M
        t = ((x - i) * cinv) % M
        assert t ^ (t >> 30) == u
