"""The FP32 tree's culling bound (yk_bvh.hpp kF32Cone), checked on the CPU.

render<float>'s sphere test (sphere.hpp:25-48 evaluated in float) is far less exact near
tangency than the FP64 one, so the FP32 kernel culls with boxes and a per-ray cone sized by a
proven bound: a root the float test accepts puts the exact point o + r d within
2^-8.9 (|o - c| + R) of the float sphere, hence within 2^-8.9 (r |d| + 2R).  This replays the test
in numpy float32 (same operations in the same order, no FMA; the reference's Newton square root
from the oracle) on rays aimed at silhouettes and surfaces over four decades of scale, and checks
its three forms (linear, cone,
quadratic) and the margins of the constants built on them.
"""
import numpy as np

import oracle_lib

BOUND = 2.0 ** -8.9
K_F32_CONE = 2.0 ** -8 * (1 + 2.0 ** -10)  # yk_bvh.hpp kF32Cone
QUAD = 72.7 * 2.0 ** -24                   # dev <= QUAD (|o - c|^2 + R^2) / R, DESIGN.md §4.1
K_F32_BIG_GROW = 2.0 ** -15                # yk_bvh.hpp kF32BigGrow
F = np.float32


def float_test(o, d, c, R, tmin=F(0.001)):
    """sphere::hit_impl<float> without t_max: (root, accepted) per ray."""
    rr = R * R
    oc = o - c
    a = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]
    hb = oc[:, 0] * d[:, 0] + oc[:, 1] * d[:, 1] + oc[:, 2] * d[:, 2]
    cc = (oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1] + oc[:, 2] * oc[:, 2]) - rr
    disc = hb * hb - a * cc
    ok = disc >= 0
    sq = oracle_lib.newton_sqrt_f32(np.where(ok, disc, F(1)))
    r1 = (-hb - sq) / a
    r2 = (-hb + sq) / a
    r = np.where(r1 >= tmin, r1, r2)
    return r, ok & (r >= tmin) & np.isfinite(r)


def near_tangent_rays(rng, n):
    """Spheres and origins over four decades of scale; directions at the silhouette seen from the
    origin (tangent rays) or at surface points, perturbed by 1e-9 .. 1e-2 of the radius."""
    scale = 10.0 ** rng.uniform(-1, 3, n)
    c = (rng.uniform(-1, 1, (n, 3)) * scale[:, None]).astype(F)
    R = scale * 10.0 ** rng.uniform(-3, 0, n)
    R = np.where(rng.random(n) < 0.1, -R, R).astype(F)
    o = (rng.uniform(-1, 1, (n, 3)) * (10.0 ** rng.uniform(-1, 3.3, n))[:, None]).astype(F)
    c64, o64 = c.astype(np.float64), o.astype(np.float64)
    Ra = np.abs(R.astype(np.float64))
    v = c64 - o64
    D = np.linalg.norm(v, axis=1)
    e = v / D[:, None]
    w = rng.normal(size=(n, 3))
    w -= (w * e).sum(1)[:, None] * e
    w /= np.linalg.norm(w, axis=1)[:, None]
    cosa = np.clip(Ra / D, 0.0, 1.0)
    sina = np.sqrt(1.0 - cosa ** 2)
    sil = c64 + Ra[:, None] * (-cosa[:, None] * e + sina[:, None] * w)  # (p-c).(p-o) = 0
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    surf = c64 + Ra[:, None] * u
    p = np.where(((rng.random(n) < 0.7) & (D > Ra))[:, None], sil, surf)
    p += rng.normal(size=(n, 3)) * (Ra * 10.0 ** rng.uniform(-9, -2, n))[:, None]
    d = ((p - o64) * (10.0 ** rng.uniform(-2, 1, n))[:, None]).astype(F)
    return o, d, c, R


def test_float_sphere_test_error_bound():
    rng = np.random.default_rng(20261016)
    worst, worst_cone, worst_quad, accepted = 0.0, 0.0, 0.0, 0
    for _ in range(4):
        o, d, c, R = near_tangent_rays(rng, 250_000)
        r, ok = float_test(o, d, c, R)
        o64, d64, c64 = (x.astype(np.float64) for x in (o, d, c))
        rad = np.sqrt((R * R).astype(np.float64))  # the float sphere: radius^2 = fl(R * R)
        P = o64 + r.astype(np.float64)[:, None] * d64
        dev = np.abs(np.linalg.norm(P - c64, axis=1) - rad)
        oc = np.linalg.norm(o64 - c64, axis=1)
        dn = np.linalg.norm(d64, axis=1)
        worst = max(worst, float(np.max(np.where(ok, dev / (oc + rad), 0.0))))
        worst_cone = max(worst_cone, float(np.max(np.where(ok, dev / (r * dn + 2 * rad), 0.0))))
        # the quadratic form the big-sphere growth rests on (yk_bvh.hpp kF32BigGrow)
        worst_quad = max(worst_quad, float(np.max(np.where(ok, dev * rad / (oc ** 2 + rad ** 2), 0.0))))
        accepted += int(ok.sum())
    assert accepted > 300_000
    assert worst <= BOUND, np.log2(worst)
    assert worst_cone <= BOUND, np.log2(worst_cone)
    assert K_F32_CONE >= 1.85 * BOUND
    assert worst_quad <= QUAD, worst_quad / QUAD
    assert K_F32_BIG_GROW / 2 >= 3.5 * QUAD
