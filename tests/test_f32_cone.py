"""The FP32 kernel's cone slab test never culls a box its cone reaches.

render<float> culls with a per-ray cone of slope s = kF32Cone |d| (ykgpu_render.hip, cone_axis and
the slow-axis bound): per axis, near planes at (plane - o) / (d + s sign d); far planes at
(plane - o) / (d - s sign d) scaled by (1 + 2^-17) when |d| >= s (1 + 2^-10); and on ONE slow axis
(|d| < s (1 - 2^-10), y first, then x, then z) the far-side plane's crossing, a LOWER bound, folded
into the max with the near distances.  This replays that arithmetic in float32 (reciprocals
perturbed by up to an ulp, as v_rcp_f32 may be) against the exact cone-box intersection in
float64 (per axis, o + (d - s) t <= hi and o + (d + s) t >= lo), boxes grown by delta = 2^-21 x
the origin bound as the FP32 tree grows them, and checks: every box the exact cone meets passes
(no false culls), and the slow-axis bound really culls boxes the plain rule keeps.
Test infrastructure only (numpy model of device arithmetic)."""
import numpy as np

import refscenes

KCONE = np.float32(2.0 ** -8 * (1 + 2.0 ** -10))
FAR_AT = np.float32(1 + 2.0 ** -10)
SLOW_AT = np.float32(1 - 2.0 ** -10)
F32 = np.float32


def fma32(a, b, c):
    # float32 FMA: the product of two floats is exact in float64, one rounding to 53 bits, then to 24
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def rcp32(x, rng):
    r = (F32(1) / x).astype(np.float32)
    k = rng.integers(-1, 2, size=r.shape)  # v_rcp_f32: within an ulp
    return np.where(k < 0, np.nextafter(r, F32(-np.inf)), np.where(k > 0, np.nextafter(r, F32(np.inf)), r))


def kernel_pass(o, d, lo, hi, tmin, ustar, slow_bound, rng):
    """o, d: (N, 3) float32; lo, hi: (N, M, 3) grown boxes; returns (N, M) bool."""
    a = (d * d).sum(axis=1, dtype=np.float32)
    s = (np.sqrt(a).astype(np.float32) * KCONE).astype(np.float32)
    tn = np.full(lo.shape[:2], F32(tmin) * F32(1 - 2.0 ** -17), dtype=np.float32)
    tf = np.full(lo.shape[:2], np.float32(ustar * (1 + 2.0 ** -18)) if np.isfinite(ustar) else F32(np.inf),
                 dtype=np.float32)
    slow_axis = np.full(len(o), -1)
    for k in (2, 0, 1):  # the kernel's assignment order: the last slow axis (y, then x, then z) wins
        slow_axis = np.where(np.abs(d[:, k]) < s * SLOW_AT, k, slow_axis)
    for k in range(3):
        dk, ok = d[:, k], o[:, k]
        sg = np.where(dk < 0, -s, s).astype(np.float32)
        inv = rcp32((dk + sg).astype(np.float32), rng)
        nc = (-(ok * inv)).astype(np.float32)
        qn = np.where((dk < 0)[:, None], hi[:, :, k], lo[:, :, k]).astype(np.float32)
        qf = np.where((dk < 0)[:, None], lo[:, :, k], hi[:, :, k]).astype(np.float32)
        near = fma32(qn, inv[:, None], nc[:, None])
        tn = np.maximum(tn, near)
        far_ok = np.abs(dk) >= s * FAR_AT
        with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
            jf = np.where(far_ok, (rcp32((dk - sg).astype(np.float32), rng) * F32(1 + 2.0 ** -17)).astype(np.float32), F32(0))
            fc = np.where(far_ok, (-(ok * jf)).astype(np.float32), F32(np.inf))
            far = np.where(far_ok[:, None], fma32(qf, jf[:, None], fc[:, None]), F32(np.inf))
        tf = np.minimum(tf, far)
        if slow_bound:
            use = slow_axis == k
            with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
                jl = np.where(use, rcp32((dk - sg).astype(np.float32), rng), F32(0))
                cl = np.where(use, (-(ok * jl)).astype(np.float32), F32(-np.inf))
                lb = np.where(use[:, None], fma32(qf, jl[:, None], cl[:, None]), F32(-np.inf))
            tn = np.maximum(tn, np.nan_to_num(lb, nan=-np.inf))
    return tn <= tf


def exact_cone_meets(o, d, lo, hi, tmin, ustar):
    """The cone {per axis: o + (d - s) t <= coordinate range <= o + (d + s) t} meets [lo, hi] at
    some t in [tmin, ustar] — float64, with s from the same float32 rounding as the kernel."""
    a = (d * d).sum(axis=1, dtype=np.float32)
    s = (np.sqrt(a).astype(np.float32) * KCONE).astype(np.float64)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    t0 = np.full(lo.shape[:2], float(tmin))
    t1 = np.full(lo.shape[:2], float(ustar))
    for k in range(3):
        for coef, rhs, ge in (((d64[:, k] + s)[:, None], lo[:, :, k] - o64[:, k:k + 1], True),
                              ((d64[:, k] - s)[:, None], hi[:, :, k] - o64[:, k:k + 1], False)):
            # ge: coef t >= rhs; else coef t <= rhs
            with np.errstate(divide="ignore", invalid="ignore"):
                b = rhs / coef
            pos = coef > 0
            neg = coef < 0
            if ge:
                t0 = np.where(pos, np.maximum(t0, b), t0)
                t1 = np.where(neg, np.minimum(t1, b), t1)
                t1 = np.where((coef == 0) & (rhs > 0), -np.inf, t1)
            else:
                t1 = np.where(pos, np.minimum(t1, b), t1)
                t0 = np.where(neg, np.maximum(t0, b), t0)
                t1 = np.where((coef == 0) & (rhs < 0), -np.inf, t1)
    return t0 <= t1


def make_case(rng, n_rays, n_boxes, bound, slow_frac):
    o = rng.uniform(-bound, bound, size=(n_rays, 3)).astype(np.float32)
    d = rng.normal(size=(n_rays, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d *= rng.uniform(0.2, 5.0, size=(n_rays, 1))
    # slow rays: one component within a few cone slopes of zero (both sides of the thresholds)
    slow = rng.random(n_rays) < slow_frac
    ax = rng.integers(0, 3, size=n_rays)
    norm = np.linalg.norm(d, axis=1)
    val = rng.uniform(-2.5, 2.5, size=n_rays) * float(KCONE) * norm
    d[slow, ax[slow]] = val[slow]
    d = d.astype(np.float32)
    # boxes scattered around the ray, most near its path
    t = rng.uniform(0.0, 60.0, size=(n_rays, n_boxes, 1))
    c = o[:, None, :] + t * d[:, None, :] + rng.normal(scale=rng.uniform(0.05, 2.0, size=(n_rays, n_boxes, 1)),
                                                       size=(n_rays, n_boxes, 3))
    half = rng.uniform(0.01, 1.0, size=(n_rays, n_boxes, 3))
    return o, d, c - half, c + half


def test_cone_never_culls_a_box_it_meets():
    rng = np.random.default_rng(2024)
    bound = 100.0
    delta = 2.0 ** -21 * bound * 2  # the tree's growth for an origin bound of 2 x the sampled |o|
    for tmin, ustar in ((0.001, np.inf), (0.001, 7.5), (0.5, 30.0)):
        o, d, lo, hi = make_case(rng, 400, 200, bound, 0.5)
        truth = exact_cone_meets(o, d, lo, hi, tmin, ustar)
        glo = np.nextafter((lo - delta).astype(np.float32), np.float32(-np.inf))
        ghi = np.nextafter((hi + delta).astype(np.float32), np.float32(np.inf))
        got = kernel_pass(o, d, glo, ghi, tmin, ustar, True, rng)
        missed = truth & ~got
        assert not missed.any(), (tmin, ustar, int(missed.sum()))
        assert truth.sum() > 1000  # the case really exercises intersecting boxes


def test_slow_axis_bound_culls():
    rng = np.random.default_rng(7)
    o, d, lo, hi = make_case(rng, 400, 200, 50.0, 1.0)
    a = (d * d).sum(axis=1)
    s = np.sqrt(a) * float(KCONE)
    slow = (np.abs(d) < s[:, None] * float(SLOW_AT)).any(axis=1)
    lo32, hi32 = lo.astype(np.float32), hi.astype(np.float32)
    with_l = kernel_pass(o, d, lo32, hi32, 0.001, np.inf, True, rng)
    without = kernel_pass(o, d, lo32, hi32, 0.001, np.inf, False, rng)
    assert not (with_l & ~without).any()  # the bound only ever removes boxes
    culled = (without & ~with_l)[slow].sum()
    kept = without[slow].sum()
    assert culled > 0.2 * kept, (culled, kept)  # and for slow rays it removes many


def test_axial_scene_exercises_slow_axes():
    """The axial camera's rays are slow on x and y (|d_k| < kF32Cone |d|) for most
    pixels: the FP32 tree's slow-axis bound and its two-slow-axes case are really exercised."""
    cam = refscenes.axial_camera()
    k = 2.0 ** -8 * (1 + 2.0 ** -10)
    slow_x = slow_y = both = 0
    n = 0
    for u in np.linspace(0, 1, 41):
        for v in np.linspace(0, 1, 21):
            d = [cam.lower_left_corner[i] + u * cam.horizontal[i] + v * cam.vertical[i] - cam.origin[i] for i in range(3)]
            s = k * float(np.sqrt(sum(x * x for x in d)))
            sx, sy = abs(d[0]) < s, abs(d[1]) < s
            slow_x += sx
            slow_y += sy
            both += sx and sy
            n += 1
    assert slow_y > 0.5 * n and slow_x > 0.2 * n and both > 0.1 * n

