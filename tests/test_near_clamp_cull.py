"""The FP64 visit's culling test with distances measured from t_min and clamped near FMAs
(`YK_NEAR_CLAMP`) keeps every box the culling contract requires (CPU).

The kernel keeps a wide-node slot when max(near, tmin_lo) <= min(far * c, U*(1 + 2^-18)) (round 5,
`old` below); round 6 computes the same test in distances from tmin_lo scaled by s = 2^-24, the
near FMAs clamped to [0, 1] in place of the max with tmin_lo (`new`).  The contract (yk_bvh.hpp):
every box whose sphere — the box shrunk by delta = 2^-21 x origin_bound — meets the ray inside
[t_min, U*] is kept.  Rays grazing boxes at every distance class (at the origin, at t_min, near, far)
with U* at the shrunk box's entry point: neither formulation may cull one.  float32 arithmetic is
emulated in numpy: products of two floats are exact in float64, and an FMA is one rounding of the
float64 sum to float32 (a double rounding in rare ties, far inside the margins tested here); the
clamp is np.clip.
"""
import numpy as np

F32 = np.float32
TMIN = 0.001
EXTENT = 40.0
DELTA = 2.0 ** -21 * 4 * EXTENT  # origin_bound = 4 x the scene extent (yk_bvh.cpp)


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F32)


def cull_cases(seed, n=300_000):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-15, 15, (n, 3))
    d = rng.normal(size=(n, 3)) * rng.choice([1e-3, 0.1, 1.0, 10.0], size=(n, 1))
    d[rng.random((n, 3)) < 0.05] *= 1e-6  # rays almost parallel to an axis
    t0 = rng.choice([0.0, TMIN, 0.5, 5.0, 40.0], n) * rng.uniform(0.9, 1.1, n)
    h = rng.uniform(0.001, 3, (n, 1))
    p = o + t0[:, None] * d
    e = h * rng.uniform(-1.02, 1.02, (n, 3))  # the ray passes through, grazes or misses the box
    lo = (p + e - h).astype(F32)
    hi = (p + e + h).astype(F32)
    # the shrunk box's entry point: the earliest exact root a sphere inside the box can have
    t1 = (lo.astype(np.float64) + DELTA - o) / d
    t2 = (hi.astype(np.float64) - DELTA - o) / d
    ts_n, ts_f = np.minimum(t1, t2).max(1), np.maximum(t1, t2).min(1)
    U = np.where(rng.random(n) < 0.3, np.inf, np.maximum(ts_n, TMIN) * rng.uniform(1.0, 1.0 + 1e-6, n))
    must = np.maximum(ts_n, TMIN) <= np.minimum(ts_f, U)
    return o, d, lo, hi, U, must


def kernel_tests(o, d, lo, hi, U):
    t32 = F32(TMIN)
    if float(t32) > TMIN:  # __double2float_rd
        t32 = np.nextafter(t32, F32(0))
    tmin_lo = F32(t32 * F32(1 - 2.0 ** -17))
    ix = (F32(1) / d.astype(F32)).astype(F32)
    of = o.astype(F32)
    kfar = F32(1 + 2.0 ** -17)
    ixs = (ix * kfar).astype(F32)
    oix = (of * ix).astype(F32)
    oixs = (of * ixs).astype(F32)
    neg = ix < 0  # the planes the kernel's per-ray offsets select
    pn, pf = np.where(neg, hi, lo), np.where(neg, lo, hi)
    ustar = (U.astype(F32) * F32(1 + 2.0 ** -18)).astype(F32)
    # round 5: max(near, tmin_lo) <= min(far c, ustar_f)
    n_old, f_old = fma(pn, ix, -oix), fma(pf, ixs, -oixs)
    keep_old = np.maximum(n_old.max(1), tmin_lo) <= np.minimum(f_old.min(1), ustar)
    # round 6: s (d - tmin_lo) units, near clamped to [0, 1]; U' rounded up
    s = F32(2.0 ** -24)
    kn = ((-oix - tmin_lo).astype(F32) * s).astype(F32)
    kf = ((-oixs - tmin_lo).astype(F32) * s).astype(F32)
    n_new = np.clip(fma(pn, (ix * s).astype(F32), kn), 0, 1)
    f_new = fma(pf, (ixs * s).astype(F32), kf)
    u_new = ((ustar - tmin_lo).astype(F32) * F32((1 + 2.0 ** -22) * 2.0 ** -24)).astype(F32)
    keep_new = n_new.max(1) <= np.minimum(f_new.min(1), u_new)
    return keep_old, keep_new


def test_clamped_near_distances_keep_every_box_the_contract_requires():
    total = 0
    for seed in (1, 2, 3):
        o, d, lo, hi, U, must = cull_cases(seed)
        keep_old, keep_new = kernel_tests(o, d, lo, hi, U)
        assert not (must & ~keep_old).any()
        assert not (must & ~keep_new).any(), f"seed {seed}: {(must & ~keep_new).sum()} boxes culled"
        total += int(must.sum())
    assert total > 500_000  # the cases are mostly boxes the ray meets


def test_clamped_near_distances_cull_what_the_round5_test_culls():
    """Same efficiency: the two tests disagree on a vanishing fraction of slots (roundings only)."""
    o, d, lo, hi, U, _ = cull_cases(4)
    keep_old, keep_new = kernel_tests(o, d, lo, hi, U)
    assert 0.2 < keep_old.mean() < 0.99
    assert (keep_old != keep_new).mean() < 1e-4
