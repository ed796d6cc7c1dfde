"""The FP64 traversal's float comparisons keep every candidate, on the CPU.

Round 5's kernel kept a candidate's lower bound as l = RN_f32(L) and compared it with
ustar_f = RN_f32(RN_f32(U*) * (1 + 2^-18)); round 6's (`YK_NEAR_CLAMP`, the leaf block of
ykgpu_render.hip) measures both from tmin_lo = t_min (1 - 2^-17) in units of s = 2^-24:
l = fma(RN(L), s, -tmin_lo s) and ustar_f = RN(RN(RN(U*)(1 + 2^-18)) - tmin_lo) RN((1 + 2^-22) s)
(test_shifted_map_never_drops_a_candidate).  The host rejects
t_min < 0, so every L and U* is >= 0, and the claim is: L <= U*  implies  l <= ustar_f.  This
replays the kernel's two float32 roundings in numpy on bounds spread over the whole double
range that float can hold, on ties (L == U*), on neighbours one double ulp apart, and on values
that round to the same float or overflow it.
"""
import numpy as np

F = np.float32
SLACK = F(1.0) + F(2.0 ** -18)


def ustar_f(u):
    with np.errstate(over="ignore"):
        return (u.astype(F) * SLACK).astype(F)


def keeps(lb, u):
    with np.errstate(over="ignore"):
        return lb.astype(F) <= ustar_f(u)


def test_rn_lower_bound_never_drops_a_candidate():
    rng = np.random.default_rng(20261017)
    n = 2_000_000
    # U* over [2^-140, 2^130] (float denormals, normals and overflow), L <= U* by a random gap
    u = np.exp2(rng.uniform(-140, 130, n))
    gap = np.where(rng.random(n) < 0.5, np.exp2(rng.uniform(-60, 0, n)), rng.random(n))
    lb = u * (1 - gap)
    assert np.all(lb <= u)
    assert np.all(keeps(lb, u))
    # exact ties and the double just below U*
    assert np.all(keeps(u, u))
    assert np.all(keeps(np.nextafter(u, 0), u))
    # zero lower bounds (t_min = 0) and infinite U* (no bound yet)
    assert np.all(keeps(np.zeros(4), np.array([0.0, 1e-300, 1.0, np.inf])))
    assert np.all(keeps(np.array([0.0, 1.0, 1e300, np.inf]), np.full(4, np.inf)))


def test_the_argument_needs_nonnegative_bounds():
    # with a negative U* the scaled bound moves down, below RN(U*): the host's t_min >= 0 check
    # is what makes the comparison safe
    u = np.array([-1.0])
    assert not keeps(u, u)[0]


def test_shifted_map_never_drops_a_candidate():
    """Round 6's map, for bounds >= t_min (the kernel's lb = fmax(t_min, ...) and U* >= t_min)."""
    t_min = 0.001
    t32 = F(t_min)
    if float(t32) > t_min:  # __double2float_rd
        t32 = np.nextafter(t32, F(0))
    tmin_lo = F(t32 * F(1 - 2.0 ** -17))
    s = 2.0 ** -24
    scale_up = F((1 + 2.0 ** -22) * s)

    def l_of(lb):  # one fma of RN(lb): (RN(lb) - tmin_lo) s rounded once (s a power of two)
        return ((lb.astype(F).astype(np.float64) - np.float64(tmin_lo)) * s).astype(F)

    def u_of(u):
        with np.errstate(over="ignore"):
            return (((u.astype(F) * SLACK).astype(F) - tmin_lo).astype(F) * scale_up).astype(F)

    rng = np.random.default_rng(20261018)
    n = 2_000_000
    u = t_min * np.exp2(rng.uniform(0, 136, n))  # U* from t_min to beyond float's range
    gap = np.where(rng.random(n) < 0.5, np.exp2(rng.uniform(-60, 0, n)), rng.random(n))
    lb = np.maximum(t_min, u * (1 - gap))
    assert np.all(lb <= u)
    with np.errstate(over="ignore"):
        assert np.all(l_of(lb) <= u_of(u))
        assert np.all(l_of(u) <= u_of(u))  # ties
        assert np.all(l_of(np.nextafter(u, 0)) <= u_of(u))
        assert np.all(l_of(np.full(3, t_min)) <= u_of(np.array([t_min, 1.0, np.inf])))
