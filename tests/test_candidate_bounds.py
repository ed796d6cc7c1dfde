"""The FP64 traversal's float comparisons keep every candidate, on the CPU.

The kernel keeps a candidate's lower bound as l = RN_f32(L) and compares it with
ustar_f = RN_f32(RN_f32(U*) * (1 + 2^-18)) (ykgpu_render.hip, the leaf block).  The host rejects
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
