"""The VERT form of the leaf test (rt_kernels.hip tri_math<..., VERT>): for a ray of
direction exactly (0, 1, 0) -- every W9E1 shadow ray, light_init, w9e1.wgsl:67-73 --
the reference's intersect_triangle (w7e3.wgsl:286-332, f32, no contraction) computes
cross(ov, w) = (-ov.z, +-0, ov.x) and dot(w, n) = n.y exactly, so a and b reduce to one
product pair and one add each.  This CPU test evaluates both forms with numpy float32
(one rounding per operation, as the kernel's -ffp-contract=off build) on random and
adversarial triangles and checks that every quantity the accept predicate reads is the
same value (a zero's sign may differ, which the predicate's < / > comparisons and the
exact quotients do not see), and that the predicate itself agrees."""
import numpy as np

f32 = np.float32


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def general(ov, e0, e1, n, w):
    nom = cross(ov, w)
    return dot(w, n), dot(nom, e1), -dot(nom, e0), dot(ov, n)


def vert(ov, e0, e1, n):
    denom = n[1]
    a = (-ov[2]) * e1[0] + ov[0] * e1[2]
    b = -((-ov[2]) * e0[0] + ov[0] * e0[2])
    return denom, a, b, dot(ov, n)


def accept(denom, a, b, c, tmin, tmax):
    with np.errstate(all="ignore"):
        rej = np.abs(denom) < f32(1e-10)
        dist = c / denom
        beta = a / denom
        gamma = b / denom
        ok = ~((beta < 0) | (gamma < 0) | (beta + gamma > 1) | (dist > tmax) | (dist < tmin))
    return ~rej & ok, dist


def _cases(rng, n):
    v0 = rng.uniform(-1, 1, (3, n)).astype(f32)
    e0 = (rng.uniform(-1, 1, (3, n)) * 10.0 ** rng.uniform(-4, 0, n)).astype(f32)
    e1 = (rng.uniform(-1, 1, (3, n)) * 10.0 ** rng.uniform(-4, 0, n)).astype(f32)
    o = rng.uniform(-1, 1, (3, n)).astype(f32)
    # adversarial: zeros and ties in the components the VERT form drops or keeps
    k = n // 8
    o[0, :k] = v0[0, :k]                       # ov.x == 0
    o[2, k:2 * k] = v0[2, k:2 * k]             # ov.z == 0
    e1[0, 2 * k:3 * k] = 0.0                   # one product of a vanishes
    e0[2, 3 * k:4 * k] = -0.0                  # a signed zero edge component
    o[:, 4 * k:5 * k] = v0[:, 4 * k:5 * k]     # the ray starts on v0
    e0[1, 5 * k:6 * k] = 0.0
    e1[1, 5 * k:6 * k] = 0.0                   # n = (0, n.y, 0) ... horizontal triangles
    e0[0, 6 * k:7 * k] = e1[0, 6 * k:7 * k]    # n.y == 0 ... vertical triangles
    e0[2, 6 * k:7 * k] = e1[2, 6 * k:7 * k]
    # the rest: rays aimed up through the triangle (a point of it, from below), so that
    # the predicate accepts many of them
    h = slice(7 * k, n)
    bc = rng.uniform(0, 1, (2, n - 7 * k))
    bc = np.where(bc.sum(0) < 1, bc, 1 - bc[::-1])
    P = v0[:, h] + bc[0] * e0[:, h] + bc[1] * e1[:, h]
    o[:, h] = np.stack([P[0], P[1] - rng.uniform(0.01, 1.0, n - 7 * k), P[2]]).astype(f32)
    n_ = np.stack(cross(e0, e1)).astype(f32)   # the records' normal is e0 x e1 in f32
    return v0, e0, e1, n_, o


def test_vert_form_equals_general_form():
    rng = np.random.default_rng(7)
    v0, e0, e1, n, o = _cases(rng, 400_000)
    w = (np.zeros_like(o[0]), np.ones_like(o[0]), np.zeros_like(o[0]))
    ov = (v0[0] - o[0], v0[1] - o[1], v0[2] - o[2])
    g = general(ov, e0, e1, n, w)
    v = vert(ov, e0, e1, n)
    for name, x, y in zip(("denom", "a", "b", "c"), g, v):
        assert np.array_equal(x, y), name                        # == : +0 equals -0
        nz = x != 0
        assert np.array_equal(np.signbit(x[nz]), np.signbit(y[nz])), name   # nonzero values bit for bit
        assert np.array_equal(x[nz].view(np.uint32), y[nz].view(np.uint32)), name
    tmin, tmax = f32(1e-4), f32(999999.0 - 1e-4)
    ag, dg = accept(*g, tmin, tmax)
    av, dv = accept(*v, tmin, tmax)
    assert np.array_equal(ag, av)
    assert ag.sum() > 20_000                                   # the cases include real accepts
    assert np.array_equal(dg[ag].view(np.uint32), dv[av].view(np.uint32))
