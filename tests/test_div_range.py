"""The operand range behind the BSP walk's unchecked plane divisions
(rt_kernels.hip bsp_decide with chk = 0; rt_bsp_build.hip k_plane_range; k_path's
per-check ballot).  rt_div_by_recip (include/rt_detmath.h) equals IEEE division for
x = 0 or 2^-100 <= |x| <= 2^100 (tests/test_fastdiv.py).  The walk skips its per-lane
range test when every interior plane and every tracing ray's origin coordinate is 0 or
in [2^-76, 2^99] in magnitude; then x = RN(plane - o) must always be 0 or in that range.
Checked here in binary32 on random and boundary operands, together with the flag's
exact thresholds (a value just outside the set must raise it)."""
import numpy as np

LO, HI = np.float32(2.0 ** -76), np.float32(2.0 ** 99)


def _allowed(rng, n):
    """Floats that are 0 or of magnitude in [2^-76, 2^99], both signs, with the
    boundaries and their neighbours inside the set over-represented."""
    e = rng.integers(-76, 100, n)
    m = rng.integers(0, 1 << 23, n, dtype=np.int64)
    v = ((e + 127).astype(np.int64) << 23 | m).astype(np.uint32).view(np.float32)
    v = np.minimum(v, HI)   # 2^99 exactly is the largest allowed magnitude
    k = rng.random(n)
    edge = np.array([0.0, LO, np.nextafter(LO, np.float32(1)), HI, np.nextafter(HI, np.float32(0)), 1.0], np.float32)
    v = np.where(k < 0.2, edge[rng.integers(0, len(edge), n)], v)
    # values close to each other (small differences: the lower end of the range)
    near = np.nextafter(np.roll(v, 1), np.float32(np.inf)) if n else v
    v = np.where((k >= 0.2) & (k < 0.35), near, v)
    v = np.where(_flag(v), LO, v)   # (a neighbour past 2^99)
    return np.where(rng.random(n) < 0.5, -v, v).astype(np.float32)


def _flag(v):
    """k_plane_range's / k_path's test: True when v lies outside {0} U [2^-76, 2^99]."""
    a = np.abs(v.astype(np.float32))
    return ~((a == 0) | ((a >= LO) & (a <= HI)))


def test_plane_minus_origin_stays_in_the_exact_range():
    rng = np.random.default_rng(7)
    for _ in range(8):
        p = _allowed(rng, 1_000_000)
        o = _allowed(rng, 1_000_000)
        # pairs that differ by one or a few ulps, same sign (the smallest nonzero x)
        close = rng.random(len(p)) < 0.25
        o = np.where(close, np.nextafter(p, np.float32(np.inf) * np.sign(rng.random(len(p)) - 0.5)), o)
        o = np.where(close & _flag(o), p, o).astype(np.float32)
        assert not _flag(p).any() and not _flag(o).any()
        x = (p - o).astype(np.float32)   # RN(plane - o) in binary32, as the kernel computes it
        a = np.abs(x)
        ok = (a == 0) | ((a >= np.float32(2.0 ** -100)) & (a <= np.float32(2.0 ** 100)))
        assert ok.all(), (p[~ok][:4], o[~ok][:4], x[~ok][:4])
        # the tighter form of the argument: a nonzero x is a multiple of 2^-99
        nz = a != 0
        assert (a[nz] >= np.float32(2.0 ** -99)).all()


def test_flag_thresholds():
    below = np.nextafter(LO, np.float32(0))
    above = np.nextafter(HI, np.float32(np.inf))
    v = np.array([0.0, -0.0, LO, -LO, HI, -HI, 1.0], np.float32)
    assert not _flag(v).any()
    w = np.array([below, -below, above, -above, np.float32(2.0 ** -149), np.inf, -np.inf, np.nan], np.float32)
    assert _flag(w).all()


def test_the_range_is_needed():
    # a plane at 2^-110 and an origin coordinate of 0 give x = 2^-110, outside the exact
    # range of rt_div_by_recip; the plane raises k_plane_range's flag
    p, o = np.float32(2.0 ** -110), np.float32(0.0)
    x = np.float32(p - o)
    assert 0 < abs(x) < np.float32(2.0 ** -100) and _flag(np.array([p])).all()
    # two origins just inside the set cannot do it: their difference is a multiple of 2^-99
    a = np.float32(LO)
    b = np.nextafter(a, np.float32(1))
    assert np.float32(b - a) == np.float32(2.0 ** -99)
