"""Accuracy of the pinned transcendentals (include/rt_detmath.h) that the GPU kernels
and the CPU oracle share (VERDICT r5 "What's missing" 1: a wrong sin / cos / acos /
atan2 would agree on both sides of every parity test, so only an independent
reference can catch it).  Each function is evaluated over a dense sweep of the
argument ranges the shaders use -- and beyond -- and compared with numpy's float64
functions: the error in ulps of the float32 result (for sin / cos near their zeros,
where ulps shrink without bound, the absolute error).

The bounds asserted are the measured ones, rounded up: every function is within a
few ulps of the correctly rounded value.  For context, the WGSL specification lets a
conforming implementation (naga -> SPIR-V -> the driver, which the reference uses)
be far looser (its f32 accuracy table allows, e.g., an absolute error of 2^-11 for
sin / cos on [-pi, pi] and 4096 ulps for atan2), so the reference's own shading
results are implementation-defined at the bit level; the build pins one accurate
choice and uses it on both sides."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

FUNCS1 = ["sinf", "cosf", "acosf", "expf", "exp2f", "log2f", "sqrtf", "atanf"]


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("detmath")
    src, so = d / "shim.c", d / "shim.so"
    body = ['#include "%s"' % os.path.join(ROOT, "include", "rt_detmath.h")]
    for f in FUNCS1:
        body.append(f"void v_{f}(const float* x, float* y, long n) {{ for (long i = 0; i < n; i++) "
                    f"y[i] = rt_det_{f}(x[i]); }}")
    body.append("void v_powf(const float* x, const float* e, float* y, long n) { for (long i = 0; i < n; i++) "
                "y[i] = rt_det_powf(x[i], e[i]); }")
    body.append("void v_atan2f(const float* a, const float* b, float* y, long n) { for (long i = 0; i < n; i++) "
                "y[i] = rt_det_atan2f(a[i], b[i]); }")
    src.write_text("\n".join(body) + "\n")
    # the oracle's flags: no contraction, IEEE
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC", "-o", str(so), str(src),
                    "-lm"], check=True)
    return C.CDLL(str(so))


def _f32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _call1(lib, name, x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    getattr(lib, "v_" + name)(_f32p(x), _f32p(y), C.c_long(x.size))
    return y


def _call2(lib, name, a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    y = np.empty_like(a)
    getattr(lib, "v_" + name)(_f32p(a), _f32p(b), _f32p(y), C.c_long(a.size))
    return y


def _ulps(got, ref):
    """|got - ref| in units of the float32 spacing at ref (ref float64)."""
    sp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    return np.abs(got.astype(np.float64) - ref) / sp


def _sweep(lo, hi, n, seed):
    rng = np.random.default_rng(seed)
    return np.concatenate([np.linspace(lo, hi, n // 2, dtype=np.float32),
                           rng.uniform(lo, hi, n - n // 2).astype(np.float32)])


def test_sin_cos(lib):
    # the shaders' arguments: 2 pi x rnd (cosine-hemisphere azimuths) and similar, in
    # [0, 2 pi]; swept over [-8 pi, 8 pi]
    x = _sweep(-8 * np.pi, 8 * np.pi, 1 << 21, 1)
    for name, ref in (("sinf", np.sin), ("cosf", np.cos)):
        r = ref(x.astype(np.float64))
        g = _call1(lib, name, x)
        abs_err = np.abs(g - r)
        big = np.abs(r) > 2 ** -6   # away from the zeros: ulps; near them: absolute error
        print(f"{name}: max {_ulps(g[big], r[big]).max():.2f} ulp (|y| > 2^-6), max abs {abs_err.max():.2e}")
        assert _ulps(g[big], r[big]).max() <= 2.0   # measured 1.52
        assert abs_err.max() <= 2 ** -23            # measured 1.3 x 2^-24


def test_acos(lib):
    x = _sweep(-1.0, 1.0, 1 << 21, 2)
    x[:3] = [-1.0, 0.0, 1.0]
    r = np.arccos(x.astype(np.float64))
    g = _call1(lib, "acosf", x)
    u = _ulps(g[r > 2 ** -10], r[r > 2 ** -10])
    print(f"acosf: max {u.max():.2f} ulp, max abs {np.abs(g - r).max():.2e}")
    assert u.max() <= 2.0                    # measured 1.26
    assert np.abs(g - r).max() <= 2 ** -21   # measured 3.0e-7 (near pi)
    assert _call1(lib, "acosf", np.array([1.5, np.nan], np.float32)).tolist() != [0.0, 0.0]   # NaN outside


def test_exp_exp2_log2_pow(lib):
    x = _sweep(-87.0, 88.0, 1 << 20, 3)
    u = _ulps(_call1(lib, "expf", x), np.exp(x.astype(np.float64)))
    print(f"expf: max {u.max():.2f} ulp")
    assert u.max() <= 1.5   # measured 0.99
    x = _sweep(-126.0, 127.0, 1 << 20, 4)
    u = _ulps(_call1(lib, "exp2f", x), np.exp2(x.astype(np.float64)))
    print(f"exp2f: max {u.max():.2f} ulp")
    assert u.max() <= 1.5   # measured 1.17
    ints = np.arange(-126, 128, dtype=np.float32)
    # exact powers of two for integer exponents (the RGBE decode); the reference value is
    # ldexp (numpy's float32 exp2 itself rounds 2^127 wrongly)
    assert np.array_equal(_call1(lib, "exp2f", ints), np.ldexp(np.float32(1.0), ints.astype(np.int32)))
    x = np.exp2(_sweep(-30.0, 30.0, 1 << 20, 5).astype(np.float64)).astype(np.float32)
    r = np.log2(x.astype(np.float64))
    g = _call1(lib, "log2f", x)
    far = np.abs(r) > 0.5
    print(f"log2f: max {_ulps(g[far], r[far]).max():.2f} ulp (|y| > 0.5), max abs near 1 "
          f"{np.abs(g[~far] - r[~far]).max():.2e}")
    assert _ulps(g[far], r[far]).max() <= 1.5          # measured 0.94
    assert np.abs(g[~far] - r[~far]).max() <= 2 ** -24   # measured 3.7e-8
    # pow as the shaders use it: the Phong lobe cos^s (w6e3.wgsl:418, base in [0, 1],
    # exponents up to ~200) and the display transform x^1.5
    rng = np.random.default_rng(6)
    b = rng.uniform(0.0, 1.0, 1 << 20).astype(np.float32)
    e = rng.uniform(0.5, 200.0, 1 << 20).astype(np.float32)
    r = np.power(b.astype(np.float64), e.astype(np.float64))
    g = _call2(lib, "powf", b, e)
    ok = r > 1e-30
    rel = np.abs(g[ok] - r[ok]) / r[ok]
    print(f"powf: max relative error {rel.max():.2e} (result > 1e-30)")
    # exp2(y log2 x): log2's absolute error times y, up to ~2^-16 relative at y = 200
    assert rel.max() <= 2 ** -15   # measured 8.6e-6


def test_atan2_full_plane(lib):
    rng = np.random.default_rng(8)
    y = rng.normal(size=1 << 20).astype(np.float32) * np.float32(10.0) ** rng.uniform(-3, 3, 1 << 20).astype(np.float32)
    x = rng.normal(size=1 << 20).astype(np.float32) * np.float32(10.0) ** rng.uniform(-3, 3, 1 << 20).astype(np.float32)
    r = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    g = _call2(lib, "atan2f", y, x)
    big = np.abs(r) > 2 ** -10
    u = _ulps(g[big], r[big])
    print(f"atan2f: max {u.max():.2f} ulp (|y| > 2^-10), max abs {np.abs(g - r).max():.2e}")
    assert u.max() <= 4.0                    # measured 2.84
    assert np.abs(g - r).max() <= 2 ** -21   # measured 2.6e-7


def test_sqrt_is_correctly_rounded(lib):
    x = np.abs(_sweep(0.0, 1e6, 1 << 20, 9))
    assert np.array_equal(_call1(lib, "sqrtf", x), np.sqrt(x))
