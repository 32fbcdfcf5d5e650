"""The pinned environment_map (include/rt_detmath.h, w9e1.wgsl:232-239) on the
CPU: atan2 accuracy against numpy, the equirectangular (u, 1 - v) mapping and
the bilinear ClampToEdge weights, through the oracle's W9E1 escape path."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT, model


def _detmath():
    """Compile a tiny shim around the header (test infrastructure)."""
    src = os.path.join(ROOT, "oracle", "_detmath_shim.c")
    so = os.path.join(ROOT, "oracle", "_detmath_shim.so")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(os.path.join(ROOT, "include", "rt_detmath.h")):
        with open(src, "w") as f:
            f.write('#include "../include/rt_detmath.h"\n'
                    'float shim_atan2(float y, float x) { return rt_det_atan2f(y, x); }\n'
                    'void shim_env(const unsigned int* t, unsigned int w, unsigned int h, float x, float y, float z,'
                    ' float* o) { rt_det_env_sample(t, w, h, x, y, z, o); }\n')
        os.system(f"cc -O2 -ffp-contract=off -fno-fast-math -shared -fPIC -o {so} {src} -lm")
    lib = C.CDLL(so)
    lib.shim_atan2.restype = C.c_float
    lib.shim_atan2.argtypes = [C.c_float, C.c_float]
    lib.shim_env.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_float, C.c_float, C.c_float,
                             C.POINTER(C.c_float)]
    return lib


def test_atan2_accuracy():
    lib = _detmath()
    rng = np.random.default_rng(7)
    ys = rng.uniform(-3, 3, 20000).astype(np.float32)
    xs = rng.uniform(-3, 3, 20000).astype(np.float32)
    got = np.array([lib.shim_atan2(float(y), float(x)) for y, x in zip(ys, xs)], np.float32)
    ref = np.arctan2(ys.astype(np.float64), xs.astype(np.float64))
    ulp = np.abs(got - ref) / np.spacing(np.abs(ref).astype(np.float32))
    assert ulp.max() <= 4.0, ulp.max()
    assert lib.shim_atan2(1.0, 0.0) == np.float32(np.pi / 2)
    assert lib.shim_atan2(0.0, -1.0) == np.float32(np.pi)
    assert lib.shim_atan2(0.0, 0.0) == 0.0


def test_env_lookup_mapping():
    lib = _detmath()
    w, h = 8, 4
    tex = np.zeros((h, w, 4), np.uint8)
    tex[..., 0] = (np.arange(w) * 30)[None, :]        # red encodes the column
    tex[..., 1] = (np.arange(h) * 60)[:, None]        # green encodes the row
    t32 = tex.view(np.uint32)
    out = (C.c_float * 3)()
    # direction (0, 0, -1): u = 0.5, v = 0.5 -> the texture centre (between columns 3|4, rows 1|2)
    lib.shim_env(t32.ctypes.data, w, h, 0.0, 0.0, -1.0, out)
    assert abs(out[0] - 105.0 / 255.0) < 1e-6 and abs(out[1] - 90.0 / 255.0) < 1e-6
    # straight up (0, 1, 0): v = acos(-1)/pi = 1 -> t = 0: clamped to row 0
    lib.shim_env(t32.ctypes.data, w, h, 0.0, 1.0, 0.0, out)
    assert out[1] == 0.0
    # straight down: row h-1
    lib.shim_env(t32.ctypes.data, w, h, 0.0, -1.0, 0.0, out)
    assert abs(out[1] - 180.0 / 255.0) < 1e-6


def test_oracle_w9e1_with_texture(oracle):
    # the oracle's escape uses the texture: a constant texture equals the constant env
    O = oracle
    m = O.load_obj(model("teapot.obj"))
    bsp = O.build_bsp(m)
    tex = np.zeros((16, 32, 4), np.uint8)
    tex[..., :3] = (204, 153, 51)
    cam = ((0.15, 1.5, 10.0), (0.15, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5)
    u = O.make_uniform(*cam, 160, 90)
    a, _, _ = O.render(O.SceneRef(m, bsp, env_tex=tex), u, "W9E1", "BSP", (40, 20, 32, 24), 0, 1)
    env = (np.float32(204) / np.float32(255), np.float32(153) / np.float32(255), np.float32(51) / np.float32(255))
    b, _, _ = O.render(O.SceneRef(m, bsp, env=env), u, "W9E1", "BSP", (40, 20, 32, 24), 0, 1)
    assert np.abs(a - b).max() < 1e-6
