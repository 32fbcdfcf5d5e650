"""CPU oracle for W9E2 (w9e2.wgsl): the RGBE decode of environment_map
(rgb * pow(2, a*255 - 128), w9e2.wgsl:240-245) and the holdout plane's primary
ids.  The reference holds no W9E2 outputs and its RGBE texture
(luxo_pxr_campus.hdr.png) is missing from the checkout, so these are the
shader's closed-form values; GPU parity is tests/test_gpu_w9e2.py."""
import numpy as np
import pytest

import oracle_ffi as O
from conftest import model
from parity_util import TEAPOT_CAM


@pytest.fixture(scope="module")
def teapot_ref(rt):
    m = rt.Mesh.from_obj(model("teapot.obj"))
    V, N, I, M, L = m.arrays()
    om = O.OracleMesh(V, N, I, M, L)
    return om, O.build_bsp(om)


@pytest.mark.parametrize("alpha", [0, 1, 100, 128, 129, 200, 255])
def test_rgbe_uniform_texture_exact(teapot_ref, alpha):
    # a uniform texture filters to itself up to the rounding of the bilinear
    # weights (their f32 sum is not always 1; the exponent a*255 - 128 carries
    # that x255): the sky pixel is (c/255) * 2^(alpha - 128)
    om, bsp = teapot_ref
    tex = np.zeros((8, 16, 4), np.uint8)
    tex[..., 0], tex[..., 1], tex[..., 2], tex[..., 3] = 200, 51, 7, alpha
    sc = O.SceneRef(om, bsp, env_tex=tex)
    a, ids, _ = O.render(sc, O.make_uniform(*TEAPOT_CAM, 80, 45), "W9E2", "BSP", (0, 0, 80, 45), 0, 1)
    want = (np.array([200, 51, 7], np.float32) / np.float32(255.0)) * np.float32(2.0 ** (alpha - 128))
    assert np.allclose(a[0, 0, :3], want, rtol=2e-5, atol=0)
    assert ids[0, 0] == 0xFFFFFFFF


def test_holdout_plane_below_the_horizon(teapot_ref):
    # the camera sits at y = 1.5 looking along -z: pixels below the image
    # centre that miss the teapot look down at the plane y = 0.  W9E1 shows the
    # constant environment (1, 1, 1) there; W9E2 the holdout: the same
    # environment when the AO ray escapes, 0 when the teapot occludes it
    om, bsp = teapot_ref
    sc = O.SceneRef(om, bsp)
    u = O.make_uniform(*TEAPOT_CAM, 160, 90)
    a2, i2, c2 = O.render(sc, u, "W9E2", "BSP", (0, 0, 160, 90), 0, 1)
    a1, i1, c1 = O.render(sc, u, "W9E1", "BSP", (0, 0, 160, 90), 0, 1)
    rows = np.arange(90)[:, None] >= 46
    plane = rows & (i1 == 0xFFFFFFFF)
    assert plane.sum() > 500
    assert (i2[plane] == 0xFFFFFFFF).all()
    assert (a1[plane][:, :3] == 1.0).all()
    v = a2[plane][:, :3]
    assert set(np.unique(v)) == {0.0, 1.0}
    assert c2["shadow"] > c1["shadow"]
