"""W9E2 (res/shaders/w9e2.wgsl; scenes.rs "W9 E2 Teapot" / "W9 E2 Bunny"): W9E1
plus the holdout plane y = 0 -- tested before the mesh, shaded by an any-hit
ambient-occlusion ray (intersect_trimesh_immediate_return, bsp.wgsl:83-155)
that shows the environment behind the plane when unoccluded -- and the RGBE
decode of the environment texture.  HIP kernel through the C ABI vs the CPU
oracle; bar: bit-exact radiance and ids, equal ray counts."""
import numpy as np
import pytest

from conftest import model
from parity_util import BUNNY_CAM, TEAPOT_CAM, Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def teapot(rt, gpu):
    return rt.Mesh.from_obj(model("teapot.obj"))


@pytest.mark.parametrize("trav", ["BSP", "BVH"])
def test_w9e2_teapot(rt, teapot, trav):
    s = Scene(rt, teapot, trav)
    region = (150, 150, 500, 300)   # the teapot and the plane around and below it
    g = s.render_gpu("W9E2", TEAPOT_CAM, 800, 450, region, 0, 2)
    o = s.render_oracle("W9E2", TEAPOT_CAM, 800, 450, region, 0, 2)
    check(g, o)
    ids = g[1]
    # plane pixels report no triangle; the AO rays are counted with the shadow rays
    assert (ids == 0xFFFFFFFF).sum() > 1000 and (ids != 0xFFFFFFFF).sum() > 1000
    assert g[2]["shadow"] > g[2]["primary"] // 2


@pytest.mark.parametrize("sel", [2, 5, 6, 7])
def test_w9e2_selection(rt, teapot, sel):
    s = Scene(rt, teapot, "BSP")
    region = (250, 180, 300, 200)
    g = s.render_gpu("W9E2", TEAPOT_CAM, 800, 450, region, 0, 2, selection1=sel)
    o = s.render_oracle("W9E2", TEAPOT_CAM, 800, 450, region, 0, 2, selection1=sel)
    check(g, o)


def _rgbe_scene(rt, mesh, tex, trav="BSP"):
    s = Scene(rt, mesh, trav)
    s.ctx.set_environment_map(tex)
    s.oscene = s.oscene.__class__(s.om, s.obsp, s.obvh, s.env, env_tex=tex)
    return s


def test_w9e2_rgbe_environment(rt, teapot):
    # random RGB, exponents around 128 (filtered alphas give fractional
    # exponents) plus the extremes 0 (2^-128, subnormal) and 255 (2^127)
    rng = np.random.default_rng(5)
    tex = rng.integers(0, 256, size=(23, 41, 4), dtype=np.uint8)
    tex[..., 3] = rng.integers(120, 137, size=(23, 41), dtype=np.uint8)
    tex[0, :, 3] = 0
    tex[-1, :, 3] = 255
    s = _rgbe_scene(rt, teapot, tex)
    g = s.render_gpu("W9E2", TEAPOT_CAM, 800, 450, (0, 0, 800, 450), 0, 1)
    o = s.render_oracle("W9E2", TEAPOT_CAM, 800, 450, (0, 0, 800, 450), 0, 1)
    check(g, o)


def test_w9e2_bunny_bvh_region(rt):
    s = Scene(rt, rt.Mesh.synth_bunny(), "BVH")
    g = s.render_gpu("W9E2", BUNNY_CAM, 512, 512, (128, 192, 256, 192), 0, 2)
    o = s.render_oracle("W9E2", BUNNY_CAM, 512, 512, (128, 192, 256, 192), 0, 2)
    check(g, o)
