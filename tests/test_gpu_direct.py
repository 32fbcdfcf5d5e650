"""W6E2 / W7E1 / W7E2 (res/shaders/w6e2.wgsl, w7e1.wgsl, w7e2.wgsl; scenes.rs
"W6 E2 Cornell Box", "W7 E1 Cornell Box", "W7 E2 Cornell Box"): direct light
from every area-light triangle of CornellBoxWithBlocks.obj, through the C ABI
(k_direct) vs the CPU oracle.  Bar: bit-exact radiance and ids, equal ray
counts.  W7E1/W7E2 accumulate without max(., 0), so negative pixels (the
unclamped cos terms) must match too."""
import numpy as np
import pytest

from conftest import model
from parity_util import CORNELL_CAM, Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["BSP", "BVH"])
def blocks(request, rt, gpu):
    return Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), request.param)


@pytest.mark.parametrize("mode,spp", [("W6E2", 1), ("W7E1", 3), ("W7E2", 3)])
def test_direct_modes(blocks, mode, spp):
    g = blocks.render_gpu(mode, CORNELL_CAM, 96, 96, (0, 0, 96, 96), 0, spp)
    o = blocks.render_oracle(mode, CORNELL_CAM, 96, 96, (0, 0, 96, 96), 0, spp)
    check(g, o)
    # two light triangles: two shadow rays per primary ray that hits the box
    assert 0 < g[2]["shadow"] <= 2 * g[2]["primary"] and g[2]["shadow"] % 2 == 0


def test_w6e2_subdivision_jitter(rt, blocks):
    J = __import__("importlib").import_module("02562_raytracer_amd.jitter")
    jit = J.jitters_for(80, 3)
    g = blocks.render_gpu("W6E2", CORNELL_CAM, 80, 80, (0, 0, 80, 80), 0, 1, jitter=jit)
    o = blocks.render_oracle("W6E2", CORNELL_CAM, 80, 80, (0, 0, 80, 80), 0, 1, jitter=jit)
    check(g, o)
    assert g[2]["primary"] == 80 * 80 * 9


@pytest.mark.parametrize("mode", ["W7E1", "W7E2"])
def test_progressive_continuation_without_clamp(blocks, mode):
    full = blocks.render_gpu(mode, CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 5)
    a = blocks.render_gpu(mode, CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 2)
    b = blocks.render_gpu(mode, CORNELL_CAM, 64, 64, (0, 0, 64, 64), 2, 3, accum_in=a[0])
    assert np.array_equal(full[0].view(np.uint32), b[0].view(np.uint32))
    o = blocks.render_oracle(mode, CORNELL_CAM, 64, 64, (0, 0, 64, 64), 2, 3, accum_in=a[0].copy())
    check(b, o)
    if mode == "W7E1":
        assert (full[0][..., :3] < 0).any()   # the shader keeps negative accumulations


@pytest.mark.parametrize("name", ["W6 E2 Cornell Box", "W7 E1 Cornell Box", "W7 E2 Cornell Box"])
def test_scene_through_render_state(rt, name):
    rs = rt.RenderState(rt.find_scene(name), resolution=(48, 48))
    try:
        rs.render(2 if rs.mode != "W6E2" else 1)
        assert np.isfinite(rs.frame()).all()
        assert rs.iteration == (2 if rs.mode != "W6E2" else 0)
    finally:
        rs.ctx.close()


@pytest.fixture(scope="module", params=["BSP", "BVH"])
def balls(request, rt, gpu):
    return Scene(rt, rt.Mesh.from_obj(model("CornellBox.obj")), request.param)


def test_w6e3_mirror_and_glossy_balls(balls):
    # w6e3.wgsl: the mirror ball, the glossy ball (Phong lobe with the pinned
    # pow(., 42) + refraction, magenta under total internal reflection), the box
    g = balls.render_gpu("W6E3", CORNELL_CAM, 128, 128, (0, 0, 128, 128), 0, 1)
    o = balls.render_oracle("W6E3", CORNELL_CAM, 128, 128, (0, 0, 128, 128), 0, 1)
    check(g, o)
    assert g[2]["bounce"] > 0 and (g[1] == 0xFFFFFFFF).sum() > 100


def test_w6e3_subdivision_region(rt, balls):
    J = __import__("importlib").import_module("02562_raytracer_amd.jitter")
    jit = J.jitters_for(512, 2)
    region = (120, 290, 300, 150)   # both balls at the scene's 512x512
    g = balls.render_gpu("W6E3", CORNELL_CAM, 512, 512, region, 0, 1, jitter=jit)
    o = balls.render_oracle("W6E3", CORNELL_CAM, 512, 512, region, 0, 1, jitter=jit)
    check(g, o)
