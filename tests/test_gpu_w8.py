"""W8E1 / W8E2 / W8E3 (res/shaders/w8e{1,2,3}.wgsl; scenes.rs "W8 E1 Cornell Box
Balls", "W8 E2 Cornell Box Balls", "W8 E3 Absorption"): the Cornell box with a
mirror ball and a glass ball, through the C ABI vs the CPU oracle.  Bar: as
tests/test_gpu_parity.py -- primary-hit ids and radiance bit-exact, ray counts
equal.  The glass ball's total internal reflection turns rays into NaN rays
(sqrt of a negative cos_t^2, as the shader computes it); full frames cover
those paths on both sides."""
import numpy as np
import pytest

from conftest import model
from parity_util import CORNELL_CAM, Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu

MODES = ("W8E1", "W8E2", "W8E3")


@pytest.fixture(scope="module")
def balls_bsp(rt, gpu):
    return Scene(rt, rt.Mesh.from_obj(model("CornellBox.obj")), "BSP")


@pytest.fixture(scope="module")
def balls_bvh(rt, gpu):
    return Scene(rt, rt.Mesh.from_obj(model("CornellBox.obj")), "BVH")


@pytest.mark.parametrize("mode", MODES)
def test_w8_full_frame_bsp(balls_bsp, mode):
    g = balls_bsp.render_gpu(mode, CORNELL_CAM, 128, 128, (0, 0, 128, 128), 0, 6)
    o = balls_bsp.render_oracle(mode, CORNELL_CAM, 128, 128, (0, 0, 128, 128), 0, 6)
    check(g, o)
    assert g[2]["shadow"] > 0 and g[2]["bounce"] > 0
    assert np.isfinite(g[0]).all()


@pytest.mark.parametrize("mode", MODES)
def test_w8_full_frame_bvh(balls_bvh, mode):
    g = balls_bvh.render_gpu(mode, CORNELL_CAM, 96, 96, (0, 0, 96, 96), 0, 4)
    o = balls_bvh.render_oracle(mode, CORNELL_CAM, 96, 96, (0, 0, 96, 96), 0, 4)
    check(g, o)


@pytest.mark.parametrize("mode", MODES)
def test_w8_scene_resolution_region(balls_bsp, mode):
    # the scene's own 512x512 frame, a region over both balls (the mirror ball
    # around pixel (178, 356), the glass ball around (348, 371): grazing hits
    # with total internal reflection) and the floor below them
    g = balls_bsp.render_gpu(mode, CORNELL_CAM, 512, 512, (120, 290, 300, 150), 0, 3)
    o = balls_bsp.render_oracle(mode, CORNELL_CAM, 512, 512, (120, 290, 300, 150), 0, 3)
    check(g, o)


def test_w8e2_progressive_continuation(balls_bsp):
    full = balls_bsp.render_gpu("W8E2", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 5)
    a = balls_bsp.render_gpu("W8E2", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 2)
    b = balls_bsp.render_gpu("W8E2", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 2, 3, accum_in=a[0])
    assert np.array_equal(full[0].view(np.uint32), b[0].view(np.uint32))
    o = balls_bsp.render_oracle("W8E2", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 2, 3, accum_in=a[0].copy())
    check(b, o)


def test_w8_ball_pixels_have_no_primary_triangle(balls_bsp):
    # a primary ray that ends on a ball reports no triangle (0xFFFFFFFF), as the
    # oracle; the mesh hits around it do
    g = balls_bsp.render_gpu("W8E1", CORNELL_CAM, 128, 128, (0, 0, 128, 128), 0, 1)
    ids = g[1]
    assert (ids == 0xFFFFFFFF).sum() > 200 and (ids != 0xFFFFFFFF).sum() > 10000


def test_w8_needs_area_light(rt, gpu):
    # W8 samples area lights: a mesh without an emissive triangle is refused
    m = rt.Mesh.from_obj(model("test_object.obj"))
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh(m)
        ctx.upload_bsp(m.bsp_tree())
        ctx.set_uniforms(rt.make_uniform(*CORNELL_CAM, 16, 16))
        acc = ctx.alloc(16 * 16 * 16)
        with pytest.raises(rt.RtError):
            ctx.render("W8E2", "BSP", (0, 0, 16, 16), 0, 1, acc.ptr, None)
        acc.free()
    finally:
        ctx.close()
