"""CPU oracle for W8E1/W8E2/W8E3 (oracle/oracle_render.c, sample_w8): properties
that hold without a GPU.  The reference has no stored outputs for these
scenes (its renders go to a window), so the restatement is checked against
what the shaders fix exactly: the W8E1 background colour on escape, the
primary ids of ball pixels, the ray bookkeeping, and the clamp/absorption
bounds.  GPU parity is tests/test_gpu_w8.py."""
import numpy as np
import pytest

import oracle_ffi as O
from conftest import model
from parity_util import CORNELL_CAM


@pytest.fixture(scope="module")
def balls(rt):
    mesh = rt.Mesh.from_obj(model("CornellBox.obj"))
    V, N, I, M, L = mesh.arrays()
    om = O.OracleMesh(V, N, I, M, L)
    return O.SceneRef(om, O.build_bsp(om), O.build_bvh(om))


def _render(sc, mode, trav="BSP", W=64, H=64, spp=1):
    return O.render(sc, O.make_uniform(*CORNELL_CAM, W, H), mode, trav, (0, 0, W, H), 0, spp)


def test_w8e1_background_on_escape(balls):
    # the box is open towards the camera: the outermost pixels escape at once
    # and W8E1 returns BACKGROUND_COLOR (0.1, 0.3, 0.6) (w8e1.wgsl:4, :228)
    a, ids, _ = _render(balls, "W8E1", W=64, H=64, spp=1)
    corner = a[0, 0, :3]
    assert np.array_equal(corner, np.array([0.1, 0.3, 0.6], np.float32))
    assert ids[0, 0] == 0xFFFFFFFF
    # W8E2/W8E3: BACKGROUND_COLOR is black
    for mode in ("W8E2", "W8E3"):
        a2, _, _ = _render(balls, mode, W=64, H=64, spp=1)
        assert np.array_equal(a2[0, 0, :3], np.zeros(3, np.float32))


@pytest.mark.parametrize("mode", ["W8E1", "W8E2", "W8E3"])
def test_w8_ray_bookkeeping(balls, mode):
    W = H = 48
    spp = 4
    a, ids, c = _render(balls, mode, W=W, H=H, spp=spp)
    assert c["samples"] == W * H * spp and c["primary"] == W * H * spp
    assert c["shadow"] > 0
    assert np.isfinite(a).all() and (a[..., :3] >= 0).all() and (a[..., 3] == 1).all()
    if mode == "W8E1":
        # at most MAX_DEPTH = 10 segments per sample
        assert c["bounce"] <= 9 * c["samples"]
    # ball pixels report no primary triangle; the rest of the box does
    assert 0 < (ids == 0xFFFFFFFF).sum() < W * H // 4


@pytest.mark.parametrize("mode", ["W8E1", "W8E2", "W8E3"])
def test_w8_bsp_equals_bvh(balls, mode):
    # both walks find the same closest triangle on every ray of the scene
    a, ia, _ = _render(balls, mode, "BSP", 40, 40, 2)
    b, ib, _ = _render(balls, mode, "BVH", 40, 40, 2)
    assert np.array_equal(ia, ib)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_w8e2_clamp_bounds_one_sample(balls):
    # min(shade(), 100) per segment, at most 50 segments: one sample <= 5000
    a, _, _ = _render(balls, "W8E2", W=32, H=32, spp=1)
    assert a[..., :3].max() <= 5000.0


def test_w8e3_absorbs(balls):
    # the glass ball absorbs in W8E3 (extinction (0.5, 0.2, 0.2) on exit):
    # fewer continuation segments than W8E2 on the same samples
    _, _, c2 = _render(balls, "W8E2", W=64, H=64, spp=4)
    _, _, c3 = _render(balls, "W8E3", W=64, H=64, spp=4)
    assert c3["bounce"] < c2["bounce"]
