"""GPU HLBVH construction (rt_build_bvh_device) vs the
host builder rt_bvh_build -- itself bit-identical to the oracle's restatement
of hlbvh.rs (tests/test_host_builders.py).  Bar: the GpuNode array (including
the over-allocated 9999 filler tail) and bvh_triangles are bit-exact, for
every max_prims the reference benchmarks (src/bin/bvh_project.rs: 1, 2, 4, 6,
8, 16), and renders through the device-built BVH equal renders through the
uploaded host build."""
import numpy as np
import pytest

from conftest import model
from parity_util import BUNNY_CAM, CORNELL_CAM, TEAPOT_CAM

pytestmark = pytest.mark.gpu


def _check_build(rt, mesh, max_prims):
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh(mesh)
        times = ctx.build_bvh_device(max_prims)
        gn, gi = ctx.download_bvh()
    finally:
        ctx.close()
    hn, hi = mesh.bvh(max_prims).arrays()
    assert gn.shape == hn.shape, (gn.shape, hn.shape)
    bad = np.nonzero((gn != hn).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} nodes differ, first {bad[:5]}: gpu {gn[bad[:1]]} host {hn[bad[:1]]}"
    assert np.array_equal(gi, hi)
    assert times["nodes"] == hn.shape[0]
    return times


@pytest.mark.parametrize("name", ["test_object.obj", "plane.obj", "CornellBox.obj", "CornellBoxWithBlocks.obj",
                                  "teapot.obj"])
@pytest.mark.parametrize("max_prims", [1, 2, 4, 8, 16])
def test_assets(rt, name, max_prims):
    _check_build(rt, rt.Mesh.from_obj(model(name)), max_prims)


@pytest.mark.parametrize("max_prims", [4, 6])
def test_bunny_standin(rt, max_prims):
    t = _check_build(rt, rt.Mesh.synth_bunny(), max_prims)
    assert t["treelets"] > 1


def test_soup_large(rt):
    # ~ the reference's dragon (871,414 triangles): uniformly spread, all 4096 treelets
    t = _check_build(rt, rt.Mesh.synth_soup(871_414), 4)
    assert t["treelets"] == 4096


def test_duplicates_and_flat(rt):
    # identical triangles (equal Morton codes down to bit -1: leaves of any size),
    # a flat mesh (zero centroid extent on one axis: Bbox::offset skips the divide)
    tri = np.array([[0, 0, 0, 1], [1, 0, 0, 1], [0, 1, 0, 1]], np.float32)
    verts = np.concatenate([tri + np.array([0.001 * (i % 3), 0.0, 0.0, 0.0], np.float32) for i in range(40)])
    idx = np.array([[3 * i, 3 * i + 1, 3 * i + 2, 0] for i in range(40)], np.uint32)
    mesh = rt.Mesh.from_arrays(verts, idx)
    for mp in (1, 2, 4):
        _check_build(rt, mesh, mp)


def test_single_triangle(rt):
    mesh = rt.Mesh.from_arrays(np.array([[0, 0, 0, 1], [1, 0, 0, 1], [0, 1, 0, 1]], np.float32),
                               np.array([[0, 1, 2, 0]], np.uint32))
    _check_build(rt, mesh, 4)


@pytest.mark.parametrize("mode,name,cam,W,H,region,spp", [
    ("W7E3", "CornellBoxWithBlocks.obj", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 2),
    ("PROJECT", "teapot.obj", TEAPOT_CAM, 800, 450, (300, 150, 128, 96), 1),
])
def test_render_with_device_bvh(rt, mode, name, cam, W, H, region, spp):
    mesh = rt.Mesh.from_obj(model(name))
    out = []
    for device_build in (False, True):
        ctx = rt.Context(0)
        ctx.upload_mesh(mesh)
        if device_build:
            ctx.build_bvh_device(4)
        else:
            ctx.upload_bvh(mesh.bvh(4))
        ctx.set_uniforms(rt.make_uniform(*cam, W, H))
        x0, y0, w, h = region
        acc = ctx.alloc(w * h * 16)
        ids = ctx.alloc(w * h * 4)
        acc.zero()
        ctx.render(mode, "BVH", region, 0, spp, acc.ptr, ids.ptr)
        out.append((acc.to_numpy(np.float32, (h, w, 4)), ids.to_numpy(np.uint32, (h, w))))
        acc.free()
        ids.free()
        ctx.close()
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))
    assert np.array_equal(out[0][1], out[1][1])


def test_bunny_render_with_device_bvh(rt):
    mesh = rt.Mesh.synth_bunny()
    ctx = rt.Context(0)
    ctx.upload_mesh(mesh)
    ctx.build_bvh_device(4)
    gn, gi = ctx.download_bvh()
    hn, hi = mesh.bvh(4).arrays()
    assert np.array_equal(gn, hn) and np.array_equal(gi, hi)
    ctx.set_uniforms(rt.make_uniform(*BUNNY_CAM, 1920, 1080))
    acc = ctx.alloc(256 * 64 * 16)
    acc.zero()
    c = ctx.render("W9E1", "BVH", (832, 476, 256, 64), 0, 1, acc.ptr, None, counts=True)
    assert c["primary"] == 256 * 64
    ctx.close()
