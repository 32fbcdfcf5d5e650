"""GPU BSP construction (rt_build_bsp_device) vs the host
builder rt_bsp_build -- bit-identical to the oracle's f32 restatement of
bsp_tree.rs (tests/test_host_builders.py) and, in f64, to the reference's own
JS builder (tests/test_oracle.py).  Bar: bsp_array, planes (bitwise),
primitive_ids and the root BboxGpu are bit-exact; renders through the
device-built tree equal renders through the uploaded host build."""
import numpy as np
import pytest

from conftest import model
from parity_util import BUNNY_CAM, CORNELL_CAM

pytestmark = pytest.mark.gpu


def _check(rt, mesh, max_depth=20, max_leaf=4):
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh(mesh)
        t = ctx.build_bsp_device(max_depth, max_leaf)
        gt, gp, gi, ga = ctx.download_bsp()
    finally:
        ctx.close()
    ht, hp, hi, ha, _ = mesh.bsp_tree(max_depth, max_leaf).arrays()
    assert gt.shape == ht.shape
    bad = np.nonzero((gt != ht).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} nodes differ, first {bad[:4]}: gpu {gt[bad[:1]]} host {ht[bad[:1]]}"
    badp = np.nonzero(gp.view(np.uint32) != hp.view(np.uint32))[0]
    assert badp.size == 0, f"{badp.size} planes differ, first {badp[:4]}: gpu {gp[badp[:2]]} host {hp[badp[:2]]}"
    assert np.array_equal(gi, hi), (gi.size, hi.size)
    assert np.array_equal(ga.view(np.uint32), ha.view(np.uint32))
    assert t["nids"] == hi.size
    return t


@pytest.mark.parametrize("name", ["test_object.obj", "plane.obj", "CornellBox.obj", "CornellBoxWithBlocks.obj",
                                  "teapot.obj"])
@pytest.mark.parametrize("depth,leaf", [(20, 4), (8, 1), (12, 2), (3, 4)])
def test_assets(rt, name, depth, leaf):
    _check(rt, rt.Mesh.from_obj(model(name)), depth, leaf)


def test_bunny_standin(rt):
    t = _check(rt, rt.Mesh.synth_bunny())
    assert t["levels"] == 21


def test_soup(rt):
    _check(rt, rt.Mesh.synth_soup(300_000))


def test_grid_of_copies(rt):
    # translated copies: many coincident candidate planes and shared extents
    _check(rt, rt.Mesh.grid(rt.Mesh.synth_bunny(2000), 4, 3, 0.2))


def test_duplicates_empty_sides(rt):
    # identical / nearly identical triangles: candidate planes with an empty
    # side, so the plane moves to the objects' extent +- max(size/8, 1e-6)
    tri = np.array([[0, 0, 0, 1], [1, 0, 0, 1], [0, 1, 0, 1]], np.float32)
    verts = np.concatenate([tri + np.array([0.001 * (i % 3), 0.0, 0.0, 0.0], np.float32) for i in range(40)])
    idx = np.array([[3 * i, 3 * i + 1, 3 * i + 2, 0] for i in range(40)], np.uint32)
    mesh = rt.Mesh.from_arrays(verts, idx)
    for depth, leaf in ((20, 4), (6, 1)):
        _check(rt, mesh, depth, leaf)


def test_single_triangle(rt):
    mesh = rt.Mesh.from_arrays(np.array([[0, 0, 0, 1], [1, 0, 0, 1], [0, 1, 0, 1]], np.float32),
                               np.array([[0, 1, 2, 0]], np.uint32))
    _check(rt, mesh)


def test_render_with_device_bsp(rt):
    mesh = rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj"))
    out = []
    for device_build in (False, True):
        ctx = rt.Context(0)
        ctx.upload_mesh(mesh)
        if device_build:
            ctx.build_bsp_device(20, 4)
        else:
            ctx.upload_bsp(mesh.bsp_tree())
        ctx.set_uniforms(rt.make_uniform(*CORNELL_CAM, 64, 64))
        acc = ctx.alloc(64 * 64 * 16)
        ids = ctx.alloc(64 * 64 * 4)
        acc.zero()
        ctx.render("W7E3", "BSP", (0, 0, 64, 64), 0, 2, acc.ptr, ids.ptr)
        out.append((acc.to_numpy(np.float32, (64, 64, 4)), ids.to_numpy(np.uint32, (64, 64))))
        acc.free()
        ids.free()
        ctx.close()
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))
    assert np.array_equal(out[0][1], out[1][1])


def test_bunny_render_with_device_bsp(rt):
    mesh = rt.Mesh.synth_bunny()
    out = []
    for device_build in (False, True):
        ctx = rt.Context(0)
        ctx.upload_mesh(mesh)
        if device_build:
            ctx.build_bsp_device(20, 4)
        else:
            ctx.upload_bsp(mesh.bsp_tree())
        ctx.set_uniforms(rt.make_uniform(*BUNNY_CAM, 1920, 1080))
        acc = ctx.alloc(256 * 64 * 16)
        acc.zero()
        ctx.render("W9E1", "BSP", (832, 476, 256, 64), 0, 2, acc.ptr, None)
        out.append(acc.to_numpy(np.float32, (64, 256, 4)))
        acc.free()
        ctx.close()
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
