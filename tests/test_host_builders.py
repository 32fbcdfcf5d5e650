"""Product host builders (lib02562rt.so, no GPU needed) vs the CPU oracle:
Mesh::from_obj, BspTree::new + bsp_array + primitive_ids, hlbvh::Bvh -- bit
identical arrays."""
import numpy as np
import pytest

from conftest import model

NAMES = ["CornellBox.obj", "CornellBoxWithBlocks.obj", "test_object.obj", "plane.obj", "teapot.obj"]


@pytest.mark.parametrize("name", NAMES)
def test_obj_loader_matches_oracle(rt, oracle, name):
    V, N, I, M, L = rt.Mesh.from_obj(model(name)).arrays()
    om = oracle.load_obj(model(name))
    assert np.array_equal(V, om.pos) and np.array_equal(N, om.nrm) and np.array_equal(I, om.idx)
    assert np.array_equal(M, om.mats) and np.array_equal(L, om.lights)


@pytest.mark.parametrize("name", NAMES)
def test_bsp_matches_oracle(rt, oracle, name):
    m = rt.Mesh.from_obj(model(name))
    tree, planes, ids, aabb, md = m.bsp_tree(20, 4).arrays()
    ob = oracle.build_bsp(oracle.load_obj(model(name)), 20, 4)
    assert md == 20 and tree.shape == (2 ** 21 - 1, 4)
    assert np.array_equal(tree, ob.tree)
    assert np.array_equal(planes.view(np.uint32), ob.planes.view(np.uint32))
    assert np.array_equal(ids, ob.ids) and np.array_equal(aabb, ob.aabb)


@pytest.mark.parametrize("name", NAMES)
def test_bvh_matches_oracle(rt, oracle, name):
    nodes, tids = rt.Mesh.from_obj(model(name)).bvh(4).arrays()
    ob = oracle.build_bvh(oracle.load_obj(model(name)), 4)
    assert np.array_equal(nodes, ob.nodes) and np.array_equal(tids, ob.tri_ids)


def test_bunny_standin_builders(rt, oracle):
    m = rt.Mesh.synth_bunny()
    V, N, I, M, L = m.arrays()
    assert abs(I.shape[0] - 69451) <= 0.01 * 69451          # 69,451 +- 1%
    lo, hi = V[:, :3].min(0), V[:, :3].max(0)
    assert np.allclose((lo + hi) / 2, [-0.0168, 0.110, -0.0015], atol=0.02)
    om = oracle.OracleMesh(V, N, I, M, L)
    tree, planes, ids, aabb, _ = m.bsp_tree().arrays()
    ob = oracle.build_bsp(om)
    assert np.array_equal(tree, ob.tree) and np.array_equal(planes, ob.planes) and np.array_equal(ids, ob.ids)
    nodes, tids = m.bvh().arrays()
    obv = oracle.build_bvh(om)
    assert np.array_equal(nodes, obv.nodes) and np.array_equal(tids, obv.tri_ids)


def test_bsp_parallel_build_is_deterministic(rt):
    m = rt.Mesh.synth_bunny(20000, seed=11)
    a = m.bsp_tree(nthreads=1).arrays()
    b = m.bsp_tree(nthreads=8).arrays()
    for x, y in zip(a[:4], b[:4]):
        assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))


def test_soup_and_grid(rt, oracle):
    s = rt.Mesh.synth_soup(5000, seed=0x5EED)
    V, N, I, M, L = s.arrays()
    assert I.shape[0] == 5000 and np.abs(V[:, :3]).max() <= 1.02
    g = rt.Mesh.grid(rt.Mesh.synth_bunny(2000), 3, 2, 0.2)
    GV, GN, GI, GM, GL = g.arrays()
    assert GI.shape[0] == 6 * rt.Mesh.synth_bunny(2000).ntris
    om = oracle.OracleMesh(GV, GN, GI, GM, GL)
    tree, planes, ids, aabb, _ = g.bsp_tree(12, 4).arrays()
    ob = oracle.build_bsp(om, 12, 4)
    assert np.array_equal(tree, ob.tree) and np.array_equal(ids, ob.ids)


def test_builder_errors(rt):
    m = rt.Mesh.from_obj(model("CornellBox.obj"))
    with pytest.raises(rt.RtError):
        m.bsp_tree(0, 4)            # bsp_tree.rs:51-54: depth must be in (0, 32)
    with pytest.raises(rt.RtError):
        m.bsp_tree(32, 4)
    with pytest.raises(rt.RtError):
        m.bsp_tree(20, 0)           # :55-58 leaf objects must be positive
    with pytest.raises(rt.RtError):
        rt.Mesh.from_obj(model("does_not_exist.obj"))
    with pytest.raises(rt.RtError):
        rt.Mesh.from_arrays(np.zeros((3, 4), np.float32), np.array([[0, 1, 5, 0]], np.uint32))
