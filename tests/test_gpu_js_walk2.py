"""GPU side of the secondary-ray pin (tests/test_js_walk2.py): the shadow and
bounce rays of the committed fixtures (tests/golden/js_walk2_<scene>.npz: the
reference's own CPU walk, run under node) traced by the kernels' own walk through
the ray-query entry point rt_trace_rays, on the reference-built tree (the JS
arrays, equal to the oracle's f64 build) uploaded through rt_upload_bsp:
  * bounce rays (closest-hit, bsp.wgsl:10-81): the accepted triangle, its
    distance, the tested-triangle sequence and the interval the walk leaves
    behind equal the f32 oracle bit for bit, and the reference's walk ray for ray
    (hit, triangle, tested sequence) except the listed cause-checked rays;
  * shadow rays (the product's any-hit walk, which stops at the first accept):
    hit/miss equals the reference's, and the tests up to the first accept equal
    the prefix of the reference's sequence (gen_js_walk.js records it).
The BVH walk (bvh.wgsl:154-191; no runnable reference walk) traces the same rays
on the oracle's HLBVH and equals the oracle's walk bit for bit."""
import numpy as np
import pytest

from conftest import model
from test_js_walk import fnv
from test_js_walk2 import EXCEPTIONS, SCENES, load_fixture

pytestmark = pytest.mark.gpu

MISS = 0xFFFFFFFF


def _bits(x):
    return np.float32(x).view(np.uint32)


def _scene(rt, oracle, name, trav):
    m = oracle.load_obj(model(f"{name}.obj"))
    ctx = rt.Context(0)
    # the reference's own walk, node by node: no subtree culling (the tested-triangle
    # sequence is compared); test_secondary_rays_culled_walk_same_hits turns it on
    ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, 0)
    ctx.upload_mesh_arrays(m.pos, m.nrm, m.idx, m.mats, m.lights)
    if trav == "BSP":
        acc = oracle.build_bsp(m, 20, 4, js64=True)
        ctx.upload_bsp_arrays(acc.aabb, acc.tree, acc.planes, acc.ids, acc.max_depth)
        sc = oracle.SceneRef(m, acc)
    else:
        acc = oracle.build_bvh(m, 4)
        ctx.upload_bvh_arrays(acc.nodes, acc.tri_ids)
        sc = oracle.SceneRef(m, None, acc)
    return ctx, sc


def _rays(z):
    return np.concatenate([z["ray_o"], z["ray_d"], z["ray_tmin"][:, None], z["ray_tmax"][:, None]], axis=1)


@pytest.mark.parametrize("name", SCENES)
def test_secondary_rays_match_reference_js_walk(rt, oracle, name):
    meta, z = load_fixture(name)
    ctx, sc = _scene(rt, oracle, name, "BSP")
    try:
        shadow = z["kind"] == 1
        h = ctx.trace_rays("BSP", _rays(z), anyhit=shadow)
    finally:
        ctx.close()
    n = z["status"].shape[0]
    js_diff = set()
    for i in range(n):
        q = oracle.trace_query(sc, "BSP", z["ray_o"][i], z["ray_d"][i], float(z["ray_tmin"][i]),
                               float(z["ray_tmax"][i]))
        js_hit = int(z["status"][i]) == 1
        if not shadow[i]:
            # closest-hit: the f32 oracle bit for bit ...
            assert h["tri"][i] == (q["tri"] if q["status"] == 1 else MISS), i
            assert (h["ntested"][i], h["tested_fnv"][i]) == (len(q["tested"]), fnv(q["tested"])), i
            for k in ("tmin", "tmax"):
                assert _bits(h[k][i]) == _bits(q[k]), (i, k)
            if q["status"] == 1:
                assert _bits(h["dist"][i]) == _bits(q["dist"]), i
            # ... and the reference's walk
            same = (h["tri"][i] == (z["tri"][i] if js_hit else MISS) and h["ntested"][i] == z["ntested"][i]
                    and h["tested_fnv"][i] == z["seq_fnv"][i])
        else:
            # any-hit: hit/miss, and the tests up to the first accept
            assert (h["tri"][i] != MISS) == (q["status"] == 1), i
            same = ((h["tri"][i] != MISS) == js_hit and h["ntested"][i] == z["nfirst"][i]
                    and h["tested_fnv"][i] == z["first_fnv"][i])
            if q["status"] == 0:   # a miss tests the whole sequence: the oracle's, bit for bit
                assert (h["ntested"][i], h["tested_fnv"][i]) == (len(q["tested"]), fnv(q["tested"])), i
        if not same:
            js_diff.add(i)
    assert js_diff == set(EXCEPTIONS[name]), sorted(js_diff)
    assert int((h["tri"] != MISS).sum()) > 400


@pytest.mark.parametrize("name", SCENES)
def test_secondary_rays_bvh_walk_matches_oracle(rt, oracle, name):
    meta, z = load_fixture(name)
    ctx, sc = _scene(rt, oracle, name, "BVH")
    try:
        shadow = z["kind"] == 1
        h = ctx.trace_rays("BVH", _rays(z), anyhit=shadow)
        hc = ctx.trace_rays("BVH", _rays(z))   # every ray closest-hit
    finally:
        ctx.close()
    for i in range(z["status"].shape[0]):
        q = oracle.trace_query(sc, "BVH", z["ray_o"][i], z["ray_d"][i], float(z["ray_tmin"][i]),
                               float(z["ray_tmax"][i]))
        tri = q["tri"] if q["status"] == 1 else MISS
        assert hc["tri"][i] == tri, i
        assert (hc["ntested"][i], hc["tested_fnv"][i]) == (len(q["tested"]), fnv(q["tested"])), i
        if q["status"] == 1:
            assert _bits(hc["dist"][i]) == _bits(q["dist"]), i
        # the any-hit walk: same boolean, a prefix of the closest-hit's tests
        assert (h["tri"][i] != MISS) == (tri != MISS), i
        k = int(h["ntested"][i])
        assert k <= len(q["tested"]) and h["tested_fnv"][i] == fnv(q["tested"][:k]), i
        if shadow[i] and tri != MISS:
            assert h["tri"][i] == q["tested"][k - 1]   # it stopped at its first accept


@pytest.mark.parametrize("name", SCENES)
def test_secondary_rays_culled_walk_same_hits(rt, oracle, name):
    # with subtree culling (RT_OPT_BSP_CULL 1, the default) the walk skips subtrees
    # whose content box the ray interval misses: fewer triangles are tested (a
    # subsequence of the reference's), and every ray's hit -- triangle, distance,
    # barycentrics, the any-hit boolean -- is the same bit for bit
    meta, z = load_fixture(name)
    ctx, sc = _scene(rt, oracle, name, "BSP")
    try:
        shadow = z["kind"] == 1
        h0 = ctx.trace_rays("BSP", _rays(z), anyhit=shadow)
        ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, 1)
        h1 = ctx.trace_rays("BSP", _rays(z), anyhit=shadow)
    finally:
        ctx.close()
    for k in ("tri", "dist", "beta", "gamma"):
        assert np.array_equal(h0[k].view(np.uint32), h1[k].view(np.uint32)), k
    assert np.all(h1["ntested"] <= h0["ntested"])
    assert h1["ntested"].sum() < h0["ntested"].sum()


def test_trace_rays_edge_cases(rt, oracle):
    # no rays; a zero-length interval; a ray that starts past its tmax
    m = oracle.load_obj(model("CornellBox.obj"))
    ctx = rt.Context(0)
    ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, 0)   # the tested sequences are compared
    try:
        ctx.upload_mesh_arrays(m.pos, m.nrm, m.idx, m.mats, m.lights)
        b = oracle.build_bsp(m, 20, 4)
        ctx.upload_bsp_arrays(b.aabb, b.tree, b.planes, b.ids, b.max_depth)
        assert ctx.trace_rays("BSP", np.zeros((0, 8), np.float32)).shape == (0,)
        r = np.array([[277, 275, -570, 0, 0, 1, 1.0, 1.0], [277, 275, -570, 0, 0, 1, 10.0, 5.0],
                      [277, 275, -570, 0, 0, 1, 1e-4, 1e4]], np.float32)
        h = ctx.trace_rays("BSP", r)
        sc = oracle.SceneRef(m, b)
        for i in range(3):
            q = oracle.trace_query(sc, "BSP", r[i, :3], r[i, 3:6], float(r[i, 6]), float(r[i, 7]))
            assert h["tri"][i] == (q["tri"] if q["status"] == 1 else MISS)
            assert (h["ntested"][i], h["tested_fnv"][i]) == (len(q["tested"]), fnv(q["tested"]))
        assert h["tri"][2] != MISS
        with pytest.raises(rt.RtError):
            ctx.trace_rays("BVH", r)   # no BVH uploaded
    finally:
        ctx.close()
