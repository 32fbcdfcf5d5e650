"""Subtree culling of the BSP walk (RT_OPT_BSP_CULL, rt_kernels.hip bsp_box_miss;
DESIGN.md section 4 "Subtree culling") changes only the work, never the result:
frames rendered with certified culling (exact by proof), with the
silhouette bound and the timed choice between the two (RT_BSP_CULL_SILHOUETTE,
RT_BSP_CULL_AUTO), with the fast margin (RT_BSP_CULL_FAST) and with culling off (every node of
bsp.wgsl:10-81 visited) are equal bit for bit -- radiance, primary-hit ids and
the ray counts --
across the shaders and walks that use the BSP: the path tracers (W7E3, W9E1 with
its plane-free scenes, W8's analytic balls, W9E2/W9E3's holdout plane, whose
secondary rays start anywhere on the plane y = 0), the primary-ray kernel with the
root-AABB clip (W6E1/PROJECT) and the direct-lighting kernels (W6E2, W7E1),
including grazing and axis-aligned rays.  Every other GPU parity test runs with
culling on and compares with the CPU oracle (which walks every node)."""
import numpy as np
import pytest

from conftest import model
from parity_util import BUNNY_CAM, CORNELL_CAM, TEAPOT_CAM, Scene

pytestmark = pytest.mark.gpu


CULL_MODES = (0, 1, 2, 3, 4)   # RT_BSP_CULL_OFF, _CERTIFIED (default), _FAST, _SILHOUETTE, _AUTO


def _frames(rt, s, mode, cam, W, H, region, spp, selection1=0, jitter=None):
    out = []
    for cull in CULL_MODES:
        s.ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, cull)
        s.ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 1)
        out.append(s.render_gpu(mode, cam, W, H, region, 0, spp, selection1=selection1, jitter=jitter))
    s.ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, rt._ffi.RT_BSP_CULL_CERTIFIED)
    s.ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 0)
    for f, name in zip(out[1:], ("certified", "fast", "silhouette", "auto")):
        print(f"{mode}: {name} culls {f[2]['subtree_culls']}, interior nodes "
              f"{f[2]['node_interior'] / max(1, out[0][2]['node_interior']):.3f} of the unculled walk")
    return out


def _same(a, b, culled=True):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), "radiance differs"
    assert np.array_equal(a[1], b[1]), "primary-hit ids differ"
    for k in ("samples", "primary", "shadow", "bounce"):
        assert a[2][k] == b[2][k], k
    assert a[2]["subtree_culls"] == 0
    if culled:
        assert b[2]["subtree_culls"] > 0


def _all_same(frames, culled=True):
    off, *ons = frames   # certified, fast, silhouette, auto
    for on in ons:
        _same(off, on, culled)


def test_cornell_w7e3_full_frame(rt):
    # the whole config-2 frame (1024 x 1024) at 8 spp: flat, coplanar walls and
    # the area-light shadow rays that graze the ceiling the light sits in
    s = Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), "BSP")
    off, on, fast, sil, auto = _frames(rt, s, "W7E3", CORNELL_CAM, 1024, 1024, (0, 0, 1024, 1024), 8)
    _all_same((off, on, fast, sil, auto))
    assert on[2]["tri_tests"] <= off[2]["tri_tests"]
    s.ctx.close()


def test_bunny_w9e1_frame(rt):
    s = Scene(rt, rt.Mesh.synth_bunny(), "BSP", env=(0.8, 0.9, 1.0))
    off, on, fast, sil, auto = _frames(rt, s, "W9E1", BUNNY_CAM, 1920, 1080, (0, 0, 1920, 1080), 2)
    _all_same((off, on, fast, sil, auto))
    # the point of it: far fewer nodes and triangles
    assert on[2]["node_interior"] < 0.75 * off[2]["node_interior"]
    assert fast[2]["node_interior"] < 0.6 * off[2]["node_interior"]
    assert sil[2]["node_interior"] <= 1.01 * on[2]["node_interior"]   # (a tighter camera bound)
    s.ctx.close()


@pytest.mark.parametrize("mode", ["W8E1", "W8E2", "W8E3"])
def test_w8_balls(rt, mode):
    s = Scene(rt, rt.Mesh.from_obj(model("CornellBox.obj")), "BSP")
    _all_same(_frames(rt, s, mode, CORNELL_CAM, 256, 256, (0, 0, 256, 256), 4))
    s.ctx.close()


@pytest.mark.parametrize("mode,sel", [("W9E2", 0), ("W9E2", 2), ("W9E3", 0), ("W9E3", 3)])
def test_w9_holdout_plane(rt, mode, sel):
    # occlusion / sun rays from points anywhere on the plane y = 0, far outside the mesh's box
    s = Scene(rt, rt.Mesh.from_obj(model("teapot.obj")), "BSP")
    _all_same(_frames(rt, s, mode, TEAPOT_CAM, 400, 225, (0, 0, 400, 225), 4, selection1=sel))
    s.ctx.close()


@pytest.mark.parametrize("mode", ["W6E1", "PROJECT", "W6E2", "W7E1"])
def test_primary_and_direct_kernels(rt, mode):
    s = Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), "BSP")
    _all_same(_frames(rt, s, mode, CORNELL_CAM, 200, 200, (0, 0, 200, 200), 2), culled=False)
    s.ctx.close()


def test_grazing_and_axis_aligned_rays(rt, oracle):
    # rays that start on a triangle and leave it almost in its plane (elevation
    # 1e-7 .. 1e-2 rad) and rays with zero direction components: the same hits
    # with and without culling, and both equal to the CPU oracle's walk
    m = oracle.load_obj(model("CornellBoxWithBlocks.obj"))
    b = oracle.build_bsp(m, 20, 4)
    rng = np.random.default_rng(11)
    P = m.pos[:, :3].astype(np.float64)
    rays = []
    for _ in range(20000):
        t = int(rng.integers(m.idx.shape[0]))
        v0, v1, v2 = (P[m.idx[t, k]] for k in range(3))
        u, v = rng.random(), rng.random()
        if u + v > 1:
            u, v = 1 - u, 1 - v
        o = v0 + u * (v1 - v0) + v * (v2 - v0)
        n = np.cross(v1 - v0, v2 - v0)
        n /= np.linalg.norm(n)
        a = rng.normal(size=3)
        a -= n * np.dot(a, n)
        a /= np.linalg.norm(a)
        el = 10.0 ** rng.uniform(-7, -2) * rng.choice([-1, 1])
        rays.append([*o, *(a * np.cos(el) + n * np.sin(el)), 0.01, 5000.0])
    for _ in range(2000):
        o = rng.uniform(P.min(0), P.max(0))
        d = np.zeros(3)
        d[rng.integers(3)] = rng.choice([-1.0, 1.0])
        rays.append([*o, *d, 0.01, 5000.0])
    R = np.asarray(rays, np.float32)
    anyhit = rng.random(len(R)) < 0.5
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh_arrays(m.pos, m.nrm, m.idx, m.mats, m.lights)
        ctx.upload_bsp_arrays(b.aabb, b.tree, b.planes, b.ids, b.max_depth)
        hs = []
        for cull in CULL_MODES:
            ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, cull)
            hs.append(ctx.trace_rays("BSP", R, anyhit))
    finally:
        ctx.close()
    h0, h1 = hs[0], hs[1]
    for h in hs[1:]:
        for k in ("tri", "dist", "beta", "gamma"):
            assert np.array_equal(h0[k].view(np.uint32), h[k].view(np.uint32)), k
    sc = oracle.SceneRef(m, b)
    MISS = 0xFFFFFFFF
    for i in range(0, len(R), 7):   # a sample against the oracle
        if anyhit[i]:
            continue
        q = oracle.trace_query(sc, "BSP", R[i, :3], R[i, 3:6], float(R[i, 6]), float(R[i, 7]))
        assert h1["tri"][i] == (q["tri"] if q["status"] == 1 else MISS), i
