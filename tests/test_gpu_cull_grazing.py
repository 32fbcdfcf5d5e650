"""Subtree culling against the rays where the f32 triangle test is least
accurate (DESIGN.md section 4 "Certified culling"): rays that meet a triangle
of the scene at a grazing angle, 10^-7.5 .. 10^-3 rad from its plane.  There
intersect_triangle's hit point o + dist*w can sit far off the triangle -- the
reference's |denom| < 1e-10 reject (w7e3.wgsl:306-309) still accepts rays
within 1e-6 rad of a large triangle's plane -- and a margin that is not a
proven bound can cull a subtree the reference's walk would accept a hit in.
Each ray is aimed at a random point of a random triangle of the scene, from a
random distance (0.01 .. 1), so it grazes that triangle and crosses the cells
around it; 30 % are any-hit walks (shadow rays).  Scenes: the config-5 style
random soup (1M large, randomly oriented triangles) and the bunny stand-in.

  * the certified walk (RT_BSP_CULL_CERTIFIED), and the silhouette bound
    (RT_BSP_CULL_SILHOUETTE, round 5) -- the two kernels the default RT_BSP_CULL_AUTO
    chooses between -- equal the CPU oracle's walk
    (bsp.wgsl:10-81, every node visited) ray for ray: triangle and distance
    bit for bit, hit or miss for the any-hit rays -- 0 differences -- and the
    unculled GPU walk in every field (triangle, distance, barycentrics);
  * the fast margin (RT_BSP_CULL_FAST) is measured, not asserted exact: where
    it differs, one of the two walks accepted a hit whose computed point lies
    outside the accepted triangle's box grown by the fast margin -- the f32
    test placing its hit off the triangle (round 3: 2 of 400,000 soup rays,
    at 1.2e-6 and 1.8e-6 rad, 4-5e-3 outside the box against a 1e-3 margin)."""
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _grazing_rays(V, I, n, seed):
    rng = np.random.default_rng(seed)
    P = V[:, :3].astype(np.float64)
    t = rng.integers(I.shape[0], size=n)
    v0, v1, v2 = P[I[t, 0]], P[I[t, 1]], P[I[t, 2]]
    u, v = rng.random(n), rng.random(n)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    p = v0 + u[:, None] * (v1 - v0) + v[:, None] * (v2 - v0)
    nn = np.cross(v1 - v0, v2 - v0)
    ln = np.linalg.norm(nn, axis=1)
    ok = ln > 0
    nn[ok] /= ln[ok, None]
    a = rng.normal(size=(n, 3))
    a -= nn * np.sum(a * nn, axis=1)[:, None]
    a /= np.linalg.norm(a, axis=1)[:, None]
    el = 10.0 ** rng.uniform(-7.5, -3, n) * rng.choice([-1.0, 1.0], n)
    w = a * np.cos(el)[:, None] + nn * np.sin(el)[:, None]
    w /= np.linalg.norm(w, axis=1)[:, None]
    s = 10.0 ** rng.uniform(-2, 0, n)
    o = p - s[:, None] * w
    R = np.concatenate([o, w, np.full((n, 1), 1e-4), np.full((n, 1), 5000.0)], axis=1).astype(np.float32)
    return R[ok], (rng.random(n) < 0.3)[ok]


@pytest.mark.parametrize("scene", ["soup", "bunny"])
def test_grazing_rays_default_walk_equals_oracle(rt, gpu, oracle, scene):
    mesh = rt.Mesh.synth_soup(1_000_000) if scene == "soup" else rt.Mesh.synth_bunny()
    V, N, I, M, L = mesh.arrays()
    R, anyhit = _grazing_rays(V, I, 400_000, 17)
    ctx = rt.Context(0)
    bsp = mesh.bsp_tree()
    try:
        ctx.upload_mesh(mesh)
        ctx.upload_bsp(bsp)
        h = {}
        for name in ("OFF", "FAST", "SILHOUETTE", "CERTIFIED"):   # CERTIFIED last: the context's default again
            ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, getattr(rt._ffi, "RT_BSP_CULL_" + name))
            h[name] = ctx.trace_rays("BSP", R, anyhit)
    finally:
        ctx.close()
    MISS = 0xFFFFFFFF
    hits = int((h["OFF"]["tri"] != MISS).sum())
    assert hits > len(R) // 4

    # the oracle's walk (every node visited), closest hit per ray
    tree, planes, ids, aabb, D = bsp.arrays()
    om = types.SimpleNamespace(pos=np.ascontiguousarray(V), nrm=np.ascontiguousarray(N), idx=np.ascontiguousarray(I),
                               ntris=I.shape[0], mats=np.ascontiguousarray(M), lights=np.ascontiguousarray(L))
    sc = oracle.SceneRef(om, types.SimpleNamespace(aabb=aabb, tree=tree, planes=planes, ids=ids, max_depth=D))
    otri, odist = oracle.trace_many(sc, "BSP", R)
    cert = h["CERTIFIED"]
    closest = ~anyhit
    bad = closest & ((cert["tri"] != otri) | ((otri != MISS) & (cert["dist"].view(np.uint32) != odist.view(np.uint32))))
    bad |= anyhit & ((cert["tri"] != MISS) != (otri != MISS))
    print(f"{scene}: {len(R)} grazing rays, {hits} hits; certified walk vs oracle: {int(bad.sum())} differ")
    assert bad.sum() == 0, f"{int(bad.sum())} of {len(R)} grazing rays differ from the oracle's walk"
    for k in ("tri", "dist", "beta", "gamma"):
        assert np.array_equal(h["OFF"][k].view(np.uint32), cert[k].view(np.uint32)), k
        # RT_BSP_CULL_SILHOUETTE: exact as well (its camera bound does not apply:
        # these rays do not start at an eye)
        assert np.array_equal(h["OFF"][k].view(np.uint32), h["SILHOUETTE"][k].view(np.uint32)), k

    # the fast margin: measured; each difference is an off-triangle f32 accept
    fast = h["FAST"]
    badf = np.zeros(len(R), bool)
    for k in ("tri", "dist", "beta", "gamma"):
        badf |= h["OFF"][k].view(np.uint32) != fast[k].view(np.uint32)
    print(f"{scene}: fast margin: {int(badf.sum())} of {len(R)} differ from the unculled walk")
    assert badf.sum() <= len(R) // 20000, f"{int(badf.sum())} of {len(R)} grazing rays differ with the fast margin"
    scale = max(abs(float(x)) for x in list(aabb[:3]) + list(aabb[4:7]) if np.isfinite(x))
    P = V[:, :3].astype(np.float64)
    for i in np.nonzero(badf)[0]:
        o, w = R[i, :3].astype(np.float64), R[i, 3:6].astype(np.float64)
        m = max(float(np.abs(R[i, :3]).max()), scale) * 2.0 ** -10
        off = []
        for hh in (h["OFF"], fast):
            if hh["tri"][i] == MISS:
                continue
            v = P[I[hh["tri"][i], :3]]
            p = o + w * float(hh["dist"][i])
            off.append(float(np.max(np.maximum(v.min(0) - p, p - v.max(0)))))
        print(f"  ray {i}: hits {h['OFF']['tri'][i]} / {fast['tri'][i]}, off-box {off}, margin {m:.3g}")
        assert off and max(off) > m, (i, off, m)


@pytest.mark.parametrize("scene", ["soup", "bunny"])
def test_camera_rays_default_walk_equals_oracle(rt, gpu, oracle, scene):
    # rays from the camera eye, which take the camera bound of the certified margin
    # (the treelets' per-eye terms): aimed at points of the triangles whose planes
    # pass closest to the eye -- the silhouette, where camera rays graze -- and at
    # random points of the frame; every ray starts exactly at the eye
    mesh = rt.Mesh.synth_soup(1_000_000) if scene == "soup" else rt.Mesh.synth_bunny()
    V, N, I, M, L = mesh.arrays()
    eye = np.array([0.0, 0.0, 3.0] if scene == "soup" else [-0.02, 0.11, 0.6], np.float32)
    P = V[:, :3].astype(np.float64)
    v0, v1, v2 = P[I[:, 0]], P[I[:, 1]], P[I[:, 2]]
    n = np.cross(v1 - v0, v2 - v0)
    ln = np.linalg.norm(n, axis=1)
    ok = ln > 0
    h = np.full(len(I), np.inf)
    h[ok] = np.abs(np.sum((v0[ok] - eye) * n[ok], axis=1)) / ln[ok]
    edge_on = np.argsort(h)[:200_000]
    rng = np.random.default_rng(23)
    t = np.concatenate([edge_on, rng.integers(len(I), size=100_000)])
    u, v = rng.random(len(t)), rng.random(len(t))
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    # points on the triangle, and just beside it in its plane (misses that graze it)
    s = np.where(rng.random(len(t)) < 0.5, 1.0, 1.0 + 10.0 ** rng.uniform(-4, -1, len(t)))
    p = v0[t] + (u * s)[:, None] * (v1[t] - v0[t]) + (v * s)[:, None] * (v2[t] - v0[t])
    w = p - eye
    w /= np.linalg.norm(w, axis=1)[:, None]
    R = np.concatenate([np.tile(eye, (len(t), 1)), w, np.full((len(t), 1), 1e-4), np.full((len(t), 1), 5000.0)],
                       axis=1).astype(np.float32)
    R[:, :3] = eye   # exactly the eye
    anyhit = np.zeros(len(R), bool)
    ctx = rt.Context(0)
    bsp = mesh.bsp_tree()
    try:
        ctx.upload_mesh(mesh)
        ctx.upload_bsp(bsp)
        ctx.set_uniforms(rt.make_uniform(tuple(float(x) for x in eye), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.5, 64, 64))
        h_ = {}
        for name in ("OFF", "FAST", "SILHOUETTE", "CERTIFIED"):
            ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, getattr(rt._ffi, "RT_BSP_CULL_" + name))
            ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 0)
            h_[name] = ctx.trace_rays("BSP", R, anyhit)
            if name == "SILHOUETTE":   # the mode's node data, for this eye
                _, sil = ctx.download_bsp_treelets(silhouette=True)
                assert (sil[1:, 3] != 0).any()
    finally:
        ctx.close()
    MISS = 0xFFFFFFFF
    tree, planes, ids, aabb, D = bsp.arrays()
    om = types.SimpleNamespace(pos=np.ascontiguousarray(V), nrm=np.ascontiguousarray(N), idx=np.ascontiguousarray(I),
                               ntris=I.shape[0], mats=np.ascontiguousarray(M), lights=np.ascontiguousarray(L))
    sc = oracle.SceneRef(om, types.SimpleNamespace(aabb=aabb, tree=tree, planes=planes, ids=ids, max_depth=D))
    otri, odist = oracle.trace_many(sc, "BSP", R)
    cert = h_["CERTIFIED"]
    bad = (cert["tri"] != otri) | ((otri != MISS) & (cert["dist"].view(np.uint32) != odist.view(np.uint32)))
    hits = int((otri != MISS).sum())
    badf = np.zeros(len(R), bool)
    for k in ("tri", "dist", "beta", "gamma"):
        badf |= h_["OFF"][k].view(np.uint32) != h_["FAST"][k].view(np.uint32)
    print(f"{scene}: {len(R)} camera rays ({hits} hits): certified vs oracle {int(bad.sum())} differ, "
          f"fast vs unculled {int(badf.sum())} differ")
    sil_ = h_["SILHOUETTE"]
    bads = (sil_["tri"] != otri) | ((otri != MISS) & (sil_["dist"].view(np.uint32) != odist.view(np.uint32)))
    print(f"{scene}: silhouette-bound walk vs oracle {int(bads.sum())} differ")
    assert hits > len(R) // 4
    assert bad.sum() == 0 and bads.sum() == 0
    for k in ("tri", "dist", "beta", "gamma"):
        assert np.array_equal(h_["OFF"][k].view(np.uint32), cert[k].view(np.uint32)), k
        assert np.array_equal(h_["OFF"][k].view(np.uint32), sil_[k].view(np.uint32)), k
