"""Subtree culling against the rays its exactness argument does not cover
(DESIGN.md section 4 "Subtree culling"): rays that meet a triangle of the scene
at a grazing angle, 10^-7.5 .. 10^-3 rad from its plane, where the f32 triangle
test's hit point can sit off the triangle by more than the culling margin.
Each ray is aimed at a random point of a random triangle of the scene, from a
random distance (0.01 .. 1), so it grazes that triangle and crosses the cells
around it.  Closest-hit and any-hit walks through rt_trace_rays with culling
on and off give the same triangle, distance and barycentrics bit for bit
on the config-5 style random soup (large, randomly oriented triangles: the
reference's |denom| < 1e-10 reject still accepts rays within 1e-6 rad of their
planes) and on the bunny stand-in.

Where the two walks differ, the reason is checked ray by ray: one of the two
accepted a hit whose computed point o + dist*w lies outside the accepted
triangle's bounding box grown by the culling margin -- the f32 triangle test
at a grazing angle placing its hit off the triangle (2 of 400,000 soup rays at
1.2e-6 and 1.8e-6 rad, hit points 4-5e-3 outside the triangle's box against a
1e-3 margin).  Such rays stay bounded in number; every other ray is identical."""
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
def test_grazing_rays_cull_equals_reference_walk(rt, gpu, scene):
    mesh = rt.Mesh.synth_soup(1_000_000) if scene == "soup" else rt.Mesh.synth_bunny()
    V, N, I, M, L = mesh.arrays()
    R, anyhit = _grazing_rays(V, I, 400_000, 17)
    ctx = rt.Context(0)
    try:
        bsp = mesh.bsp_tree()
        ctx.upload_mesh(mesh)
        ctx.upload_bsp(bsp)
        ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, 0)
        h0 = ctx.trace_rays("BSP", R, anyhit)
        ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, 1)
        h1 = ctx.trace_rays("BSP", R, anyhit)
    finally:
        ctx.close()
    bad = np.zeros(len(R), bool)
    for k in ("tri", "dist", "beta", "gamma"):
        bad |= h0[k].view(np.uint32) != h1[k].view(np.uint32)
    hits = int((h0["tri"] != 0xFFFFFFFF).sum())
    print(f"{scene}: {len(R)} grazing rays, {hits} hits, {int(bad.sum())} differ with culling")
    assert hits > len(R) // 4
    assert bad.sum() <= len(R) // 20000, f"{int(bad.sum())} of {len(R)} grazing rays differ with culling"
    # each difference: one walk accepted a hit point off its triangle's box by more than the margin
    aabb = bsp.arrays()[3]
    scale = max(abs(float(x)) for x in list(aabb[:3]) + list(aabb[4:7]) if np.isfinite(x))
    P = V[:, :3].astype(np.float64)
    for i in np.nonzero(bad)[0]:
        o, w = R[i, :3].astype(np.float64), R[i, 3:6].astype(np.float64)
        m = max(float(np.abs(R[i, :3]).max()), scale) * 2.0 ** -10
        off = []
        for h in (h0, h1):
            if h["tri"][i] == 0xFFFFFFFF:
                continue
            v = P[I[h["tri"][i], :3]]
            p = o + w * float(h["dist"][i])
            off.append(float(np.max(np.maximum(v.min(0) - p, p - v.max(0)))))
        print(f"  ray {i}: hits {h0['tri'][i]} / {h1['tri'][i]}, off-box {off}, margin {m:.3g}")
        assert off and max(off) > m, (i, off, m)
