"""The data the certified culling's proof rests on (DESIGN.md section 4
"Certified culling"), as the GPU repack wrote it into the BSP treelets
(rt_bsp_build.hip k_leaf_boxes / k_node_boxes / k_bsp_repack / k_treelet_hcam),
checked node by node against an f64 recomputation on the host from the mesh and
the reference-layout tree (rt_download_bsp):

  * the content box holds every vertex of the subtree's triangles;
  * F (bf16) <= 1e-10 / E2, E2 the subtree's largest squared edge (inf-norm of
    the records' f32 edges) -- the shader's |denom| >= 1e-10 floor, normalised;
  * the normal box [c - r, c + r] (f16) holds n* / E2s for every triangle, n* =
    e0 x e1 exactly and E2s = E2 rounded up to f32 (the repack's divisor);
  * the camera term G (f16) <= (H - 128u D1) / Dinf for the uniforms' eye, H the
    subtree's least |(v0 - eye) . n*| / E_T^2 and D1, Dinf the L1 / L-inf
    distances of the stored box from the eye;
  * (round 5, RT_BSP_CULL_SILHOUETTE's node data) the two triangles of least H
    are stored as their normals n*/E_t^2 (f16, nearest) and the rest's term
    G_x <= (H3 - 128u D1) / Dinf, H3 the
    third least H of distinct triangles -- recomputed here with the GPU's own
    order (stable in H, leaves in treeIds order, a subtree's left child first),
    so the stored normals must be exactly those triangles'.

Rounding the wrong way anywhere in those kernels would break the proof without
necessarily changing a test frame; this pins each inequality."""
import numpy as np
import pytest

from conftest import model

pytestmark = pytest.mark.gpu

U = 2.0 ** -24


def _f16(bits):
    return np.asarray(bits, np.uint16).view(np.float16).astype(np.float64)


def _f32_up(x):
    """smallest f32 >= x (x >= 0, f64)"""
    f = x.astype(np.float32)
    lo = f.astype(np.float64) < x
    f[lo] = np.nextafter(f[lo], np.float32(np.inf))
    return f.astype(np.float64)


def _check(rt, mesh, eye, target):
    V, N, I, M, L = mesh.arrays()
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh(mesh)
        ctx.upload_bsp(mesh.bsp_tree())
        ctx.set_uniforms(rt.make_uniform(tuple(float(x) for x in eye), target, (0.0, 1.0, 0.0), 1.5, 64, 64))
        tl, sil = ctx.download_bsp_treelets(silhouette=True)
        tree, planes, ids, aabb = ctx.download_bsp()
    finally:
        ctx.close()
    n = tree.shape[0]
    assert tl.shape == (n + 1, 24) and sil.shape == (n + 1, 4)

    # per triangle, from the records' f32 edges (k_tri_records2)
    P = V[:, :3].astype(np.float32)
    v0, v1, v2 = P[I[:, 0]], P[I[:, 1]], P[I[:, 2]]
    e0 = (v1 - v0).astype(np.float64)
    e1 = (v2 - v0).astype(np.float64)
    ns = np.cross(e0, e1)   # exact: products of f32 values, differences well inside f64
    E = np.maximum(np.abs(e0).max(1), np.abs(e1).max(1))
    E2 = E * E
    d = v0.astype(np.float64) - eye.astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        H = np.where(E2 > 0, np.abs((d * ns).sum(1)) / E2, np.inf)
    vlo = np.minimum(np.minimum(v0, v1), v2).astype(np.float64)
    vhi = np.maximum(np.maximum(v0, v1), v2).astype(np.float64)

    # subtree aggregates, bottom-up over the heap (node i: children 2i+1, 2i+2),
    # leaves first (their id ranges tile ids in order)
    leaf = (tree[:, 0] & 3) == 3
    cnt = (tree[:, 0] >> 2).astype(np.int64)
    first = tree[:, 1].astype(np.int64)
    lv = np.nonzero(leaf & (cnt > 0))[0]
    order = np.argsort(first[lv], kind="stable")
    starts = first[lv][order]
    assert starts[0] == 0 and np.all(np.diff(np.append(starts, len(ids))) == cnt[lv][order])

    def per_leaf(vals, red, fill):
        out = np.full((n,) + vals.shape[1:], fill)
        res = np.empty((len(lv),) + vals.shape[1:])
        res[order] = red.reduceat(vals[ids.astype(np.int64)], starts, axis=0)
        out[lv] = res
        return out

    def up(arr, red):
        dmax = int(np.floor(np.log2(n + 1)))
        for dd in range(dmax, -1, -1):
            i = np.arange(2 ** dd - 1, min(2 ** (dd + 1) - 1, n))
            i = i[(~leaf[i]) & (2 * i + 2 < n)]
            arr[i] = red(arr[2 * i + 1], arr[2 * i + 2])
        return arr

    agg_E2 = up(per_leaf(E2, np.maximum, 0.0), np.maximum)
    agg_H = up(per_leaf(H, np.minimum, np.inf), np.minimum)
    agg_lo = up(per_leaf(vlo, np.minimum, np.inf), np.minimum)
    agg_hi = up(per_leaf(vhi, np.maximum, -np.inf), np.maximum)
    agg_nlo = up(per_leaf(ns, np.minimum, np.inf), np.minimum)
    agg_nhi = up(per_leaf(ns, np.maximum, -np.inf), np.maximum)

    # reachable nodes (children of interior nodes), 1-based treelet row M = i + 1
    reach = np.zeros(n, bool)
    reach[0] = True
    dmax = int(np.floor(np.log2(n + 1)))
    for dd in range(dmax + 1):
        i = np.arange(2 ** dd - 1, min(2 ** (dd + 1) - 1, n))
        i = i[reach[i] & ~leaf[i] & (2 * i + 2 < n)]
        reach[2 * i + 1] = reach[2 * i + 2] = True
    idx = np.nonzero(reach)[0]
    rows = tl[idx + 1]
    box = rows[:, :6].view(np.float32).astype(np.float64)
    F = ((rows[:, 20] & 0xFFFF) << 16).view(np.float32).astype(np.float64)
    G = _f16((rows[:, 20] >> 16).astype(np.uint16))
    c = np.stack([_f16(rows[:, 21] & 0xFFFF), _f16(rows[:, 21] >> 16), _f16(rows[:, 22] & 0xFFFF)], 1)
    r = np.stack([_f16(rows[:, 22] >> 16), _f16(rows[:, 23] & 0xFFFF), _f16(rows[:, 23] >> 16)], 1)

    has = np.isfinite(agg_lo[idx]).all(1)   # subtrees with triangles
    assert has.sum() > len(idx) // 4
    # content box
    assert (box[has, :3] <= agg_lo[idx][has]).all() and (box[has, 3:] >= agg_hi[idx][has]).all()
    ext = agg_E2[idx] > 0
    # floor
    assert (F[ext] <= 1e-10 / agg_E2[idx][ext]).all()
    assert np.isinf(F[~ext]).all()
    # normal box
    E2s = _f32_up(agg_E2[idx][ext])
    lo_n = agg_nlo[idx][ext] / E2s[:, None]
    hi_n = agg_nhi[idx][ext] / E2s[:, None]
    assert (c[ext] - r[ext] <= lo_n).all(), "normal box misses a normal (low side)"
    assert (c[ext] + r[ext] >= hi_n).all(), "normal box misses a normal (high side)"
    # camera term
    dl = np.abs(box[:, :3] - eye.astype(np.float64))
    dh = np.abs(box[:, 3:] - eye.astype(np.float64))
    dd = np.maximum(dl, dh)
    D1, Dinf = dd.sum(1), dd.max(1)
    fin = np.isfinite(agg_H[idx]) & has
    with np.errstate(divide="ignore", invalid="ignore"):
        Gt = np.where(Dinf > 0, (agg_H[idx] - 128 * U * D1) / Dinf, 0.0)
    Gt = np.maximum(Gt, 0.0)
    assert (G[fin] <= Gt[fin]).all(), "camera term above its bound"
    assert (G[fin] >= 0).all()
    # the excluded pair and G_x (k_leaf_hcam / k_node_hcam / k_treelet_hcam), in the
    # GPU's own f32 values of H (tri_hcam: |dot| less its error bound, rounded down)
    dot = d[:, 0] * ns[:, 0] + d[:, 1] * ns[:, 1] + d[:, 2] * ns[:, 2]
    err = 2.0 ** -45 * (np.abs(d[:, 0] * ns[:, 0]) + np.abs(d[:, 1] * ns[:, 1]) + np.abs(d[:, 2] * ns[:, 2]))
    with np.errstate(divide="ignore", invalid="ignore"):
        hx = np.where(np.abs(dot) - err > 0, (np.abs(dot) - err) / E2 * (1.0 - 2.0 ** -19), 0.0)
    hg = hx.astype(np.float32)
    up_ = hg.astype(np.float64) > hx
    hg[up_] = np.nextafter(hg[up_], np.float32(-np.inf))
    Hg = np.where(E2 > 0, hg.astype(np.float64), np.inf)
    h3, t3 = _top3(tree, ids, Hg, leaf, n)
    with np.errstate(divide="ignore", invalid="ignore"):
        Gx_t = np.where(np.isinf(h3[idx, 2]), np.inf,
                        np.maximum(np.where(Dinf > 0, (h3[idx, 2] - 128 * U * D1) / Dinf, 0.0), 0.0))
        nt = np.where(E2[:, None] > 0, ns / E2[:, None], np.nan).astype(np.float32).astype(np.float16).view(np.uint16)
    srow = sil[idx + 1]
    Gx = _f16((srow[:, 3] & 0xFFFF).astype(np.uint16))
    assert (Gx <= Gx_t).all(), "excluded camera term above its bound"
    xs = np.stack([srow[:, 0] & 0xFFFF, srow[:, 0] >> 16, srow[:, 1] & 0xFFFF,
                   srow[:, 1] >> 16, srow[:, 2] & 0xFFFF, srow[:, 2] >> 16], 1).astype(np.uint16)
    for j in range(2):
        tj = t3[idx, j]
        ok = tj >= 0
        assert np.array_equal(xs[ok, 3 * j:3 * j + 3], nt[tj[ok]]), f"excluded normal {j}"
        assert (xs[~ok, 3 * j:3 * j + 3] == 0x7E00).all()
    bound = int((G[fin] > 0).sum())
    print(f"{len(idx)} reachable treelets ({int(has.sum())} with triangles): content boxes, floors, normal boxes "
          f"and {bound} positive camera terms within their bounds")
    return bound


def _top3(tree, ids, H, leaf, n):
    """Per node the three least H of distinct triangles of its subtree and the
    triangles (-1: none), as k_leaf_hcam / k_node_hcam build them: stable in H
    over the leaf's treeIds order / the left child's list then the right's, a
    repeated triangle kept once, +inf never taken."""
    h3 = np.full((n, 3), np.inf)
    t3 = np.full((n, 3), -1, np.int64)

    def take(hc, tc):
        # rows of candidates in insertion order -> the first three of a stable sort
        o = np.argsort(hc, axis=1, kind="stable")
        hs = np.take_along_axis(hc, o, 1)
        ts = np.take_along_axis(tc, o, 1)
        for j in range(1, ts.shape[1]):   # a triangle seen earlier in the row (same H) is dropped
            dup = (ts[:, j:j + 1] == ts[:, :j]).any(1) & (ts[:, j] >= 0)
            hs[dup, j] = np.inf
            ts[dup, j] = -1
        o = np.argsort(hs, axis=1, kind="stable")
        hs = np.take_along_axis(hs, o, 1)[:, :3]
        ts = np.take_along_axis(ts, o, 1)[:, :3]
        ts[~np.isfinite(hs)] = -1
        return hs, ts

    cnt = (tree[:, 0] >> 2).astype(np.int64)
    first = tree[:, 1].astype(np.int64)
    lvs = np.nonzero(leaf & (cnt > 0))[0]
    w = int(cnt[lvs].max()) if len(lvs) else 1
    hc = np.full((len(lvs), w), np.inf)
    tc = np.full((len(lvs), w), -1, np.int64)
    for k in range(w):
        has = cnt[lvs] > k
        t = ids[(first[lvs] + k)[has]].astype(np.int64)
        hc[has, k] = H[t]
        tc[has, k] = t
    h3[lvs], t3[lvs] = take(hc, tc)
    dmax = int(np.floor(np.log2(n + 1)))
    for dd in range(dmax, -1, -1):
        i = np.arange(2 ** dd - 1, min(2 ** (dd + 1) - 1, n))
        i = i[(~leaf[i]) & (2 * i + 2 < n)]
        if len(i):
            h3[i], t3[i] = take(np.concatenate([h3[2 * i + 1], h3[2 * i + 2]], 1),
                                np.concatenate([t3[2 * i + 1], t3[2 * i + 2]], 1))
    return h3, t3


def test_teapot_treelets(rt):
    mesh = rt.Mesh.from_obj(model("teapot.obj"))
    assert _check(rt, mesh, np.array([0.15, 1.5, 6.0], np.float32), (0.0, 1.0, 0.0)) > 0


def test_bunny_treelets(rt):
    assert _check(rt, rt.Mesh.synth_bunny(), np.array([-0.02, 0.11, 0.6], np.float32), (-0.02, 0.1, 0.0)) > 0


def test_soup_treelets(rt):
    assert _check(rt, rt.Mesh.synth_soup(20_000), np.array([0.0, 0.0, 3.0], np.float32), (0.0, 0.0, 0.0)) > 0
