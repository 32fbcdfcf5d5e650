"""The trace stage of a wavefront renderer (rt_trace_batch, k_trace: a
traversal-only persistent kernel) and the counting renders' ray capture
(rt_set_ray_capture), DESIGN.md section 4 "Outside the megakernel".

* Random closest-hit and any-hit rays through the BSP: every ray's result equals
  the query kernel's walk (rt_trace_rays, one walk per lane, pinned to the
  oracle and to the reference's JS walk elsewhere) -- hit or miss, triangle, the
  distance bits -- in every culling mode, including rays with zero and tiny
  direction components.
* A counting render of the config-2 Cornell box captures exactly the rays it
  counts (camera + shadow + bounce), camera rays first in each path; the batch
  trace of the captured stream equals rt_trace_rays on it, and its camera rays
  hit the primary ids the render wrote."""
import numpy as np
import pytest

from conftest import model
from parity_util import Scene

pytestmark = pytest.mark.gpu


def _rays(rng, n, lo, hi):
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    # axis-parallel and tiny components (the cull's zero-component slab, bsp_inv1's flags)
    d[: n // 16, 0] = 0.0
    d[n // 16: n // 8, 1] = np.float32(3e-9)
    d[n // 8: n // 8 + n // 32] = np.array([0.0, 1.0, 0.0], np.float32)
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = o
    r[:, 3:6] = d
    r[:, 6] = 1e-4
    r[:, 7] = np.where(rng.random(n) < 0.5, 5000.0, 999999.0 - 1e-4)
    return r


def _batch(ctx, rays, anyhit):
    n = rays.shape[0]
    rb, fb, hb = ctx.alloc(rays.nbytes), ctx.alloc(4 * n), ctx.alloc(8 * n)
    try:
        rb.from_numpy(np.ascontiguousarray(rays))
        fb.from_numpy(np.ascontiguousarray(anyhit.astype(np.uint32)))
        ctx.trace_batch("BSP", rb.ptr, fb.ptr, n, hb.ptr)
        return hb.to_numpy(np.uint32, (n, 2))
    finally:
        for b in (rb, fb, hb):
            b.free()


def _check(ctx, rays, anyhit):
    import importlib
    rt_ffi = importlib.import_module("02562_raytracer_amd._ffi")
    q = ctx.trace_rays("BSP", rays, anyhit)
    h = _batch(ctx, rays, anyhit)
    tree, _, ids, _ = ctx.download_bsp()
    rec_off = ((tree.shape[0] + 1) * rt_ffi.BSP_TREELET_BYTES + 255) & ~255   # (rt_upload_bsp)
    found = h[:, 0] != 0xFFFFFFFF
    assert np.array_equal(found, q["tri"] != 0xFFFFFFFF)
    assert np.array_equal(h[found & anyhit, 0], np.full(int((found & anyhit).sum()), 0xFFFFFFFE, np.uint32))
    ch = found & ~anyhit
    tri = ids[(h[ch, 0] - rec_off) // 48]
    assert np.array_equal(tri, q["tri"][ch])
    assert np.array_equal(h[found, 1], q["dist"][found].view(np.uint32))
    return found.mean()


@pytest.mark.parametrize("cull", [1, 2, 0, 3])
def test_batch_trace_equals_query_walk(rt, gpu, cull):
    s = Scene(rt, rt.Mesh.from_obj(model("teapot.obj")), "BSP")
    s.ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, cull)
    rng = np.random.default_rng(5 + cull)
    rays = _rays(rng, 60000, -3.0, 3.0)
    anyhit = rng.random(rays.shape[0]) < 0.4
    frac = _check(s.ctx, rays, anyhit)
    assert 0.05 < frac < 0.95   # both hits and misses
    s.ctx.close()


def test_capture_stream_equals_render_rays(rt, gpu):
    s = Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), "BSP")
    ctx = s.ctx
    W, H, spp = 64, 48, 4
    cam = ((277.0, 275.0, -570.0), (277.0, 275.0, 0.0), (0.0, 1.0, 0.0), 1.0)
    ctx.set_uniforms(rt.make_uniform(*cam, W, H))
    cap = 200000
    rb, fb = ctx.alloc(32 * cap), ctx.alloc(4 * cap)
    acc, ids = ctx.alloc(W * H * 16), ctx.alloc(W * H * 4)
    try:
        acc.zero()
        ctx.set_ray_capture(rb.ptr, fb.ptr, cap)
        ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 1)
        c = ctx.render("W7E3", "BSP", (0, 0, W, H), 0, spp, acc.ptr, ids.ptr, counts=True)
        ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 0)
        n = ctx.ray_capture_count()
        ctx.set_ray_capture(None)
        assert n == c["primary"] + c["shadow"] + c["bounce"] and n <= cap
        rays = rb.to_numpy(np.float32, (cap, 8))[:n]
        flags = fb.to_numpy(np.uint32, (cap,))[:n]
        prim_ids = ids.to_numpy(np.uint32, (H, W))
    finally:
        for b in (rb, fb, acc, ids):
            b.free()
    anyhit = (flags & 1).astype(bool)
    assert int(anyhit.sum()) == c["shadow"]
    eye = np.asarray(cam[0], np.float32)
    camera = (rays[:, :3] == eye).all(axis=1) & ~anyhit
    assert int(camera.sum()) == c["primary"]
    _check(ctx, rays, anyhit)
    # the camera rays hit what the render's primary ids say (the last iteration's
    # id per pixel is among the camera rays' hits)
    q = ctx.trace_rays("BSP", rays[camera], None)
    assert set(np.unique(prim_ids)) <= set(np.unique(q["tri"]))
    ctx.close()


def test_batch_rejects_2_pow_31_rays(rt, gpu):
    # k_trace's 2^28-capped shard heads would hand out the same block
    # forever past 2^31 rays; the ABI refuses such a batch before any launch
    with pytest.raises(rt._ffi.RtError) as e:
        gpu.trace_batch("BSP", 256, 256, 1 << 31, 256)   # (the pointers are never read)
    assert e.value.code == rt._ffi.RT_E_INVALID
