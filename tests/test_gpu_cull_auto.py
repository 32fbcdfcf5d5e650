"""RT_BSP_CULL_AUTO (rt_api.cpp probe_take / probe_launch / probe_finish; DESIGN.md
section 4 "The auto probe"): the W9E1 BSP renders time the certified and the
silhouette kernels on four of their own launches (certified, silhouette,
certified, silhouette; each >= 2^20 samples) and run the faster once the probe's
events have completed -- read at a later render, never waited for.  Both forms
are exact, so an automatic render equals the certified render bit for bit
whichever ran; the choice holds for the scene until the BSP or the option
changes or the eye's reach leaves [1/2, 2] of the probed one; other modes and
walks run the certified kernel without probing."""
import time

import numpy as np
import pytest

from conftest import model
from parity_util import BUNNY_CAM, CORNELL_CAM, Scene

pytestmark = pytest.mark.gpu

REGION = (0, 0, 640, 360)   # 230,400 px: a probe launch takes 5 iterations (>= 2^20 samples)
CAM2 = ((0.25, 0.18, 0.45), (-0.02, 0.09, 0.0), (0.0, 1.0, 0.0), 2.5)
FAR = ((-0.02, 0.11, 3.0), (-0.02, 0.11, 0.0), (0.0, 1.0, 0.0), 3.5)   # reach > 2x the bunny cam's


def _same(a, b):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), "radiance differs"
    assert np.array_equal(a[1], b[1]), "primary-hit ids differ"
    for k in ("samples", "primary", "shadow", "bounce"):
        assert a[2][k] == b[2][k], k


def _render(s, cam, spp=32, first_iter=0, accum_in=None):
    return s.render_gpu("W9E1", cam, 640, 360, REGION, first_iter, spp, accum_in=accum_in)


def test_auto_probes_inside_the_render_and_matches_certified(rt):
    F = rt._ffi
    s = Scene(rt, rt.Mesh.synth_bunny(), "BSP", env=(0.8, 0.9, 1.0))
    ctx = s.ctx
    ref = {}
    for cam in (BUNNY_CAM, CAM2, FAR):
        ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
        ref[cam] = _render(s, cam)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    assert ctx.bsp_cull_in_use() == (F.RT_BSP_CULL_CERTIFIED, 0.0, 0.0)   # not probed yet: the certified kernel
    assert ctx.bsp_cull_probes() == (0, 0)
    # a counting render (RT_OPT_DETAIL_COUNTERS: other kernels) does not probe
    ctx.set_option(F.RT_OPT_DETAIL_COUNTERS, 1)
    _same(ref[BUNNY_CAM], _render(s, BUNNY_CAM))
    ctx.set_option(F.RT_OPT_DETAIL_COUNTERS, 0)
    assert ctx.bsp_cull_probes() == (0, 0)
    # a render too small for a timed launch (4 iterations x 230,400 < 2^20 samples) does not probe
    small = _render(s, BUNNY_CAM, spp=4)
    assert ctx.bsp_cull_probes() == (0, 0)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
    _same(_render(s, BUNNY_CAM, spp=4), small)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    # 32 iterations: four probe launches of 5 iterations, then 12 on the certified kernel
    got = _render(s, BUNNY_CAM)
    _same(ref[BUNNY_CAM], got)
    assert ctx.bsp_cull_probes() == (1, 4)
    mode, mc, ms = ctx.bsp_cull_in_use()   # (the render's results were read: its events are done)
    print(f"probe: certified {mc:.4f}, silhouette {ms:.4f} ms per 2^20 samples -> mode {mode}")
    assert mc > 0 and ms > 0
    assert mode == (F.RT_BSP_CULL_SILHOUETTE if ms < 0.95 * mc else F.RT_BSP_CULL_CERTIFIED)
    # the choice holds: the same eye again, a progressive continuation, and a new eye at
    # a similar reach -- no second probe, the same frames
    _same(ref[BUNNY_CAM], _render(s, BUNNY_CAM))
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
    cont_ref = _render(s, BUNNY_CAM, first_iter=32, accum_in=ref[BUNNY_CAM][0])
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    _render(s, BUNNY_CAM)   # (the option change started over: a second probe)
    assert ctx.bsp_cull_probes() == (2, 8)
    _same(cont_ref, _render(s, BUNNY_CAM, first_iter=32, accum_in=got[0]))
    _same(ref[CAM2], _render(s, CAM2))
    assert ctx.bsp_cull_probes() == (2, 8)
    assert ctx.bsp_cull_in_use()[1:] != (0.0, 0.0)
    # an eye five times as far: a new probe
    _same(ref[FAR], _render(s, FAR))
    assert ctx.bsp_cull_probes() == (3, 12)
    m2, mc2, ms2 = ctx.bsp_cull_in_use()
    assert mc2 > 0 and ms2 > 0
    assert m2 == (F.RT_BSP_CULL_SILHOUETTE if ms2 < 0.95 * mc2 else F.RT_BSP_CULL_CERTIFIED)
    # the query kernel follows the choice (same hits as certified either way)
    rng = np.random.default_rng(3)
    R = np.zeros((4096, 8), np.float32)
    R[:, :3] = np.asarray(CAM2[0], np.float32)
    d = rng.normal(size=(4096, 3)) * [0.3, 0.3, 1.0] + [0.0, 0.0, -1.0]
    R[:, 3:6] = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    R[:, 6], R[:, 7] = 1e-4, 1e6
    h_auto = ctx.trace_rays("BSP", R, None)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
    h_cert = ctx.trace_rays("BSP", R, None)
    for k in ("tri", "dist", "beta", "gamma"):
        assert np.array_equal(h_auto[k].view(np.uint32), h_cert[k].view(np.uint32)), k
    ctx.close()


def test_auto_with_async_fold(rt):
    # the probe launches are passes of the render: double-buffered scratch, folds on the second stream
    F = rt._ffi
    s = Scene(rt, rt.Mesh.synth_bunny(), "BSP", env=(0.8, 0.9, 1.0))
    ctx = s.ctx
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
    ref = [_render(s, BUNNY_CAM), _render(s, CAM2)]
    ctx.set_option(F.RT_OPT_ASYNC_FOLD, 1)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    got = [_render(s, BUNNY_CAM), _render(s, CAM2)]
    ctx.set_option(F.RT_OPT_ASYNC_FOLD, 0)
    for a, b in zip(ref, got):
        _same(a, b)
    assert ctx.bsp_cull_probes() == (1, 4)
    ctx.close()


def test_cull_option_range(rt):
    F = rt._ffi
    ctx = rt.Context(0)
    try:
        assert ctx.bsp_cull_in_use() == (F.RT_BSP_CULL_CERTIFIED, 0.0, 0.0)   # the default auto, before a probe
        for bad in (-1, F.RT_BSP_CULL_AUTO + 1):
            with pytest.raises(Exception):
                ctx.set_option(F.RT_OPT_BSP_CULL, bad)
        ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_FAST)
        assert ctx.bsp_cull_in_use()[0] == F.RT_BSP_CULL_FAST
        ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_SILHOUETTE)
        assert ctx.bsp_cull_in_use()[0] == F.RT_BSP_CULL_CERTIFIED   # no camera terms yet: the certified kernel
    finally:
        ctx.close()


def test_auto_other_modes_do_not_probe(rt):
    F = rt._ffi
    s = Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), "BSP")
    ctx = s.ctx
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
    ref = s.render_gpu("W7E3", CORNELL_CAM, 1024, 1024, (0, 0, 1024, 1024), 0, 4)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    got = s.render_gpu("W7E3", CORNELL_CAM, 1024, 1024, (0, 0, 1024, 1024), 0, 4)
    _same(ref, got)
    assert ctx.bsp_cull_in_use() == (F.RT_BSP_CULL_CERTIFIED, 0.0, 0.0)
    assert ctx.bsp_cull_probes() == (0, 0)
    ctx.close()


def test_held_camera_key_probes_once(rt):
    """the reference's interactive loop (src/lib.rs:331-363 +
    render_state.rs:467-481: one 1-spp frame, then the camera update) on the config-3
    scene at 1920x1080 with the Left key held for 32 frames.  RT_BSP_CULL_AUTO probes
    once (its four launches are four of the frames), never waits on the host, costs
    at most 10 % over the certified kernel, and renders the same frames bit for bit."""
    F = rt._ffi
    scene = rt.find_scene("W9 E1 Bunny")

    def run(cull, keep=True):
        rs = rt.RenderState(scene, resolution=(1920, 1080), env=(0.8, 0.9, 1.0))
        try:
            rs.ctx.set_option(F.RT_OPT_BSP_CULL, cull)
            rs.set_samples(4096, True)
            rs.input("Left", True)
            rs.step()   # (first frame: the kernels' first launch, not timed)
            rs.ctx.synchronize()
            frames, t = [], 0.0
            for _ in range(32):
                t0 = time.perf_counter()
                assert rs.step()
                rs.ctx.synchronize()
                t += time.perf_counter() - t0
                if keep:
                    frames.append((rs.frame().copy(), rs.hit_ids().copy()))
            return t, frames, rs.ctx.bsp_cull_probes(), rs.ctx.bsp_cull_in_use()
        finally:
            rs.ctx.close()

    t_cert, f_cert, _, _ = run(F.RT_BSP_CULL_CERTIFIED)
    t_auto, f_auto, probes, used = run(F.RT_BSP_CULL_AUTO)
    # timing without the frame downloads: best of three runs each
    for _ in range(2):
        t_cert = min(t_cert, run(F.RT_BSP_CULL_CERTIFIED, keep=False)[0])
        t_auto = min(t_auto, run(F.RT_BSP_CULL_AUTO, keep=False)[0])
    print(f"32 held-key frames: certified {t_cert * 1e3:.1f} ms, auto {t_auto * 1e3:.1f} ms; probes {probes}; "
          f"in use {used}")
    assert probes == (1, 4)
    assert used[1] > 0 and used[2] > 0
    assert t_auto <= 1.10 * t_cert
    for (ac, ic), (aa, ia) in zip(f_cert, f_auto):
        assert np.array_equal(ac.view(np.uint32), aa.view(np.uint32))
        assert np.array_equal(ic, ia)
