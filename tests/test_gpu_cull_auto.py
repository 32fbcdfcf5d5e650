"""RT_BSP_CULL_AUTO (rt_api.cpp probe_auto_cull; DESIGN.md section 4 "Round 5"):
the first W9E1 BSP render for a scene and eye times the certified and the
silhouette kernels on a probe of itself and runs the faster.  Both forms are
exact, so an automatic render equals the certified render bit for bit whichever
it picked; the probe writes only the per-sample scratch (accum and ids come from
the real passes); the choice holds until the eye (or the BSP) changes; other
modes and walks run the certified kernel without probing."""
import numpy as np
import pytest

from conftest import model
from parity_util import BUNNY_CAM, CORNELL_CAM, Scene

pytestmark = pytest.mark.gpu

REGION = (0, 0, 640, 360)
CAM2 = ((0.25, 0.18, 0.45), (-0.02, 0.09, 0.0), (0.0, 1.0, 0.0), 2.5)


def _same(a, b):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), "radiance differs"
    assert np.array_equal(a[1], b[1]), "primary-hit ids differ"
    for k in ("samples", "primary", "shadow", "bounce"):
        assert a[2][k] == b[2][k], k


def _render(s, cam, spp=8, first_iter=0, accum_in=None):
    return s.render_gpu("W9E1", cam, 640, 360, REGION, first_iter, spp, accum_in=accum_in)


def test_auto_picks_a_form_and_matches_certified(rt):
    F = rt._ffi
    s = Scene(rt, rt.Mesh.synth_bunny(), "BSP", env=(0.8, 0.9, 1.0))
    ctx = s.ctx
    ref = {}
    for cam in (BUNNY_CAM, CAM2):
        ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
        ref[cam] = _render(s, cam)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    mode, mc, ms = ctx.bsp_cull_in_use()
    assert (mode, mc, ms) == (F.RT_BSP_CULL_CERTIFIED, 0.0, 0.0)   # not probed yet: the certified kernel
    got = _render(s, BUNNY_CAM)
    mode, mc, ms = ctx.bsp_cull_in_use()
    print(f"probe: certified {mc:.3f} ms, silhouette {ms:.3f} ms -> mode {mode}")
    assert mc > 0 and ms > 0
    assert mode == (F.RT_BSP_CULL_SILHOUETTE if ms < 0.97 * mc else F.RT_BSP_CULL_CERTIFIED)
    _same(ref[BUNNY_CAM], got)
    # the choice holds for the eye (no second probe) and renders the same frame again
    _same(ref[BUNNY_CAM], _render(s, BUNNY_CAM))
    assert ctx.bsp_cull_in_use() == (mode, mc, ms)
    # a progressive continuation (iterations 8..15 on top of the first 8) as well
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_CERTIFIED)
    cont_ref = _render(s, BUNNY_CAM, first_iter=8, accum_in=ref[BUNNY_CAM][0])
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    _same(cont_ref, _render(s, BUNNY_CAM, first_iter=8, accum_in=got[0]))
    # a new eye: new camera terms, a new probe
    _same(ref[CAM2], _render(s, CAM2))
    m2, mc2, ms2 = ctx.bsp_cull_in_use()
    assert mc2 > 0 and ms2 > 0 and (mc2, ms2) != (mc, ms)
    assert m2 == (F.RT_BSP_CULL_SILHOUETTE if ms2 < 0.97 * mc2 else F.RT_BSP_CULL_CERTIFIED)
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
    # the probe writes the per-sample scratch a pending fold may still read: it joins it first
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
    ref = s.render_gpu("W7E3", CORNELL_CAM, 256, 256, (0, 0, 256, 256), 0, 4)
    ctx.set_option(F.RT_OPT_BSP_CULL, F.RT_BSP_CULL_AUTO)
    got = s.render_gpu("W7E3", CORNELL_CAM, 256, 256, (0, 0, 256, 256), 0, 4)
    _same(ref, got)
    assert ctx.bsp_cull_in_use() == (F.RT_BSP_CULL_CERTIFIED, 0.0, 0.0)
    ctx.close()
