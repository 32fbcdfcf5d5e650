"""GPU parity: HIP kernels (through the C ABI) vs the CPU oracle on the same
seeded inputs.  Bar: primary-hit triangle ids bit-exact; accumulated radiance
within L-inf 1e-4 (north_star) -- and in fact bit-exact, which is asserted
separately so a precision drift is reported as such."""
import numpy as np
import pytest

from conftest import model
from parity_util import (BASIC_CAM, BUNNY_CAM, CORNELL_CAM, RADIANCE_TOL, TEAPOT_CAM, Scene, compare)

pytestmark = pytest.mark.gpu


def check(gpu, ora, exact=True, counts=True):
    linf, bits, idm = compare(gpu, ora)
    assert idm == 0, f"{idm} primary-hit ids differ"
    assert linf <= RADIANCE_TOL, f"L-inf {linf}"
    if exact:
        assert bits == 0, f"{bits} radiance words differ bitwise (L-inf {linf})"
    if counts:
        for k in ("samples", "primary", "shadow", "bounce"):
            assert gpu[2][k] == ora[2][k], (k, gpu[2][k], ora[2][k])


def test_math_selftest(gpu):
    # sqrt, division, pinned transcendentals: device == host bit for bit
    assert gpu.selftest_math(1 << 20, -4.0, 4.0) == 0
    assert gpu.selftest_math(1 << 16, -1e4, 1e4) == 0


def test_w1e6_analytic(rt, gpu, oracle):
    # config 1: scenes.rs W1 E6, 512x512, 1 spp, no mesh
    u = rt.make_uniform(*BASIC_CAM, 512, 512)
    gpu.set_uniforms(u)
    acc = gpu.alloc(512 * 512 * 16)
    ids = gpu.alloc(512 * 512 * 4)
    cnt = gpu.render("W1E6", "NONE", (0, 0, 512, 512), 0, 1, acc.ptr, ids.ptr, counts=True)
    g = (acc.to_numpy(np.float32, (512, 512, 4)), ids.to_numpy(np.uint32, (512, 512)), cnt)
    ou = oracle.make_uniform(*BASIC_CAM, 512, 512)
    o = oracle.render(oracle.SceneRef(None), ou, "W1E6", "NONE", (0, 0, 512, 512), 0, 1)
    check(g, o)
    assert set(np.unique(g[1])) <= {0, 1, 2, 0xFFFFFFFF}


@pytest.fixture(scope="module")
def cornell_bsp(rt, gpu):
    return Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), "BSP")


def test_cornell_w7e3_bsp(cornell_bsp):
    # config 2 (reduced): W7 E3 Cornell Box, BSP D20/leaf 4, 4 progressive iterations
    g = cornell_bsp.render_gpu("W7E3", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 4)
    o = cornell_bsp.render_oracle("W7E3", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 4)
    check(g, o)
    assert g[2]["shadow"] > 0 and g[2]["bounce"] > 0
    assert np.all(g[0][..., 3] == 1.0)


def test_cornell_w7e3_progressive_continuation(cornell_bsp):
    # iterations 0..1 then 2..5 from the accumulation buffer == 0..5 in one launch
    full = cornell_bsp.render_gpu("W7E3", CORNELL_CAM, 96, 80, (16, 8, 48, 40), 0, 6)
    a = cornell_bsp.render_gpu("W7E3", CORNELL_CAM, 96, 80, (16, 8, 48, 40), 0, 2)
    b = cornell_bsp.render_gpu("W7E3", CORNELL_CAM, 96, 80, (16, 8, 48, 40), 2, 4, accum_in=a[0])
    assert np.array_equal(full[0].view(np.uint32), b[0].view(np.uint32))
    assert np.array_equal(full[1], b[1])
    o = cornell_bsp.render_oracle("W7E3", CORNELL_CAM, 96, 80, (16, 8, 48, 40), 2, 4, accum_in=a[0])
    check(b, o)


@pytest.mark.parametrize("chunk,order,budget_mb", [(1, 1, None), (3, 0, None), (1, 0, 1), (5, 1, 1), (64, 1, None)])
def test_work_units_and_passes(rt, cornell_bsp, chunk, order, budget_mb):
    # k_path work units of `chunk` iterations in either order, and renders split
    # into passes by the per-sample scratch budget (1 MiB = 10 iterations of
    # 160x160 px): the progressive fold reproduces the in-order accumulation bit
    # for bit, for any unit shape (regions with ragged 8x8 tiles)
    s = cornell_bsp
    try:
        s.ctx.set_option(rt._ffi.RT_OPT_SAMPLE_CHUNK, chunk)
        s.ctx.set_option(rt._ffi.RT_OPT_UNIT_ORDER, order)
        if budget_mb:
            s.ctx.set_option(rt._ffi.RT_OPT_SAMPLE_BUDGET_MB, budget_mb)
        accum_in = s.render_gpu("W7E3", CORNELL_CAM, 200, 180, (20, 10, 160, 160), 0, 3)[0]
        g = s.render_gpu("W7E3", CORNELL_CAM, 200, 180, (20, 10, 160, 160), 3, 13, accum_in=accum_in)
        o = s.render_oracle("W7E3", CORNELL_CAM, 200, 180, (20, 10, 160, 160), 3, 13, accum_in=accum_in.copy())
    finally:
        s.ctx.set_option(rt._ffi.RT_OPT_SAMPLE_CHUNK, 1)
        s.ctx.set_option(rt._ffi.RT_OPT_UNIT_ORDER, 1)
        s.ctx.set_option(rt._ffi.RT_OPT_SAMPLE_BUDGET_MB, 16384)
    check(g, o)


def test_cornell_w7e3_bvh(rt, gpu):
    s = Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), "BVH")
    g = s.render_gpu("W7E3", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 2)
    o = s.render_oracle("W7E3", CORNELL_CAM, 64, 64, (0, 0, 64, 64), 0, 2)
    check(g, o)


@pytest.mark.parametrize("mode,trav,name", [("W6E1", "BSP", "teapot.obj"), ("PROJECT", "BVH", "teapot.obj"),
                                            ("PROJECT", "BSP", "teapot.obj"), ("PROJECT", "BVH", "test_object.obj"),
                                            ("PROJECT", "BVH", "plane.obj"),
                                            ("PROJECT", "BVH", "CornellBoxWithBlocks.obj")])
def test_primary_modes(rt, gpu, mode, trav, name):
    cam = {"teapot.obj": TEAPOT_CAM, "CornellBoxWithBlocks.obj": CORNELL_CAM}.get(name, BASIC_CAM)
    W, H = (800, 450) if name == "teapot.obj" else (512, 512)
    s = Scene(rt, rt.Mesh.from_obj(model(name)), trav)
    region = (200, 100, 240, 136)
    g = s.render_gpu(mode, cam, W, H, region)
    o = s.render_oracle(mode, cam, W, H, region)
    check(g, o)


@pytest.mark.parametrize("mode,trav", [("W6E1", "BSP"), ("PROJECT", "BSP"), ("PROJECT", "BVH")])
def test_axis_aligned_and_tiny_direction_components(rt, gpu, mode, trav):
    """An axis-aligned camera and a hand-made jitter table (uniform.rs:254-277
    jitter[] with subdivision 2) put exact zeros, tiny negatives (|d| < 1e-8:
    bsp.wgsl:63 divides by +1e-8 while the near child follows the sign) and
    near-threshold values into ray directions around the centre pixel."""
    cam = ((0.0, 1.5, 10.0), (0.0, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5)
    W, H = 801, 451                         # odd: the centre pixel has uv = (0, 0)
    jitter = [(0.0, 0.0), (-1e-9, 1e-9), (-2e-8, -3e-9), (1e-10, -5e-9)]
    s = Scene(rt, rt.Mesh.from_obj(model("teapot.obj")), trav)
    region = (368, 209, 64, 32)
    g = s.render_gpu(mode, cam, W, H, region, jitter=jitter)
    o = s.render_oracle(mode, cam, W, H, region, jitter=jitter)
    check(g, o)
    assert (g[1] != 0xFFFFFFFF).any()


@pytest.mark.parametrize("sel", [2, 5, 6, 4, 7])
def test_shader_selection(rt, gpu, sel):
    # uniforms.selection1 switch of shade(): mirror, normal, base colour, default (error colour)
    s = Scene(rt, rt.Mesh.from_obj(model("teapot.obj")), "BSP")
    region = (300, 150, 128, 96)
    for mode in ("W6E1", "W9E1"):
        g = s.render_gpu(mode, TEAPOT_CAM, 800, 450, region, 0, 1, selection1=sel)
        o = s.render_oracle(mode, TEAPOT_CAM, 800, 450, region, 0, 1, selection1=sel)
        check(g, o)


@pytest.fixture(scope="module")
def bunny(rt, gpu):
    return Scene(rt, rt.Mesh.synth_bunny(), "BSP", env=(0.8, 0.9, 1.0))


def test_bunny_w9e1_bsp_region(bunny):
    # config 3 geometry and camera at 1920x1080 (a sampled region), 2 spp
    region = (704, 412, 512, 128)
    g = bunny.render_gpu("W9E1", BUNNY_CAM, 1920, 1080, region, 0, 2)
    o = bunny.render_oracle("W9E1", BUNNY_CAM, 1920, 1080, region, 0, 2)
    check(g, o)
    assert (g[1] != 0xFFFFFFFF).mean() > 0.3


def test_bunny_w9e1_bvh_region(rt, gpu):
    s = Scene(rt, rt.Mesh.synth_bunny(), "BVH", env=(0.8, 0.9, 1.0))
    region = (832, 476, 256, 64)
    g = s.render_gpu("W9E1", BUNNY_CAM, 1920, 1080, region, 0, 2)
    o = s.render_oracle("W9E1", BUNNY_CAM, 1920, 1080, region, 0, 2)
    check(g, o)


@pytest.mark.parametrize("depth", [20, 9])
def test_shade_threshold_is_scheduling_only(rt, gpu, depth):
    # The shading threshold only schedules: every setting -- fixed 8, 16, 24 or 32,
    # lockstep (0 and 64), an explicit per-wave pair, and the default per-wave choice
    # from the wave's share of lanes inside a leaf (k_path; T_lo 16 / T_hi 32 with
    # the certified and auto culling, 8 / 24 with the fast margin) -- renders the same
    # bits.  Depth 9 makes a test-dominated walk (~300 triangles per leaf: the share
    # is high and the waves choose T_hi), depth 20 a walk-dominated one (T_lo).
    s = Scene(rt, rt.Mesh.synth_soup(150_000), "BSP", oracle_accel_from_product=True, bsp_depth=depth)
    cam = ((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.5)
    region = (600, 300, 96, 64)
    frames = {}
    try:
        for t in (-1, 8, 16, 24, 32, 0, 64, 0x10000 | (32 << 8) | 12):
            s.ctx.set_option(rt._ffi.RT_OPT_SHADE_THRESHOLD, t)
            frames[t] = s.render_gpu("W9E1", cam, 1280, 720, region, 0, 3)
    finally:
        s.ctx.set_option(rt._ffi.RT_OPT_SHADE_THRESHOLD, -1)
    o = s.render_oracle("W9E1", cam, 1280, 720, region, 0, 3)
    check(frames[-1], o)
    for t, g in frames.items():
        assert np.array_equal(g[0].view(np.uint32), frames[-1][0].view(np.uint32)), t
        assert np.array_equal(g[1], frames[-1][1]), t
    s.ctx.close()


@pytest.mark.parametrize("waves,chunk,order", [(1, 1, 1), (3, 3, 0), (32, 1, 0), (32, 5, 1)])
def test_bvh_work_shards(rt, gpu, waves, chunk, order):
    # the BVH walk's 8 per-XCD work queues: a wave draws from its XCD's shard,
    # then from the others once that is drained, so every (pixel, iteration)
    # unit is rendered exactly once for any grid size and unit shape
    s = Scene(rt, rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj")), "BVH")
    try:
        s.ctx.set_option(rt._ffi.RT_OPT_WAVES_PER_CU, waves)
        s.ctx.set_option(rt._ffi.RT_OPT_SAMPLE_CHUNK, chunk)
        s.ctx.set_option(rt._ffi.RT_OPT_UNIT_ORDER, order)
        g = s.render_gpu("W7E3", CORNELL_CAM, 120, 100, (4, 6, 100, 90), 0, 7)
    finally:
        s.ctx.set_option(rt._ffi.RT_OPT_WAVES_PER_CU, 32)
        s.ctx.set_option(rt._ffi.RT_OPT_SAMPLE_CHUNK, 1)
        s.ctx.set_option(rt._ffi.RT_OPT_UNIT_ORDER, 1)
    o = s.render_oracle("W7E3", CORNELL_CAM, 120, 100, (4, 6, 100, 90), 0, 7)
    check(g, o)


def test_tileset_unpack_equals_region(rt, cornell_bsp):
    # multi-GPU framebuffer tiling: every rank's packed tiles, gathered and
    # unpacked, reproduce the single-device frame bit for bit (8x8 tiles,
    # global pixel seeds), including ragged edge tiles (W,H not multiples of 8)
    W, H, nr = 70, 45, 3
    ref = cornell_bsp.render_gpu("W7E3", CORNELL_CAM, W, H, (0, 0, W, H), 0, 2)
    gpu = cornell_bsp.ctx
    u = rt.make_uniform(*CORNELL_CAM, W, H)
    gpu.set_uniforms(u)
    lt = rt.local_tiles(W, H, nr)
    pa = gpu.alloc(nr * lt * 64 * 16)
    pi = gpu.alloc(nr * lt * 64 * 4)
    for r in range(nr):
        gpu.render_tiles("W7E3", "BSP", r, nr, 0, 2, pa.ptr + r * lt * 64 * 16, pi.ptr + r * lt * 64 * 4)
    fa = gpu.alloc(W * H * 16)
    fi = gpu.alloc(W * H * 4)
    gpu.unpack_tiles(W, H, nr, pa.ptr, pi.ptr, fa.ptr, fi.ptr)
    a = fa.to_numpy(np.float32, (H, W, 4))
    i = fi.to_numpy(np.uint32, (H, W))
    assert np.array_equal(a.view(np.uint32), ref[0].view(np.uint32))
    assert np.array_equal(i, ref[1])


def test_empty_region_and_zero_spp(rt, cornell_bsp):
    gpu = cornell_bsp.ctx
    u = rt.make_uniform(*CORNELL_CAM, 64, 64)
    gpu.set_uniforms(u)
    acc = gpu.alloc(16)
    c = gpu.render("W7E3", "BSP", (0, 0, 0, 0), 0, 1, acc.ptr, None, counts=True)
    assert c["samples"] == 0
    acc2 = gpu.alloc(8 * 8 * 16)
    c = gpu.render("W7E3", "BSP", (0, 0, 8, 8), 0, 0, acc2.ptr, None, counts=True)
    assert c["samples"] == 0


def test_detail_counters_match_oracle(rt, cornell_bsp):
    # the algorithmic-bytes inputs: traversal counters of the counting
    # instantiation equal the oracle's for primary rays (W6E1-style closest hit
    # only; shadow rays use any-hit on the GPU, a strict subset of the work)
    # (with subtree culling off: the reference's node-by-node walk, whose counts
    # the oracle restates; tests/test_gpu_cull.py compares culled and full walks)
    s = cornell_bsp
    gpu = s.ctx
    gpu.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 1)
    gpu.set_option(rt._ffi.RT_OPT_BSP_CULL, 0)
    try:
        g = s.render_gpu("PROJECT", CORNELL_CAM, 64, 64, (0, 0, 64, 64))
    finally:
        gpu.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 0)
        gpu.set_option(rt._ffi.RT_OPT_BSP_CULL, 1)
    o = s.render_oracle("PROJECT", CORNELL_CAM, 64, 64, (0, 0, 64, 64))
    check(g, o)
    for k in ("node_interior", "node_leaf", "ids_read", "tri_tests", "tri_accepts"):
        assert g[2][k] == o[2][k], (k, g[2][k], o[2][k])


def _envmap_scene(rt, tex, mesh):
    s = Scene(rt, mesh, "BSP")
    s.ctx.set_environment_map(tex)
    s.oscene = s.oscene.__class__(s.om, s.obsp, s.obvh, s.env, env_tex=tex)
    return s


@pytest.mark.parametrize("spp", [1, 3])
def test_w9e1_environment_texture_synthetic(rt, spp):
    # hdri0 sampling (w9e1.wgsl:232-239) on an odd-sized random RGBA8 texture
    rng = np.random.default_rng(11)
    tex = rng.integers(0, 256, size=(19, 37, 4), dtype=np.uint8)
    s = _envmap_scene(rt, tex, rt.Mesh.synth_bunny())
    region = (704, 412, 256, 96)
    g = s.render_gpu("W9E1", BUNNY_CAM, 1920, 1080, region, 0, spp)
    o = s.render_oracle("W9E1", BUNNY_CAM, 1920, 1080, region, 0, spp)
    check(g, o)


def test_w9e1_teapot_campus_scene(rt):
    # scenes.rs "W9 E1 Teapot": teapot.obj, utah teapot camera, 800x450, the
    # luxo_pxr_campus.jpg background (decoded with PIL: texel values unpinned,
    # identical on both sides here)
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "textures",
                        "luxo_pxr_campus.jpg")
    tex = rt.load_texture_rgba8(path)
    assert tex.shape == (2000, 4000, 4)
    s = _envmap_scene(rt, tex, rt.Mesh.from_obj(model("teapot.obj")))
    region = (0, 180, 800, 40)   # teapot and background
    g = s.render_gpu("W9E1", TEAPOT_CAM, 800, 450, region, 0, 2)
    o = s.render_oracle("W9E1", TEAPOT_CAM, 800, 450, region, 0, 2)
    check(g, o)
    assert (g[1] != 0xFFFFFFFF).any() and (g[1] == 0xFFFFFFFF).any()


def test_display_frame_rgba8(rt):
    # fs_main's frame output through rt_frame_rgba8: saturate(pow(accum, 1.5)) in
    # 8-bit sRGB, checked against a float64 host evaluation of the same pinned
    # definition (exact 8-bit rounding away from the code thresholds)
    rs = rt.RenderState(rt.find_scene("W7 E3 Cornell Box"), resolution=(64, 48))
    rs.render(spp=4)
    acc = rs.frame().astype(np.float64)
    img = rs.frame_rgba8()
    v = np.clip(np.maximum(acc[..., :3], 0) ** 1.5, 0, 1)
    enc = np.where(v <= 0.0031308, 12.92 * v, 1.055 * v ** (1 / 2.4) - 0.055)
    ref = np.floor(enc * 255 + 0.5)
    near = np.abs(enc * 255 - np.floor(enc * 255) - 0.5) < 1e-3   # float rounding of pow/sqrt may flip these
    assert np.all((img[..., :3] == ref) | near)
    assert np.all(img[..., 3] == 255)
    rs.ctx.close()


def test_resolution_limit(rt, gpu):
    # k_path packs a lane's pixel as x | y << 16: larger frames are refused
    # at the boundary, not rendered wrongly
    with pytest.raises(rt.RtError):
        gpu.set_uniforms(rt.make_uniform(*BASIC_CAM, 65536, 16))
    with pytest.raises(rt.RtError):
        gpu.set_uniforms(rt.make_uniform(*BASIC_CAM, 16, 65536))
    gpu.set_uniforms(rt.make_uniform(*BASIC_CAM, 65535, 16))
