"""BASELINE configs at their full sizes, checked through properties that do
not depend on size, plus the oracle where it finishes in seconds:

* config 3 (bunny stand-in, 1920x1080, W9E1, BSP, 256 spp -- the bench frame):
  - the whole frame at 1 spp equals the CPU oracle bit for bit (ids and radiance);
  - 256 iterations in one launch equal 128 + 128 continued from the
    accumulation buffer, and equal a second run (the persistent work queue
    hands out units in a different order each run; the fold does not care);
  - the 8-rank tile split of the frame, gathered and unpacked, equals the
    single-device frame (the N>1 data path of bench.py, all ranks on one GPU);
  - 24 pixels spread over the frame equal the oracle at all 256 iterations;
  - the whole frame at its BASELINE 256 spp, rendered with the default
    (certified) culling exactly as the bench renders it, equals the oracle's 256
    iterations in every pixel's accumulation bits and primary id (the oracle
    walks every node, as bsp.wgsl does: ~26 s on the box's 16 threads).
* config 5 (10M-triangle soup, 3840x2160, W9E1, BSP): split identity at 2 spp.
"""
import numpy as np
import pytest

from parity_util import BUNNY_CAM, Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu

W, H = 1920, 1080


@pytest.fixture(scope="module")
def bunny(rt, gpu):
    return Scene(rt, rt.Mesh.synth_bunny(), "BSP")


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def test_config3_full_frame_1spp_equals_oracle(bunny):
    g = bunny.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, 1)
    o = bunny.render_oracle("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, 1)
    check(g, o)
    assert g[2]["samples"] == W * H


def test_config3_256spp_split_and_rerun_identity(bunny):
    full = bunny.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, 256)
    again = bunny.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, 256)
    assert np.array_equal(_bits(full[0]), _bits(again[0])) and np.array_equal(full[1], again[1])
    half = bunny.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, 128)
    rest = bunny.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 128, 128, accum_in=half[0])
    assert np.array_equal(_bits(full[0]), _bits(rest[0])) and np.array_equal(full[1], rest[1])
    assert full[2]["samples"] == W * H * 256
    # 24 pixels across the frame, all 256 iterations, against the oracle
    rng = np.random.default_rng(3)
    for x, y in zip(rng.integers(0, W, 24), rng.integers(0, H, 24)):
        o = bunny.render_oracle("W9E1", BUNNY_CAM, W, H, (int(x), int(y), 1, 1), 0, 256)
        assert np.array_equal(_bits(full[0][y, x]), _bits(o[0][0, 0])), (x, y, full[0][y, x], o[0][0, 0])
        assert full[1][y, x] == o[1][0, 0]


def test_config3_full_frame_baseline_spp_equals_oracle(rt, bunny):
    # the headline frame whole, not by transitivity through the
    # unculled walk -- every one of its 530.8 M samples, in one launch
    assert rt._ffi.RT_BSP_CULL_CERTIFIED == 1
    # (the bench's own kernel instantiation: no counting build; that culling is
    # active on this frame is test_gpu_cull_fullframe.py's business)
    bunny.ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, rt._ffi.RT_BSP_CULL_CERTIFIED)
    g = bunny.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, 256)
    assert g[2]["samples"] == W * H * 256
    o = bunny.render_oracle("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, 256)
    check(g, o)


def test_config3_eight_rank_tiles_equal_frame(rt, bunny):
    spp = 4
    ref = bunny.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, spp)
    gpu = bunny.ctx
    gpu.set_uniforms(rt.make_uniform(*BUNNY_CAM, W, H))
    nr = 8
    lt = rt.local_tiles(W, H, nr)
    pa = gpu.alloc(nr * lt * 64 * 16)
    pi = gpu.alloc(nr * lt * 64 * 4)
    total = 0
    for r in range(nr):
        c = gpu.render_tiles("W9E1", "BSP", r, nr, 0, spp, pa.ptr + r * lt * 64 * 16, pi.ptr + r * lt * 64 * 4,
                             counts=True)
        total += c["samples"]
    fa = gpu.alloc(W * H * 16)
    fi = gpu.alloc(W * H * 4)
    gpu.unpack_tiles(W, H, nr, pa.ptr, pi.ptr, fa.ptr, fi.ptr)
    a = fa.to_numpy(np.float32, (H, W, 4))
    i = fi.to_numpy(np.uint32, (H, W))
    for b in (pa, pi, fa, fi):
        b.free()
    assert total == W * H * spp   # every pixel-sample on exactly one rank
    assert np.array_equal(_bits(a), _bits(ref[0])) and np.array_equal(i, ref[1])


@pytest.mark.slow
def test_config5_full_frame_split_identity(rt):
    mesh = rt.Mesh.synth_soup(10_000_000)
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh(mesh)
        ctx.build_bsp_device(20, 4)
        cam = ((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.5)
        W5, H5 = 3840, 2160
        ctx.set_uniforms(rt.make_uniform(*cam, W5, H5))
        out = []
        for parts in ((0, 2), (0, 1), (1, 1)):
            acc = ctx.alloc(W5 * H5 * 16)
            if parts == (1, 1):
                acc.from_numpy(out[1])
            else:
                acc.zero()
            ctx.render("W9E1", "BSP", (0, 0, W5, H5), parts[0], parts[1], acc.ptr, None)
            out.append(acc.to_numpy(np.float32, (H5, W5, 4)))
            acc.free()
        assert np.array_equal(_bits(out[0]), _bits(out[2]))
        assert np.isfinite(out[0]).all() and (out[0][..., 3] == 1.0).all()
    finally:
        ctx.close()
