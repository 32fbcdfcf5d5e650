"""GPU parity on the BASELINE.json workloads other than the headline
(02562_raytracer_amd/configs.py): regions of the full-size frames, GPU vs the
CPU oracle: bit-exact triangle ids, radiance within RADIANCE_TOL and, as
everywhere else, bit for bit.

  config 2: Cornell box with blocks, 1024x1024, W7E3, BSP -- the whole frame at
            its BASELINE 64 spp
  config 4: 10 x 10 grid of bunny stand-ins (6.96M triangles), W9E1, BSP
  config 5: 10M random-triangle soup, 3840x2160, W9E1, BSP (and BVH)

For configs 4 and 5 the oracle renders from the product builder's arrays
(bit-identical builders, tests/test_host_builders.py), sparing its
single-threaded build of a 7M/10M-triangle BSP."""
import importlib

import numpy as np
import pytest

from parity_util import RADIANCE_TOL, Scene, compare

pytestmark = pytest.mark.gpu


def check(g, o):
    linf, bits, idm = compare(g, o)
    assert idm == 0, f"{idm} primary-hit id mismatches"
    assert linf <= RADIANCE_TOL, f"radiance L-inf {linf}"
    assert bits == 0, f"{bits} radiance words differ bitwise (L-inf {linf})"
    for k in ("samples", "primary", "shadow", "bounce"):
        assert g[2][k] == o[2][k], (k, g[2][k], o[2][k])


@pytest.fixture(scope="module")
def configs():
    return importlib.import_module("02562_raytracer_amd.configs").WORKLOADS


def test_config2_cornell_region(rt, gpu, configs):
    wl = configs[2]
    s = Scene(rt, wl.mesh(), wl.traversal, env=wl.env)
    region = (448, 400, 128, 96)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, 4)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, 4)
    check(g, o)
    assert (g[1] != 0xFFFFFFFF).all()


def test_config2_full_frame_baseline_spp(rt, gpu, configs):
    # the whole BASELINE config-2 frame: 1024x1024 at 64 spp in one launch, every
    # pixel's accumulation and primary id against the oracle's 64 iterations
    wl = configs[2]
    assert (wl.width, wl.height, wl.spp) == (1024, 1024, 64)
    s = Scene(rt, wl.mesh(), wl.traversal, env=wl.env)
    region = (0, 0, wl.width, wl.height)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    check(g, o)
    assert g[2]["samples"] == wl.width * wl.height * wl.spp and g[2]["bounce"] > 0
    s.ctx.close()


def test_config4_bunny_grid_region(rt, gpu, configs):
    wl = configs[4]
    mesh = wl.mesh()
    assert abs(mesh.ntris - 6945100) <= 0.01 * 6945100
    s = Scene(rt, mesh, wl.traversal, env=wl.env, oracle_accel_from_product=True)
    region = (832, 420, 256, 96)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, 16)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, 16)
    check(g, o)
    assert (g[1] != 0xFFFFFFFF).mean() > 0.3
    # iterations 16..31 continued from that accumulation
    g2 = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 16, 16, accum_in=g[0])
    o2 = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 16, 16, accum_in=g[0])
    check(g2, o2)
    s.ctx.close()


def test_config4_baseline_spp_region(rt, gpu, configs):
    # config 4's BASELINE 256 spp, in one launch, on the centre quarter of the
    # frame (960 x 540: 133 M samples, where the grid's bunnies overlap on screen
    # and paths bounce longest; the oracle walks every node of the 7M-triangle
    # BSP: about a minute on the box's 16 threads).  Round 4 compared a 32 x 32
    # region.
    wl = configs[4]
    assert wl.spp == 256
    s = Scene(rt, wl.mesh(), wl.traversal, env=wl.env, oracle_accel_from_product=True)
    region = (480, 270, 960, 540)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    check(g, o)
    assert g[2]["samples"] == 960 * 540 * wl.spp and g[2]["bounce"] > 0
    s.ctx.close()


@pytest.mark.parametrize("trav", ["BSP", "BVH"])
def test_config5_soup_region(rt, gpu, configs, trav):
    wl = configs[5]
    mesh = wl.mesh()
    assert mesh.ntris == 10_000_000
    s = Scene(rt, mesh, trav, env=wl.env, oracle_accel_from_product=True)
    region = (1856, 1040, 128, 80)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, 8)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, 8)
    check(g, o)
    assert (g[1] != 0xFFFFFFFF).mean() > 0.5
    s.ctx.close()


def test_config5_baseline_spp_region(rt, gpu, configs):
    # config 5's BASELINE 1024 spp, in one launch, on a 32x32 region at the frame
    # centre (the oracle walks a 10M-triangle BSP per sample)
    wl = configs[5]
    assert wl.spp == 1024
    s = Scene(rt, wl.mesh(), "BSP", env=wl.env, oracle_accel_from_product=True)
    region = (1904, 1064, 32, 32)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    check(g, o)
    assert g[2]["samples"] == 32 * 32 * 1024
    s.ctx.close()
