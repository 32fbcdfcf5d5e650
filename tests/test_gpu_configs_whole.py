"""Whole frames of the two 8-GPU workloads against the CPU oracle in the suite
(VERDICT r5 "What's weak" 1(b): they were pinned whole only by one-off runs of
tests/pin_full_frame.py, profiles/r05/final/pin_full_frame_c{4,5}.txt).

  config 4 (10 x 10 bunny grid, 6.96M triangles, 1920x1080, W9E1, BSP) at its
  BASELINE 256 spp: test_gpu_configs.py compares the centre 960x540; the four
  bands around it here complete the frame;
  config 5 (10M-triangle soup, 3840x2160, W9E1, BSP) at 16 of its 1024 spp (its
  1024 spp are compared on a 32x32 region in test_gpu_configs.py): the four
  1920x1080 quadrants.

Each piece is its own test (the oracle takes 20-40 s per piece on the box's 16
threads, walking every node as bsp.wgsl does) and renders the piece as a region
of the full frame: global pixel coordinates, so the PRNG seeds and rays are the
whole frame's.  The default culling (RT_BSP_CULL_AUTO) renders on the GPU.  The
oracle renders from the product builder's arrays (bit-identical builders,
tests/test_host_builders.py)."""
import importlib

import pytest

from parity_util import Scene
from test_gpu_configs import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def workloads():
    return importlib.import_module("02562_raytracer_amd.configs").WORKLOADS


@pytest.fixture(scope="module")
def scene4(rt, gpu, workloads):
    wl = workloads[4]
    s = Scene(rt, wl.mesh(), "BSP", env=wl.env, oracle_accel_from_product=True)
    yield wl, s
    s.ctx.close()


@pytest.fixture(scope="module")
def scene5(rt, gpu, workloads):
    wl = workloads[5]
    s = Scene(rt, wl.mesh(), "BSP", env=wl.env, oracle_accel_from_product=True)
    yield wl, s
    s.ctx.close()


# the frame minus test_gpu_configs.py's centre (480, 270, 960, 540)
C4_BANDS = [(0, 0, 1920, 270), (0, 810, 1920, 270), (0, 270, 480, 540), (1440, 270, 480, 540)]


@pytest.mark.parametrize("region", C4_BANDS, ids=["top", "bottom", "left", "right"])
def test_config4_whole_frame_baseline_spp(scene4, region):
    wl, s = scene4
    assert (wl.width, wl.height, wl.spp) == (1920, 1080, 256)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, wl.spp)
    check(g, o)
    assert g[2]["samples"] == region[2] * region[3] * wl.spp


C5_QUADRANTS = [(0, 0, 1920, 1080), (1920, 0, 1920, 1080), (0, 1080, 1920, 1080), (1920, 1080, 1920, 1080)]


@pytest.mark.parametrize("region", C5_QUADRANTS, ids=["q00", "q10", "q01", "q11"])
def test_config5_whole_frame_16spp(scene5, region):
    wl, s = scene5
    assert (wl.width, wl.height) == (3840, 2160)
    g = s.render_gpu(wl.mode, wl.camera, wl.width, wl.height, region, 0, 16)
    o = s.render_oracle(wl.mode, wl.camera, wl.width, wl.height, region, 0, 16)
    check(g, o)
    assert g[2]["samples"] == region[2] * region[3] * 16
