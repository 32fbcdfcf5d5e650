"""The headline frame's shape on the reference's only organic, non-convex mesh,
res/models/justElephant.obj (12,064 triangles after tobj's fan triangulation; copied
into assets/models; no scenes.rs scene uses it, so tools/mesh_frame.py's ELEPHANT_CAM
three-quarter view): W9E1 path tracer at 1920x1080.  The bunny
stand-in is a near-convex displaced sphere; the elephant's legs, trunk and ears give
concave, self-shadowing geometry and long bounce paths.

* the whole frame at the headline's 256 spp, BSP walk with the default culling
  (RT_BSP_CULL_AUTO: its probe launches run inside the render), equals the CPU
  oracle's 256 iterations in every pixel's accumulation bits and primary id;
* the whole frame with the HLBVH walk at 32 spp equals the oracle's;
* every culling mode renders the whole 64-spp frame bit for bit like the unculled walk.
"""
import numpy as np
import pytest

from conftest import model
from parity_util import Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu

W, H = 1920, 1080
ENV = (0.8, 0.9, 1.0)
ELEPHANT_CAM = ((15.0, 4.0, 14.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 3.5)   # tools/mesh_frame.py


@pytest.fixture(scope="module")
def mesh(rt):
    m = rt.Mesh.from_obj(model("justElephant.obj"))
    assert m.ntris == 12064
    return m


def test_elephant_full_frame_256spp_bsp_equals_oracle(rt, gpu, mesh):
    s = Scene(rt, mesh, "BSP", env=ENV)
    try:
        assert s.ctx.bsp_cull_in_use()[0] == rt._ffi.RT_BSP_CULL_CERTIFIED   # (the default auto, not yet probed)
        g = s.render_gpu("W9E1", ELEPHANT_CAM, W, H, (0, 0, W, H), 0, 256)
        assert g[2]["samples"] == W * H * 256
        probes = s.ctx.bsp_cull_probes()
        o = s.render_oracle("W9E1", ELEPHANT_CAM, W, H, (0, 0, W, H), 0, 256)
        check(g, o)
        hit = float((g[1] != 0xFFFFFFFF).mean())
        print(f"elephant 256 spp: {hit:.3f} of the pixels hit, bounce rays per primary "
              f"{g[2]['bounce'] / g[2]['primary']:.3f}, probes {probes}, kernel {s.ctx.bsp_cull_in_use()}")
        assert probes == (1, 4)
        assert 0.2 < hit < 0.9   # the framing: the elephant fills part of the frame
    finally:
        s.ctx.close()


def test_elephant_full_frame_bvh_equals_oracle(rt, gpu, mesh):
    s = Scene(rt, mesh, "BVH", env=ENV)
    try:
        g = s.render_gpu("W9E1", ELEPHANT_CAM, W, H, (0, 0, W, H), 0, 32)
        o = s.render_oracle("W9E1", ELEPHANT_CAM, W, H, (0, 0, W, H), 0, 32)
        check(g, o)
    finally:
        s.ctx.close()


def test_elephant_every_culling_mode_equals_the_unculled_walk(rt, gpu, mesh):
    F = rt._ffi
    s = Scene(rt, mesh, "BSP", env=ENV)
    try:
        out = {}
        for mode in (F.RT_BSP_CULL_OFF, F.RT_BSP_CULL_CERTIFIED, F.RT_BSP_CULL_FAST, F.RT_BSP_CULL_SILHOUETTE,
                     F.RT_BSP_CULL_AUTO):
            s.ctx.set_option(F.RT_OPT_BSP_CULL, mode)
            out[mode] = s.render_gpu("W9E1", ELEPHANT_CAM, W, H, (0, 0, W, H), 0, 64)
        ref = out[F.RT_BSP_CULL_OFF]
        for mode, g in out.items():
            assert np.array_equal(ref[0].view(np.uint32), g[0].view(np.uint32)), mode
            assert np.array_equal(ref[1], g[1]), mode
            for k in ("samples", "primary", "shadow", "bounce"):
                assert ref[2][k] == g[2][k], (mode, k)
    finally:
        s.ctx.close()
