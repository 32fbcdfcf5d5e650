"""The tile gather behind the C ABI (include/rt.h "multi-GPU": rt_comm_unique_id,
rt_comm_init, rt_gather_tiles) on the box's one GPU: a 1-rank
RCCL communicator opened through the library -- no torch.distributed -- gathers
the packed tiles of rt_render_tiles and unpacks them into a frame that equals
the plain region render bit for bit.  Multi-rank frames through the same code
path run on the 8-GPU node (bench.py, --gpus N)."""
import numpy as np
import pytest

from conftest import model

pytestmark = pytest.mark.gpu


def test_one_rank_communicator_gather_equals_region_render(rt):
    W, H, spp = 200, 136, 2
    ctx = rt.Context(0)
    try:
        mesh = rt.Mesh.from_obj(model("CornellBoxWithBlocks.obj"))
        ctx.upload_mesh(mesh)
        ctx.upload_bsp(mesh.bsp_tree())
        wl = __import__("importlib").import_module("02562_raytracer_amd.configs").WORKLOADS[2]
        ctx.set_uniforms(rt.make_uniform(*wl.camera, W, H))
        uid = rt.Context.comm_unique_id()
        assert len(uid) == 128
        ctx.comm_init(1, 0, uid)
        lt = rt.local_tiles(W, H, 1)
        la, li = ctx.alloc(lt * 64 * 16), ctx.alloc(lt * 64 * 4)
        fa, fi = ctx.alloc(W * H * 16), ctx.alloc(W * H * 4)
        ra, ri = ctx.alloc(W * H * 16), ctx.alloc(W * H * 4)
        ctx.render_tiles("W7E3", "BSP", 0, 1, 0, spp, la.ptr, li.ptr)
        ctx.gather_tiles(W, H, la.ptr, li.ptr, fa.ptr, fi.ptr)
        ctx.render("W7E3", "BSP", (0, 0, W, H), 0, spp, ra.ptr, ri.ptr)
        ctx.synchronize()
        g = fa.to_numpy(np.uint32, (H, W, 4)), fi.to_numpy(np.uint32, (H, W))
        r = ra.to_numpy(np.uint32, (H, W, 4)), ri.to_numpy(np.uint32, (H, W))
        assert np.array_equal(g[0], r[0]) and np.array_equal(g[1], r[1])
        # a second communicator on the same context is refused; destroy, then re-init works
        with pytest.raises(rt.RtError):
            ctx.comm_init(1, 0, uid)
        ctx.comm_destroy()
        ctx.comm_init(1, 0, rt.Context.comm_unique_id())
        ctx.gather_tiles(W, H, la.ptr, None, fa.ptr, None)   # accumulation only
        ctx.synchronize()
        assert np.array_equal(fa.to_numpy(np.uint32, (H, W, 4)), r[0])
        for b in (la, li, fa, fi, ra, ri):
            b.free()
    finally:
        ctx.close()


def test_gather_without_communicator_is_refused(rt):
    ctx = rt.Context(0)
    try:
        with pytest.raises(rt.RtError):
            ctx.gather_tiles(64, 64, 1, None, 1, None)
    finally:
        ctx.close()
