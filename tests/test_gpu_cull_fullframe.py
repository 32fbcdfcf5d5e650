"""Subtree culling (RT_OPT_BSP_CULL, DESIGN.md section 4 "Subtree culling") on
the BASELINE workloads at full size: every frame rendered with culling on --
certified (exact by proof), silhouette (round 5's camera bound,
exact by proof), the timed choice between those two (auto) and fast (the round-3 margin, exact by these
measurements only) -- equals the frame rendered with it off -- the reference's walk,
bsp.wgsl:10-81, which the rest of the suite pins to the oracle and the oracle
to the reference's own JS walk -- bit for bit: every pixel's accumulated
radiance (any single sample that differed would change its pixel's average),
the primary-hit ids and the ray counts.  These are the frames the bench
renders: config 2 at its 64 spp, configs 3 and 4 at their 256 spp (800 M and
180 M rays per frame, with the silhouette and grazing rays of the whole
image), config 5 at 4K with 16 of its 1024 spp."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def configs():
    return importlib.import_module("02562_raytracer_amd.configs").WORKLOADS


def _frame(rt, ctx, wl, spp, cull):
    W, H = wl.width, wl.height
    ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, cull)
    ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 1)
    acc = ctx.alloc(W * H * 16)
    ids = ctx.alloc(W * H * 4)
    try:
        c = ctx.render(wl.mode, wl.traversal, (0, 0, W, H), 0, spp, acc.ptr, ids.ptr, counts=True)
        return acc.to_numpy(np.uint32, (H, W, 4)), ids.to_numpy(np.uint32, (H, W)), c
    finally:
        acc.free()
        ids.free()


@pytest.mark.parametrize("config,spp", [(2, 64), (3, 256), (4, 256), (5, 16)])
def test_full_frame_cull_equals_reference_walk(rt, gpu, configs, config, spp):
    wl = configs[config]
    mesh = wl.mesh()
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh(mesh)
        ctx.upload_bsp(mesh.bsp_tree())
        ctx.set_environment(wl.env)
        ctx.set_uniforms(rt.make_uniform(*wl.camera, wl.width, wl.height))
        off = _frame(rt, ctx, wl, spp, rt._ffi.RT_BSP_CULL_OFF)
        ons = [_frame(rt, ctx, wl, spp, m) for m in (rt._ffi.RT_BSP_CULL_CERTIFIED, rt._ffi.RT_BSP_CULL_FAST,
                                                      rt._ffi.RT_BSP_CULL_SILHOUETTE, rt._ffi.RT_BSP_CULL_AUTO)]
        chosen = ctx.bsp_cull_in_use()
    finally:
        ctx.close()
    assert off[2]["subtree_culls"] == 0
    for on, name in zip(ons, ("certified", "fast", "silhouette", "auto")):
        diff = int((off[0] != on[0]).any(axis=2).sum())
        assert diff == 0, f"config {config}: {diff} pixels' radiance differs with {name} culling"
        assert np.array_equal(off[1], on[1]), f"primary-hit ids differ with {name} culling"
        for k in ("samples", "primary", "shadow", "bounce"):
            assert off[2][k] == on[2][k], (name, k, off[2][k], on[2][k])
        # the work culling saves (printed for the log; the bench reports it too)
        print(f"config {config} {name}: culls {on[2]['subtree_culls']}, interior nodes "
              f"{on[2]['node_interior'] / off[2]['node_interior']:.3f}, "
              f"triangle tests {on[2]['tri_tests'] / off[2]['tri_tests']:.3f} of the unculled walk")
    # both modes really cull (the certified one too: a mode that culled nothing
    # would pass the equalities above trivially)
    assert all(on[2]["subtree_culls"] > 0 for on in ons)
    print(f"config {config}: RT_BSP_CULL_AUTO ran mode {chosen[0]} (probe: certified {chosen[1]:.2f} ms, "
          f"silhouette {chosen[2]:.2f} ms)")
