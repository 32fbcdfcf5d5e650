"""Subtree culling at the BASELINE spp of the 8-GPU workloads (DESIGN.md section 4
"Subtree culling"): the whole config-4 frame at 256 spp and the whole config-5
frame at 1024 spp (and config 3's at 256), rendered with RT_OPT_BSP_CULL 1
(certified margin, the default), 3 (certified with the silhouette bound), 2 (fast
margin) and 0 (every node of bsp.wgsl's walk), compared bit for bit: every pixel's accumulation, the primary-hit ids and
the ray counts.  Too long for the GPU
suite (the unculled config-5 frame takes about a minute); run once per kernel
change, its output committed under profiles/.

  python tools/cull_stress.py [configs, default 3,4,5]
"""
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def frame(rt, ctx, wl, cull):
    W, H = wl.width, wl.height
    ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, cull)
    acc = ctx.alloc(W * H * 16)
    ids = ctx.alloc(W * H * 4)
    try:
        t0 = time.perf_counter()
        c = ctx.render(wl.mode, wl.traversal, (0, 0, W, H), 0, wl.spp, acc.ptr, ids.ptr, counts=True)
        ctx.synchronize()
        el = time.perf_counter() - t0
        return acc.to_numpy(np.uint32, (H, W, 4)), ids.to_numpy(np.uint32, (H, W)), c, el
    finally:
        acc.free()
        ids.free()


def main():
    rt = importlib.import_module("02562_raytracer_amd")
    wls = importlib.import_module("02562_raytracer_amd.configs").WORKLOADS
    cfgs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "3,4,5").split(",")]
    bad_total = 0
    for n in cfgs:
        wl = wls[n]
        mesh = wl.mesh()
        ctx = rt.Context(0)
        try:
            ctx.upload_mesh(mesh)
            ctx.upload_bsp(mesh.bsp_tree())
            ctx.set_environment(wl.env)
            ctx.set_uniforms(rt.make_uniform(*wl.camera, wl.width, wl.height))
            frames = {}
            for cull, name in ((1, "certified"), (3, "silhouette"), (2, "fast"), (0, "unculled")):
                frames[name] = frame(rt, ctx, wl, cull)
                print(f"config {n}: {name} frame {frames[name][3]:.1f} s", flush=True)
        finally:
            ctx.close()
        off = frames["unculled"]
        for name in ("certified", "silhouette", "fast"):
            on = frames[name]
            px = int((on[0] != off[0]).any(axis=2).sum())
            idm = int((on[1] != off[1]).sum())
            cnt = {k: (on[2][k], off[2][k]) for k in ("samples", "primary", "shadow", "bounce")}
            same = all(a == b for a, b in cnt.values())
            rays = sum(on[2][k] for k in ("primary", "shadow", "bounce"))
            print(f"config {n}, {name}: {wl.width}x{wl.height} x {wl.spp} spp, {rays} rays: {px} pixels' accumulation "
                  f"differ, {idm} primary ids differ, ray counts {'equal' if same else cnt}", flush=True)
            bad_total += px + idm + (0 if same else 1)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
