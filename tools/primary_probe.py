"""Diagnostics for the primary-ray kernel on the reference's teapot W6E1 frame:
counters of the counting instantiation and kernel time vs waves per CU."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rt = importlib.import_module("02562_raytracer_amd")
    mesh = rt.Mesh.from_obj(os.path.join(ROOT, "assets", "models", "teapot.obj"))
    ctx = rt.Context(0)
    ctx.upload_mesh(mesh)
    ctx.upload_bsp(mesh.bsp_tree())
    W, H = 800, 450
    ctx.set_uniforms(rt.make_uniform((0.15, 1.5, 10.0), (0.15, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5, W, H))
    acc = ctx.alloc(W * H * 16)
    ids = ctx.alloc(W * H * 4)
    ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 1)
    c = ctx.render("W6E1", "BSP", (0, 0, W, H), 0, 1, acc.ptr, ids.ptr, counts=True)
    ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 0)
    print(json.dumps({k: v for k, v in c.items() if v}))
    for wpc in (4, 8, 16, 32):
        ctx.set_option(rt._ffi.RT_OPT_WAVES_PER_CU, wpc)
        ctx.render("W6E1", "BSP", (0, 0, W, H), 0, 1, acc.ptr, ids.ptr)
        ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 1)
        ctx.kernel_time(reset=True)
        for _ in range(20):
            ctx.render("W6E1", "BSP", (0, 0, W, H), 0, 1, acc.ptr, ids.ptr)
        t, n = ctx.kernel_time(reset=True)
        ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 0)
        print(json.dumps({"waves_per_cu": wpc, "kernel_ms": round(t / n, 4)}))
    ctx.close()


if __name__ == "__main__":
    main()
