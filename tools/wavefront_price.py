"""Price of a wavefront split of the W9E1 path tracer (DESIGN.md
section 4 "Outside the megakernel"), measured on the real ray stream.

One process on one GPU:
  1. a counting render of the workload (k_path's counting instantiation) with the
     ray capture armed (rt_set_ray_capture): every camera, shadow and bounce ray
     the frame traces, in issue order, lands in HBM (36 B per ray, rt_trace_rays' layout);
  2. the megakernel frame, timed (HIP events around each k_path launch);
  3. the captured stream through the traversal-only persistent kernel
     (rt_trace_batch, k_trace: the walk with no shading state), timed the same
     way -- the trace stage of a wavefront renderer, on exactly the rays the
     megakernel traced;
  4. the split's queue traffic per ray, priced at the HBM peak (its best case):
     the ray written by the shade stage and read by the trace stage (32 + 32 B),
     the hit record written and read (8 + 8 B), the path state read and written
     by the shade stage (2 x 64 B: radiance, blocked sum, throughput, PRNG state,
     pixel, iteration, primary id, bounce count, flags).
Prints one JSON line.  usage: python tools/wavefront_price.py [--config 3] [--spp N] [--reps 3]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12
QUEUE_BYTES_PER_RAY = 32 + 32 + 8 + 8 + 2 * 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--bsp-cull", type=int, default=None)
    ap.add_argument("--threshold", type=int, default=None, help="k_trace's refill threshold (default 16)")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    rt = importlib.import_module("02562_raytracer_amd")
    wl = importlib.import_module("02562_raytracer_amd.configs").WORKLOADS[args.config]
    W, H, spp = wl.width, wl.height, args.spp or wl.spp
    if args.config == 5 and args.spp is None:
        spp = 32   # 650 M rays, 23 GB of captured stream (the full 1024 spp would not fit)
    t0 = time.perf_counter()
    mesh = wl.mesh()
    ctx = rt.Context(0)
    if args.bsp_cull is not None:
        ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, args.bsp_cull)
    ctx.upload_mesh(mesh)
    ctx.upload_bsp(mesh.bsp_tree())
    ctx.set_environment(wl.env)
    ctx.set_uniforms(rt.make_uniform(*wl.camera, W, H))
    acc, ids = ctx.alloc(W * H * 16), ctx.alloc(W * H * 4)
    print(f"[wf] setup {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)

    def frame(counting=False):
        ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 1 if counting else 0)
        c = ctx.render(wl.mode, "BSP", (0, 0, W, H), 0, spp, acc.ptr, ids.ptr, counts=True)
        ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 0)
        return c

    c = frame(counting=True)
    nrays = c["primary"] + c["shadow"] + c["bounce"]
    cap = int(nrays * 1.02) + 1024
    rb, fb, hb = ctx.alloc(32 * cap), ctx.alloc(4 * cap), ctx.alloc(8 * cap)
    ctx.set_ray_capture(rb.ptr, fb.ptr, cap)
    frame(counting=True)
    n = ctx.ray_capture_count()
    ctx.set_ray_capture(None)
    assert n == nrays <= cap, (n, nrays, cap)
    print(f"[wf] captured {n} rays", file=sys.stderr, flush=True)

    ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 1)
    frame()
    ctx.kernel_time(reset=True)
    for _ in range(args.reps):
        frame()
    kp, kl = ctx.kernel_time(reset=True)
    if args.threshold is not None:
        ctx.set_option(rt._ffi.RT_OPT_SHADE_THRESHOLD, args.threshold)
    ctx.trace_batch("BSP", rb.ptr, fb.ptr, n, hb.ptr)
    ctx.kernel_time(reset=True)
    for _ in range(args.reps):
        ctx.trace_batch("BSP", rb.ptr, fb.ptr, n, hb.ptr)
    tt, tl = ctx.kernel_time(reset=True)
    ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 0)
    hits = hb.to_numpy(np.uint32, (n, 2))
    kpath_ms = kp / args.reps          # one frame: all its k_path launches
    trace_ms = tt / args.reps
    queue_ms = n * QUEUE_BYTES_PER_RAY / HBM_PEAK * 1e3
    line = {
        "config": args.config, "workload": f"{wl.name}, {W}x{H}, {spp} spp", "culling": args.bsp_cull,
        "rays_traced": int(n), "primary": int(c["primary"]), "shadow": int(c["shadow"]), "bounce": int(c["bounce"]),
        "k_path_ms_per_frame": round(kpath_ms, 3), "k_path_launches_per_frame": kl // args.reps,
        "k_trace_ms": round(trace_ms, 3),
        "k_trace_grays_per_s": round(n / trace_ms / 1e6, 3),
        "k_path_grays_per_s_traced": round(n / kpath_ms / 1e6, 3),
        "trace_over_megakernel": round(trace_ms / kpath_ms, 4),
        "queue_bytes_per_ray": QUEUE_BYTES_PER_RAY,
        "queue_ms_at_hbm_peak": round(queue_ms, 3),
        "wavefront_floor_ms": round(trace_ms + queue_ms, 3),
        "wavefront_floor_over_megakernel": round((trace_ms + queue_ms) / kpath_ms, 4),
        "hit_fraction": round(float((hits[:, 0] != 0xFFFFFFFF).mean()), 4),
        "note": "wavefront_floor = the trace stage alone + its queue traffic at the HBM peak (no shading "
                "arithmetic, no launch gaps): a lower bound on a wavefront frame",
    }
    print(json.dumps(line), flush=True)
    for b in (rb, fb, hb, acc, ids):
        b.free()
    ctx.close()


if __name__ == "__main__":
    main()
