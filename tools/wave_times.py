"""Where a k_path launch's fixed cost goes: every wave's start and end time (the
diagnostic build `make DEFS=-DRT_DBG_WAVE_TIMES`, run through RT_LIBRARY; the product
build has no such code), for the full config-3 frame and rank 0's share of an N-rank
split.  Prints, per launch, the kernel time (HIP events), when the waves started
(spread), the quantiles of their end times, and the tail: the time from the moment
half / 90 % / 99 % of the waves had finished to the last one.  Tool code.

  RT_LIBRARY=02562_raytracer_amd/variants/wt/lib02562rt.so python tools/wave_times.py [--shares 1,8] [--spp 256]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shares", default="1,8")
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    rt = importlib.import_module("02562_raytracer_amd")
    wl = importlib.import_module("02562_raytracer_amd.configs").WORKLOADS[a.config]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    W, H = wl.width, wl.height
    mesh = wl.mesh()
    ctx = rt.Context(0)
    ctx.set_stream(stream.cuda_stream)
    ctx.upload_mesh(mesh)
    ctx.build_bsp_device(20, 4)
    ctx.set_environment(wl.env)
    ctx.set_uniforms(rt.make_uniform(*wl.camera, W, H))
    ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, rt._ffi.RT_BSP_CULL_CERTIFIED)
    nw = 256 * 32   # waves of the persistent grid (num_CUs x 32)
    buf = torch.zeros((nw, 4), dtype=torch.float32, device=dev)
    flg = torch.zeros((nw,), dtype=torch.int32, device=dev)
    for n in [int(x) for x in a.shares.split(",")]:
        lt = rt.local_tiles(W, H, n)
        acc = torch.empty((lt * 64, 4), dtype=torch.float32, device=dev)
        ids = torch.empty((lt * 64,), dtype=torch.int32, device=dev)
        ctx.render_tiles(wl.mode, "BSP", 0, n, 0, a.spp, acc.data_ptr(), ids.data_ptr())   # warm
        torch.cuda.synchronize(dev)
        for rep in range(a.reps):
            buf.zero_()
            ctx.set_ray_capture(buf.data_ptr(), flg.data_ptr(), nw)
            ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 1)
            ctx.kernel_time(reset=True)
            ctx.render_tiles(wl.mode, "BSP", 0, n, 0, a.spp, acc.data_ptr(), ids.data_ptr())
            torch.cuda.synchronize(dev)
            kms, _ = ctx.kernel_time(reset=True)
            ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 0)
            ctx.set_ray_capture(None)
            b = buf.cpu().numpy().view(np.uint32)
            used = (b[:, 0] | b[:, 1]) != 0
            t0 = (b[used, 0].astype(np.uint64) | (b[used, 1].astype(np.uint64) << np.uint64(32))).astype(np.float64)
            t1 = b[used, 2].astype(np.float64)   # low 32 bits of the end time
            t1 = t1 + np.floor((t0 - (t0 % 2 ** 32)) / 1.0)   # same high word (a launch is far below 42 s)
            t1 = np.where(t1 < t0, t1 + 2 ** 32, t1)
            xcc = b[used, 3]
            base = t0.min()
            s, e = (t0 - base) / 100.0, (t1 - base) / 100.0   # 100-MHz clock -> microseconds
            q = np.percentile(e, [50, 90, 99, 100])
            out = {"share": f"rank 0 of {n}", "spp": a.spp, "kernel_ms": round(kms, 3), "waves": int(used.sum()),
                   "start_spread_us": round(float(s.max()), 1),
                   "end_us_p50_p90_p99_max": [round(float(x), 1) for x in q],
                   "tail_after_p50_us": round(float(q[3] - q[0]), 1),
                   "tail_after_p90_us": round(float(q[3] - q[1]), 1),
                   "tail_after_p99_us": round(float(q[3] - q[2]), 1),
                   "last_end_per_xcd_us": [round(float(e[xcc == k].max()), 1) if (xcc == k).any() else None
                                           for k in range(8)]}
            print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
