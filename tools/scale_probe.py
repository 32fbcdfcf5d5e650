"""Projected strong scaling on one GPU: renders the rank-r share of the
interleaved tile partition for every r < N (one rank at a time, HIP-event
timed) and reports the slowest rank's kernel time per N.  Diagnostic only:
the N>1 bench runs one process per GPU.

  python tools/scale_probe.py [--config 3] [--spp 256] [--ns 1,2,4,8]
"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--trav", default=None)
    ap.add_argument("--chunks", default="1")   # the bench's one-iteration units
    ap.add_argument("--warm", type=int, default=1, help="untimed render of every share before timing it (0: only "
                    "one warm-up render, for the long configs 4 and 5)")
    args = ap.parse_args()
    import torch
    rt = importlib.import_module("02562_raytracer_amd")
    wl = importlib.import_module("02562_raytracer_amd.configs").WORKLOADS[args.config]
    W, H, spp = wl.width, wl.height, args.spp or wl.spp
    trav = args.trav or wl.traversal
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    mesh = wl.mesh(None)
    ctx = rt.Context(0)
    ctx.set_stream(stream.cuda_stream)
    ctx.upload_mesh(mesh)
    ctx.upload_bsp(mesh.bsp_tree()) if trav == "BSP" else ctx.upload_bvh(mesh.bvh())
    ctx.set_environment(wl.env)
    ctx.set_uniforms(rt.make_uniform(*wl.camera, W, H, selection1=0))
    for chunk in [int(x) for x in args.chunks.split(",")]:
        ctx.set_option(rt._ffi.RT_OPT_SAMPLE_CHUNK, chunk)
        probe(ctx, rt, wl, trav, W, H, spp, dev, stream, args, chunk)
    ctx.close()


def probe(ctx, rt, wl, trav, W, H, spp, dev, stream, args, chunk):
    import torch
    out = {}
    if not args.warm:   # one warm-up launch for the whole probe
        lt = rt.local_tiles(W, H, 8)
        acc = torch.empty((lt * 64, 4), dtype=torch.float32, device=dev)
        ctx.render_tiles(wl.mode, trav, 0, 8, 0, min(spp, 4), acc.data_ptr(), None)
        torch.cuda.synchronize(dev)
    for n in [int(x) for x in args.ns.split(",")]:
        lt = rt.local_tiles(W, H, n)
        acc = torch.empty((lt * 64, 4), dtype=torch.float32, device=dev)
        ids = torch.empty((lt * 64,), dtype=torch.int32, device=dev)
        ms = []
        for r in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if args.warm:
                ctx.render_tiles(wl.mode, trav, r, n, 0, spp, acc.data_ptr(), ids.data_ptr())   # warm
                # (drained before timing, as the bench drains its warm-up: RT_BSP_CULL_AUTO reads
                # its probe's events at the next render only once they have completed)
                torch.cuda.synchronize(dev)
            e0.record(stream)
            ctx.render_tiles(wl.mode, trav, r, n, 0, spp, acc.data_ptr(), ids.data_ptr())
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms.append(e0.elapsed_time(e1))
        out[n] = {"max_ms": round(max(ms), 3), "mean_ms": round(sum(ms) / n, 3),
                  "rank_ms": [round(x, 3) for x in ms]}
        print(json.dumps({"chunk": chunk, "n": n, **out[n]}), flush=True)
    t1 = out[min(out)]["max_ms"]
    print(json.dumps({"chunk": chunk, "projected_speedup": {n: round(t1 / v["max_ms"], 2) for n, v in out.items()}}))


if __name__ == "__main__":
    main()
