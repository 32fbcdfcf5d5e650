"""Whole-frame parity pin of a BASELINE workload at its BASELINE spp, too long for the
GPU suite (test infrastructure: run on the GPU box, its output committed under
profiles/).  The GPU frame (the library's default culling, one launch per pass) and
the CPU oracle's frame (every node of bsp.wgsl's walk, the product builder's arrays,
every thread of the box's share) are compared bit for bit: every pixel's accumulated
radiance word, the primary-hit id, the ray counts.  Config 4 (the 7M-triangle bunny
grid, 1920x1080 x 256 spp = 531 M samples) extends tests/test_gpu_configs.py's centre
quarter to the whole frame.

  python tests/pin_full_frame.py --config 4 [--spp N] [--trav BVH]
Prints one JSON line; exit status 1 if anything differs."""
import argparse
import importlib
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from parity_util import Scene, compare  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--trav", default=None, choices=["BSP", "BVH"], help="the walk (default: the workload's)")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    rt = importlib.import_module("02562_raytracer_amd")
    wl = importlib.import_module("02562_raytracer_amd.configs").WORKLOADS[a.config]
    spp = a.spp or wl.spp
    W, H = wl.width, wl.height
    t0 = time.perf_counter()
    trav = a.trav or wl.traversal
    s = Scene(rt, wl.mesh(), trav, env=wl.env, oracle_accel_from_product=True)
    t1 = time.perf_counter()
    g = s.render_gpu(wl.mode, wl.camera, W, H, (0, 0, W, H), 0, spp)
    used = s.ctx.bsp_cull_in_use()
    t2 = time.perf_counter()
    print(f"[pin] setup {t1 - t0:.1f} s, GPU frame {t2 - t1:.1f} s; oracle frame on {a.threads} threads ...",
          file=sys.stderr, flush=True)
    # heartbeat: the oracle call runs for minutes without output (ctypes releases the GIL)
    stop = threading.Event()

    def beat():
        while not stop.wait(30.0):
            print(f"[pin] oracle running, {time.perf_counter() - t2:.0f} s", file=sys.stderr, flush=True)

    hb = threading.Thread(target=beat, daemon=True)
    hb.start()
    try:
        o = s.render_oracle(wl.mode, wl.camera, W, H, (0, 0, W, H), 0, spp, nthreads=a.threads)
    finally:
        stop.set()
    t3 = time.perf_counter()
    linf, bits, idm = compare(g, o)
    counts = {k: [int(g[2][k]), int(o[2][k])] for k in ("samples", "primary", "shadow", "bounce")}
    same = bits == 0 and idm == 0 and all(x == y for x, y in counts.values())
    print(json.dumps({
        "config": a.config, "workload": f"{wl.name}, {W}x{H}, {spp} spp", "samples": W * H * spp, "traversal": trav,
        "gpu_culling": {0: "off", 1: "certified", 2: "fast", 3: "silhouette"}[used[0]] if trav == "BSP" else None,
        "radiance_words_differing": int(bits), "primary_ids_differing": int(idm), "radiance_linf": linf,
        "ray_counts_gpu_oracle": counts, "equal": bool(same),
        "oracle_s": round(t3 - t2, 1), "oracle_threads": a.threads}), flush=True)
    s.ctx.close()
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
