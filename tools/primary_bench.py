"""Primary-ray frames the reference publishes frame times for (BASELINE.md,
journal/src/project.md:973-992, journal/src/img/w6_e1_*_performance.png):
one 1-spp frame of the W6E1 / PROJECT shader, BSP depth 20 (or HLBVH leaf 4).
The teapot (6,320 tris) is the reference's own asset; the bunny and dragon
files are missing from the reference, so their rows use the stand-ins
(displaced-sphere bunny, 871,414-triangle soup) and are marked as such.

  python tools/primary_bench.py [--runs 50] [--out FILE]
"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TEAPOT_CAM = ((0.15, 1.5, 10.0), (0.15, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5)      # scenes.rs teapot scenes
BUNNY_CAM = ((-0.02, 0.11, 0.6), (-0.02, 0.11, 0.0), (0.0, 1.0, 0.0), 3.5)    # scenes.rs:71-77
DRAGON_CAM = ((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.5)         # stand-in soup framing

# (name, mesh, mode, trav, W, H, camera, published ms/frame range, source)
ROWS = [
    ("teapot w6e1 BSP", "teapot", "W6E1", "BSP", 800, 450, TEAPOT_CAM, (1.79, 1.98),
     "journal/src/img/w6_e1_teapot_performance.png"),
    ("bunny w6e1 BSP (stand-in mesh)", "bunny", "W6E1", "BSP", 512, 512, BUNNY_CAM, (1.985, 2.009),
     "journal/src/img/w6_e1_bunny_performance.png"),
    ("dragon project BSP (stand-in soup)", "dragon", "PROJECT", "BSP", 800, 450, DRAGON_CAM, (13.66, 14.26),
     "journal/src/project.md:973-980"),
    ("dragon project HLBVH (stand-in soup)", "dragon", "PROJECT", "BVH", 800, 450, DRAGON_CAM, (7.78, 8.40),
     "journal/src/project.md:988-992"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=50)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rt = importlib.import_module("02562_raytracer_amd")
    meshes = {"teapot": lambda: rt.Mesh.from_obj(os.path.join(ROOT, "assets", "models", "teapot.obj")),
              "bunny": lambda: rt.Mesh.synth_bunny(), "dragon": lambda: rt.Mesh.synth_soup(871_414)}
    cache = {}
    lines = []
    for name, mk, mode, trav, W, H, cam, pub, src in ROWS:
        if mk not in cache:
            cache[mk] = meshes[mk]()
        mesh = cache[mk]
        ctx = rt.Context(0)
        ctx.upload_mesh(mesh)
        if trav == "BSP":
            ctx.upload_bsp(mesh.bsp_tree())
        else:
            ctx.upload_bvh(mesh.bvh(4))
        ctx.set_uniforms(rt.make_uniform(*cam, W, H))
        acc = ctx.alloc(W * H * 16)
        ids = ctx.alloc(W * H * 4)
        ctx.render(mode, trav, (0, 0, W, H), 0, 1, acc.ptr, ids.ptr)   # warm-up
        ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 1)
        ctx.kernel_time(reset=True)
        for _ in range(a.runs):
            ctx.render(mode, trav, (0, 0, W, H), 0, 1, acc.ptr, ids.ptr)
        tot, n = ctx.kernel_time(reset=True)
        ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 0)
        ms = tot / max(1, n)
        line = {"row": name, "ntris": mesh.ntris, "mode": mode, "traversal": trav, "resolution": [W, H],
                "kernel_ms_per_frame": round(ms, 4), "primary_mrays_s": round(W * H / ms / 1e3, 1),
                "reference_published_ms_per_frame": list(pub),
                "reference_primary_mrays_s": round(W * H / (sum(pub) / 2) / 1e3, 1), "source": src}
        lines.append(line)
        print(json.dumps(line), flush=True)
        acc.free()
        ids.free()
        ctx.close()
    if a.out:
        with open(a.out, "w") as f:
            for l in lines:
                f.write(json.dumps(l) + "\n")


if __name__ == "__main__":
    main()
