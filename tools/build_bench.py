"""Acceleration-structure build benchmark, after the reference's
src/bin/bvh_project.rs: HLBVH construction time per phase (morton codes, radix
sort, treelet init, treelet build, upper tree, flattening) averaged over runs,
for the teapot (6,320 tris, the real asset), the bunny stand-in (69,564) and a
dragon-sized soup (871,414; dragon.obj is missing from the reference), and the
dragon-size sweep over max leaf primitives 1..16.  Beside each: this repo's
multi-threaded C++ host builder (rt_bvh_build) and the reference's published
CPU times (journal/src/benchmark.md:9-32, Ryzen 7 7735HS, leaf 4).

  python tools/build_bench.py [--runs 20] [--out FILE]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PUBLISHED_MS = {("teapot", 4): 0.993, ("bunny", 4): 4.305, ("dragon", 4): 49.28}   # benchmark.md:9-32
PUBLISHED_BSP_MS = {"teapot": 31.47, "bunny": 144.38, "dragon": 827.93}   # benchmark.md:132-171 (depth 20, leaf 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rt = importlib.import_module("02562_raytracer_amd")
    meshes = {
        "teapot": rt.Mesh.from_obj(os.path.join(ROOT, "assets", "models", "teapot.obj")),
        "bunny": rt.Mesh.synth_bunny(),
        "dragon": rt.Mesh.synth_soup(871_414),
    }
    cases = [(m, 4) for m in meshes] + [("dragon", k) for k in (1, 2, 6, 8, 16)]
    ctx = rt.Context(0)
    lines = []
    for name, mp in cases:
        mesh = meshes[name]
        ctx.upload_mesh(mesh)
        ctx.build_bvh_device(mp)   # warm-up (module load, allocations)
        acc = {}
        for _ in range(a.runs):
            t = ctx.build_bvh_device(mp)
            for k, v in t.items():
                acc[k] = acc.get(k, 0.0) + v
        gpu = {k: round(v / a.runs, 4) for k, v in acc.items() if k not in ("treelets", "nodes")}
        t0 = time.perf_counter()
        hruns = max(1, a.runs // 4)
        for _ in range(hruns):
            mesh.bvh(mp)
        host_ms = (time.perf_counter() - t0) / hruns * 1e3
        line = {"mesh": name, "ntris": mesh.ntris, "max_prims": mp, "runs": a.runs, "gpu_ms": gpu,
                "treelets": int(acc["treelets"] / a.runs), "nodes": int(acc["nodes"] / a.runs),
                "host_cpp_ms": round(host_ms, 3), "host_threads": os.cpu_count(),
                "reference_published_cpu_ms": PUBLISHED_MS.get((name, mp))}
        lines.append(line)
        print(json.dumps(line), flush=True)
    # BSP, depth 20 / leaf 4 (run_single_bsp, bvh_project.rs:90-106), plus the 10M soup of config 5
    meshes["soup10M"] = rt.Mesh.synth_soup(10_000_000)
    for name in ("teapot", "bunny", "dragon", "soup10M"):
        mesh = meshes[name]
        ctx.upload_mesh(mesh)
        ctx.build_bsp_device(20, 4)   # warm-up
        runs = a.runs if name != "soup10M" else 3
        acc = {}
        for _ in range(runs):
            t = ctx.build_bsp_device(20, 4)
            for k, v in t.items():
                acc[k] = acc.get(k, 0.0) + v
        gpu = {k: round(acc[k] / runs, 3) for k in ("subdivision_ms", "flattening_ms", "total_ms")}
        t0 = time.perf_counter()
        hruns = 1 if name == "soup10M" else max(1, runs // 4)
        for _ in range(hruns):
            mesh.bsp_tree(20, 4)
        host_ms = (time.perf_counter() - t0) / hruns * 1e3
        line = {"bsp_mesh": name, "ntris": mesh.ntris, "max_depth": 20, "max_leaf": 4, "runs": runs, "gpu_ms": gpu,
                "leaves": int(acc["leaves"] / runs), "nids": int(acc["nids"] / runs),
                "host_cpp_ms": round(host_ms, 2), "reference_published_cpu_ms": PUBLISHED_BSP_MS.get(name)}
        lines.append(line)
        print(json.dumps(line), flush=True)
    ctx.close()
    if a.out:
        with open(a.out, "w") as f:
            for l in lines:
                f.write(json.dumps(l) + "\n")


if __name__ == "__main__":
    main()
