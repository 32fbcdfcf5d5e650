"""How often the reference's HLBVH walk reaches its 1000-pop cap (bvh.wgsl:162-164) on the
BASELINE scenes: camera rays of random pixels walked by the CPU oracle (the same walk as
the kernel: the slab test on [0, 1e27] ignores the ray interval, bvh.wgsl:16-83, so a ray
visits every box its whole line crosses).  One W6E1 sample per 1x1 region (camera ray
only) gives that ray's pop count.  Tool code (CPU), not part of the product.

  python tools/bvh_cap_probe.py [configs, default 3,4,5] [rays per config, default 300]
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ffi as O  # noqa: E402


def main():
    cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "3,4,5").split(",")]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    rt = importlib.import_module("02562_raytracer_amd")
    W = importlib.import_module("02562_raytracer_amd.configs").WORKLOADS
    for c in cfgs:
        wl = W[c]
        mesh = wl.mesh()
        V, N, I, M, L = mesh.arrays()
        om = O.OracleMesh(V, N, I, M, L)
        sc = O.SceneRef(om, None, O.OracleBvh(*mesh.bvh().arrays()), env=wl.env)
        u = O.make_uniform(*wl.camera, wl.width, wl.height)
        rng = np.random.default_rng(5)
        pops, hits = [], 0
        for _ in range(n):
            x, y = int(rng.integers(wl.width)), int(rng.integers(wl.height))
            _, ids, cnt = O.render(sc, u, "W6E1", "BVH", (x, y, 1, 1), 0, 1, nthreads=1)
            pops.append(cnt["bvh_pops"])
            hits += int(ids[0, 0] != 0xFFFFFFFF)
        p = np.array(pops)
        print(f"config {c} ({mesh.ntris} tris): camera rays {n}, hit {hits / n:.3f}; pops per ray mean {p.mean():.1f}, "
              f"median {np.median(p):.0f}, p90 {np.percentile(p, 90):.0f}; at the 1000-pop cap {np.mean(p >= 1000):.3f}",
              flush=True)


if __name__ == "__main__":
    main()
