"""Generates tests/golden/js_walk_<scene>.npz: results of the reference's own
CPU BSP walk (js/bsp_tree/modules/BspTree_interleaved.js:237-352, run under node
by gen_js_walk.js) on a committed ray set.

Rays (float32, stored exactly):
  * the 64x64 camera rays of fs_main (w6e1.wgsl / project.wgsl: tmin ETA = 1e-5,
    tmax 1e5, root-AABB clip first), made by the oracle's camera (the kernel's
    camera is bit-identical to it: tests/test_gpu_parity.py);
  * random rays from inside / around the mesh box (no clip; tmin 1e-4, tmax 1e4);
  * axis-aligned rays (zero direction components; no clip).
Each result: [status (-1 clipped / 0 miss / 1 hit), triangle id of the last accept,
distance (f64), ray tmin / tmax after the walk (f64), number of triangle tests,
FNV-1a of the tested ids in order].  The tree hash (SHA-256 of the JS bspTree,
bspPlanes and treeIds arrays) pins the builder of that same file.

usage: python tests/golden/gen_js_walk.py [/root/reference]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import oracle_ffi as O   # noqa: E402

BASIC = ((2.0, 1.5, 2.0), (0.0, 0.5, 0.0), (0.0, 1.0, 0.0), 1.0)          # scenes.rs:47-53
CORNELL = ((277.0, 275.0, -570.0), (277.0, 275.0, 0.0), (0.0, 1.0, 0.0), 1.0)   # scenes.rs:63-69
TEAPOT = ((0.15, 1.5, 10.0), (0.15, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5)     # scenes.rs:55-61
SCENES = {"test_object": BASIC, "CornellBox": CORNELL, "CornellBoxWithBlocks": CORNELL, "teapot": TEAPOT}
RES = 64
N_RANDOM = 1024
F = np.float32


def rays_for(mesh, cam, seed):
    rays = []
    u = O.make_uniform(*cam, RES, RES)
    for y in range(RES):
        for x in range(RES):
            o, d = O.camera_ray(u, x, y)
            rays.append((o, d, F(1e-5), F(1e5), 1))
    p = mesh.pos[:, :3]
    lo, hi = p.min(axis=0), p.max(axis=0)
    ext = hi - lo
    rng = np.random.default_rng(seed)
    for _ in range(N_RANDOM):
        o = rng.uniform(lo - 0.2 * ext, hi + 0.2 * ext).astype(F)
        d = rng.normal(size=3).astype(F)
        d = (d / F(np.sqrt(F(np.dot(d, d))))).astype(F)
        rays.append((o, d, F(1e-4), F(1e4), 0))
    for _ in range(64):
        o = rng.uniform(lo - 0.2 * ext, hi + 0.2 * ext).astype(F)
        d = np.zeros(3, dtype=F)
        k = rng.integers(0, 3)
        d[k] = F(1.0) if rng.random() < 0.5 else F(-1.0)
        if rng.random() < 0.5:   # two components, one zero
            j = (k + 1 + rng.integers(0, 2)) % 3
            d[j] = F(rng.uniform(-1, 1))
            d = (d / F(np.sqrt(F(np.dot(d, d))))).astype(F)
        rays.append((o, d, F(1e-4), F(1e4), 0))
    return rays


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    mod = os.path.join(ref, "js", "bsp_tree", "modules")
    for i, (name, cam) in enumerate(SCENES.items()):
        m = O.load_obj(os.path.join(ROOT, "assets", "models", f"{name}.obj"))
        rays = rays_for(m, cam, 100 + i)
        jr = [[[float(v) for v in o], [float(v) for v in d], float(t0), float(t1), c] for o, d, t0, t1, c in rays]
        inp = {"pos": [float(v) for v in m.pos[:, :3].reshape(-1)], "idx": [int(v) for v in m.idx.reshape(-1)],
               "rays": jr}
        with tempfile.TemporaryDirectory() as td:
            ip, op = os.path.join(td, "in.json"), os.path.join(td, "out.json")
            with open(ip, "w") as f:
                json.dump(inp, f)
            subprocess.run(["node", os.path.join(HERE, "gen_js_walk.js"), mod, ip, op], check=True)
            with open(op) as f:
                out = json.load(f)
        res = out["results"]
        path = os.path.join(HERE, f"js_walk_{name}.npz")
        np.savez_compressed(
            path,
            meta=np.array(json.dumps({"scene": name, "camera": cam, "res": RES, "ntris": out["ntris"],
                                      "nids": out["nids"], "tree_sha256": out["tree_sha256"]})),
            ray_o=np.array([r[0] for r in rays], dtype=F), ray_d=np.array([r[1] for r in rays], dtype=F),
            ray_tmin=np.array([r[2] for r in rays], dtype=F), ray_tmax=np.array([r[3] for r in rays], dtype=F),
            ray_clip=np.array([r[4] for r in rays], dtype=np.int32),
            status=np.array([r[0] for r in res], dtype=np.int32), tri=np.array([r[1] for r in res], dtype=np.int64),
            dist=np.array([r[2] for r in res], dtype=np.float64), tmin=np.array([r[3] for r in res], dtype=np.float64),
            tmax=np.array([r[4] for r in res], dtype=np.float64), ntested=np.array([r[5] for r in res], dtype=np.int64),
            seq_fnv=np.array([r[6] for r in res], dtype=np.uint32))
        st = np.array([r[0] for r in res])
        print(f"{name}: {len(rays)} rays, hits {int((st == 1).sum())}, clipped {int((st == -1).sum())}, "
              f"{os.path.getsize(path) // 1024} KiB")


if __name__ == "__main__":
    main()
