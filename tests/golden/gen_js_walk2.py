"""Generates tests/golden/js_walk2_<scene>.npz: the reference's own CPU BSP walk
(js/bsp_tree/modules/BspTree_interleaved.js:237-352, run under node by
gen_js_walk.js) on SECONDARY rays -- the shadow and bounce rays the path
tracers trace from a surface point:
  * CornellBoxWithBlocks, W7E3 (w7e3.wgsl:427-470): the area-light shadow ray
    (origin on the surface, tmin = ETA = 0.01, tmax = |light point - origin| - ETA,
    :442-449) and the cosine bounce (tmin 0.01, tmax 5000, :472-489);
  * teapot, W9E1 (w9e1.wgsl:428-470): the dummy-light shadow ray (direction
    (0, 1, 0), tmin 1e-4, tmax 999999 - 1e-4) and the cosine bounce (tmin 1e-4).
The rays are the ones the CPU oracle's renders of those scenes trace (every ray
its trace() receives, oracle or_render_raylog) on the reference-built tree (the
oracle's f64 builder, equal to build_bsp_tree of the same JS file by SHA-256),
minus the camera rays, subsampled with a fixed seed.  No root-AABB clip (the
path tracers do not clip).  Each result row: status (0 miss / 1 hit), triangle
id of the last accept, distance (f64), ray tmin / tmax after the walk, number of
tested triangles and FNV-1a of their ids in order, and the same two for the tests
up to and including the first accept (what an any-hit walk tests).

usage: python tests/golden/gen_js_walk2.py [/root/reference]
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

CORNELL = ((277.0, 275.0, -570.0), (277.0, 275.0, 0.0), (0.0, 1.0, 0.0), 1.0)   # scenes.rs:63-69
TEAPOT = ((0.15, 1.5, 10.0), (0.15, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5)     # scenes.rs:55-61
# scene -> (shader, camera, resolution, spp)
SCENES = {"CornellBoxWithBlocks": ("W7E3", CORNELL, 48, 2), "teapot": ("W9E1", TEAPOT, 64, 4)}
PER_KIND = 1500
F = np.float32


def secondary_rays(name, mode, cam, res, spp):
    m = O.load_obj(os.path.join(ROOT, "assets", "models", f"{name}.obj"))
    b = O.build_bsp(m, 20, 4, js64=True)
    u = O.make_uniform(*cam, res, res, selection1=0)
    _, _, rays = O.render_raylog(O.SceneRef(m, b), u, mode, "BSP", (0, 0, res, res), 0, spp)
    eye = np.array(cam[0], F)
    sec = rays[~np.all(rays[:, :3] == eye, axis=1)]
    if mode == "W7E3":
        shadow = sec[:, 7] != F(5000.0)
    else:
        shadow = np.all(sec[:, 3:6] == np.array([0, 1, 0], F), axis=1) & (sec[:, 7] == F(999999.0) - F(1e-4))
    rng = np.random.default_rng(7)
    keep = []
    for k in (False, True):
        idx = np.nonzero(shadow == k)[0]
        keep.append(np.sort(rng.choice(idx, size=min(PER_KIND, idx.size), replace=False)))
    sel = np.sort(np.concatenate(keep))
    return m, sec[sel], shadow[sel].astype(np.int32)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    mod = os.path.join(ref, "js", "bsp_tree", "modules")
    for name, (mode, cam, res, spp) in SCENES.items():
        m, rays, kind = secondary_rays(name, mode, cam, res, spp)
        jr = [[[float(v) for v in r[:3]], [float(v) for v in r[3:6]], float(r[6]), float(r[7]), 0] for r in rays]
        inp = {"pos": [float(v) for v in m.pos[:, :3].reshape(-1)], "idx": [int(v) for v in m.idx.reshape(-1)],
               "rays": jr}
        with tempfile.TemporaryDirectory() as td:
            ip, op = os.path.join(td, "in.json"), os.path.join(td, "out.json")
            with open(ip, "w") as f:
                json.dump(inp, f)
            subprocess.run(["node", os.path.join(HERE, "gen_js_walk.js"), mod, ip, op], check=True)
            with open(op) as f:
                out = json.load(f)
        res_ = out["results"]
        col = lambda k, t: np.array([r[k] for r in res_], dtype=t)   # noqa: E731
        path = os.path.join(HERE, f"js_walk2_{name}.npz")
        np.savez_compressed(
            path,
            meta=np.array(json.dumps({"scene": name, "mode": mode, "camera": cam, "res": res, "spp": spp,
                                      "ntris": out["ntris"], "nids": out["nids"],
                                      "tree_sha256": out["tree_sha256"]})),
            ray_o=rays[:, :3].copy(), ray_d=rays[:, 3:6].copy(), ray_tmin=rays[:, 6].copy(),
            ray_tmax=rays[:, 7].copy(), kind=kind,
            status=col(0, np.int32), tri=col(1, np.int64), dist=col(2, np.float64), tmin=col(3, np.float64),
            tmax=col(4, np.float64), ntested=col(5, np.int64), seq_fnv=col(6, np.uint32),
            nfirst=col(7, np.int64), first_fnv=col(8, np.uint32))
        st = col(0, np.int32)
        print(f"{name} ({mode}): {len(rays)} rays ({int(kind.sum())} shadow), hits {int((st == 1).sum())}, "
              f"{os.path.getsize(path) // 1024} KiB")


if __name__ == "__main__":
    main()
