"""Trip-count model of k_path's BSP walk under walk variants (tools/walk_sim.c).
Rays: camera rays of a workload (random pixels, jittered), the W9E1 shadow ray
of every hit (any-hit, direction (0, 1, 0), [1e-4, 999999 - 1e-4]) and a
cosine bounce about the face normal.  usage: python tools/walk_sim.py [config] [rays]"""
import ctypes
import os
import subprocess
import sys
import time
from importlib import import_module

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ffi as O  # noqa: E402

NAMES = ["walk_trips", "leaf_trips", "decisions", "leaf_visits", "empty_leaves", "tests", "pushes", "pops", "hits",
         "mismatch", "box_tests"]


def lib():
    src = os.path.join(ROOT, "tools", "walk_sim.c")
    so = "/tmp/walk_sim.so"
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", so, src], check=True)
    return ctypes.CDLL(so)


def main():
    cfgn = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    cfg = import_module("02562_raytracer_amd.configs").WORKLOADS[cfgn]
    mesh = cfg.mesh()
    tree, planes, ids, aabb, D = mesh.bsp_tree(20, 4).arrays()
    pos, nrm, idx, mats, lights = mesh.arrays()
    import types
    m = types.SimpleNamespace(pos=pos, nrm=nrm, idx=idx, ntris=idx.shape[0], mats=np.ascontiguousarray(mats),
                              lights=lights)
    b = types.SimpleNamespace(aabb=aabb, tree=tree, planes=planes, ids=ids, max_depth=D)
    sc = O.SceneRef(m, b)
    u = O.make_uniform(*cfg.camera, cfg.width, cfg.height)
    rng = np.random.default_rng(1)
    rays, flags = [], []
    t0 = time.time()
    # WALK_COHERENT=k: k consecutive samples of each pixel (the kernel's pixel-major units)
    coh = int(os.environ.get("WALK_COHERENT", "1"))
    for r_ in range(nr):
        if r_ % coh == 0:
            x, y = int(rng.integers(cfg.width)), int(rng.integers(cfg.height))
        o, d = O.camera_ray(u, x, y, float(rng.random()) / cfg.height, float(rng.random()) / cfg.height)
        rays.append([*o, *d, 1e-4, 5000.0])
        flags.append(0)
        hit, tri, dist = O.trace_one(sc, "BSP", o, d, 1e-4, 5000.0)
        if hit:
            p = (o + d * np.float32(dist)).astype(np.float32)
            rays.append([*p, 0.0, 1.0, 0.0, 1e-4, np.float32(999999.0) - np.float32(1e-4)])
            flags.append(1)
            v0, v1, v2 = (pos[idx[tri, k], :3] for k in range(3))
            n = np.cross(v1 - v0, v2 - v0)
            n = n / np.linalg.norm(n)
            if np.dot(n, d) > 0:
                n = -n
            a = rng.normal(size=3)
            a = a - n * np.dot(a, n)
            a /= np.linalg.norm(a)
            c = np.sqrt(rng.random())
            w = (n * np.sqrt(1 - c * c) + a * c).astype(np.float32)
            rays.append([*p, *w, 1e-4, 5000.0])
            flags.append(0)
    if os.environ.get("WALK_STRESS"):
        # grazing secondary rays: origin on a random triangle, direction nearly in
        # its plane (elevation 1e-7 .. 1e-2 rad), tmin = 1e-4 (the W9E1 ETA)
        rays, flags = [], []
        P3 = pos[:, :3].astype(np.float64)
        for _ in range(nr):
            tri = int(rng.integers(idx.shape[0]))
            v0, v1, v2 = (P3[idx[tri, k]] for k in range(3))
            u, v = rng.random(), rng.random()
            if u + v > 1:
                u, v = 1 - u, 1 - v
            p = (v0 + u * (v1 - v0) + v * (v2 - v0)).astype(np.float32)
            n = np.cross(v1 - v0, v2 - v0)
            n /= np.linalg.norm(n)
            a = rng.normal(size=3)
            a -= n * np.dot(a, n)
            a /= np.linalg.norm(a)
            el = 10.0 ** rng.uniform(-7, -2) * (1 if rng.random() < 0.5 else -1)
            w = (a * np.cos(el) + n * np.sin(el)).astype(np.float32)
            rays.append([*p, *w, 1e-4, 5000.0])
            flags.append(int(rng.random() < 0.5))
    R = np.ascontiguousarray(np.array(rays, np.float32))
    F = np.ascontiguousarray(np.array(flags, np.uint32))
    if os.environ.get("WALK_RAYS"):   # 0: camera rays only, 1: shadow, 2: bounce (the list's 3-ray groups)
        kind = np.zeros(len(R), int)
        i = 0
        while i < len(R):   # camera ray, then its shadow + bounce when it hit
            if i + 2 < len(R) and F[i + 1] == 1:
                kind[i + 1], kind[i + 2] = 1, 2
                i += 3
            else:
                i += 1
        keep = kind == int(os.environ["WALK_RAYS"])
        R, F = np.ascontiguousarray(R[keep]), np.ascontiguousarray(F[keep])
    out = np.zeros(55, np.float64)
    # content boxes of every node's subtree (v3), bottom-up from the leaves' triangles
    boxes = None
    if os.environ.get("WALK_BOXES"):
        n = tree.shape[0]
        boxes = np.empty((n, 6), np.float32)
        boxes[:, :3] = np.inf
        boxes[:, 3:] = -np.inf
        P3 = pos[:, :3]
        tb_lo = np.minimum(np.minimum(P3[idx[:, 0]], P3[idx[:, 1]]), P3[idx[:, 2]])
        tb_hi = np.maximum(np.maximum(P3[idx[:, 0]], P3[idx[:, 1]]), P3[idx[:, 2]])
        leaf = (tree[:, 0] & 3) == 3
        cnt = tree[:, 0] >> 2
        lv = np.nonzero(leaf & (cnt > 0))[0]
        first = tree[lv, 1].astype(np.int64)

        def leaf_reduce(vals, red):
            # per non-empty leaf: red over its triangles' vals (leaf ranges are contiguous in ids order)
            order = np.argsort(first, kind="stable")
            st = first[order]
            v = vals[ids]
            out = np.empty((len(lv),) + vals.shape[1:], vals.dtype)
            out[order] = red.reduceat(v, st, axis=0)
            return out

        def up(arr, red):
            # bottom-up union over interior nodes, one depth level at a time
            dmax = int(np.floor(np.log2(n + 1)))
            for dd in range(dmax, -1, -1):
                a, b = 2 ** dd - 1, min(2 ** (dd + 1) - 1, n)
                i = np.arange(a, b)
                i = i[(~leaf[i]) & (2 * i + 2 < n)]
                arr[i] = red(arr[2 * i + 1], arr[2 * i + 2])

        boxes[lv, :3] = leaf_reduce(tb_lo, np.minimum)
        boxes[lv, 3:] = leaf_reduce(tb_hi, np.maximum)
        up(boxes, lambda x, y: np.concatenate([np.minimum(x[:, :3], y[:, :3]), np.maximum(x[:, 3:], y[:, 3:])], 1))
        # conservative expansion: 2^-k of the scene's coordinate magnitude (WALK_MARGIN_LG, default 14)
        scale = float(np.abs(pos[:, :3]).max())
        mg = np.float32(scale * 2.0 ** -float(os.environ.get("WALK_MARGIN_LG", "14")))
        boxes[:, :3] -= mg
        boxes[:, 3:] += mg
        boxes = np.ascontiguousarray(boxes)
        if os.environ.get("WALK_CERT"):
            # raw content boxes (the certified margin is applied per ray) and the
            # per-subtree certification data: E2 and the box of n*/(2 E2)
            boxes[:, :3] += mg
            boxes[:, 3:] -= mg
            V32 = pos[:, :3].astype(np.float32)
            v0, v1, v2 = V32[idx[:, 0]], V32[idx[:, 1]], V32[idx[:, 2]]
            e0 = (v1 - v0).astype(np.float32).astype(np.float64)
            e1 = (v2 - v0).astype(np.float32).astype(np.float64)
            nst = np.cross(e0, e1)
            Et2 = np.maximum(np.abs(e0).max(1), np.abs(e1).max(1)) ** 2
            cert = np.zeros((n, 7))
            e2 = np.zeros(n)
            e2[lv] = leaf_reduce(Et2, np.maximum)
            up(e2, np.maximum)
            cert[:, 0] = e2
            lo_raw = np.full((n, 3), np.inf)
            hi_raw = np.full((n, 3), -np.inf)
            lo_raw[lv] = leaf_reduce(nst, np.minimum)
            hi_raw[lv] = leaf_reduce(nst, np.maximum)
            up(lo_raw, np.minimum)
            up(hi_raw, np.maximum)
            ok = cert[:, 0] > 0
            cert[ok, 1:4] = lo_raw[ok] / (2 * cert[ok, 0, None])
            cert[ok, 4:7] = hi_raw[ok] / (2 * cert[ok, 0, None])
            cert[~ok, 0] = 1.0
            cert = np.ascontiguousarray(cert)
            if os.environ.get("WALK_CELLS"):
                cells = np.empty((n, 6))
                cells[0, :3] = -np.inf
                cells[0, 3:] = np.inf
                for dd in range(0, int(np.floor(np.log2(n + 1)))):
                    a, b = 2 ** dd - 1, min(2 ** (dd + 1) - 1, n)
                    i = np.arange(a, b)
                    i = i[(~leaf[i]) & (2 * i + 2 < n)]
                    ax = (tree[i, 0] & 3).astype(np.int64)
                    pl = planes[i].astype(np.float64)
                    L_, R_ = 2 * i + 1, 2 * i + 2
                    cells[L_] = cells[i]
                    cells[R_] = cells[i]
                    cells[L_, 3 + ax] = pl
                    cells[R_, ax] = pl
                occ = np.empty((n, 6))
                occ[:, :3] = np.inf
                occ[:, 3:] = -np.inf
                occ[lv] = cells[lv]
                up(occ, lambda x, y: np.concatenate([np.minimum(x[:, :3], y[:, :3]), np.maximum(x[:, 3:], y[:, 3:])], 1))
                occ = np.ascontiguousarray(occ)
                print("occupied-cell boxes: unbounded sides at the root", int(np.isinf(occ[0]).sum()))
            boxes = np.ascontiguousarray(boxes)
    L = lib()
    P = ctypes.c_void_p
    L.walk_sim_levels(int(os.environ.get("WALK_LEVELS", "3")))
    L.walk_sim_boxes(P(boxes.ctypes.data) if boxes is not None else None)
    if boxes is not None and os.environ.get("WALK_CERT"):
        L.walk_sim_cert.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_int]
        L.walk_sim_cert(cert.ctypes.data, float(np.abs(pos[:, :3]).max()), int(os.environ.get("WALK_CERT_FLOOR", "0")))
        if os.environ.get("WALK_CELLS"):
            L.walk_sim_cells(P(occ.ctypes.data))
        if os.environ.get("WALK_SHADOW"):
            hy = np.full(n, np.inf)
            hy[lv] = leaf_reduce(np.abs(nst[:, 1]), np.minimum)
            up(hy, np.minimum)
            hy = np.ascontiguousarray(np.where(np.isfinite(hy), hy / cert[:, 0], 0.0))
            L.walk_sim_hy(P(hy.ctypes.data))
        if os.environ.get("WALK_CAM"):
            eye = np.asarray(cfg.camera[0], np.float32)
            hn = np.abs(((v0.astype(np.float64) - eye.astype(np.float64)) * nst).sum(1)) / np.maximum(Et2, 1e-300)
            hcam = np.full(n, np.inf)
            hcam[lv] = leaf_reduce(hn, np.minimum)
            up(hcam, np.minimum)
            hcam = np.ascontiguousarray(hcam)
            if os.environ.get("WALK_CAMX"):
                hn_c = np.ascontiguousarray(hn)
                L.walk_sim_camx(P(tree.ctypes.data), P(ids.ctypes.data), ctypes.c_uint32(n), P(hn_c.ctypes.data),
                                int(os.environ["WALK_CAMX"]))
                L.walk_sim_camx_bound(int(os.environ.get("WALK_CAMX_BOUND", "0")))
            L.walk_sim_cam.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float]
            L.walk_sim_cam(hcam.ctypes.data, *[float(x) for x in eye])
    L.walk_sim_spec(int(os.environ.get("WALK_SPEC", "0")))
    L.walk_sim_root_only(int(os.environ.get("WALK_ROOT_ONLY", "0")))
    L.walk_sim_axis(int(os.environ.get("WALK_AXIS", "1")))
    L.walk_sim_cull_every(int(os.environ.get("WALK_CULL_EVERY", "0")))
    L.walk_sim_clip(int(os.environ.get("WALK_CLIP", "0")))
    L.walk_sim_chunk.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float]
    L.walk_sim_chunk(int(os.environ.get("WALK_CHUNK", "0")), int(os.environ.get("WALK_CHUNK_MIN", "0")),
                     int(os.environ.get("WALK_CHUNK_FREE", "0")),
                     float(np.abs(pos[:, :3]).max()) * 2.0 ** -float(os.environ.get("WALK_MARGIN_LG", "14")))
    trace = toff = None
    if os.environ.get("WALK_TRACE"):   # the v4 walk's per-ray trip sequences -> an .npz (two_ray_price.py)
        trace = np.zeros(len(R) * 4096, np.uint8)
        toff = np.zeros(len(R) + 1, np.uint64)
        L.walk_sim_trace(P(trace.ctypes.data), ctypes.c_uint64(trace.size), P(toff.ctypes.data))
    L.walk_sim(P(tree.ctypes.data), P(planes.ctypes.data), P(ids.ctypes.data), P(np.ascontiguousarray(pos).ctypes.data),
               P(np.ascontiguousarray(idx).ctypes.data), P(R.ctypes.data), P(F.ctypes.data), ctypes.c_uint32(len(R)),
               P(out.ctypes.data))
    out = out.reshape(5, 11)
    if trace is not None:
        L.walk_sim_trace_len.restype = ctypes.c_uint64
        n = int(L.walk_sim_trace_len())
        toff[len(R)] = n
        kind = np.zeros(len(R), np.uint8)   # 0 camera, 1 shadow, 2 bounce (generation order, as WALK_RAYS)
        i = 0
        while i < len(R):
            if i + 2 < len(R) and F[i + 1] == 1:
                kind[i + 1], kind[i + 2] = 1, 2
                i += 3
            else:
                i += 1
        np.savez(os.environ["WALK_TRACE"], trace=trace[:n], off=toff, kind=kind)
        L.walk_sim_trace(None, ctypes.c_uint64(0), None)
    ks = np.array([4, 6, 8, 10, 12, 16], np.uint32)
    tr = np.zeros(4 * len(ks), np.float64)
    L.trail_sim(P(tree.ctypes.data), P(planes.ctypes.data), P(ids.ctypes.data), P(np.ascontiguousarray(pos).ctypes.data),
                P(np.ascontiguousarray(idx).ctypes.data), P(R.ctypes.data), P(F.ctypes.data), ctypes.c_uint32(len(R)),
                P(ks.ctypes.data), ctypes.c_uint32(len(ks)), P(tr.ctypes.data))
    tr = tr.reshape(len(ks), 4) / len(R)
    for k, row in zip(ks, tr):
        print(f"compact trail K={k}: per ray {row[0]:.2f} pushes, {row[1]:.3f} overwrite a pending entry, "
              f"{row[2]:.2f} pops, {row[3]:.3f} pops of a lost entry (recompute)")
    bad = np.zeros(256)
    nb = L.walk_sim_bad(P(bad.ctypes.data))
    for k in range(nb):
        i, v, t0, tv = bad[4 * k:4 * k + 4]
        r = R[int(i)]
        print(f"MISMATCH ray {int(i)} v{int(v)}: v0 tri {int(t0)} vs {int(tv)}; ray {r.tolist()} anyhit {F[int(i)]}")
        if t0 >= 0:
            tri = int(t0)
            vv = pos[idx[tri, :3], :3]
            print("   v0 hit triangle verts", vv.tolist())
    if boxes is not None:
        cu = np.zeros(33)
        L.walk_sim_culls(P(cu.ctypes.data))
        print("culls per ray by depth:", {d: round(v / len(R), 3) for d, v in enumerate(cu[:32]) if v},
              "of which at leaves:", round(cu[32] / len(R), 3))
    if boxes is not None and os.environ.get("WALK_CERT"):
        L.walk_sim_cert_mean.restype = ctypes.c_double
        print("mean certified margin", L.walk_sim_cert_mean())
        lo_ = np.zeros(4)
        L.walk_sim_lost(P(lo_.ctypes.data))
        print("fast culls lost by the certified test per ray: cone regime %.3f, floor regime %.3f" % (lo_[0] / len(R), lo_[1] / len(R)))
        if os.environ.get("WALK_CAMX"):
            cx = np.zeros(4)
            L.walk_sim_camx_stats(P(cx.ctypes.data))
            print("camx per ray: culls won %.3f, excluded-triangle tests %.3f, refused %.4f, checks %.3f"
                  % tuple(v / len(R) for v in cx))
    if os.environ.get("WALK_SPEC"):
        sp = np.zeros(8)
        L.walk_sim_spec_stats(P(sp.ctypes.data))
        print("speculative cull per ray: flagged %.4f, spec-only culls %.4f, spec-only clip decisions %.4f, "
              "proven culls %.3f, re-walk trips %.3f, re-walk tests %.3f" % tuple(v / len(R) for v in sp[:6]))
    print(f"config {cfgn}: {len(R)} rays ({sum(flags)} any-hit), {time.time() - t0:.1f} s")
    for v in range(5 if boxes is not None else 3):
        s = {k: round(out[v, i] / len(R), 3) for i, k in enumerate(NAMES)}
        s["mismatch"] = int(out[v, 9])
        s["box_tests"] = round(out[v, 10] / len(R), 3)
        tr = out[v, 0] + out[v, 1]
        print(f"v{v}", s, "trips/ray", round(tr / len(R), 3), "vs v0", round(tr / (out[0, 0] + out[0, 1]), 4))


if __name__ == "__main__":
    main()
