"""Shared helpers for GPU-vs-oracle parity tests (test infrastructure)."""
import numpy as np

import oracle_ffi as O

CORNELL_CAM = ((277.0, 275.0, -570.0), (277.0, 275.0, 0.0), (0.0, 1.0, 0.0), 1.0)
BUNNY_CAM = ((-0.02, 0.11, 0.6), (-0.02, 0.11, 0.0), (0.0, 1.0, 0.0), 3.5)
TEAPOT_CAM = ((0.15, 1.5, 10.0), (0.15, 1.5, 0.0), (0.0, 1.0, 0.0), 2.5)
BASIC_CAM = ((2.0, 1.5, 2.0), (0.0, 0.5, 0.0), (0.0, 1.0, 0.0), 1.0)

RADIANCE_TOL = 1e-4   # north_star: image L-infinity < 1e-4 vs the reference path


class Scene:
    """One mesh + acceleration structure on both sides: the product builds and
    uploads its own (rt.Mesh -> BspTree/Bvh -> Context), the oracle builds its
    own from the same triangle arrays."""

    def __init__(self, rt, mesh, trav, env=(1.0, 1.0, 1.0), oracle_mesh=None, device=0, oracle_accel_from_product=False,
                 bsp_depth=20, bsp_leaf=4):
        """oracle_accel_from_product: the oracle renders from the product
        builder's arrays instead of building its own (they are bit-identical,
        tests/test_host_builders.py) -- for the 7M/10M-triangle configs, where
        the single-threaded oracle build would dominate the test."""
        ctx = rt.Context(device)   # one context per scene: uploads never clobber another test's scene
        self.rt, self.ctx, self.trav, self.env = rt, ctx, trav, env
        self.mesh = mesh
        V, N, I, M, L = mesh.arrays()
        self.om = oracle_mesh if oracle_mesh is not None else O.OracleMesh(V, N, I, M, L)
        ctx.upload_mesh(mesh)
        self.obsp = self.obvh = None
        if trav == "BSP":
            bsp = mesh.bsp_tree(bsp_depth, bsp_leaf)
            ctx.upload_bsp(bsp)
            self.obsp = (O.OracleBsp(*bsp.arrays()) if oracle_accel_from_product
                         else O.build_bsp(self.om, bsp_depth, bsp_leaf))
        elif trav == "BVH":
            bvh = mesh.bvh()
            ctx.upload_bvh(bvh)
            self.obvh = O.OracleBvh(*bvh.arrays()) if oracle_accel_from_product else O.build_bvh(self.om)
        ctx.set_environment(env)
        self.oscene = O.SceneRef(self.om, self.obsp, self.obvh, env)

    def render_gpu(self, mode, cam, W, H, region, first_iter=0, spp=1, selection1=0, accum_in=None,
                   tileset=None, jitter=None):
        rt, ctx = self.rt, self.ctx
        subdiv = 1 if jitter is None else int(round(np.sqrt(len(jitter))))
        u = rt.make_uniform(*cam, W, H, selection1=selection1, subdiv=subdiv)
        ctx.set_uniforms(u, None if jitter is None else np.ascontiguousarray(jitter, dtype=np.float32))
        x0, y0, w, h = region
        acc = ctx.alloc(w * h * 16)
        ids = ctx.alloc(w * h * 4)
        if accum_in is not None:
            acc.from_numpy(np.ascontiguousarray(accum_in, dtype=np.float32))
        else:
            acc.zero()
        cnt = ctx.render(mode, self.trav, region, first_iter, spp, acc.ptr, ids.ptr, counts=True)
        a = acc.to_numpy(np.float32, (h, w, 4))
        i = ids.to_numpy(np.uint32, (h, w))
        acc.free()
        ids.free()
        return a, i, cnt

    def render_oracle(self, mode, cam, W, H, region, first_iter=0, spp=1, selection1=0, accum_in=None,
                      nthreads=None, jitter=None):
        subdiv = 1 if jitter is None else int(round(np.sqrt(len(jitter))))
        u = O.make_uniform(*cam, W, H, selection1=selection1, subdiv=subdiv)
        return O.render(self.oscene, u, mode, self.trav, region, first_iter, spp, accum=accum_in, nthreads=nthreads,
                        jitter=None if jitter is None else np.ascontiguousarray(jitter, dtype=np.float32))


def compare(gpu, ora, what=""):
    """Returns (max abs radiance diff, #bit mismatches, #id mismatches).  The
    L-inf is infinite when the two sides disagree on a non-finite value: NaN
    against a number, an infinity against a finite value, or +inf against -inf
    (such differences vanish from a finite-only max)."""
    ga, gi, gc = gpu
    oa, oi, oc = ora
    diff = np.abs(ga.astype(np.float64) - oa.astype(np.float64))
    finite = np.isfinite(diff)
    linf = float(diff[finite].max()) if finite.any() else 0.0
    both_nan = np.isnan(ga) & np.isnan(oa)   # NaN payload/sign is not a value (x86 0/0 = -qNaN)
    nan_mismatch = int((np.isnan(ga) != np.isnan(oa)).sum())
    inf_mismatch = int(((np.isinf(ga) | np.isinf(oa)) & (ga != oa)).sum())
    bits = int(((ga.view(np.uint32) != oa.view(np.uint32)) & ~both_nan).sum())
    idm = int((gi != oi).sum())
    return linf + (np.inf if nan_mismatch or inf_mismatch else 0.0), bits, idm
