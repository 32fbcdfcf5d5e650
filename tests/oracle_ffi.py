"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE.

The oracle is the CPU checker (see oracle/oracle.h).  Only tests/, the
smoke() of __graft_entry__ and bench.py's cpu_baseline leg may use it.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

u32p = C.POINTER(C.c_uint32)
f32p = C.POINTER(C.c_float)


class Material(C.Structure):
    _fields_ = [("diffuse", C.c_float * 4), ("ambient", C.c_float * 4), ("specular", C.c_float * 4),
                ("emissive", C.c_uint32), ("_pad", C.c_uint32 * 3)]


class GpuNode(C.Structure):
    _fields_ = [("min", C.c_float * 3), ("offset_ptr", C.c_uint32), ("max", C.c_float * 3),
                ("n_prims", C.c_uint32)]


class Uniform(C.Structure):
    _fields_ = [("camera_pos", C.c_float * 3), ("camera_constant", C.c_float),
                ("camera_look_at", C.c_float * 3), ("aspect_ratio", C.c_float),
                ("camera_up", C.c_float * 3), ("selection1", C.c_uint32), ("selection2", C.c_uint32),
                ("subdivision_level", C.c_uint32), ("use_texture", C.c_uint32), ("iteration", C.c_uint32),
                ("uv_scale", C.c_float * 2), ("resolution", C.c_uint32 * 2)]


class Scene(C.Structure):
    _fields_ = [("pos", f32p), ("nrm", f32p), ("nverts", C.c_uint32),
                ("idx", u32p), ("ntris", C.c_uint32),
                ("mats", C.POINTER(Material)), ("nmats", C.c_uint32),
                ("lights", u32p), ("nlights", C.c_uint32),
                ("aabb", f32p), ("tree", u32p), ("planes", f32p), ("nnodes", C.c_uint32),
                ("ids", u32p), ("nids", C.c_uint32), ("max_depth", C.c_uint32),
                ("bvh_nodes", C.POINTER(GpuNode)), ("bvh_nnodes", C.c_uint32),
                ("bvh_ids", u32p), ("bvh_nids", C.c_uint32),
                ("env", C.c_float * 3), ("env_tex", u32p), ("env_w", C.c_uint32), ("env_h", C.c_uint32)]


COUNT_FIELDS = ["samples", "primary", "shadow", "bounce", "node_interior", "node_leaf", "bvh_pops",
                "ids_read", "tri_tests", "tri_accepts"]


class Counts(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in COUNT_FIELDS]

    def asdict(self):
        return {n: int(getattr(self, n)) for n in COUNT_FIELDS}


class Mesh(C.Structure):
    _fields_ = [("pos", f32p), ("nrm", f32p), ("idx", u32p), ("mats", C.POINTER(Material)),
                ("lights", u32p), ("nverts", C.c_uint32), ("ntris", C.c_uint32), ("nmats", C.c_uint32),
                ("nlights", C.c_uint32)]


class Bsp(C.Structure):
    _fields_ = [("tree", u32p), ("planes", f32p), ("ids", u32p), ("aabb", C.c_float * 8),
                ("nnodes", C.c_uint32), ("nids", C.c_uint32), ("max_depth", C.c_uint32)]


class Bvh(C.Structure):
    _fields_ = [("nodes", C.POINTER(GpuNode)), ("tri_ids", u32p), ("nnodes", C.c_uint32),
                ("nids", C.c_uint32)]


MODES = {"W1E6": 0, "W6E1": 1, "PROJECT": 2, "W7E3": 3, "W9E1": 4, "W8E1": 5, "W8E2": 6, "W8E3": 7, "W9E2": 8, "W6E2": 9, "W7E1": 10, "W7E2": 11, "W6E3": 12, "W9E3": 13}
TRAVS = {"BSP": 0, "BVH": 1, "NONE": 2}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(LIB_PATH)
        L.or_load_obj.argtypes = [C.c_char_p, C.POINTER(Mesh)]
        L.or_free_mesh.argtypes = [C.POINTER(Mesh)]
        L.or_bsp_build.argtypes = [f32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(Bsp)]
        L.or_free_bsp.argtypes = [C.POINTER(Bsp)]
        L.or_bsp_build_js64.argtypes = L.or_bsp_build.argtypes
        L.or_bvh_build.argtypes = [f32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32, C.POINTER(Bvh)]
        L.or_free_bvh.argtypes = [C.POINTER(Bvh)]
        L.or_light_list.argtypes = [u32p, C.c_uint32, C.POINTER(Material), C.c_uint32,
                                    C.POINTER(u32p), u32p]
        L.or_render.argtypes = [C.POINTER(Scene), C.POINTER(Uniform), f32p, C.c_int, C.c_int,
                                C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                f32p, u32p, C.POINTER(Counts), C.c_int]
        L.or_trace_one.argtypes = [C.POINTER(Scene), C.c_int, C.c_int, f32p, f32p, C.c_float, C.c_float,
                                   u32p, f32p]
        L.or_camera_ray.argtypes = [C.POINTER(Uniform), C.c_uint32, C.c_uint32, C.c_float, C.c_float, f32p, f32p]
        L.or_camera_ray.restype = None
        L.or_trace_query.argtypes = [C.POINTER(Scene), C.c_int, C.c_int, f32p, f32p, C.c_float, C.c_float,
                                     u32p, f32p, f32p, f32p, u32p, C.c_uint32, u32p]
        L.or_trace_brute.argtypes = [C.POINTER(Scene), f32p, f32p, C.c_float, C.c_float, u32p, f32p]
        L.or_render_raylog.argtypes = [C.POINTER(Scene), C.POINTER(Uniform), C.c_int, C.c_int, C.c_uint32,
                                       C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, f32p, u32p, f32p,
                                       C.c_uint32, u32p]
        for n in ("or_det_sinf", "or_det_cosf", "or_det_acosf"):
            getattr(L, n).argtypes = [C.c_float]
            getattr(L, n).restype = C.c_float
        _lib = L
    return _lib


def _arr(ptr, n, dtype, width=1):
    if n == 0:
        return np.zeros((0, width) if width > 1 else 0, dtype=dtype)
    a = np.ctypeslib.as_array(ptr, shape=(n * width,)).copy()
    return a.reshape(n, width) if width > 1 else a


def mats_to_np(mats_ptr, n):
    out = np.zeros((n, 16), dtype=np.float32)
    raw = np.ctypeslib.as_array(C.cast(mats_ptr, f32p), shape=(n * 16,)).copy()
    out[:] = raw.reshape(n, 16)
    return out


class OracleMesh:
    """Host arrays in the reference's GPU layout (src/mesh.rs:35-41)."""

    def __init__(self, pos, nrm, idx, mats, lights=None):
        self.pos = np.ascontiguousarray(pos, dtype=np.float32).reshape(-1, 4)
        self.nrm = np.ascontiguousarray(nrm if nrm is not None else np.zeros_like(self.pos),
                                        dtype=np.float32).reshape(-1, 4)
        self.idx = np.ascontiguousarray(idx, dtype=np.uint32).reshape(-1, 4)
        self.mats = np.ascontiguousarray(mats, dtype=np.float32).reshape(-1, 16)
        if lights is None:
            lights = light_list(self.idx, self.mats)
        self.lights = np.ascontiguousarray(lights, dtype=np.uint32)

    @property
    def ntris(self):
        return self.idx.shape[0]


def light_list(idx, mats):
    L = lib()
    out = u32p()
    n = C.c_uint32()
    idx = np.ascontiguousarray(idx, dtype=np.uint32)
    mats = np.ascontiguousarray(mats, dtype=np.float32)
    L.or_light_list(idx.ctypes.data_as(u32p), idx.shape[0], C.cast(mats.ctypes.data, C.POINTER(Material)),
                    mats.shape[0], C.byref(out), C.byref(n))
    arr = _arr(out, n.value, np.uint32)
    C.CDLL(None).free(out)
    return arr


def load_obj(path):
    L = lib()
    m = Mesh()
    rc = L.or_load_obj(path.encode(), C.byref(m))
    if rc != 0:
        raise IOError(f"or_load_obj({path}) = {rc}")
    res = OracleMesh(_arr(m.pos, m.nverts, np.float32, 4), _arr(m.nrm, m.nverts, np.float32, 4),
                     _arr(m.idx, m.ntris, np.uint32, 4), mats_to_np(m.mats, m.nmats),
                     _arr(m.lights, m.nlights, np.uint32))
    L.or_free_mesh(C.byref(m))
    return res


class OracleBsp:
    def __init__(self, tree, planes, ids, aabb, max_depth):
        self.tree, self.planes, self.ids, self.aabb, self.max_depth = tree, planes, ids, aabb, max_depth


def build_bsp(mesh, max_depth=20, max_leaf=4, js64=False):
    L = lib()
    b = Bsp()
    fn = L.or_bsp_build_js64 if js64 else L.or_bsp_build
    rc = fn(mesh.pos.ctypes.data_as(f32p), mesh.pos.shape[0], mesh.idx.ctypes.data_as(u32p),
                        mesh.ntris, max_depth, max_leaf, C.byref(b))
    if rc != 0:
        raise ValueError(f"or_bsp_build = {rc}")
    res = OracleBsp(_arr(b.tree, b.nnodes, np.uint32, 4), _arr(b.planes, b.nnodes, np.float32),
                    _arr(b.ids, b.nids, np.uint32), np.array(list(b.aabb), dtype=np.float32), b.max_depth)
    L.or_free_bsp(C.byref(b))
    return res


class OracleBvh:
    def __init__(self, nodes, tri_ids):
        self.nodes, self.tri_ids = nodes, tri_ids


def build_bvh(mesh, max_prims=4):
    L = lib()
    b = Bvh()
    rc = L.or_bvh_build(mesh.pos.ctypes.data_as(f32p), mesh.pos.shape[0], mesh.idx.ctypes.data_as(u32p),
                        mesh.ntris, max_prims, C.byref(b))
    if rc != 0:
        raise ValueError(f"or_bvh_build = {rc}")
    raw = np.ctypeslib.as_array(C.cast(b.nodes, u32p), shape=(b.nnodes * 8,)).copy().reshape(b.nnodes, 8)
    res = OracleBvh(raw, _arr(b.tri_ids, b.nids, np.uint32))
    L.or_free_bvh(C.byref(b))
    return res


def make_uniform(eye, target, up, constant, width, height, selection1=0, subdiv=1, aspect=None):
    u = Uniform()
    u.camera_pos[:] = [float(v) for v in eye]
    u.camera_look_at[:] = [float(v) for v in target]
    u.camera_up[:] = [float(v) for v in up]
    u.camera_constant = constant
    u.aspect_ratio = np.float32(width) / np.float32(height) if aspect is None else aspect
    u.selection1 = selection1
    u.subdivision_level = subdiv
    u.uv_scale[:] = [1.0, 1.0]
    u.resolution[:] = [width, height]
    return u


class SceneRef:
    """Keeps numpy arrays alive behind an or_scene."""

    def __init__(self, mesh, bsp=None, bvh=None, env=(1.0, 1.0, 1.0), env_tex=None):
        """env_tex: RGBA8 equirectangular texture as uint8[h, w, 4] (or None)."""
        self.mesh, self.bsp, self.bvh = mesh, bsp, bvh
        self.env_tex = None if env_tex is None else np.ascontiguousarray(env_tex, dtype=np.uint8).view(np.uint32)
        s = Scene()
        if mesh is not None:
            s.pos = mesh.pos.ctypes.data_as(f32p)
            s.nrm = mesh.nrm.ctypes.data_as(f32p)
            s.nverts = mesh.pos.shape[0]
            s.idx = mesh.idx.ctypes.data_as(u32p)
            s.ntris = mesh.ntris
            s.mats = C.cast(mesh.mats.ctypes.data, C.POINTER(Material))
            s.nmats = mesh.mats.shape[0]
            s.lights = mesh.lights.ctypes.data_as(u32p)
            s.nlights = mesh.lights.shape[0]
        if bsp is not None:
            s.aabb = bsp.aabb.ctypes.data_as(f32p)
            s.tree = bsp.tree.ctypes.data_as(u32p)
            s.planes = bsp.planes.ctypes.data_as(f32p)
            s.nnodes = bsp.tree.shape[0]
            s.ids = bsp.ids.ctypes.data_as(u32p)
            s.nids = bsp.ids.shape[0]
            s.max_depth = bsp.max_depth
        if bvh is not None:
            s.bvh_nodes = C.cast(bvh.nodes.ctypes.data, C.POINTER(GpuNode))
            s.bvh_nnodes = bvh.nodes.shape[0]
            s.bvh_ids = bvh.tri_ids.ctypes.data_as(u32p)
            s.bvh_nids = bvh.tri_ids.shape[0]
        s.env[:] = list(env)
        if self.env_tex is not None:
            s.env_tex = self.env_tex.ctypes.data_as(u32p)
            s.env_h, s.env_w = self.env_tex.shape[0], self.env_tex.shape[1]
        self.s = s


def render(scene, uniform, mode, trav, region, first_iter=0, spp=1, accum=None, jitter=None, nthreads=None):
    """Returns (accum[h,w,4] float32, ids[h,w] uint32, counts dict)."""
    L = lib()
    x0, y0, w, h = region
    if accum is None:
        accum = np.zeros((h, w, 4), dtype=np.float32)
    accum = np.ascontiguousarray(accum, dtype=np.float32)
    ids = np.zeros((h, w), dtype=np.uint32)
    cnt = Counts()
    jp = None
    if jitter is not None:
        jitter = np.ascontiguousarray(jitter, dtype=np.float32)
        jp = jitter.ctypes.data_as(f32p)
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)   # the GPU box shares 16 host threads per GPU
    rc = L.or_render(C.byref(scene.s), C.byref(uniform), jp, MODES[mode] if isinstance(mode, str) else mode,
                     TRAVS[trav] if isinstance(trav, str) else trav, x0, y0, w, h, first_iter, spp,
                     accum.ctypes.data_as(f32p), ids.ctypes.data_as(u32p), C.byref(cnt), nthreads)
    if rc != 0:
        raise ValueError(f"or_render = {rc}")
    return accum, ids, cnt.asdict()


def render_raylog(scene, uniform, mode, trav, region, first_iter=0, spp=1, cap=1 << 20):
    """render() on one thread that also returns every ray the walk received, in
    trace order: float32[n, 8] = origin, direction, tmin, tmax."""
    L = lib()
    x0, y0, w, h = region
    accum = np.zeros((h, w, 4), dtype=np.float32)
    ids = np.zeros((h, w), dtype=np.uint32)
    rays = np.zeros((cap, 8), dtype=np.float32)
    n = C.c_uint32()
    rc = L.or_render_raylog(C.byref(scene.s), C.byref(uniform), MODES[mode], TRAVS[trav], x0, y0, w, h, first_iter,
                            spp, accum.ctypes.data_as(f32p), ids.ctypes.data_as(u32p), rays.ctypes.data_as(f32p), cap,
                            C.byref(n))
    if rc != 0 or n.value > cap:
        raise ValueError(f"or_render_raylog = {rc}, {n.value} rays")
    return accum, ids, rays[:n.value].copy()


def trace_one(scene, trav, o, d, tmin, tmax, face_normals=1):
    L = lib()
    o = np.asarray(o, dtype=np.float32)
    d = np.asarray(d, dtype=np.float32)
    tri = C.c_uint32()
    dist = C.c_float()
    hit = L.or_trace_one(C.byref(scene.s), TRAVS[trav], face_normals, o.ctypes.data_as(f32p),
                         d.ctypes.data_as(f32p), tmin, tmax, C.byref(tri), C.byref(dist))
    return bool(hit), tri.value, dist.value


def trace_many(scene, trav, rays, nthreads=None):
    """or_trace_many: closest hits of rays float32[n, 8] -> (tri uint32[n], dist float32[n])."""
    rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
    n = rays.shape[0]
    tri = np.zeros(n, np.uint32)
    dist = np.zeros(n, np.float32)
    nt = nthreads or min(16, os.cpu_count() or 1)
    lib().or_trace_many(C.byref(scene.s), TRAVS[trav], n, rays.ctypes.data_as(f32p), tri.ctypes.data_as(u32p),
                        dist.ctypes.data_as(f32p), nt)
    return tri, dist


def camera_ray(uniform, x, y, jx=0.0, jy=0.0):
    """fs_main's camera ray for pixel (x, y): (origin, direction) float32[3]."""
    o = np.zeros(3, dtype=np.float32)
    d = np.zeros(3, dtype=np.float32)
    lib().or_camera_ray(C.byref(uniform), x, y, jx, jy, o.ctypes.data_as(f32p), d.ctypes.data_as(f32p))
    return o, d


def trace_query(scene, trav, o, d, tmin, tmax, clip=False, cap=4096):
    """One walk as w6e1/project issue it (optional root-AABB clip first).
    Returns dict(status -1 clipped / 0 miss / 1 hit, tri, dist, tmin, tmax,
    tested = triangle ids in test order)."""
    L = lib()
    o = np.asarray(o, dtype=np.float32)
    d = np.asarray(d, dtype=np.float32)
    tri, n = C.c_uint32(), C.c_uint32()
    dist, t0, t1 = C.c_float(), C.c_float(), C.c_float()
    log = np.zeros(cap, dtype=np.uint32)
    st = L.or_trace_query(C.byref(scene.s), TRAVS[trav], int(clip), o.ctypes.data_as(f32p), d.ctypes.data_as(f32p),
                          tmin, tmax, C.byref(tri), C.byref(dist), C.byref(t0), C.byref(t1),
                          log.ctypes.data_as(u32p), cap, C.byref(n))
    assert n.value <= cap
    return {"status": st, "tri": tri.value, "dist": dist.value, "tmin": t0.value, "tmax": t1.value,
            "tested": log[:n.value].copy()}


def trace_brute(scene, o, d, tmin, tmax):
    L = lib()
    o = np.asarray(o, dtype=np.float32)
    d = np.asarray(d, dtype=np.float32)
    tri = C.c_uint32()
    dist = C.c_float()
    hit = L.or_trace_brute(C.byref(scene.s), o.ctypes.data_as(f32p), d.ctypes.data_as(f32p), tmin, tmax,
                           C.byref(tri), C.byref(dist))
    return bool(hit), tri.value, dist.value
