"""ctypes binding of lib02562rt.so (include/rt.h).

The shared library holds the gfx950 kernels, the C ABI and the host builders.
There is no fallback: if the library is missing every call raises, so a GPU
test can never pass on a silent CPU path.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RT_LIBRARY selects an experimental build variant (see the Makefile knobs);
# the default is the in-tree library
LIB_PATH = os.environ.get("RT_LIBRARY") or os.path.join(PKG_DIR, "lib02562rt.so")

RT_OK = 0
RT_E_INVALID = -1
RT_E_OOM = -2
RT_E_DEVICE = -3
RT_E_NOT_READY = -4
RT_E_IO = -5
RT_E_UNSUPPORTED = -6

(RT_MODE_W1E6, RT_MODE_W6E1, RT_MODE_PROJECT, RT_MODE_W7E3, RT_MODE_W9E1, RT_MODE_W8E1, RT_MODE_W8E2, RT_MODE_W8E3,
 RT_MODE_W9E2, RT_MODE_W6E2, RT_MODE_W7E1, RT_MODE_W7E2, RT_MODE_W6E3, RT_MODE_W9E3) = range(14)
RT_TRAVERSE_BSP, RT_TRAVERSE_BVH, RT_TRAVERSE_NONE = range(3)
RT_OPT_DETAIL_COUNTERS = 1
RT_OPT_WAVES_PER_CU = 2
RT_OPT_SHADE_THRESHOLD = 3
RT_OPT_SAMPLE_CHUNK = 4
RT_OPT_SAMPLE_BUDGET_MB = 5
RT_OPT_UNIT_ORDER = 6
RT_OPT_BSP_CULL = 9
RT_OPT_ASYNC_FOLD = 10
RT_BSP_CULL_OFF, RT_BSP_CULL_CERTIFIED, RT_BSP_CULL_FAST, RT_BSP_CULL_SILHOUETTE, RT_BSP_CULL_AUTO = range(5)
BSP_TREELET_BYTES = 96   # rt_internal.h: the BSP walk's treelet (rt_download_bsp_treelets)
RT_OPT_KERNEL_TIMING = 7
RT_COMM_ID_BYTES = 128

MODES = {"W1E6": RT_MODE_W1E6, "W6E1": RT_MODE_W6E1, "PROJECT": RT_MODE_PROJECT, "W7E3": RT_MODE_W7E3,
         "W9E1": RT_MODE_W9E1, "W8E1": RT_MODE_W8E1, "W8E2": RT_MODE_W8E2, "W8E3": RT_MODE_W8E3,
         "W9E2": RT_MODE_W9E2, "W6E2": RT_MODE_W6E2, "W7E1": RT_MODE_W7E1, "W7E2": RT_MODE_W7E2,
         "W6E3": RT_MODE_W6E3, "W9E3": RT_MODE_W9E3}
# progressive path tracers (per-iteration samples folded in order)
PATH_MODES = ("W7E3", "W9E1", "W8E1", "W8E2", "W8E3", "W9E2", "W7E1", "W7E2", "W9E3")
TRAVERSALS = {"BSP": RT_TRAVERSE_BSP, "BVH": RT_TRAVERSE_BVH, "NONE": RT_TRAVERSE_NONE}

u32p = C.POINTER(C.c_uint32)
f32p = C.POINTER(C.c_float)
vp = C.c_void_p


class Material(C.Structure):          # src/mesh.rs:12-20
    _fields_ = [("diffuse", C.c_float * 4), ("ambient", C.c_float * 4), ("specular", C.c_float * 4),
                ("emissive", C.c_uint32), ("_pad", C.c_uint32 * 3)]


class GpuNode(C.Structure):           # src/data_structures/hlbvh.rs:508-515
    _fields_ = [("min", C.c_float * 3), ("offset_ptr", C.c_uint32), ("max", C.c_float * 3),
                ("n_prims", C.c_uint32)]


class BvhBuildTimes(C.Structure):    # include/rt.h rt_bvh_build_times (bvh_util.rs BvhConstructionTime)
    _fields_ = [(n, C.c_double) for n in ("morton_codes_ms", "radix_sort_ms", "treelet_init_ms",
                                          "treelet_build_ms", "upper_tree_ms", "upper_tree_host_ms",
                                          "flattening_ms", "total_ms")] + [("treelets", C.c_uint32),
                                                                            ("nodes", C.c_uint32)]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class BspBuildTimes(C.Structure):    # include/rt.h rt_bsp_build_times
    _fields_ = [("subdivision_ms", C.c_double), ("flattening_ms", C.c_double), ("total_ms", C.c_double),
                ("levels", C.c_uint32), ("leaves", C.c_uint32), ("nids", C.c_uint32)]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class Uniform(C.Structure):           # src/bindings/uniform.rs:6-34
    _fields_ = [("camera_pos", C.c_float * 3), ("camera_constant", C.c_float),
                ("camera_look_at", C.c_float * 3), ("aspect_ratio", C.c_float),
                ("camera_up", C.c_float * 3), ("selection1", C.c_uint32), ("selection2", C.c_uint32),
                ("subdivision_level", C.c_uint32), ("use_texture", C.c_uint32), ("iteration", C.c_uint32),
                ("uv_scale", C.c_float * 2), ("resolution", C.c_uint32 * 2)]


class Tile(C.Structure):
    _fields_ = [("x0", C.c_uint32), ("y0", C.c_uint32), ("w", C.c_uint32), ("h", C.c_uint32)]


class Tileset(C.Structure):
    _fields_ = [("rank", C.c_uint32), ("nranks", C.c_uint32)]


COUNT_FIELDS = ["samples", "primary", "shadow", "bounce", "node_interior", "node_leaf", "bvh_pops",
                "ids_read", "tri_tests", "tri_accepts", "trips", "lane_steps", "leaf_lane_steps",
                "node_trips", "leaf_trips", "exact_tests", "exact_nodes", "shade_passes",
                "shade_lanes", "trav_cycles", "shade_cycles", "memwait_cycles", "subtree_culls"]


class RayCounts(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in COUNT_FIELDS]

    def asdict(self):
        return {n: int(getattr(self, n)) for n in COUNT_FIELDS}


class MeshView(C.Structure):
    _fields_ = [("vertices", f32p), ("normals", f32p), ("indices", u32p), ("materials", C.POINTER(Material)),
                ("lights", u32p), ("nverts", C.c_uint32), ("ntris", C.c_uint32), ("nmats", C.c_uint32),
                ("nlights", C.c_uint32)]


class BspView(C.Structure):
    _fields_ = [("tree", u32p), ("planes", f32p), ("ids", u32p), ("aabb", C.c_float * 8),
                ("nnodes", C.c_uint32), ("nids", C.c_uint32), ("max_depth", C.c_uint32)]


class BvhView(C.Structure):
    _fields_ = [("nodes", C.POINTER(GpuNode)), ("tri_ids", u32p), ("nnodes", C.c_uint32), ("nids", C.c_uint32)]


# name -> (restype, argtypes); mirrors include/rt.h one to one
SIGNATURES = {
    "rt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rt_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "rt_destroy": (None, [vp]),
    "rt_set_stream": (C.c_int, [vp, vp]),
    "rt_get_stream": (vp, [vp]),
    "rt_synchronize": (C.c_int, [vp]),
    "rt_set_option": (C.c_int, [vp, C.c_int, C.c_int64]),
    "rt_bsp_cull_in_use": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_float), C.POINTER(C.c_uint32)]),
    "rt_last_error": (C.c_char_p, [vp]),
    "rt_device_alloc": (C.c_int, [vp, C.c_size_t, C.POINTER(vp)]),
    "rt_device_free": (C.c_int, [vp, vp]),
    "rt_memcpy_to_host": (C.c_int, [vp, vp, vp, C.c_size_t]),
    "rt_memcpy_to_device": (C.c_int, [vp, vp, vp, C.c_size_t]),
    "rt_memset_device": (C.c_int, [vp, vp, C.c_int, C.c_size_t]),
    "rt_timer_start": (C.c_int, [vp]),
    "rt_timer_stop": (C.c_int, [vp, f32p]),
    "rt_frame_rgba8": (C.c_int, [vp, vp, C.c_uint32, vp]),
    "rt_kernel_time": (C.c_int, [vp, C.c_int, C.POINTER(C.c_double), u32p]),
    "rt_gather_time": (C.c_int, [vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), u32p]),
    "rt_build_bvh_device": (C.c_int, [vp, C.c_uint32, C.POINTER(BvhBuildTimes)]),
    "rt_build_bsp_device": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.POINTER(BspBuildTimes)]),
    "rt_download_bsp": (C.c_int, [vp, u32p, f32p, C.c_uint32, u32p, C.c_uint32, f32p, u32p, u32p]),
    "rt_download_bsp_treelets": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "rt_download_bvh": (C.c_int, [vp, C.POINTER(GpuNode), C.c_uint32, u32p, C.c_uint32, u32p, u32p]),
    "rt_upload_mesh": (C.c_int, [vp, f32p, f32p, C.c_uint32, u32p, C.c_uint32, C.POINTER(Material), C.c_uint32,
                                 u32p, C.c_uint32]),
    "rt_upload_bsp": (C.c_int, [vp, f32p, u32p, f32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32]),
    "rt_upload_bvh": (C.c_int, [vp, C.POINTER(GpuNode), C.c_uint32, u32p, C.c_uint32]),
    "rt_set_uniforms": (C.c_int, [vp, C.POINTER(Uniform), f32p]),
    "rt_set_environment": (C.c_int, [vp, f32p]),
    "rt_set_environment_map": (C.c_int, [vp, C.POINTER(C.c_uint8), C.c_uint32, C.c_uint32]),
    "rt_render": (C.c_int, [vp, C.c_int, C.c_int, C.POINTER(Tile), C.c_uint32, C.c_uint32, vp, vp,
                            C.POINTER(RayCounts)]),
    "rt_render_tiles": (C.c_int, [vp, C.c_int, C.c_int, C.POINTER(Tileset), C.c_uint32, C.c_uint32, vp, vp,
                                  C.POINTER(RayCounts)]),
    "rt_tileset_local_tiles": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32]),
    "rt_unpack_tiles": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, vp]),
    "rt_comm_unique_id": (C.c_int, [vp]),
    "rt_comm_init": (C.c_int, [vp, C.c_uint32, C.c_uint32, vp]),
    "rt_comm_destroy": (C.c_int, [vp]),
    "rt_gather_tiles": (C.c_int, [vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp]),
    "rt_trace_rays": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint32, vp]),
    "rt_trace_batch": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint32, vp]),
    "rt_set_ray_capture": (C.c_int, [vp, vp, vp, C.c_uint64]),
    "rt_ray_capture_count": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
    "rt_last_counts": (C.c_int, [vp, C.POINTER(RayCounts)]),
    "rt_selftest_math": (C.c_int, [vp, C.c_uint32, C.c_float, C.c_float, u32p]),
    "rt_mesh_load_obj": (C.c_int, [C.c_char_p, C.POINTER(vp)]),
    "rt_mesh_from_arrays": (C.c_int, [f32p, f32p, C.c_uint32, u32p, C.c_uint32, C.POINTER(Material), C.c_uint32,
                                      C.POINTER(vp)]),
    "rt_mesh_synth_bunny": (C.c_int, [C.c_uint32, C.c_uint32, C.POINTER(vp)]),
    "rt_mesh_synth_soup": (C.c_int, [C.c_uint32, C.c_uint32, C.POINTER(vp)]),
    "rt_mesh_synth_grid": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_float, C.POINTER(vp)]),
    "rt_mesh_scale": (C.c_int, [vp, C.c_float]),
    "rt_mesh_view_get": (C.c_int, [vp, C.POINTER(MeshView)]),
    "rt_mesh_free": (None, [vp]),
    "rt_bsp_build": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(vp)]),
    "rt_bsp_view_get": (C.c_int, [vp, C.POINTER(BspView)]),
    "rt_bsp_free": (None, [vp]),
    "rt_bvh_build": (C.c_int, [vp, C.c_uint32, C.POINTER(vp)]),
    "rt_bvh_view_get": (C.c_int, [vp, C.POINTER(BvhView)]),
    "rt_bvh_free": (None, [vp]),
    "rt_upload_mesh_host": (C.c_int, [vp, vp]),
    "rt_upload_bsp_host": (C.c_int, [vp, vp]),
    "rt_upload_bvh_host": (C.c_int, [vp, vp]),
}

_lib = None


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


def lib():
    """Load lib02562rt.so (raises loudly when it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C 02562_raytracer_amd)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("RT_LIBRARY") and not hasattr(L, name):
                continue   # an A/B variant built from an earlier tree (tools/ab.sh) may lack a newer entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != RT_OK:
        msg = lib().rt_last_error(ctx)
        raise RtError(rc, msg.decode() if msg else "")
    return rc


def as_f32p(a):
    return a.ctypes.data_as(f32p)


def as_u32p(a):
    return a.ctypes.data_as(u32p)


def np_from(ptr, n, dtype, width=1):
    """Copy n*width elements from a C pointer into a new numpy array."""
    if n == 0:
        return np.zeros((0, width) if width > 1 else (0,), dtype=dtype)
    raw = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n * width,))
    out = raw.copy()
    return out.reshape(n, width) if width > 1 else out
