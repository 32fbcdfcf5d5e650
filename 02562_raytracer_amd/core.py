"""Host-side objects over the C ABI: Mesh, BspTree, Bvh (the Rust structures
that feed the GPU, src/mesh.rs and src/data_structures/) and Context (the
HIP device/stream handle that replaces src/gpu_handles.rs plus the GPU
binding layer src/bindings/)."""
import ctypes as C

import numpy as np

from . import _ffi as F


def _mats_from(ptr, n):
    if n == 0:
        return np.zeros((0, 16), dtype=np.float32)
    raw = np.ctypeslib.as_array(C.cast(ptr, F.f32p), shape=(n * 16,)).copy()
    return raw.reshape(n, 16)


class Mesh:
    """Mesh (src/mesh.rs:35-41): vertices/normals float4, indices (v0,v1,v2,material)."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle) if not isinstance(handle, C.c_void_p) else handle

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and F._lib is not None:
            F._lib.rt_mesh_free(self._h)
            self._h = C.c_void_p(None)

    @property
    def handle(self):
        return self._h

    # -- constructors -----------------------------------------------------
    @classmethod
    def from_obj(cls, path):
        """Mesh::from_obj (src/mesh.rs:78-92)."""
        h = C.c_void_p()
        F.check(F.lib().rt_mesh_load_obj(str(path).encode(), C.byref(h)))
        return cls(h)

    @classmethod
    def from_arrays(cls, vertices, indices, normals=None, materials=None):
        pos = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 4)
        idx = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1, 4)
        nrm = None if normals is None else np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 4)
        mats = None if materials is None else np.ascontiguousarray(materials, dtype=np.float32).reshape(-1, 16)
        h = C.c_void_p()
        F.check(F.lib().rt_mesh_from_arrays(F.as_f32p(pos), None if nrm is None else F.as_f32p(nrm), pos.shape[0],
                                            F.as_u32p(idx), idx.shape[0],
                                            None if mats is None else C.cast(mats.ctypes.data, C.POINTER(F.Material)),
                                            0 if mats is None else mats.shape[0], C.byref(h)))
        return cls(h)

    @classmethod
    def synth_bunny(cls, ntris=69451, seed=0x0B0B):
        h = C.c_void_p()
        F.check(F.lib().rt_mesh_synth_bunny(ntris, seed, C.byref(h)))
        return cls(h)

    @classmethod
    def synth_soup(cls, ntris, seed=0x5EED):
        h = C.c_void_p()
        F.check(F.lib().rt_mesh_synth_soup(ntris, seed, C.byref(h)))
        return cls(h)

    @classmethod
    def grid(cls, src, nx, nz, spacing):
        h = C.c_void_p()
        F.check(F.lib().rt_mesh_synth_grid(src.handle, nx, nz, spacing, C.byref(h)))
        return cls(h)

    def scale(self, factor):
        """Mesh::scale (src/mesh.rs:246-252)."""
        F.check(F.lib().rt_mesh_scale(self._h, factor))
        return self

    # -- views --------------------------------------------------------------
    def _view(self):
        v = F.MeshView()
        F.check(F.lib().rt_mesh_view_get(self._h, C.byref(v)))
        return v

    @property
    def ntris(self):
        return int(self._view().ntris)

    def arrays(self):
        """Copies: (vertices[n,4], normals[n,4], indices[t,4], materials[m,16], lights[l])."""
        v = self._view()
        return (F.np_from(v.vertices, v.nverts, np.float32, 4), F.np_from(v.normals, v.nverts, np.float32, 4),
                F.np_from(v.indices, v.ntris, np.uint32, 4), _mats_from(v.materials, v.nmats),
                F.np_from(v.lights, v.nlights, np.uint32))

    # -- acceleration structures (src/mesh.rs:229-239) -------------------
    def bsp_tree(self, max_depth=20, max_leaf=4, nthreads=0):
        return BspTree.build(self, max_depth, max_leaf, nthreads)

    def bvh(self, max_prims=4):
        return Bvh.build(self, max_prims)


class BspTree:
    """BspTree + BspTreeIntermediate (src/data_structures/bsp_tree.rs:45-347)."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and F._lib is not None:
            F._lib.rt_bsp_free(self._h)
            self._h = C.c_void_p(None)

    @classmethod
    def build(cls, mesh, max_depth=20, max_leaf=4, nthreads=0):
        h = C.c_void_p()
        F.check(F.lib().rt_bsp_build(mesh.handle, max_depth, max_leaf, nthreads, C.byref(h)))
        return cls(h)

    @property
    def handle(self):
        return self._h

    def arrays(self):
        """(bsp_tree[n,4] u32, bsp_planes[n] f32, tree_ids[k] u32, aabb[8] f32, max_depth)."""
        v = F.BspView()
        F.check(F.lib().rt_bsp_view_get(self._h, C.byref(v)))
        return (F.np_from(v.tree, v.nnodes, np.uint32, 4), F.np_from(v.planes, v.nnodes, np.float32),
                F.np_from(v.ids, v.nids, np.uint32), np.array(list(v.aabb), dtype=np.float32), int(v.max_depth))


class Bvh:
    """hlbvh::Bvh flattened (src/data_structures/hlbvh.rs:195-239)."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and F._lib is not None:
            F._lib.rt_bvh_free(self._h)
            self._h = C.c_void_p(None)

    @classmethod
    def build(cls, mesh, max_prims=4):
        h = C.c_void_p()
        F.check(F.lib().rt_bvh_build(mesh.handle, max_prims, C.byref(h)))
        return cls(h)

    @property
    def handle(self):
        return self._h

    def arrays(self):
        """(nodes[n,8] u32 view of GpuNode, tri_ids[k] u32)."""
        v = F.BvhView()
        F.check(F.lib().rt_bvh_view_get(self._h, C.byref(v)))
        raw = F.np_from(C.cast(v.nodes, F.u32p), v.nnodes, np.uint32, 8)
        return raw, F.np_from(v.tri_ids, v.nids, np.uint32)


def make_uniform(eye, target, up, constant, width, height, selection1=0, subdiv=1, aspect=None, iteration=0):
    """Uniform (src/bindings/uniform.rs:6-34) for a headless W x H frame."""
    u = F.Uniform()
    u.camera_pos[:] = [float(v) for v in eye]
    u.camera_look_at[:] = [float(v) for v in target]
    u.camera_up[:] = [float(v) for v in up]
    u.camera_constant = float(constant)
    u.aspect_ratio = float(np.float32(width) / np.float32(height)) if aspect is None else float(aspect)
    u.selection1 = selection1
    u.subdivision_level = subdiv
    u.iteration = iteration
    u.uv_scale[:] = [1.0, 1.0]
    u.resolution[:] = [width, height]
    return u


# include/rt.h rt_ray_hit
RAY_HIT_DTYPE = np.dtype([("tri", "<u4"), ("dist", "<f4"), ("beta", "<f4"), ("gamma", "<f4"), ("ntested", "<u4"),
                          ("tested_fnv", "<u4"), ("tmin", "<f4"), ("tmax", "<f4")])


class DeviceBuffer:
    """HBM allocation owned by a Context (frame buffers)."""

    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        F.check(F.lib().rt_device_alloc(ctx.handle, self.nbytes, C.byref(p)), ctx.handle)
        self.ptr = p.value

    def free(self):
        if self.ptr:
            F.lib().rt_device_free(self.ctx.handle, C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            if self.ptr and F._lib is not None and self.ctx.handle:
                self.free()
        except Exception:
            pass

    def to_numpy(self, dtype, shape):
        out = np.empty(shape, dtype=dtype)
        assert out.nbytes <= self.nbytes
        F.check(F.lib().rt_memcpy_to_host(self.ctx.handle, out.ctypes.data, C.c_void_p(self.ptr), out.nbytes),
                self.ctx.handle)
        return out

    def from_numpy(self, arr):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        F.check(F.lib().rt_memcpy_to_device(self.ctx.handle, C.c_void_p(self.ptr), arr.ctypes.data, arr.nbytes),
                self.ctx.handle)

    def zero(self):
        F.check(F.lib().rt_memset_device(self.ctx.handle, C.c_void_p(self.ptr), 0, self.nbytes), self.ctx.handle)


class Context:
    """One HIP device + stream + the device-resident scene (rt_ctx)."""

    def __init__(self, device=0):
        h = C.c_void_p()
        F.check(F.lib().rt_create(device, C.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h and self._h.value:
            F.lib().rt_destroy(self._h)
            self._h = C.c_void_p(None)

    def __del__(self):
        try:
            if F._lib is not None:
                self.close()
        except Exception:
            pass

    @staticmethod
    def device_count():
        n = C.c_int(0)
        rc = F.lib().rt_device_count(C.byref(n))
        return n.value if rc == F.RT_OK else 0

    def _chk(self, rc):
        return F.check(rc, self._h)

    def set_stream(self, hip_stream):
        self._chk(F.lib().rt_set_stream(self._h, C.c_void_p(hip_stream) if hip_stream else None))

    def synchronize(self):
        self._chk(F.lib().rt_synchronize(self._h))

    def set_option(self, opt, value):
        self._chk(F.lib().rt_set_option(self._h, opt, int(value)))

    def bsp_cull_in_use(self):
        """(mode, certified probe ms, silhouette probe ms): the culling mode the BSP
        kernels run now (rt_bsp_cull_in_use; RT_BSP_CULL_AUTO's choice once probed)."""
        m = C.c_int()
        ms = (C.c_float * 2)()
        self._chk(F.lib().rt_bsp_cull_in_use(self._h, C.byref(m), ms, None))
        return m.value, ms[0], ms[1]

    def bsp_cull_probes(self):
        """(probes started, probe launches) of RT_BSP_CULL_AUTO on this context
        (rt_bsp_cull_in_use's probes)."""
        m = C.c_int()
        n = (C.c_uint32 * 2)()
        self._chk(F.lib().rt_bsp_cull_in_use(self._h, C.byref(m), None, n))
        return n[0], n[1]

    def upload_mesh(self, mesh):
        self._chk(F.lib().rt_upload_mesh_host(self._h, mesh.handle))

    def upload_bsp(self, bsp):
        self._chk(F.lib().rt_upload_bsp_host(self._h, bsp.handle))

    def upload_bvh(self, bvh):
        self._chk(F.lib().rt_upload_bvh_host(self._h, bvh.handle))

    def build_bvh_device(self, max_prims=4):
        """HLBVH construction on the device from the uploaded mesh
        (hlbvh::Bvh::new + flatten + triangles, rt_build_bvh_device); becomes
        this context's BVH.  Returns the per-phase times (ms)."""
        t = F.BvhBuildTimes()
        self._chk(F.lib().rt_build_bvh_device(self._h, max_prims, C.byref(t)))
        return t.asdict()

    def build_bsp_device(self, max_depth=20, max_leaf=4):
        """BSP construction on the device from the uploaded mesh
        (BspTree::new + bsp_array + primitive_ids, rt_build_bsp_device);
        becomes this context's BSP.  Returns the phase times (ms)."""
        t = F.BspBuildTimes()
        self._chk(F.lib().rt_build_bsp_device(self._h, max_depth, max_leaf, C.byref(t)))
        return t.asdict()

    def download_bsp(self):
        """(tree[n,4] u32, planes[n] f32, ids[k] u32, aabb[8] f32) of this context's BSP."""
        nn, ni = C.c_uint32(), C.c_uint32()
        self._chk(F.lib().rt_download_bsp(self._h, None, None, 0, None, 0, None, C.byref(nn), C.byref(ni)))
        tree = np.zeros((max(1, nn.value), 4), np.uint32)
        planes = np.zeros(max(1, nn.value), np.float32)
        ids = np.zeros(max(1, ni.value), np.uint32)
        aabb = np.zeros(8, np.float32)
        self._chk(F.lib().rt_download_bsp(self._h, tree.ctypes.data_as(F.u32p), planes.ctypes.data_as(F.f32p),
                                          nn.value, ids.ctypes.data_as(F.u32p), ni.value,
                                          aabb.ctypes.data_as(F.f32p), C.byref(nn), C.byref(ni)))
        return tree[:nn.value], planes[:nn.value], ids[:ni.value], aabb

    def download_bsp_treelets(self, silhouette=False):
        """The BSP walk's 96-B treelets as u32[nnodes + 1, 24] (rt_download_bsp_treelets;
        diagnostics: the certified culling's per-subtree data); with silhouette=True
        also RT_BSP_CULL_SILHOUETTE's node data as u32[nnodes + 1, 4]."""
        nb = C.c_uint64()
        self._chk(F.lib().rt_download_bsp_treelets(self._h, None, 0, C.byref(nb)))
        out = np.zeros(nb.value // 4, np.uint32)
        self._chk(F.lib().rt_download_bsp_treelets(self._h, out.ctypes.data_as(C.c_void_p), nb.value, C.byref(nb)))
        w = F.BSP_TREELET_BYTES // 4
        slots = out.size // (w + 4)
        tl = out[:slots * w].reshape(-1, w)
        return (tl, out[slots * w:].reshape(-1, 4)) if silhouette else tl

    def download_bvh(self):
        """(nodes[n,8] u32 view of GpuNode, tri_ids[k] u32) of this context's BVH."""
        nn, ni = C.c_uint32(), C.c_uint32()
        self._chk(F.lib().rt_download_bvh(self._h, None, 0, None, 0, C.byref(nn), C.byref(ni)))
        nodes = (F.GpuNode * max(1, nn.value))()
        ids = np.zeros(max(1, ni.value), np.uint32)
        self._chk(F.lib().rt_download_bvh(self._h, nodes, nn.value, ids.ctypes.data_as(F.u32p), ni.value,
                                          C.byref(nn), C.byref(ni)))
        raw = np.frombuffer(nodes, dtype=np.uint32).reshape(-1, 8)[:nn.value].copy()
        return raw, ids[:ni.value].copy()

    def upload_mesh_arrays(self, vertices, normals, indices, materials, lights=None):
        pos = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 4)
        nrm = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 4)
        idx = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1, 4)
        mats = np.ascontiguousarray(materials, dtype=np.float32).reshape(-1, 16)
        lp = None
        nl = 0
        if lights is not None:
            lights = np.ascontiguousarray(lights, dtype=np.uint32)
            lp, nl = F.as_u32p(lights), lights.shape[0]
        self._chk(F.lib().rt_upload_mesh(self._h, F.as_f32p(pos), F.as_f32p(nrm), pos.shape[0], F.as_u32p(idx),
                                         idx.shape[0], C.cast(mats.ctypes.data, C.POINTER(F.Material)),
                                         mats.shape[0], lp, nl))

    def upload_bsp_arrays(self, aabb, tree, planes, ids, max_depth):
        aabb = np.ascontiguousarray(aabb, dtype=np.float32)
        tree = np.ascontiguousarray(tree, dtype=np.uint32).reshape(-1, 4)
        planes = np.ascontiguousarray(planes, dtype=np.float32)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        self._chk(F.lib().rt_upload_bsp(self._h, F.as_f32p(aabb), F.as_u32p(tree), F.as_f32p(planes), tree.shape[0],
                                        F.as_u32p(ids), ids.shape[0], max_depth))

    def upload_bvh_arrays(self, nodes_u32x8, tri_ids):
        nodes = np.ascontiguousarray(nodes_u32x8, dtype=np.uint32).reshape(-1, 8)
        ids = np.ascontiguousarray(tri_ids, dtype=np.uint32)
        self._chk(F.lib().rt_upload_bvh(self._h, C.cast(nodes.ctypes.data, C.POINTER(F.GpuNode)), nodes.shape[0],
                                        F.as_u32p(ids), ids.shape[0]))

    def set_uniforms(self, uniform, jitter=None):
        jp = None
        if jitter is not None:
            self._jitter = np.ascontiguousarray(jitter, dtype=np.float32)
            jp = F.as_f32p(self._jitter)
        self._chk(F.lib().rt_set_uniforms(self._h, C.byref(uniform), jp))

    def set_environment(self, rgb):
        a = np.ascontiguousarray(rgb, dtype=np.float32)
        self._chk(F.lib().rt_set_environment(self._h, F.as_f32p(a)))

    def set_environment_map(self, rgba8):
        """hdri0 equirectangular background for W9E1: uint8[h, w, 4] (RGBA), or None."""
        if rgba8 is None:
            self._chk(F.lib().rt_set_environment_map(self._h, None, 0, 0))
            return
        a = np.ascontiguousarray(rgba8, dtype=np.uint8)
        if a.ndim != 3 or a.shape[2] != 4:
            raise ValueError("environment map must be uint8[h, w, 4]")
        self._env_keep = a
        self._chk(F.lib().rt_set_environment_map(self._h, a.ctypes.data_as(C.POINTER(C.c_uint8)), a.shape[1],
                                                 a.shape[0]))

    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)

    def render(self, mode, trav, region, first_iter, spp, accum_ptr, ids_ptr=None, counts=False):
        """rt_render on a region (x0, y0, w, h); device pointers in/out."""
        t = F.Tile(*region)
        cnt = F.RayCounts() if counts else None
        self._chk(F.lib().rt_render(self._h, F.MODES.get(mode, mode), F.TRAVERSALS.get(trav, trav), C.byref(t),
                                    first_iter, spp, C.c_void_p(accum_ptr), C.c_void_p(ids_ptr) if ids_ptr else None,
                                    C.byref(cnt) if counts else None))
        return cnt.asdict() if counts else None

    def render_tiles(self, mode, trav, rank, nranks, first_iter, spp, accum_ptr, ids_ptr=None, counts=False):
        ts = F.Tileset(rank, nranks)
        cnt = F.RayCounts() if counts else None
        self._chk(F.lib().rt_render_tiles(self._h, F.MODES.get(mode, mode), F.TRAVERSALS.get(trav, trav),
                                          C.byref(ts), first_iter, spp, C.c_void_p(accum_ptr),
                                          C.c_void_p(ids_ptr) if ids_ptr else None,
                                          C.byref(cnt) if counts else None))
        return cnt.asdict() if counts else None

    def unpack_tiles(self, width, height, nranks, packed_accum, packed_ids, frame_accum, frame_ids):
        vpn = (lambda p: C.c_void_p(p) if p else None)
        self._chk(F.lib().rt_unpack_tiles(self._h, width, height, nranks, vpn(packed_accum), vpn(packed_ids),
                                          vpn(frame_accum), vpn(frame_ids)))

    # ---- the tile gather over RCCL (include/rt.h "multi-GPU")
    @staticmethod
    def comm_unique_id():
        """rt_comm_unique_id: a new communicator id (bytes, RT_COMM_ID_BYTES)."""
        buf = (C.c_uint8 * F.RT_COMM_ID_BYTES)()
        F.check(F.lib().rt_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        """rt_comm_init: join communicator `uid` as `rank` of `nranks` (collective)."""
        buf = (C.c_uint8 * F.RT_COMM_ID_BYTES).from_buffer_copy(uid)
        self._chk(F.lib().rt_comm_init(self._h, nranks, rank, buf))

    def comm_destroy(self):
        self._chk(F.lib().rt_comm_destroy(self._h))

    def gather_tiles(self, width, height, local_accum, local_ids, frame_accum=None, frame_ids=None):
        """rt_gather_tiles: every rank's packed tiles to rank 0's frame (device pointers)."""
        vpn = (lambda p: C.c_void_p(p) if p else None)
        self._chk(F.lib().rt_gather_tiles(self._h, width, height, vpn(local_accum), vpn(local_ids), vpn(frame_accum),
                                          vpn(frame_ids)))

    def trace_rays(self, trav, rays, anyhit=None):
        """rt_trace_rays on host arrays: rays float32[n, 8] (origin, direction,
        tmin, tmax), anyhit bool[n] or None.  Returns a structured array with the
        fields of rt_ray_hit (tri, dist, beta, gamma, ntested, tested_fnv, tmin, tmax)."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        n = rays.shape[0]
        out = np.zeros(n, dtype=RAY_HIT_DTYPE)
        if n == 0:
            return out
        rb = self.alloc(rays.nbytes)
        hb = self.alloc(out.nbytes)
        fb = None
        try:
            rb.from_numpy(rays)
            if anyhit is not None:
                fb = self.alloc(4 * n)
                fb.from_numpy(np.ascontiguousarray(np.asarray(anyhit).astype(np.uint32)))
            self._chk(F.lib().rt_trace_rays(self._h, F.TRAVERSALS.get(trav, trav), C.c_void_p(rb.ptr),
                                            C.c_void_p(fb.ptr) if fb else None, n, C.c_void_p(hb.ptr)))
            return hb.to_numpy(RAY_HIT_DTYPE, (n,))
        finally:
            for b in (rb, hb, fb):
                if b is not None:
                    b.free()

    def last_counts(self):
        cnt = F.RayCounts()
        self._chk(F.lib().rt_last_counts(self._h, C.byref(cnt)))
        return cnt.asdict()

    def timer_start(self):
        self._chk(F.lib().rt_timer_start(self._h))

    def timer_stop(self):
        ms = C.c_float()
        self._chk(F.lib().rt_timer_stop(self._h, C.byref(ms)))
        return ms.value

    def frame_rgba8(self, accum_ptr, npix, out_ptr):
        """Display transform of npix accumulated pixels into 8-bit sRGB RGBA (device pointers)."""
        self._chk(F.lib().rt_frame_rgba8(self._h, C.c_void_p(accum_ptr), npix, C.c_void_p(out_ptr)))

    def kernel_time(self, reset=True):
        """(summed ms, launches) of the traversal-kernel launches timed since the
        last reset (RT_OPT_KERNEL_TIMING must be on); synchronizes."""
        ms = C.c_double()
        n = C.c_uint32()
        self._chk(F.lib().rt_kernel_time(self._h, int(reset), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def trace_batch(self, trav, rays_ptr, flags_ptr, n, hits_ptr):
        """rt_trace_batch: the traversal-only kernel over n device rays (8 f32 each;
        flags bit 0 any-hit, or None) into n x {record offset | 0xFFFFFFFE | ~0, dist}."""
        self._chk(F.lib().rt_trace_batch(self._h, F.TRAVERSALS.get(trav, trav), C.c_void_p(rays_ptr),
                                          C.c_void_p(flags_ptr) if flags_ptr else None, n, C.c_void_p(hits_ptr)))

    def set_ray_capture(self, rays_ptr=None, flags_ptr=None, cap=0):
        """Arm (device buffers of cap rays) or disarm (None) the counting renders' ray capture."""
        self._chk(F.lib().rt_set_ray_capture(self._h, C.c_void_p(rays_ptr) if rays_ptr else None,
                                              C.c_void_p(flags_ptr) if flags_ptr else None, cap))

    def ray_capture_count(self):
        n = C.c_uint64()
        self._chk(F.lib().rt_ray_capture_count(self._h, C.byref(n)))
        return n.value

    def gather_time(self, reset=True):
        """(transfer ms, unpack ms, calls) of the frame assembly timed since the last
        reset (rt_gather_time: rt_gather_tiles' RCCL transfers and every unpack;
        RT_OPT_KERNEL_TIMING must be on); synchronizes."""
        tx = C.c_double()
        up = C.c_double()
        n = C.c_uint32()
        self._chk(F.lib().rt_gather_time(self._h, int(reset), C.byref(tx), C.byref(up), C.byref(n)))
        return tx.value, up.value, n.value

    def selftest_math(self, n=1 << 20, lo=-4.0, hi=4.0):
        bad = C.c_uint32()
        self._chk(F.lib().rt_selftest_math(self._h, n, lo, hi, C.byref(bad)))
        return bad.value


def load_texture_rgba8(path):
    """Texture::from_file (src/bindings/texture.rs:98, image.to_rgba8()): a
    JPEG/PNG as uint8[h, w, 4].  Decoded with PIL (the reference's image 0.24
    decoder is not available: texel values are parity-unpinned)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGBA"), dtype=np.uint8).copy()


def local_tiles(width, height, nranks):
    return int(F.lib().rt_tileset_local_tiles(width, height, nranks))
