// rt_internal.h -- launch interface between the C ABI layer (rt_api.cpp) and
// the gfx950 kernels (rt_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/rt.h"

namespace rtk {

// Device-resident scene, in the layout the kernels read (DESIGN.md "Data layout in HBM").
struct DevScene {
    // mesh (src/bindings/storage_mesh.rs): positions/normals float4, index uint4 (v0,v1,v2,mat)
    const float4* pos;
    const float4* nrm;
    const uint4* tri_idx;
    const rt_material* mats;
    const uint32_t* lights;
    uint32_t nverts, ntris, nmats, nlights;
    // BSP: one allocation [96-B treelets | 48-B records] (rt_api.cpp rt_upload_bsp):
    // treelet of 1-based node M at 96*M holds M's content box (min.xyz, max.xyz: the
    // triangles its subtree references), nodes M, 2M, 2M+1, 4M..4M+3 (8 B each:
    // interior {axis, plane bits}, leaf {3 | (48*count) << 2, first record's byte
    // offset}; children implicit, 2i+1, 2i+2 0-based, src/data_structures/bsp_tree.rs:137-140)
    // and the certification data of its subtree (rt_bsp_build.hip k_bsp_repack).
    const uint2* bsp_nodes;       // start of the allocation
    const float4* bsp_recs;       // = bsp_nodes + bsp_rec_off: v0, e0=v1-v0, e1=v2-v0, n=cross(e0,e1)
    uint32_t bsp_bytes;           // size of the allocation (buffer-resource range)
    uint32_t bsp_rec_off;         // byte offset of the records
    const uint32_t* bsp_ids;      // treeIds
    uint32_t bsp_depth;           // MAX_LEVEL
    float aabb[6];                // root BboxGpu min.xyz, max.xyz
    // BVH: one allocation [32-B node records | 48-B triangle records in bvh_triangles
    // order] (rt_api.cpp rt_upload_bvh; links and leaf ranges as byte offsets)
    const uint8_t* bvh_base;
    uint32_t bvh_bytes;
    uint32_t bvh_rec_off;
    const uint32_t* bvh_ids;
    uint32_t bvh_nnodes;
    // RT_OPT_BSP_CULL: the BSP walk skips a subtree whose content box, grown by a
    // margin, the ray misses by more than this fraction of |tn| + |tf| (2^-18; +inf
    // turns culling off without a branch on a uniform flag, rt_kernels.hip bsp_box_miss)
    float bsp_cull_gap;
    // the margin, as data for both culling modes (bsp_box_miss):
    //   m = D1 * (cull_k1 * w1 / max(F, 2 Dlb - 20u w1) + cull_k3) + max(|o|inf * cull_ko, bsp_margin)
    // certified (RT_BSP_CULL_CERTIFIED): k1 = 36u, k3 = 2u, ko = 2^-19, bsp_margin = 2^-19 x scene;
    // fast (RT_BSP_CULL_FAST): k1 = k3 = 0, ko = 2^-10, bsp_margin = 2^-10 x scene
    float bsp_margin;
    float cull_k1, cull_k3, cull_ko;
    // the eye the treelets' camera terms are for (rt_bsp_build.hip
    // launch_bsp_camera): rays starting exactly there use them (NaN: none)
    float cam_eye[3];
    // the cap of the cull's gap tolerance (bsp_box_miss): FLT_MAX with culling on, so a
    // slab that is +-inf (an axis whose direction component is exactly zero and whose
    // origin coordinate lies outside the grown box) culls; +inf with culling off
    // (kept last: a field added mid-struct once moved the trip loop into spills)
    float bsp_cull_emax;
    // per BSP record slot: {triangle id, material} (treeIds[k], tri_idx[treeIds[k]].w),
    // so shading resolves a hit with one load (rt_kernels.hip resolve)
    const uint2* bsp_tm;
    // RT_BSP_CULL_SILHOUETTE: per 1-based node M, the camera term's two excluded
    // triangles' normals and the rest's term, 16 B at [M] (rt_bsp_build.hip k_treelet_hcam)
    const uint4* bsp_sil;
    uint32_t bsp_cull_mode;   // RT_BSP_CULL_* (the host picks k_path's instantiation by it)
    // 1: some interior plane lies outside {0} U [2^-76, 2^99] in magnitude, so the walk's
    // divisions keep their per-decision range check for every ray (launch_plane_range)
    uint32_t bsp_div_checked;
};

// Work mapping + outputs of one launch.
struct DevLaunch {
    rt_uniform u;
    float cam[14];                // camera basis e, v, b1, b2, d, aspect (get_camera_ray, w7e3.wgsl:211-228)
    const float* jitter;          // subdiv^2 float2 (device), may be null when subdiv == 1
    float env[3];
    const uint32_t* env_tex;      // RGBA8 equirectangular hdri0, or null for the constant env
    uint32_t env_w, env_h;
    // region mode (tileset == 0): 8x8 tiles over [x0,x0+w) x [y0,y0+h), row-major region output
    // tileset mode (tileset == 1): the 8x8 tile at sequence position s = l*nranks + rank
    // (rt.h rt_tileset: rows rotated by their index mod 8), packed output
    uint32_t tileset;
    uint32_t x0, y0, w, h;
    uint32_t rank, nranks;
    uint32_t tiles_x, tiles_y;    // tile grid (of the region, or of the frame)
    uint32_t nwork;               // work items (tiles) in this launch
    uint32_t first_iter, spp;     // this pass: iterations first_iter .. first_iter+spp-1
    uint32_t shade_threshold;     // k_path: shade when <= this many lanes still trace
    uint32_t reserved0;           // (was the retired trip-half postponement; kept for the argument layout)
    // k_path work units: (chunk of `chunk` iterations, pixel slot), chunk-major;
    // per-iteration radiance + primary id go to samples[(it - first_iter) * stride + out]
    // and k_fold applies the progressive average in order (w7e3.wgsl:261-271)
    uint32_t chunk, nchunks;
    uint32_t unit_order;          // 0: chunk-major, 1: pixel-major
    uint32_t stride;              // output pixels of the launch (region w*h, or nwork*64 packed)
    float4* samples;
    float4* accum;
    uint32_t* ids;
    uint32_t* work_counter;       // zeroed before launch
    unsigned long long* counters; // 32 x u64, zeroed before launch (rt_ray_counts order)
    uint32_t* bvh_deep;           // BVH stack entries beyond the LDS share: (50 - K) x grid lanes
    // ray capture (rt_set_ray_capture; the counting instantiation only): every ray
    // the path kernel's walks trace, appended as {o.xyz, w.xyz, tmin, tmax} + flags
    // (bit 0 any-hit); cap_count counts them all, cap_max bounds what is written
    float4* cap_rays;
    uint32_t* cap_flags;
    unsigned long long* cap_count;
    unsigned long long cap_max;
};

// Launch the kernel for (mode, trav); detail = counting instantiation.
int launch_render(const DevScene& s, const DevLaunch& l, rt_mode mode, rt_traverse trav, bool detail,
                  int num_cus, int waves_per_cu, hipStream_t stream);
// bytes of the deep BVH stack for a grid of at most num_cus x waves_per_cu waves
size_t bvh_deep_bytes(int num_cus, int waves_per_cu);

// rt_trace_rays: one walk per ray (k_query); bvh_deep sized bvh_deep_bytes(num_cus, 16)
int launch_query(const DevScene& s, rt_traverse trav, const float* rays, const uint32_t* flags, uint32_t n,
                 rt_ray_hit* out, uint32_t* bvh_deep, int num_cus, hipStream_t stream);

// rt_trace_batch: the traversal-only persistent kernel (k_trace) over n device
// rays (8 floats each) into n x {record offset | 0xFFFFFFFE any-hit | ~0 miss, dist};
// work: 1 KiB of shard heads (zeroed here); BSP only
int launch_trace_batch(const DevScene& s, const float* rays, const uint32_t* flags, uint32_t n, uint32_t* hits,
                       uint32_t* work, uint32_t threshold, int num_cus, hipStream_t stream);

// Progressive average of one pass's per-iteration samples into accum/ids (after k_path).
int launch_fold(const DevLaunch& l, hipStream_t stream);

// display frame: RGBA32F accum -> 8-bit sRGB (thr: 255 device floats, srgb_code_thresholds)
int launch_frame(const float4* accum, uint32_t npix, const float* thr, uchar4* out, hipStream_t stream);

int launch_unpack(uint32_t width, uint32_t height, uint32_t nranks, uint32_t local_tiles,
                  const float4* packed_accum, const uint32_t* packed_ids, float4* frame_accum,
                  uint32_t* frame_ids, hipStream_t stream);

// GPU HLBVH build (rt_build.hip): reference-layout arrays (GpuNode + bvh_triangles),
// device allocations owned by the caller afterwards (hipFree).
struct BvhDeviceOut {
    rt_gpu_node* nodes = nullptr;
    uint32_t* ids = nullptr;
    uint32_t nnodes = 0, nids = 0;
};
int build_bvh_device(const float4* pos, const uint4* idx, uint32_t ntris, uint32_t max_prims, int num_cus,
                     hipStream_t stream, BvhDeviceOut& out, rt_bvh_build_times* times, std::string& err);
// traversal layout of a BVH from its reference-layout arrays (rt_upload_bvh's repack, on device)
int launch_bvh_repack(const rt_gpu_node* nodes, uint32_t nnodes, uint32_t rec_off, void* blob, const float4* pos,
                      const uint4* idx, const uint32_t* ids, uint32_t nids, hipStream_t stream);

// GPU BSP build (rt_bsp_build.hip): reference-layout arrays (bsp_array, planes,
// primitive_ids, BboxGpu), device allocations owned by the caller afterwards.
struct BspDeviceOut {
    uint32_t* tree = nullptr;    // nnodes x vec4u
    float* planes = nullptr;     // nnodes
    uint32_t* ids = nullptr;     // nids
    float aabb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t nnodes = 0, nids = 0;
};
int build_bsp_device(const float4* pos, const uint4* idx, uint32_t ntris, uint32_t max_depth, uint32_t max_leaf,
                     int num_cus, hipStream_t stream, BspDeviceOut& out, rt_bsp_build_times* times, std::string& err);
// traversal layout of a BSP from its reference-layout arrays (rt_upload_bsp's repack, on device):
// 96-B treelets (content box + 7 nodes + certification data, BSP_TREELET_BYTES)
// then the 48-B records; box_scratch: nnodes x 64 B of device memory for the
// content boxes and the certification data
constexpr uint32_t BSP_TREELET_BYTES = 96;
// the camera terms of every treelet for the camera-ray eye, and each node's
// silhouette data for RT_BSP_CULL_SILHOUETTE (sil: (nnodes + 1) x 16 B; scratch: nnodes x 24 B)
int launch_bsp_camera(const uint32_t* tree, uint32_t nnodes, const float4* pos, const uint4* idx, const uint32_t* ids,
                      uint32_t nids, const float eye[3], void* blob, uint32_t* sil, void* scratch, hipStream_t stream);
// flag (device, 4 B) = 1 when an interior plane lies outside {0} U [2^-76, 2^99] in magnitude
int launch_plane_range(const uint32_t* tree, const float* planes, uint32_t nnodes, uint32_t* flag, hipStream_t stream);
// tm: nids x {triangle id, material} in treeIds order (or null)
int launch_bsp_repack(const uint32_t* tree, const float* planes, uint32_t nnodes, uint32_t rec_off, void* blob,
                      const float4* pos, const uint4* idx, const uint32_t* ids, uint32_t nids, float margin,
                      void* box_scratch, uint2* tm, hipStream_t stream);
// device primitives shared by the builders (rt_build.hip)
int scan_exclusive_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* scratch, hipStream_t s);
size_t scan_scratch_words(uint32_t n);
int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, uint32_t passes,
                     uint32_t* hist, hipStream_t s, int& result_in_second);
size_t radix_hist_words(uint32_t n);

int launch_selftest_math(const float* in, float* out, uint32_t n, hipStream_t stream);

// get_camera_ray's basis from the uniforms (host, same f32 operations as the shader)
void camera_basis(const rt_uniform& u, float cam[14]);

// Host reference of the pinned math for the self test (same header, host compile).
void host_math(const float* in, float* out, uint32_t n);

constexpr int kMathOuts = 16;   // outputs per input in the math self test

}  // namespace rtk
