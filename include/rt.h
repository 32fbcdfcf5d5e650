/*
 * rt.h -- C ABI of the MI355X-native hot path of cakarsubasi/02562_raytracer.
 *
 * The reference renders one frame per `RenderState::render()` call
 * (src/render_state.rs:483-561): a full-screen quad whose fragment shader
 * (`fs_main` of res/shaders/{w6e1,project,w7e3,w9e1,w1e6}.wgsl) traces one path
 * per pixel through the BSP (res/shaders/bsp.wgsl:10-81) or HLBVH
 * (res/shaders/bvh.wgsl:154-191).  This library replaces, behind plain C
 * pointers and sizes:
 *   - the wgpu device/queue wrapper          src/gpu_handles.rs:9-14, 72-92
 *   - the storage-buffer uploads             src/bindings/{storage_mesh,bsp_tree,bvh,uniform}.rs
 *   - the render pass + accumulation copy    src/render_state.rs:483-561
 *   - the fragment shader itself             res/shaders/<scene>.wgsl (HIP kernels for gfx950)
 * and exposes the host-side builders that feed it (the reference computes these
 * in Rust before upload):
 *   - Mesh::from_obj / Mesh::load            src/mesh.rs:78-202
 *   - BspTree::new + bsp_array + primitive_ids  src/data_structures/bsp_tree.rs:45,120,79
 *   - hlbvh::Bvh::new + flatten + triangles  src/data_structures/hlbvh.rs:36,195,237
 *
 * Conventions:
 *   - every function returns RT_OK (0) or a negative RT_E_* code; no exceptions
 *     cross the ABI; rt_last_error() gives a message for the last failure;
 *   - uploads copy from caller-owned host arrays (as wgpu create_buffer_init);
 *     the context owns all device memory it allocates;
 *   - a context is bound to one HIP device and is not thread-safe: use one
 *     context per GPU and per host thread (the reference uses its RenderState
 *     from the single "Render Thread", src/lib.rs:305-307);
 *   - output buffers passed to rt_render* are DEVICE pointers (HBM resident);
 *     their layout is documented per function.
 */
#ifndef RT02562_RT_H
#define RT02562_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
#define RT_OK            0
#define RT_E_INVALID    (-1)  /* bad argument / malformed structure          */
#define RT_E_OOM        (-2)  /* device allocation failed (SurfaceError::OutOfMemory, src/lib.rs:345) */
#define RT_E_DEVICE     (-3)  /* HIP runtime error                           */
#define RT_E_NOT_READY  (-4)  /* render called before the needed upload      */
#define RT_E_IO         (-5)  /* file could not be read / parsed             */
#define RT_E_UNSUPPORTED (-6) /* mode/traversal combination not implemented  */

/* ---- plain data types (byte-compatible with the reference GPU structs) -- */

/* Material, 64 B: src/mesh.rs:12-20 (WGSL struct src/bindings/storage_mesh.rs:392-397) */
typedef struct rt_material {
    float diffuse[4];
    float ambient[4];
    float specular[4];
    uint32_t emissive;      /* MTL illum; == 1 marks an area light (storage_mesh.rs:322) */
    uint32_t _pad[3];
} rt_material;

/* HLBVH GpuNode, 32 B: src/data_structures/hlbvh.rs:508-515 */
typedef struct rt_gpu_node {
    float min[3];
    uint32_t offset_ptr;    /* leaf: first index into tri_ids; interior: right child */
    float max[3];
    uint32_t n_prims;       /* 0 = interior (left child is node+1) */
} rt_gpu_node;

/* Uniform block, 80 B: src/bindings/uniform.rs:6-34 */
typedef struct rt_uniform {
    float camera_pos[3];
    float camera_constant;
    float camera_look_at[3];
    float aspect_ratio;
    float camera_up[3];
    uint32_t selection1;     /* shader selector (0 = Lambertian) */
    uint32_t selection2;
    uint32_t subdivision_level;
    uint32_t use_texture;
    uint32_t iteration;      /* progressive frame index (overridden by first_iter) */
    float uv_scale[2];
    uint32_t resolution[2];  /* full-frame W, H (global pixel space) */
} rt_uniform;

/* Which scene shader the kernel restates (SceneDescriptor.shader, src/scenes.rs:19-29). */
typedef enum rt_mode {
    RT_MODE_W1E6    = 0,  /* res/shaders/w1e6.wgsl: analytic sphere/plane/triangle, no mesh  */
    RT_MODE_W6E1    = 1,  /* res/shaders/w6e1.wgsl: primary rays, directional light, split vertex layout */
    RT_MODE_PROJECT = 2,  /* res/shaders/project.wgsl: as W6E1, combined layout, ambient*0.1 */
    RT_MODE_W7E3    = 3,  /* res/shaders/w7e3.wgsl: area-light path tracer, progressive       */
    RT_MODE_W9E1    = 4,  /* res/shaders/w9e1.wgsl: dummy-light path tracer, environment escape */
    RT_MODE_W8E1    = 5,  /* res/shaders/w8e1.wgsl: Cornell box + mirror and glass balls, direct light */
    RT_MODE_W8E2    = 6,  /* res/shaders/w8e2.wgsl: as W8E1, path traced (Russian roulette, clamp 100) */
    RT_MODE_W8E3    = 7,  /* res/shaders/w8e3.wgsl: as W8E2, Beer-Lambert absorption in the glass ball */
    RT_MODE_W9E2    = 8,  /* res/shaders/w9e2.wgsl: W9E1 + holdout plane y=0 (AO any-hit), RGBE environment */
    RT_MODE_W6E2    = 9,  /* res/shaders/w6e2.wgsl: direct light from every area-light centre, subdiv^2 samples */
    RT_MODE_W7E1    = 10, /* res/shaders/w7e1.wgsl: as W6E2, progressive (TEA jitter), no max(., 0) */
    RT_MODE_W7E2    = 11, /* res/shaders/w7e2.wgsl: random area-light points, progressive */
    RT_MODE_W6E3    = 12, /* res/shaders/w6e3.wgsl: W6E2's box + mirror ball and glossy (Phong + refraction) ball */
    RT_MODE_W9E3    = 13  /* res/shaders/w9e3.wgsl: sun light, holdout plane (AO + sun rays), culled triangles */
} rt_mode;

/* SceneDescriptor.traverse_type, src/scenes.rs:13-17 */
typedef enum rt_traverse {
    RT_TRAVERSE_BSP  = 0,
    RT_TRAVERSE_BVH  = 1,
    RT_TRAVERSE_NONE = 2   /* only valid with RT_MODE_W1E6 */
} rt_traverse;

/* A rectangle of the frame in GLOBAL pixel coordinates. */
typedef struct rt_tile {
    uint32_t x0, y0, w, h;
} rt_tile;

/* Interleaved 8x8-tile partition of the full frame for multi-GPU rendering
 * (SURVEY.md 8(e)): the tiles (ceil(W/8) x ceil(H/8)) are taken in sequence
 * s = ty * tiles_x + (tx - (ty & 7)) mod tiles_x -- row-major, each row rotated
 * by its index mod 8 (not rotated when tiles_x < 8) -- and sequence position s
 * is owned by rank s % nranks (diagonal stripes: when nranks divides 8 and
 * tiles_x, rank r owns tx = r + ty mod nranks).
 * Global pixel coordinates keep PRNG seeds, and therefore images, identical
 * for every nranks. */
typedef struct rt_tileset {
    uint32_t rank;
    uint32_t nranks;
} rt_tileset;

#define RT_TILE_DIM 8u    /* tile edge in pixels: one wave64 = one 8x8 tile */

/* Per-launch counters.  primary/shadow/bounce are always filled; the traversal
 * detail counters are filled only when RT_OPT_DETAIL_COUNTERS is enabled (a
 * separate, slower kernel instantiation used to price algorithmic bytes). */
typedef struct rt_ray_counts {
    uint64_t samples;        /* pixel-samples traced                       */
    uint64_t primary;        /* camera rays                                */
    uint64_t shadow;         /* shadow (visibility) rays                   */
    uint64_t bounce;         /* indirect closest-hit rays                  */
    uint64_t node_interior;  /* BSP interior node visits                   */
    uint64_t node_leaf;      /* BSP leaf visits                            */
    uint64_t bvh_pops;       /* BVH node pops                              */
    uint64_t ids_read;       /* treeIds / bvh_triangles reads              */
    uint64_t tri_tests;      /* ray-triangle tests                         */
    uint64_t tri_accepts;    /* accepted (closer) hits                     */
    /* SIMD-efficiency diagnostics (detail instantiation only), per wave trip
     * of the traversal loop: */
    uint64_t trips;          /* traversal loop trips (sum over waves)      */
    uint64_t lane_steps;     /* lanes that advanced a ray in those trips    */
    uint64_t leaf_lane_steps;/* ... of which were inside a leaf (triangle)  */
    uint64_t node_trips;     /* trips in which some lane walked nodes       */
    uint64_t leaf_trips;     /* trips in which some lane tested a triangle  */
    uint64_t exact_tests;    /* triangle tests that needed exact division   */
    uint64_t exact_nodes;    /* node decisions that needed exact division   */
    /* path kernels, per wave: shading passes, lanes shaded, and wave cycles
     * (s_memtime) spent in the traversal and in the shading/refill phases */
    uint64_t shade_passes;
    uint64_t shade_lanes;
    uint64_t trav_cycles;
    uint64_t shade_cycles;
    uint64_t memwait_cycles; /* BSP trips: wave cycles from load issue to data */
    uint64_t subtree_culls;  /* BSP walking trips that skipped their node's subtree (content box missed) */
} rt_ray_counts;

/* ---- options (rt_set_option) ------------------------------------------- */
#define RT_OPT_DETAIL_COUNTERS 1  /* 0/1: use the counting kernel instantiation    */
#define RT_OPT_WAVES_PER_CU    2  /* persistent grid size: waves per CU (default 32; capped by LDS) */
#define RT_OPT_SHADE_THRESHOLD 3  /* path kernels: shade once <= N of 64 lanes still trace; 0 or 64 = all lanes finish their rays first (lockstep); -1 = the default: 24 for W7E3 on the BSP walk, 4 for the BVH walk, and for the other modes on the BSP walk a per-wave choice from the share of its tracing lanes inside a leaf (the higher when >= 1/2): 20 or 32 with certified culling (24 or 32 when the silhouette kernel runs), 8 or 24 otherwise; 0x10000 | hi << 8 | lo sets that choice's two thresholds */
#define RT_OPT_SAMPLE_CHUNK    4  /* W7E3/W9E1: progressive iterations per work unit (default 1) */
#define RT_OPT_SAMPLE_BUDGET_MB 5 /* W7E3/W9E1: device scratch for per-sample results, MiB (default 16384);
                                     a render whose spp x pixels x 16 B exceed it runs in several passes */
#define RT_OPT_KERNEL_TIMING   7  /* 0/1: record HIP events around every traversal-kernel launch */
/* option 8 is retired (trip-half postponement: slower on every BASELINE workload, and its
   per-trip test cost 1.7-4.4 % even when off, profiles/r02/sweep_KH_c5.txt, ab_nokh.txt) */
#define RT_OPT_UNIT_ORDER      6  /* W7E3/W9E1 work-unit order: 0 chunk-major, 1 pixel-major (default) */
#define RT_OPT_ASYNC_FOLD     10  /* 0 (default) / 1: pipelined frames.  The path tracers' progressive fold (the
                                     last step of rt_render / rt_render_tiles) runs on a second, context-owned
                                     stream, and so do the calls that consume its outputs (rt_unpack_tiles,
                                     rt_gather_tiles; rt_frame_rgba8 joins that stream and runs on the
                                     context stream); the per-sample scratch is double-buffered.
                                     The next render's traversal kernel then overlaps this frame's fold and
                                     gather.  rt_synchronize, the memcpy/memset calls and every other entry point
                                     wait for that stream first; a caller reading the outputs through its own
                                     stream synchronizes the device (or calls rt_synchronize) first. */
#define RT_OPT_BSP_CULL        9  /* subtree culling in the BSP walk: a subtree whose content
                                     box (the union of its triangles' bounding boxes), grown by a margin, the ray
                                     interval misses is skipped, and the walk's decisions use the interval clipped to
                                     that box.  One of RT_BSP_CULL_*: */
#define RT_BSP_CULL_OFF        0  /* every node of bsp.wgsl's walk is visited: the reference's walk and tested-
                                     triangle sequence, by construction */
#define RT_BSP_CULL_CERTIFIED  1  /* the margin is a proven bound on how far an f32 accept of
                                     intersect_triangle (w7e3.wgsl:286-332) can lie from its triangle's box, from the
                                     subtree's largest edge, its box of normals and, for rays that start at the
                                     uniforms' camera eye, its per-eye plane distance: every hit (triangle, distance,
                                     barycentrics) is bit-identical to RT_BSP_CULL_OFF for every ray; only hitless
                                     work is skipped */
#define RT_BSP_CULL_FAST       2  /* the margin is 2^-10 of the scene's / the ray origin's coordinate magnitude: not
                                     a proven bound.  A ray within ~1e-5 rad of a large triangle's plane, where the
                                     f32 test's hit point can sit off the triangle by more than the margin, can get
                                     a different hit (measured: 2 of 400,000 deliberately grazing rays on a random
                                     soup, none in any rendered frame) */
#define RT_BSP_CULL_SILHOUETTE 3  /* the certified margin, exact as RT_BSP_CULL_CERTIFIED, with a tighter bound for
                                     camera rays: each subtree's two triangles nearest the eye's plane-distance
                                     floor (its silhouette) are bounded per ray by their own normals, the rest by
                                     their camera term.  Fewer trips for far, many-object views (config 4: +15 %),
                                     more arithmetic per trip (config 3: -4 %, config 5: -3 %).  The W9E1
                                     path kernel and rt_trace_batch use it; other kernels run the certified form */
#define RT_BSP_CULL_AUTO       4  /* (default) exact as RT_BSP_CULL_CERTIFIED: the W9E1 BSP renders time the
                                     certified and the silhouette kernels on four of their own launches (certified,
                                     silhouette, certified, silhouette; each at least 2^20 samples: a big render
                                     splits its first iterations, up to an eighth of it or 2^26 samples per
                                     launch, 1-spp frames give one launch each), with no extra
                                     work and no host wait (the events are read at a later render; the certified
                                     kernel runs until then), and run the faster from then on (the silhouette
                                     kernel must be 5 % faster to be chosen), until the BSP or this option changes
                                     or the eye's reach (farthest distance to the scene box) leaves [1/2, 2] of the
                                     reach the probe ran at.  rt_bsp_cull_in_use reports the choice */

/* ---- device / context (replaces src/gpu_handles.rs) -------------------- */

typedef struct rt_ctx rt_ctx;   /* one HIP device + stream + the device-resident scene */

/* Number of HIP devices (~ gpu_handles::self_test, src/gpu_handles.rs:72-92). */
int rt_device_count(int* count);

/* Create a context on HIP device `device` (~ GPUHandles::new / RenderState::new
 * device part, src/render_state.rs:66-106).  Creates its own non-blocking stream. */
int rt_create(int device, rt_ctx** out);
void rt_destroy(rt_ctx* ctx);

/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream)
 * instead of the context's own stream; NULL restores the own stream. */
int rt_set_stream(rt_ctx* ctx, void* hip_stream);
void* rt_get_stream(rt_ctx* ctx);
int rt_synchronize(rt_ctx* ctx);

int rt_set_option(rt_ctx* ctx, int option, int64_t value);

/* The culling mode the W9E1 BSP path kernel (and the query and batch kernels) run now
 * (RT_BSP_CULL_*): the option's value, except that RT_BSP_CULL_SILHOUETTE without the
 * eye's camera terms runs CERTIFIED and RT_BSP_CULL_AUTO runs its probe's choice
 * (CERTIFIED or SILHOUETTE; CERTIFIED until a probe has decided for the current BSP).
 * Kernels without a silhouette form (the other modes, W9E1's transparent shader) run
 * CERTIFIED under SILHOUETTE and AUTO.  probe_ms (2 floats, or NULL): the probe's best
 * certified and silhouette times in milliseconds per 2^20 samples, 0 until it has decided.
 * probes (2 uint32, or NULL): the probes this context has started and their launches. */
int rt_bsp_cull_in_use(rt_ctx* ctx, int* mode, float* probe_ms, uint32_t* probes);

/* Message describing the last failure on this context (or the last
 * context-less failure when ctx == NULL).  Never NULL. */
const char* rt_last_error(const rt_ctx* ctx);

/* Device memory for frame buffers (the RenderSource/RenderDestination
 * textures of src/bindings/texture.rs:285-407 become plain HBM arrays).
 * Copies synchronize the context stream; memset is asynchronous on it. */
int rt_device_alloc(rt_ctx* ctx, size_t bytes, void** dptr);
int rt_device_free(rt_ctx* ctx, void* dptr);
int rt_memcpy_to_host(rt_ctx* ctx, void* dst, const void* src_dev, size_t bytes);
int rt_memcpy_to_device(rt_ctx* ctx, void* dst_dev, const void* src, size_t bytes);
int rt_memset_device(rt_ctx* ctx, void* dst_dev, int value, size_t bytes);

/* HIP-event timer on the context stream (RenderStats, src/tools.rs:4-61,
 * times render() on the host; this times the device work). */
int rt_timer_start(rt_ctx* ctx);
int rt_timer_stop(rt_ctx* ctx, float* ms);   /* synchronizes */

/* Per-launch timing of the traversal kernels (k_path / k_primary / k_w1e6),
 * enabled by RT_OPT_KERNEL_TIMING: HIP events around every such launch on the
 * context stream.  rt_kernel_time synchronizes and returns the summed
 * duration and the number of launches since the last reset (reset != 0
 * clears them).  At most 4096 launches are kept between resets. */
int rt_kernel_time(rt_ctx* ctx, int reset, double* total_ms, uint32_t* launches);

/* The same for the frame's assembly (RT_OPT_KERNEL_TIMING): HIP events on the
 * output stream around the RCCL transfers of rt_gather_tiles (rank 0: the copy of
 * its own tiles and every peer's receive; another rank: its send) and around the
 * unpack kernel (rt_gather_tiles on rank 0, rt_unpack_tiles).  Synchronizes and
 * returns the summed times and the number of calls since the last reset (at
 * most 4096 calls are kept between resets).  For a multi-GPU host's per-rank
 * diagnostics (bench.py's N>1 line). */
int rt_gather_time(rt_ctx* ctx, int reset, double* transfer_ms, double* unpack_ms, uint32_t* calls);

/* ---- uploads (replace the src/bindings/ create_buffer_init calls) ------------- */

/* Mesh + materials + light list (src/bindings/storage_mesh.rs:13-26, 82-110,
 * 201-236, 297-332).  pos_vec4 / nrm_vec4: nverts x float4 (w ignored);
 * nrm_vec4 may be NULL (zero normals, as mesh.rs:165-171).  idx_vec4u: ntris x
 * (v0, v1, v2, material).  light_idx[0] must be the UINT32_MAX sentinel
 * (storage_mesh.rs:325-326); light_idx may be NULL to derive the list from
 * materials[].emissive == 1. */
int rt_upload_mesh(rt_ctx* ctx,
                   const float* pos_vec4, const float* nrm_vec4, uint32_t nverts,
                   const uint32_t* idx_vec4u, uint32_t ntris,
                   const rt_material* mats, uint32_t nmats,
                   const uint32_t* light_idx, uint32_t nlight);

/* Flattened BSP (src/bindings/bsp_tree.rs:167-203): aabb = BboxGpu (min.xyz,
 * pad, max.xyz, pad); tree_vec4u = nnodes x (axis|count<<2, first_id, left,
 * right) with nnodes == 2^(max_depth+1)-1; planes = nnodes floats; ids = nids
 * triangle indices.  Requires a prior rt_upload_mesh (triangles are repacked
 * in treeIds order on upload). */
int rt_upload_bsp(rt_ctx* ctx, const float aabb[8],
                  const uint32_t* tree_vec4u, const float* planes, uint32_t nnodes,
                  const uint32_t* ids, uint32_t nids, uint32_t max_depth);

/* Flattened HLBVH (src/bindings/bvh.rs:75-93). Requires a prior rt_upload_mesh. */
int rt_upload_bvh(rt_ctx* ctx, const rt_gpu_node* nodes, uint32_t nnodes,
                  const uint32_t* tri_ids, uint32_t nids);

/* Uniforms + jitter table (src/bindings/uniform.rs:163-176).  jitter holds
 * subdivision_level^2 float2 offsets (may be NULL when subdivision_level == 1:
 * compute_jitters returns (0,0), uniform.rs:261-263).  RT_E_INVALID for a zero
 * resolution or one above 65535 in either axis (the path kernel packs a pixel's
 * coordinates into one 32-bit register). */
int rt_set_uniforms(rt_ctx* ctx, const rt_uniform* u, const float* jitter);

/* ---- acceleration-structure construction on the GPU ---- */

/* Per-phase times of a device build, the reference's BvhConstructionTime
 * split (src/data_structures/bvh_util.rs:6-13, src/bin/bvh_project.rs). */
typedef struct rt_bvh_build_times {
    double morton_codes_ms, radix_sort_ms, treelet_init_ms, treelet_build_ms;
    double upper_tree_ms;        /* device-to-host of the treelet roots + host collapse + upload */
    double upper_tree_host_ms;   /* of which the host collapse                                    */
    double flattening_ms;        /* DFS offsets, GpuNode array, filler                            */
    double total_ms;             /* wall clock of the whole call                                  */
    uint32_t treelets, nodes;
} rt_bvh_build_times;

/* hlbvh::Bvh::new(mesh, max_prims) + flatten() + triangles()
 * (src/data_structures/hlbvh.rs:36-239) on the device from the context's
 * uploaded mesh: the same arrays as rt_bvh_build (equal Morton codes in
 * primitive-index order), installed as the context's BVH as rt_upload_bvh
 * would.  times may be NULL.  Synchronizes the context stream. */
int rt_build_bvh_device(rt_ctx* ctx, uint32_t max_prims, rt_bvh_build_times* times);

/* Per-phase times of a device BSP build (src/bin/bvh_project.rs
 * BspConstructionTime: subdivision, flattening). */
typedef struct rt_bsp_build_times {
    double subdivision_ms;   /* the level-by-level subdivide_node of every depth       */
    double flattening_ms;    /* leaf first-ids in DFS order + primitive_ids            */
    double total_ms;         /* wall clock of the whole call                           */
    uint32_t levels, leaves, nids;
} rt_bsp_build_times;

/* BspTree::new(mesh.bboxes(), max_depth, max_leaf) + bsp_array() +
 * primitive_ids() (src/data_structures/bsp_tree.rs:45-189, 195-323) on the
 * device from the context's uploaded mesh: the same arrays as rt_bsp_build,
 * installed as the context's BSP as rt_upload_bsp would.  Subdivision runs
 * one depth level at a time over all nodes of that level.  times may be NULL.
 * Synchronizes the context stream. */
int rt_build_bsp_device(rt_ctx* ctx, uint32_t max_depth, uint32_t max_leaf, rt_bsp_build_times* times);

/* Copy the context's BSP in the reference layout (bsp_array vec4u, planes,
 * primitive_ids, BboxGpu aabb[8]) to host arrays; sizes stored in nnodes/nids
 * (pass NULL arrays to query them). */
int rt_download_bsp(rt_ctx* ctx, uint32_t* tree, float* planes, uint32_t cap_nodes, uint32_t* ids,
                    uint32_t cap_ids, float aabb[8], uint32_t* nnodes, uint32_t* nids);

/* Diagnostics (no reference counterpart; tests/test_gpu_cert_data.py): copy the
 * BSP walk's 96-B treelets (slot 0 unused, then one per 1-based node M:
 * content box, nodes M, 2M, 2M+1, 4M..4M+3, and the certified culling's data
 * -- F bf16 | camera term G f16 << 16, normal-box centre and radius as f16;
 * rt_bsp_build.hip k_bsp_repack) to dst, (nnodes + 1) * 96 bytes, followed by
 * RT_BSP_CULL_SILHOUETTE's node data ((nnodes + 1) * 16 bytes: the two excluded
 * triangles' n* / E^2 as f16 triples, the rest's camera term G_x f16; zero when
 * not computed), after bringing the camera terms up to date for the uniforms'
 * eye (certified culling).  The size is stored in *bytes (pass dst NULL to
 * query it). */
int rt_download_bsp_treelets(rt_ctx* ctx, void* dst, uint64_t cap_bytes, uint64_t* bytes);

/* Copy the context's BVH in the reference layout (GpuNode array, bvh_triangles)
 * to host arrays of capacity cap_nodes / cap_ids; the sizes are stored in
 * nnodes / nids (pass NULL arrays to query them). */
int rt_download_bvh(rt_ctx* ctx, rt_gpu_node* nodes, uint32_t cap_nodes, uint32_t* tri_ids, uint32_t cap_ids,
                    uint32_t* nnodes, uint32_t* nids);

/* Environment radiance returned on escape by RT_MODE_W9E1 (stands in for the
 * equirectangular hdri0 texture, res/shaders/w9e1.wgsl:232-241). Default (1,1,1). */
int rt_set_environment(rt_ctx* ctx, const float rgb[3]);

/* The hdri0 equirectangular background of the W9E1 scenes (src/scenes.rs
 * background_hdri; src/bindings/texture.rs: Rgba8Unorm, image.to_rgba8()):
 * width x height RGBA8 texels, row 0 at the top (v = 0).  Sampled by
 * environment_map (w9e1.wgsl:232-239) as include/rt_detmath.h pins it.
 * NULL removes it (the constant of rt_set_environment applies again). */
int rt_set_environment_map(rt_ctx* ctx, const uint8_t* rgba8, uint32_t width, uint32_t height);

/* ---- render (replaces RenderState::render, src/render_state.rs:483-561) -- */

/* Trace `spp` progressive iterations first_iter .. first_iter+spp-1 for every
 * pixel of `region` (global pixel coordinates inside uniforms.resolution).
 * W7E3/W9E1 split the iterations of a pixel into work units of
 * RT_OPT_SAMPLE_CHUNK iterations that run in parallel; each unit writes its
 * per-iteration radiance to device scratch, and a fold kernel then applies the
 * reference's progressive average in iteration order (bit-identical to
 * `spp` sequential render() calls).
 *   accum_rgba32f: DEVICE, region.w*region.h float4, row-major over the region,
 *     in/out: holds the accumulation of iterations < first_iter (read when
 *     first_iter > 0; the RenderDestination texture, render_state.rs:541-555),
 *     and receives max(vec4(accum,1),0) (w7e3.wgsl:261-271).  For W1E6/W6E1/
 *     PROJECT it receives the linear per-frame result (before pow(.,1.5)).
 *   primary_hit_ids: DEVICE or NULL, region.w*region.h u32: triangle index of
 *     the primary hit of the LAST traced iteration, UINT32_MAX on miss.
 *   counts: host pointer or NULL; when non-NULL the call synchronizes and
 *     stores this launch's counters. */
int rt_render(rt_ctx* ctx, rt_mode mode, rt_traverse trav, const rt_tile* region,
              uint32_t first_iter, uint32_t spp,
              float* accum_rgba32f, uint32_t* primary_hit_ids,
              rt_ray_counts* counts);

/* Same, over the 8x8 tiles owned by `ts` (multi-GPU framebuffer tiling).
 * Outputs are PACKED: local tile l (the tile at sequence position
 * s = l*nranks + rank, rt_tileset above) occupies pixels [l*64, l*64+64),
 * row-major inside the tile.  Buffers hold rt_tileset_local_tiles() * 64 px. */
int rt_render_tiles(rt_ctx* ctx, rt_mode mode, rt_traverse trav, const rt_tileset* ts,
                    uint32_t first_iter, uint32_t spp,
                    float* accum_rgba32f, uint32_t* primary_hit_ids,
                    rt_ray_counts* counts);

/* Number of local tiles rank `rank` owns for a W x H frame (equal for all ranks
 * rounded up, so packed buffers have one size: ceil(ntiles / nranks)). */
uint32_t rt_tileset_local_tiles(uint32_t width, uint32_t height, uint32_t nranks);

/* The displayed frame of fs_main (w7e3.wgsl:261-271): saturate(pow(accum, 1.5))
 * as the sRGB surface stores it (render_state.rs:108-115), 8-bit RGBA, for
 * npix pixels; device pointers, asynchronous on the context stream.  The
 * pow and the sRGB rounding are pinned here (the display path is outside
 * the parity contract). */
int rt_frame_rgba8(rt_ctx* ctx, const float* accum_rgba32f, uint32_t npix, uint8_t* frame_rgba8);

/* Scatter gathered packed buffers (nranks x local_tiles x 64 px, rank-major as
 * a gather to the root produces them) into a row-major W x H frame, on the context's
 * stream.  Either pair of pointers may be NULL. */
int rt_unpack_tiles(rt_ctx* ctx, uint32_t width, uint32_t height, uint32_t nranks,
                    const float* packed_accum, const uint32_t* packed_ids,
                    float* frame_accum, uint32_t* frame_ids);

/* ---- multi-GPU: the tile gather over RCCL -----------------
 * One process per GPU, each with its own context: every rank renders its
 * interleaved tiles (rt_render_tiles with rt_tileset {rank, nranks}), then
 * rt_gather_tiles collects them on rank 0 -- one grouped RCCL receive of each
 * peer's packed accumulation (16 B/px) and primary-hit ids (4 B/px), point to
 * point over xGMI, no other collective -- and scatters them into rank 0's frame
 * (rt_unpack_tiles).  Replaces, for a Rust host that tiles one
 * RenderState::render (src/render_state.rs:483-561, driven per frame by
 * src/lib.rs:331-363) across the GPUs of a node, what bench.py did with
 * torch.distributed.  RCCL is loaded at rt_comm_init (librccl.so.1; a process
 * that already holds one, e.g. through PyTorch, shares it). */
#define RT_COMM_ID_BYTES 128u

/* A new communicator id (ncclGetUniqueId), made on rank 0 and handed to every
 * rank out of band (a file, a socket, the launcher's store). */
int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);

/* Join the communicator `id` as `rank` of `nranks` on the context's device
 * (ncclCommInitRank; collective: every rank calls it).  One communicator per
 * context; rt_comm_destroy (or rt_destroy) releases it. */
int rt_comm_init(rt_ctx* ctx, uint32_t nranks, uint32_t rank, const uint8_t id[RT_COMM_ID_BYTES]);
int rt_comm_destroy(rt_ctx* ctx);

/* Gather the ranks' packed tiles of a width x height frame (each rank:
 * rt_tileset_local_tiles(width, height, nranks) * 64 px in local_accum /
 * local_ids, device pointers) to rank 0 and unpack them into rank 0's
 * row-major frame_accum (W*H RGBA32F) and frame_ids (W*H u32); the other ranks
 * pass NULL frames.  Collective over the context's communicator, asynchronous
 * on the context's stream (RCCL runs on it); the frame is complete once the
 * stream has drained.  Either id pointer may be NULL on every rank (accum only). */
int rt_gather_tiles(rt_ctx* ctx, uint32_t width, uint32_t height, const float* local_accum,
                    const uint32_t* local_ids, float* frame_accum, uint32_t* frame_ids);

/* ---- the trace stage of a wavefront renderer ---------------------------------
 * rt_trace_batch walks n device-resident rays through the context's BSP with the
 * render kernels' step function in a traversal-only persistent kernel (no
 * shading state; refills by ballot + mbcnt from per-XCD queues): rays_dev = n x
 * {o.xyz, w.xyz, tmin, tmax} (f32, rt_trace_rays' layout), flags_dev = n x u32 (bit 0: any-hit, the
 * shadow walk; NULL: every ray closest-hit), hits_dev = n x {u32 record byte
 * offset of the accepted triangle (closest hit), 0xFFFFFFFE (any-hit: blocked) or
 * 0xFFFFFFFF (miss), f32 dist}.  The results are rt_trace_rays' walks (same
 * culling mode).  Asynchronous on the context stream; timed by
 * RT_OPT_KERNEL_TIMING like the render kernels.  RT_OPT_SHADE_THRESHOLD's low
 * byte (default 16) is the lanes-still-tracing count at which finished lanes
 * refill.  n must stay below 2^31 (the per-XCD work queues count 64-ray blocks in
 * 32-bit heads; RT_E_INVALID above).  DESIGN.md section 4 "Outside the megakernel".
 *
 * rt_set_ray_capture arms a capture: every counting render (RT_OPT_DETAIL_COUNTERS)
 * of a W7E3 / W9E1 path mode appends each ray its walks start -- camera, shadow
 * and bounce rays, in issue order -- to rays_dev / flags_dev in the layout above
 * (up to cap rays; NULL disarms); rt_ray_capture_count returns how many were
 * traced since it was armed (more than cap: the rest were not written). */
int rt_trace_batch(rt_ctx* ctx, rt_traverse trav, const float* rays_dev, const uint32_t* flags_dev, uint32_t n,
                   uint32_t* hits_dev);
int rt_set_ray_capture(rt_ctx* ctx, float* rays_dev, uint32_t* flags_dev, uint64_t cap);
int rt_ray_capture_count(rt_ctx* ctx, uint64_t* n);

/* ---- ray queries: the walk alone ------------------------------------------ */

/* One walk per ray through the context's BSP or BVH, with the render kernels'
 * own traversal step: intersect_trimesh (res/shaders/bsp.wgsl:10-81) /
 * intersect_bvh (bvh.wgsl:154-191) for a closest-hit ray; with bit 0 of
 * flags[i] set, the any-hit walk of the shadow and occlusion rays (it stops at
 * the first accepted triangle, as intersect_trimesh_immediate_return,
 * bsp.wgsl:83-155, does).  The query form of the reference's CPU walk
 * intersect_bsp_array (js/bsp_tree/modules/BspTree_interleaved.js:287-352).
 *   rays:  DEVICE, n x 8 floats: origin.xyz, direction.xyz, tmin, tmax;
 *   flags: DEVICE, n u32, or NULL (all closest-hit);
 *   hits:  DEVICE, n x rt_ray_hit.
 * Asynchronous on the context stream. */
typedef struct rt_ray_hit {
    uint32_t tri;          /* the accepted triangle (the last accept), UINT32_MAX on a miss */
    float dist;            /* its distance (the ray's tmax when the walk ends) */
    float beta, gamma;     /* its barycentrics (0 for an any-hit walk, which keeps none) */
    uint32_t ntested;      /* triangles tested, in walk order */
    uint32_t tested_fnv;   /* FNV-1a 32 of the tested triangle ids (little-endian u32) in order */
    float tmin, tmax;      /* the ray interval the walk leaves behind (bsp.wgsl narrows it in place) */
} rt_ray_hit;
int rt_trace_rays(rt_ctx* ctx, rt_traverse trav, const float* rays, const uint32_t* flags, uint32_t n,
                  rt_ray_hit* hits);

/* Counters of the most recent launch (synchronizes). */
int rt_last_counts(rt_ctx* ctx, rt_ray_counts* counts);

/* Device-vs-host self check of the pinned f32 math (sqrt, division, the
 * rt_detmath.h transcendentals) over n inputs in [lo, hi]; returns the number
 * of bit mismatches in *mismatches. */
int rt_selftest_math(rt_ctx* ctx, uint32_t n, float lo, float hi, uint32_t* mismatches);

/* ---- host-side builders (the Rust code above the reference's GPU boundary) */

typedef struct rt_mesh_host rt_mesh_host;   /* owns Mesh arrays (src/mesh.rs:35-41) */
typedef struct rt_mesh_view {
    const float* vertices;     /* nverts x float4 */
    const float* normals;      /* nverts x float4 */
    const uint32_t* indices;   /* ntris x (v0,v1,v2,material) */
    const rt_material* materials;
    const uint32_t* lights;    /* nlights entries, [0] = UINT32_MAX sentinel */
    uint32_t nverts, ntris, nmats, nlights;
} rt_mesh_view;

/* Mesh::from_obj with tobj 4.0 semantics (single_index, fan triangulation,
 * per-group models, MTL Kd/Ka/Ks/illum), src/mesh.rs:78-202. */
int rt_mesh_load_obj(const char* path, rt_mesh_host** out);
/* Wrap caller arrays into a host mesh (copies). normals/materials may be NULL. */
int rt_mesh_from_arrays(const float* pos_vec4, const float* nrm_vec4, uint32_t nverts,
                        const uint32_t* idx_vec4u, uint32_t ntris,
                        const rt_material* mats, uint32_t nmats, rt_mesh_host** out);
/* Deterministic synthetic meshes for the configs the reference cannot supply:
 *   kind 0: displaced-sphere "bunny" stand-in (~ntris triangles, bunny bbox);
 *   kind 1: 10M-style random triangle soup, centres U[-1,1]^3, half-size 0.01;
 *   kind 2: nx x nz grid of copies of `src` translated by `spacing` (instancing
 *           flattened into one mesh; the reference has no instancing). */
int rt_mesh_synth_bunny(uint32_t ntris_target, uint32_t seed, rt_mesh_host** out);
int rt_mesh_synth_soup(uint32_t ntris, uint32_t seed, rt_mesh_host** out);
int rt_mesh_synth_grid(const rt_mesh_host* src, uint32_t nx, uint32_t nz, float spacing,
                       rt_mesh_host** out);
int rt_mesh_scale(rt_mesh_host* m, float factor);   /* Mesh::scale, src/mesh.rs:246-252 */
int rt_mesh_view_get(const rt_mesh_host* m, rt_mesh_view* view);
void rt_mesh_free(rt_mesh_host* m);

typedef struct rt_bsp_host rt_bsp_host;
typedef struct rt_bsp_view {
    const uint32_t* tree;     /* nnodes x vec4u */
    const float* planes;      /* nnodes */
    const uint32_t* ids;      /* nids */
    float aabb[8];            /* BboxGpu */
    uint32_t nnodes, nids, max_depth;
} rt_bsp_view;

/* BspTree::new(bboxes, max_depth, max_leaf) + bsp_array() + primitive_ids(),
 * bit-identical to the reference's f32 arithmetic; nthreads <= 0 = hardware. */
int rt_bsp_build(const rt_mesh_host* mesh, uint32_t max_depth, uint32_t max_leaf,
                 int nthreads, rt_bsp_host** out);
int rt_bsp_view_get(const rt_bsp_host* b, rt_bsp_view* view);
void rt_bsp_free(rt_bsp_host* b);

typedef struct rt_bvh_host rt_bvh_host;
typedef struct rt_bvh_view {
    const rt_gpu_node* nodes;
    const uint32_t* tri_ids;
    uint32_t nnodes, nids;
} rt_bvh_view;

/* hlbvh::Bvh::new(mesh, max_prims) + flatten() + triangles(). Equal Morton
 * codes are ordered by primitive index (the reference's rdst order is
 * implementation-defined). */
int rt_bvh_build(const rt_mesh_host* mesh, uint32_t max_prims, rt_bvh_host** out);
int rt_bvh_view_get(const rt_bvh_host* b, rt_bvh_view* view);
void rt_bvh_free(rt_bvh_host* b);

/* Convenience: upload a host mesh / BSP / BVH built above. */
int rt_upload_mesh_host(rt_ctx* ctx, const rt_mesh_host* m);
int rt_upload_bsp_host(rt_ctx* ctx, const rt_bsp_host* b);
int rt_upload_bvh_host(rt_ctx* ctx, const rt_bvh_host* b);

#ifdef __cplusplus
}
#endif
#endif /* RT02562_RT_H */
