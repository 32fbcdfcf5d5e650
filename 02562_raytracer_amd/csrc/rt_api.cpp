// rt_api.cpp -- the extern "C" boundary (include/rt.h): HIP device/stream
// wrapper (replaces src/gpu_handles.rs), storage-buffer uploads (replaces
// src/bindings/*.rs create_buffer_init) with the MI355X data layout repack,
// and RenderState::render (src/render_state.rs:483-561).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "host_types.h"
#include "rt_internal.h"

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    ~DevBuf() { reset(); }
    void reset()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t bytes)
    {
        reset();
        if (bytes == 0) bytes = 16;
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        n = bytes;
        return hipSuccess;
    }
    hipError_t ensure(size_t bytes)   // at least `bytes`, keeping a large enough block
    {
        return p && n >= bytes ? hipSuccess : alloc(bytes);
    }
    void adopt(void* q, size_t bytes)   // take ownership of a hipMalloc'ed block
    {
        reset();
        p = q;
        n = bytes;
    }
    template <class T>
    T* as() const
    {
        return reinterpret_cast<T*>(p);
    }
};

}  // namespace

struct rt_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    int num_cus = 256;
    int waves_per_cu = 32;   // 8 waves per SIMD: the k_path register budget (RT_PATH_WAVES_PER_EU)
    int shade_threshold = -1;   // -1: per walk (BSP 8, BVH 4); pixel-major units refill together (coherent samples)
    uint32_t sample_chunk = 1;          // iterations per k_path work unit
    uint32_t unit_order = 1;            // 0: chunk-major, 1: pixel-major
    uint32_t bsp_cull = RT_BSP_CULL_AUTO;   // RT_OPT_BSP_CULL: subtree culling by content boxes in the BSP walk
    float bsp_scale = 0.0f;             // the scene's coordinate magnitude (set on upload; the margins' scale)
    uint32_t bsp_div_checked = 1;       // DevScene.bsp_div_checked (launch_plane_range, on upload)
    uint64_t sample_budget_mb = 16384;  // per-sample scratch (one pass at 1080p x 256 spp needs 8.1 GiB)
    DevBuf samples;
    bool detail = false;
    // host copies needed to build the triangle records on BSP/BVH upload
    std::vector<float> h_pos;
    std::vector<uint32_t> h_idx;
    uint32_t nverts = 0, ntris = 0, nmats = 0, nlights = 0;
    bool has_mesh = false;
    DevBuf pos, nrm, idx, mats, lights;
    DevBuf bsp_nodes, bsp_ids;   // bsp_nodes: [8-B nodes | 48-B records]
    DevBuf bsp_tm;               // per record slot {triangle id, material} (DevScene.bsp_tm)
    DevBuf plane_flag;           // launch_plane_range's 4-B result
    DevBuf bsp_ref_tree, bsp_ref_planes;   // bsp_array + planes in the reference layout (rt_download_bsp)
    float bsp_aabb8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t bsp_nnodes = 0, bsp_nids = 0;
    uint32_t bsp_rec_off = 0;
    uint32_t bsp_depth = 0;
    float aabb[6] = {0, 0, 0, 0, 0, 0};
    bool has_bsp = false;
    // the treelets' camera terms (rtk::launch_bsp_camera) are for this eye
    bool hcam_valid = false;
    float hcam_eye[3] = {0, 0, 0};
    DevBuf hcam_scratch;
    DevBuf bsp_sil;   // RT_BSP_CULL_SILHOUETTE's node data ((nnodes + 1) x 16 B)
    // RT_BSP_CULL_AUTO (probe_plan / probe_finish): the exact kernel the W9E1 BSP walk
    // runs for this scene (0: not decided yet), the probe's four timed launches --
    // certified, silhouette, certified, silhouette, each one of the renders' own
    // launches -- with their sample counts, the best time per 2^20 samples of each
    // kernel, the eye reach the choice was made at (a reach outside [1/2, 2] of it
    // probes again), and how many probes / probe launches this context has run
    uint32_t auto_cull = 0;
    uint32_t probe_n = 0;
    uint64_t probe_samples[4] = {0, 0, 0, 0};
    float auto_ms[2] = {0, 0};
    float probe_reach = 0.0f;
    uint32_t probes = 0, probe_launches = 0;
    hipEvent_t auto_ev[8] = {};
    DevBuf bvh_nodes, bvh_ids;   // bvh_nodes: [32-B nodes | 48-B records]
    DevBuf bvh_ref;              // the GpuNode array in the reference layout (rt_download_bvh)
    uint32_t bvh_rec_off = 0;
    uint32_t bvh_nnodes = 0, bvh_nids = 0;
    bool has_bvh = false;
    rt_uniform u;
    bool has_u = false;
    DevBuf jitter;
    bool has_jitter = false;
    float env[3] = {1.0f, 1.0f, 1.0f};
    DevBuf env_tex;   // RGBA8 equirectangular hdri0 (rt_set_environment_map)
    uint32_t env_w = 0, env_h = 0;
    DevBuf work, counters;
    DevBuf bvh_deep;   // BVH stack entries beyond the kernels' LDS share
    DevBuf srgb_thr;   // rt_frame_rgba8's 8-bit sRGB code thresholds
    rt_ray_counts last;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // RT_OPT_KERNEL_TIMING: event pairs around traversal-kernel launches (pool reused after reset)
    bool ktiming = false;
    std::vector<hipEvent_t> kev;
    size_t kused = 0;   // events recorded since the last reset (2 per launch)
    // ... and around the tile gather's transfers and the unpack kernel (rt_gather_time):
    // triples {before the transfers, after them, after the unpack} per call (an
    // rt_unpack_tiles call: its transfer part is empty)
    std::vector<hipEvent_t> gev;
    size_t gused = 0;
    // rt_comm_init: the tile gather's RCCL communicator (rt_gather_tiles)
    // RT_OPT_ASYNC_FOLD: the fold and its consumers on a second stream, the
    // per-sample scratch double-buffered (ev_free[b]: the fold that last read buffer b)
    bool async_fold = false;
    hipStream_t fold_stream = nullptr;
    hipEvent_t ev_path = nullptr, ev_enter = nullptr, ev_fold = nullptr, ev_free[2] = {nullptr, nullptr};
    DevBuf samples2;
    uint32_t sbuf = 0;
    bool fold_pending = false;   // work on fold_stream the context stream has not joined yet
    // rt_set_ray_capture: the counting renders append their traced rays here (device)
    float* cap_rays = nullptr;
    uint32_t* cap_flags = nullptr;
    uint64_t cap_max = 0;
    DevBuf cap_count;
    ncclComm_t comm = nullptr;
    uint32_t comm_nranks = 0, comm_rank = 0;
    DevBuf gather_accum, gather_ids;   // rank 0: every rank's packed tiles, rank-major
};

namespace {

int fail(rt_ctx* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    else rthost::set_error(msg);
    return code;
}

#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(ctx, e_ == hipErrorOutOfMemory ? RT_E_OOM : RT_E_DEVICE,                   \
                        std::string(#expr ": ") + hipGetErrorString(e_));                          \
    } while (0)

int upload(rt_ctx* c, DevBuf& b, const void* src, size_t bytes)
{
    hipError_t e = b.alloc(bytes);
    if (e != hipSuccess)
        return fail(c, e == hipErrorOutOfMemory ? RT_E_OOM : RT_E_DEVICE,
                    std::string("hipMalloc: ") + hipGetErrorString(e));
    if (bytes) HIPCHK(c, hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
    return RT_OK;
}

// 48-byte triangle record {v0, e0 = v1 - v0, e1 = v2 - v0, n = cross(e0, e1)}
// for every slot of `ids` (IEEE f32, no contraction: identical to computing
// them per test in the shader).
void build_recs(const std::vector<float>& pos, const std::vector<uint32_t>& idx, const uint32_t* ids, size_t nids,
                std::vector<float>& out)
{
    out.resize(nids * 12);
    auto work = [&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; k++) {
            const uint32_t* ix = &idx[(size_t)ids[k] * 4];
            const float* a = &pos[(size_t)ix[0] * 4];
            const float* b = &pos[(size_t)ix[1] * 4];
            const float* c = &pos[(size_t)ix[2] * 4];
            const float e0[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
            const float e1[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
            const float n[3] = {e0[1] * e1[2] - e0[2] * e1[1], e0[2] * e1[0] - e0[0] * e1[2],
                                e0[0] * e1[1] - e0[1] * e1[0]};
            float* o = &out[k * 12];
            o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = e0[0];
            o[4] = e0[1]; o[5] = e0[2]; o[6] = e1[0]; o[7] = e1[1];
            o[8] = e1[2]; o[9] = n[0]; o[10] = n[1]; o[11] = n[2];
        }
    };
    const size_t nthr = std::min<size_t>(std::max(1u, std::thread::hardware_concurrency()), 32);
    if (nids < 65536 || nthr == 1) {
        work(0, nids);
        return;
    }
    std::vector<std::thread> th;
    const size_t chunk = (nids + nthr - 1) / nthr;
    for (size_t t = 0; t < nthr; t++) {
        const size_t lo = t * chunk, hi = std::min(nids, lo + chunk);
        if (lo < hi) th.emplace_back(work, lo, hi);
    }
    for (auto& t : th) t.join();
}

// The current device, without joining the fold stream (RT_OPT_ASYNC_FOLD): the
// render calls and the fold's consumers, which order themselves against it.
int set_dev_nojoin(rt_ctx* c)
{
    HIPCHK(c, hipSetDevice(c->device));
    return RT_OK;
}

// The current device, with the fold stream's pending work joined into the
// context stream first (every entry point but the renders and the fold's
// consumers), so that synchronising the context stream covers it.
int set_dev(rt_ctx* c)
{
    HIPCHK(c, hipSetDevice(c->device));
    if (c->fold_pending) {
        HIPCHK(c, hipEventRecord(c->ev_fold, c->fold_stream));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_fold, 0));
        c->fold_pending = false;
    }
    return RT_OK;
}

// The stream the fold's consumers (unpack, gather, sRGB frame) run on: the fold
// stream under RT_OPT_ASYNC_FOLD, after the context stream's work so far.
int out_stream(rt_ctx* c, hipStream_t* s)
{
    if (!c->async_fold || !c->fold_stream) {
        *s = c->stream;
        return RT_OK;
    }
    HIPCHK(c, hipEventRecord(c->ev_enter, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->fold_stream, c->ev_enter, 0));
    c->fold_pending = true;
    *s = c->fold_stream;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_device_count(int* count)
{
    if (!count) return fail(nullptr, RT_E_INVALID, "rt_device_count: null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(nullptr, RT_E_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *count = n;
    return RT_OK;
}

int rt_create(int device, rt_ctx** out)
{
    if (!out) return fail(nullptr, RT_E_INVALID, "rt_create: null");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(nullptr, RT_E_DEVICE, "rt_create: no such HIP device");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return fail(nullptr, RT_E_DEVICE, "rt_create: hipGetDeviceProperties failed");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, RT_E_DEVICE, std::string("rt_create: kernels are built for gfx950, device is ") +
                                              prop.gcnArchName);
    rt_ctx* c = new rt_ctx();
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    memset(&c->u, 0, sizeof c->u);
    memset(&c->last, 0, sizeof c->last);
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess ||
        c->work.alloc(4096) != hipSuccess || c->counters.alloc(32 * sizeof(unsigned long long)) != hipSuccess) {
        delete c;
        return fail(nullptr, RT_E_DEVICE, "rt_create: stream/buffer setup failed");
    }
    c->stream = c->own;
    *out = c;
    return RT_OK;
}

void rt_destroy(rt_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    (void)rt_comm_destroy(c);
    for (hipEvent_t e : {c->ev_path, c->ev_enter, c->ev_fold, c->ev_free[0], c->ev_free[1]})
        if (e) (void)hipEventDestroy(e);
    if (c->fold_stream) (void)hipStreamDestroy(c->fold_stream);
    for (hipEvent_t e : c->kev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->gev) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (hipEvent_t e : c->auto_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int rt_set_stream(rt_ctx* c, void* s)
{
    if (!c) return RT_E_INVALID;
    c->stream = s ? (hipStream_t)s : c->own;
    return RT_OK;
}

void* rt_get_stream(rt_ctx* c) { return c ? (void*)c->stream : nullptr; }

int rt_synchronize(rt_ctx* c)
{
    if (!c) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_set_option(rt_ctx* c, int option, int64_t value)
{
    if (!c) return RT_E_INVALID;
    switch (option) {
    case RT_OPT_DETAIL_COUNTERS:
        c->detail = value != 0;
        return RT_OK;
    case RT_OPT_WAVES_PER_CU:
        if (value < 1 || value > 32) return fail(c, RT_E_INVALID, "waves per CU must be in [1,32]");
        c->waves_per_cu = (int)value;
        return RT_OK;
    case RT_OPT_SHADE_THRESHOLD:
        // 0x10000 | hi << 8 | lo: the per-wave choice between lo and hi (BSP walk)
        if ((value < -1 || value > 64) &&
            !((value & ~0x1FFFF) == 0 && (value & 0x10000) && (value & 0xFF) <= 64 && ((value >> 8) & 0xFF) <= 64))
            return fail(c, RT_E_INVALID, "shade threshold must be in [0,64] (64 = lockstep), 0x10000 | hi << 8 | lo "
                                         "(a per-wave choice, hi and lo in [0,64]), or -1 (the default)");
        c->shade_threshold = (int)value;
        return RT_OK;
    case RT_OPT_SAMPLE_CHUNK:
        if (value < 1 || value > (1 << 20)) return fail(c, RT_E_INVALID, "sample chunk must be in [1,2^20]");
        c->sample_chunk = (uint32_t)value;
        return RT_OK;
    case RT_OPT_KERNEL_TIMING:
        c->ktiming = value != 0;
        return RT_OK;
    case RT_OPT_BSP_CULL:
        if (value < RT_BSP_CULL_OFF || value > RT_BSP_CULL_AUTO)
            return fail(c, RT_E_INVALID, "BSP cull must be RT_BSP_CULL_OFF, _CERTIFIED, _FAST, _SILHOUETTE or _AUTO");
        if (c->bsp_cull != (uint32_t)value) {   // (RT_BSP_CULL_AUTO starts over)
            c->auto_cull = 0;
            c->probe_n = 0;
        }
        c->bsp_cull = (uint32_t)value;
        return RT_OK;
    case RT_OPT_UNIT_ORDER:
        if (value < 0 || value > 1) return fail(c, RT_E_INVALID, "unit order must be 0 or 1");
        c->unit_order = (uint32_t)value;
        return RT_OK;
    case RT_OPT_ASYNC_FOLD:
        if (value < 0 || value > 1) return fail(c, RT_E_INVALID, "async fold must be 0 or 1");
        if (int r = set_dev(c)) return r;   // joins pending fold work
        if (value && !c->fold_stream) {
            HIPCHK(c, hipStreamCreateWithFlags(&c->fold_stream, hipStreamNonBlocking));
            for (hipEvent_t* e : {&c->ev_path, &c->ev_enter, &c->ev_fold, &c->ev_free[0], &c->ev_free[1]})
                HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableTiming));
        }
        c->async_fold = value != 0;
        return RT_OK;
    case RT_OPT_SAMPLE_BUDGET_MB:
        if (value < 1 || value > (1 << 20)) return fail(c, RT_E_INVALID, "sample budget must be in [1,2^20] MiB");
        c->sample_budget_mb = (uint64_t)value;
        return RT_OK;
    default:
        return fail(c, RT_E_INVALID, "unknown option");
    }
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : rthost::get_error(); }

int rt_device_alloc(rt_ctx* c, size_t bytes, void** dptr)
{
    if (!c || !dptr) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    *dptr = nullptr;
    HIPCHK(c, hipMalloc(dptr, bytes ? bytes : 16));
    return RT_OK;
}

int rt_device_free(rt_ctx* c, void* dptr)
{
    if (!c) return RT_E_INVALID;
    if (!dptr) return RT_OK;
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(dptr));
    return RT_OK;
}

int rt_memcpy_to_host(rt_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c || (!dst && bytes) || (!src && bytes)) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_memcpy_to_device(rt_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c || (!dst && bytes) || (!src && bytes)) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_memset_device(rt_ctx* c, void* dst, int value, size_t bytes)
{
    if (!c || (!dst && bytes)) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipMemsetAsync(dst, value, bytes, c->stream));
    return RT_OK;
}

int rt_timer_start(rt_ctx* c)
{
    if (!c) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    if (!c->ev0) {
        HIPCHK(c, hipEventCreate(&c->ev0));
        HIPCHK(c, hipEventCreate(&c->ev1));
    }
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    return RT_OK;
}

int rt_kernel_time(rt_ctx* c, int reset, double* total_ms, uint32_t* launches)
{
    if (!c) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    double tot = 0.0;
    for (size_t i = 0; i + 1 < c->kused; i += 2) {
        HIPCHK(c, hipEventSynchronize(c->kev[i + 1]));
        float ms = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->kev[i], c->kev[i + 1]));
        tot += ms;
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = (uint32_t)(c->kused / 2);
    if (reset) c->kused = 0;
    return RT_OK;
}

int rt_timer_stop(rt_ctx* c, float* ms)
{
    if (!c || !ms || !c->ev0) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipEventSynchronize(c->ev1));
    HIPCHK(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
    return RT_OK;
}

int rt_upload_mesh(rt_ctx* c, const float* pos_vec4, const float* nrm_vec4, uint32_t nverts,
                   const uint32_t* idx_vec4u, uint32_t ntris, const rt_material* mats, uint32_t nmats,
                   const uint32_t* light_idx, uint32_t nlight)
{
    if (!c) return RT_E_INVALID;
    if ((!pos_vec4 && nverts) || (!idx_vec4u && ntris) || !mats || nmats == 0)
        return fail(c, RT_E_INVALID, "rt_upload_mesh: missing arrays (need >= 1 material)");
    for (size_t t = 0; t < ntris; t++)
        for (int k = 0; k < 3; k++)
            if (idx_vec4u[t * 4 + k] >= nverts) return fail(c, RT_E_INVALID, "rt_upload_mesh: vertex index out of range");
    std::vector<uint32_t> lights;
    if (light_idx) {
        if (nlight == 0 || light_idx[0] != 0xFFFFFFFFu)
            return fail(c, RT_E_INVALID, "rt_upload_mesh: light list must start with the UINT32_MAX sentinel");
        lights.assign(light_idx, light_idx + nlight);
        for (uint32_t i = 1; i < nlight; i++)
            if (lights[i] >= ntris) return fail(c, RT_E_INVALID, "rt_upload_mesh: light index out of range");
    } else {
        std::vector<uint32_t> ix(idx_vec4u, idx_vec4u + (size_t)ntris * 4);
        std::vector<rt_material> mv(mats, mats + nmats);
        lights = rthost::light_list(ix, mv);
    }
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->has_mesh = c->has_bsp = c->has_bvh = false;
    c->h_pos.assign(pos_vec4, pos_vec4 + (size_t)nverts * 4);
    c->h_idx.assign(idx_vec4u, idx_vec4u + (size_t)ntris * 4);
    std::vector<float> nrm;
    if (nrm_vec4) nrm.assign(nrm_vec4, nrm_vec4 + (size_t)nverts * 4);
    else nrm.assign((size_t)nverts * 4, 0.0f);
    int r;
    if ((r = upload(c, c->pos, c->h_pos.data(), c->h_pos.size() * 4))) return r;
    if ((r = upload(c, c->nrm, nrm.data(), nrm.size() * 4))) return r;
    if ((r = upload(c, c->idx, c->h_idx.data(), c->h_idx.size() * 4))) return r;
    if ((r = upload(c, c->mats, mats, (size_t)nmats * sizeof(rt_material)))) return r;
    if ((r = upload(c, c->lights, lights.data(), lights.size() * 4))) return r;
    c->nverts = nverts;
    c->ntris = ntris;
    c->nmats = nmats;
    c->nlights = (uint32_t)lights.size();
    c->has_mesh = true;
    return RT_OK;
}

// The traversal layout of the context's BSP (reference arrays already in
// bsp_ref_tree / bsp_ref_planes / bsp_ids, mesh in pos / idx): content boxes,
// 96-B treelets and the 48-B records (rt_bsp_build.hip launch_bsp_repack), and
// the scale of the content boxes' margins: the largest coordinate magnitude of
// the BSP's root box (bsp_box_miss in rt_kernels.hip adds the ray origin's).
static int repack_bsp(rt_ctx* c, uint32_t nnodes, uint32_t nids, size_t rec_off, size_t total, const float aabb[8])
{
    c->hcam_valid = false;
    c->auto_cull = 0;   // (a new scene: RT_BSP_CULL_AUTO probes again)
    c->probe_n = 0;
    HIPCHK(c, c->bsp_nodes.alloc(total));
    DevBuf boxes;
    HIPCHK(c, boxes.alloc((size_t)nnodes * 64));
    HIPCHK(c, c->bsp_tm.alloc((size_t)std::max<uint32_t>(nids, 1u) * 8));
    if (rtk::launch_bsp_repack(c->bsp_ref_tree.as<uint32_t>(), c->bsp_ref_planes.as<float>(), nnodes,
                               (uint32_t)rec_off, c->bsp_nodes.p, c->pos.as<float4>(), c->idx.as<uint4>(),
                               c->bsp_ids.as<uint32_t>(), nids, 0.0f, boxes.p, c->bsp_tm.as<uint2>(), c->stream))
        return fail(c, RT_E_DEVICE, "BSP repack launch failed");
    if (!c->plane_flag.p) HIPCHK(c, c->plane_flag.alloc(4));
    if (rtk::launch_plane_range(c->bsp_ref_tree.as<uint32_t>(), c->bsp_ref_planes.as<float>(), nnodes,
                                c->plane_flag.as<uint32_t>(), c->stream))
        return fail(c, RT_E_DEVICE, "BSP plane range launch failed");
    uint32_t pflag = 1;
    HIPCHK(c, hipMemcpyAsync(&pflag, c->plane_flag.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->bsp_div_checked = pflag != 0u;
    float scale = 0.0f;
    for (int k : {0, 1, 2, 4, 5, 6})
        if (std::isfinite(aabb[k])) scale = std::max(scale, std::fabs(aabb[k]));
    c->bsp_scale = scale;
    return RT_OK;
}

int rt_upload_bsp(rt_ctx* c, const float aabb[8], const uint32_t* tree, const float* planes, uint32_t nnodes,
                  const uint32_t* ids, uint32_t nids, uint32_t max_depth)
{
    if (!c) return RT_E_INVALID;
    if (!c->has_mesh) return fail(c, RT_E_NOT_READY, "rt_upload_bsp: upload the mesh first");
    if (!aabb || !tree || !planes || (!ids && nids)) return fail(c, RT_E_INVALID, "rt_upload_bsp: null array");
    if (max_depth == 0 || max_depth >= 32 || (uint64_t)nnodes != ((uint64_t)1 << (max_depth + 1)) - 1)
        return fail(c, RT_E_INVALID, "rt_upload_bsp: nnodes must be 2^(max_depth+1)-1, max_depth in [1,31]");
    for (uint32_t k = 0; k < nids; k++)
        if (ids[k] >= c->ntris) return fail(c, RT_E_INVALID, "rt_upload_bsp: triangle id out of range");
    // validate the reachable tree (implicit children, leaves inside ids)
    std::vector<uint32_t> stack{0};
    while (!stack.empty()) {
        const uint32_t i = stack.back();
        stack.pop_back();
        const uint32_t* n = tree + 4 * (size_t)i;
        if ((n[0] & 3u) == 3u) {
            if ((uint64_t)n[1] + (n[0] >> 2) > nids)
                return fail(c, RT_E_INVALID, "rt_upload_bsp: leaf range outside treeIds");
            if ((n[0] >> 2) >= (1u << 24))
                return fail(c, RT_E_UNSUPPORTED, "rt_upload_bsp: leaf with 2^24 or more triangles");
            continue;
        }
        const uint64_t l = 2ull * i + 1, rgt = 2ull * i + 2;
        if (rgt >= nnodes || n[2] != l || n[3] != rgt)
            return fail(c, RT_E_INVALID, "rt_upload_bsp: interior node children are not 2i+1, 2i+2 inside the array");
        stack.push_back((uint32_t)l);
        stack.push_back((uint32_t)rgt);
    }
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->has_bsp = false;
    int r;
    // One allocation [treelets | records], read through one buffer resource
    // with 32-bit offsets (DESIGN.md "Data layout in HBM"), laid out on the
    // device by launch_bsp_repack from the reference arrays (the same code as
    // rt_build_bsp_device):
    //  * treelet of node M (1-based heap index), 96 B at 96*M: M's content box,
    //    the 8-B nodes {M | 2M, 2M+1 | 4M, 4M+1 | 4M+2, 4M+3} and the certified
    //    culling's 16 B of subtree data -- everything a 3-level walk from M reads;
    //  * 8-B node: interior {axis, plane bits}; leaf {3 | (48*count) << 2, byte
    //    offset of its first record} (children implicit: 2i+1, 2i+2 0-based);
    //  * record k (treeIds slot k): 48 B {v0, e0, e1, n} at rec_off + 48*k.
    const size_t slots = (size_t)nnodes + 1;
    const size_t rec_off = (slots * rtk::BSP_TREELET_BYTES + 255) & ~(size_t)255;
    const size_t total = rec_off + (size_t)nids * 48;
    if (total >= ((size_t)1 << 32))
        return fail(c, RT_E_UNSUPPORTED, "rt_upload_bsp: BSP treelets + records must stay below 4 GiB (96-B treelets: "
                                              "max_depth 24 takes 3.2 GB, leaving room for ~22M records)");
    if ((r = upload(c, c->bsp_ref_tree, tree, (size_t)nnodes * 16))) return r;
    if ((r = upload(c, c->bsp_ref_planes, planes, (size_t)nnodes * 4))) return r;
    if ((r = upload(c, c->bsp_ids, ids, (size_t)nids * 4))) return r;
    if ((r = repack_bsp(c, nnodes, nids, rec_off, total, aabb))) return r;
    c->bsp_rec_off = (uint32_t)rec_off;
    memcpy(c->bsp_aabb8, aabb, sizeof c->bsp_aabb8);
    c->bsp_nnodes = nnodes;
    c->bsp_nids = nids;
    c->bsp_depth = max_depth;
    c->aabb[0] = aabb[0];
    c->aabb[1] = aabb[1];
    c->aabb[2] = aabb[2];
    c->aabb[3] = aabb[4];
    c->aabb[4] = aabb[5];
    c->aabb[5] = aabb[6];
    c->has_bsp = true;
    return RT_OK;
}

int rt_upload_bvh(rt_ctx* c, const rt_gpu_node* nodes, uint32_t nnodes, const uint32_t* tri_ids, uint32_t nids)
{
    if (!c) return RT_E_INVALID;
    if (!c->has_mesh) return fail(c, RT_E_NOT_READY, "rt_upload_bvh: upload the mesh first");
    if (!nodes || nnodes == 0 || (!tri_ids && nids)) return fail(c, RT_E_INVALID, "rt_upload_bvh: null array");
    for (uint32_t k = 0; k < nids; k++)
        if (tri_ids[k] >= c->ntris) return fail(c, RT_E_INVALID, "rt_upload_bvh: triangle id out of range");
    // validate nodes reachable from the root (bvh.wgsl:168-179 walk)
    std::vector<uint8_t> seen(nnodes, 0);
    std::vector<uint32_t> stack{0};
    while (!stack.empty()) {
        const uint32_t i = stack.back();
        stack.pop_back();
        if (seen[i]) continue;
        seen[i] = 1;
        const rt_gpu_node& n = nodes[i];
        if (n.n_prims > 0) {
            if ((uint64_t)n.offset_ptr + n.n_prims > nids) return fail(c, RT_E_INVALID, "rt_upload_bvh: leaf range");
        } else {
            if ((uint64_t)i + 1 >= nnodes || n.offset_ptr >= nnodes)
                return fail(c, RT_E_INVALID, "rt_upload_bvh: child index out of range");
            stack.push_back(i + 1);
            stack.push_back(n.offset_ptr);
        }
    }
    std::vector<float> recs;
    build_recs(c->h_pos, c->h_idx, tri_ids, nids, recs);
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->has_bvh = false;
    int r;
    // One allocation [32-B node records | 48-B triangle records], read through
    // one buffer resource with 32-bit offsets.  Node record: {min.xyz, w0}
    // {max.xyz, w1}; interior: w0 = byte offset of the right child (offset_ptr),
    // w1 = 0; leaf: w0 = byte offset of its first triangle record, w1 = 48*n_prims.
    const size_t rec_off = ((size_t)nnodes * 32 + 255) & ~(size_t)255;
    const size_t total = rec_off + recs.size() * 4;
    if (total >= ((size_t)1 << 32))
        return fail(c, RT_E_UNSUPPORTED, "rt_upload_bvh: BVH nodes + records must stay below 4 GiB");
    {
        std::vector<uint8_t> blob(total, 0);
        for (uint32_t i = 0; i < nnodes; i++) {
            const rt_gpu_node& n = nodes[i];
            uint32_t* o = reinterpret_cast<uint32_t*>(blob.data() + 32 * (size_t)i);
            memcpy(o, n.min, 12);
            memcpy(o + 4, n.max, 12);
            if (n.n_prims > 0) {
                o[3] = (uint32_t)(rec_off + 48ull * n.offset_ptr);
                o[7] = 48u * n.n_prims;
            } else {
                o[3] = (uint32_t)(32ull * n.offset_ptr);
                o[7] = 0u;
            }
        }
        memcpy(blob.data() + rec_off, recs.data(), recs.size() * 4);
        if ((r = upload(c, c->bvh_nodes, blob.data(), blob.size()))) return r;
    }
    c->bvh_rec_off = (uint32_t)rec_off;
    if ((r = upload(c, c->bvh_ids, tri_ids, (size_t)nids * 4))) return r;
    if ((r = upload(c, c->bvh_ref, nodes, (size_t)nnodes * sizeof(rt_gpu_node)))) return r;
    c->bvh_nnodes = nnodes;
    c->bvh_nids = nids;
    c->has_bvh = true;
    return RT_OK;
}

int rt_build_bvh_device(rt_ctx* c, uint32_t max_prims, rt_bvh_build_times* times)
{
    if (!c) return RT_E_INVALID;
    if (!c->has_mesh) return fail(c, RT_E_NOT_READY, "rt_build_bvh_device: upload the mesh first");
    if (max_prims == 0) return fail(c, RT_E_INVALID, "rt_build_bvh_device: max_prims must be >= 1");
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->has_bvh = false;
    rtk::BvhDeviceOut o;
    std::string err;
    const int r = rtk::build_bvh_device(c->pos.as<float4>(), c->idx.as<uint4>(), c->ntris, max_prims, c->num_cus,
                                        c->stream, o, times, err);
    DevBuf nodes_ref, ids;   // own the outputs from here on
    if (o.nodes) nodes_ref.adopt(o.nodes, (size_t)o.nnodes * sizeof(rt_gpu_node));
    if (o.ids) ids.adopt(o.ids, (size_t)o.nids * 4);
    if (r) return fail(c, r, err);
    // traversal layout, as rt_upload_bvh (records of the bvh_triangles slots)
    const size_t rec_off = ((size_t)o.nnodes * 32 + 255) & ~(size_t)255;
    const size_t total = rec_off + (size_t)o.nids * 48;
    if (total >= ((size_t)1 << 32))
        return fail(c, RT_E_UNSUPPORTED, "rt_build_bvh_device: BVH nodes + records must stay below 4 GiB");
    HIPCHK(c, c->bvh_nodes.alloc(total));
    if (rtk::launch_bvh_repack(nodes_ref.as<rt_gpu_node>(), o.nnodes, (uint32_t)rec_off, c->bvh_nodes.p,
                               c->pos.as<float4>(), c->idx.as<uint4>(), ids.as<uint32_t>(), o.nids, c->stream))
        return fail(c, RT_E_DEVICE, "rt_build_bvh_device: repack launch failed");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->bvh_ref.adopt(nodes_ref.p, nodes_ref.n);
    nodes_ref.p = nullptr;
    c->bvh_ids.adopt(ids.p, ids.n);
    ids.p = nullptr;
    c->bvh_rec_off = (uint32_t)rec_off;
    c->bvh_nnodes = o.nnodes;
    c->bvh_nids = o.nids;
    c->has_bvh = true;
    return RT_OK;
}

int rt_build_bsp_device(rt_ctx* c, uint32_t max_depth, uint32_t max_leaf, rt_bsp_build_times* times)
{
    if (!c) return RT_E_INVALID;
    if (!c->has_mesh) return fail(c, RT_E_NOT_READY, "rt_build_bsp_device: upload the mesh first");
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->has_bsp = false;
    rtk::BspDeviceOut o;
    std::string err;
    const int r = rtk::build_bsp_device(c->pos.as<float4>(), c->idx.as<uint4>(), c->ntris, max_depth, max_leaf,
                                        c->num_cus, c->stream, o, times, err);
    DevBuf tree, planes, ids;   // own the outputs from here on
    if (o.tree) tree.adopt(o.tree, (size_t)o.nnodes * 16);
    if (o.planes) planes.adopt(o.planes, (size_t)o.nnodes * 4);
    if (o.ids) ids.adopt(o.ids, std::max<size_t>(16, (size_t)o.nids * 4));
    if (r) return fail(c, r, err);
    const size_t slots = (size_t)o.nnodes + 1;
    const size_t rec_off = (slots * rtk::BSP_TREELET_BYTES + 255) & ~(size_t)255;
    const size_t total = rec_off + (size_t)o.nids * 48;
    if (total >= ((size_t)1 << 32))
        return fail(c, RT_E_UNSUPPORTED, "rt_build_bsp_device: BSP treelets + records must stay below 4 GiB");
    c->bsp_ref_tree.adopt(tree.p, tree.n);
    tree.p = nullptr;
    c->bsp_ref_planes.adopt(planes.p, planes.n);
    planes.p = nullptr;
    c->bsp_ids.adopt(ids.p, ids.n);
    ids.p = nullptr;
    if (int rr = repack_bsp(c, o.nnodes, o.nids, rec_off, total, o.aabb)) return rr;
    c->bsp_rec_off = (uint32_t)rec_off;
    c->bsp_depth = max_depth;
    memcpy(c->bsp_aabb8, o.aabb, sizeof c->bsp_aabb8);
    c->aabb[0] = o.aabb[0];
    c->aabb[1] = o.aabb[1];
    c->aabb[2] = o.aabb[2];
    c->aabb[3] = o.aabb[4];
    c->aabb[4] = o.aabb[5];
    c->aabb[5] = o.aabb[6];
    c->bsp_nnodes = o.nnodes;
    c->bsp_nids = o.nids;
    c->has_bsp = true;
    return RT_OK;
}

int rt_download_bsp(rt_ctx* c, uint32_t* tree, float* planes, uint32_t cap_nodes, uint32_t* ids, uint32_t cap_ids,
                    float aabb[8], uint32_t* nnodes, uint32_t* nids)
{
    if (!c) return RT_E_INVALID;
    if (!c->has_bsp) return fail(c, RT_E_NOT_READY, "rt_download_bsp: no BSP on the context");
    if (nnodes) *nnodes = c->bsp_nnodes;
    if (nids) *nids = c->bsp_nids;
    if (aabb) memcpy(aabb, c->bsp_aabb8, sizeof c->bsp_aabb8);
    if (int r = set_dev(c)) return r;
    if ((tree || planes) && cap_nodes < c->bsp_nnodes) return fail(c, RT_E_INVALID, "rt_download_bsp: arrays too small");
    if (ids && cap_ids < c->bsp_nids) return fail(c, RT_E_INVALID, "rt_download_bsp: id array too small");
    if (tree)
        HIPCHK(c, hipMemcpyAsync(tree, c->bsp_ref_tree.p, (size_t)c->bsp_nnodes * 16, hipMemcpyDeviceToHost, c->stream));
    if (planes)
        HIPCHK(c, hipMemcpyAsync(planes, c->bsp_ref_planes.p, (size_t)c->bsp_nnodes * 4, hipMemcpyDeviceToHost,
                                 c->stream));
    if (ids && c->bsp_nids)
        HIPCHK(c, hipMemcpyAsync(ids, c->bsp_ids.p, (size_t)c->bsp_nids * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

static int ensure_hcam(rt_ctx* c);

// the culling modes whose margin is the certified bound (their treelets carry the camera terms)
static bool cull_certified(const rt_ctx* c)
{
    return c->bsp_cull == RT_BSP_CULL_CERTIFIED || c->bsp_cull == RT_BSP_CULL_SILHOUETTE ||
           c->bsp_cull == RT_BSP_CULL_AUTO;
}

// whether a render's walk has a silhouette instantiation: W9E1's BSP path kernel (not
// its transparent form, selection1 7, launch_render); the query and batch kernels have
// one too.  Every other kernel runs the certified form under SILHOUETTE and AUTO.
static bool has_silhouette(const rt_ctx* c, rt_mode mode, rt_traverse trav)
{
    return mode == RT_MODE_W9E1 && trav == RT_TRAVERSE_BSP && c->u.selection1 != 7u;
}

// the mode a BSP kernel runs (sil: it has a silhouette instantiation): the silhouette
// bound needs its node data, made with the camera terms (ensure_hcam), so without them
// (no uniforms, or a non-finite eye) it runs the certified kernel; RT_BSP_CULL_AUTO runs
// its probe's choice (certified until the probe has decided)
static uint32_t cull_in_use(const rt_ctx* c, bool sil = true)
{
    if (c->bsp_cull == RT_BSP_CULL_SILHOUETTE || c->bsp_cull == RT_BSP_CULL_AUTO) {
        const bool s = sil && c->hcam_valid &&
                       (c->bsp_cull == RT_BSP_CULL_SILHOUETTE || c->auto_cull == RT_BSP_CULL_SILHOUETTE);
        return s ? RT_BSP_CULL_SILHOUETTE : RT_BSP_CULL_CERTIFIED;
    }
    return c->bsp_cull;
}
int rt_download_bsp_treelets(rt_ctx* c, void* dst, uint64_t cap_bytes, uint64_t* bytes)
{
    if (!c) return RT_E_INVALID;
    if (!c->has_bsp) return fail(c, RT_E_NOT_READY, "rt_download_bsp_treelets: no BSP on the context");
    const uint64_t nt = ((uint64_t)c->bsp_nnodes + 1) * rtk::BSP_TREELET_BYTES;
    const uint64_t ns = ((uint64_t)c->bsp_nnodes + 1) * 16;
    const uint64_t n = nt + ns;
    if (bytes) *bytes = n;
    if (!dst) return RT_OK;
    if (cap_bytes < n) return fail(c, RT_E_INVALID, "rt_download_bsp_treelets: buffer too small");
    if (int r = set_dev(c)) return r;   // (first: ensure_hcam may launch the camera-term kernels)
    if (int r = ensure_hcam(c)) return r;
    HIPCHK(c, hipMemcpyAsync(dst, c->bsp_nodes.p, nt, hipMemcpyDeviceToHost, c->stream));
    // the silhouette section only when it was made for this BSP and the uniforms' eye
    // (ensure_hcam leaves it alone in the uncertified modes)
    const bool sil_now = c->hcam_valid && cull_certified(c) && c->has_u &&
                         memcmp(c->u.camera_pos, c->hcam_eye, sizeof c->hcam_eye) == 0;
    if (sil_now && c->bsp_sil.n >= ns) HIPCHK(c, hipMemcpyAsync(static_cast<uint8_t*>(dst) + nt, c->bsp_sil.p, ns,
                                                     hipMemcpyDeviceToHost, c->stream));
    else memset(static_cast<uint8_t*>(dst) + nt, 0, ns);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_download_bvh(rt_ctx* c, rt_gpu_node* nodes, uint32_t cap_nodes, uint32_t* tri_ids, uint32_t cap_ids,
                    uint32_t* nnodes, uint32_t* nids)
{
    if (!c) return RT_E_INVALID;
    if (!c->has_bvh) return fail(c, RT_E_NOT_READY, "rt_download_bvh: no BVH on the context");
    if (nnodes) *nnodes = c->bvh_nnodes;
    if (nids) *nids = c->bvh_nids;
    if (int r = set_dev(c)) return r;
    if (nodes) {
        if (cap_nodes < c->bvh_nnodes) return fail(c, RT_E_INVALID, "rt_download_bvh: node array too small");
        HIPCHK(c, hipMemcpyAsync(nodes, c->bvh_ref.p, (size_t)c->bvh_nnodes * sizeof(rt_gpu_node),
                                 hipMemcpyDeviceToHost, c->stream));
    }
    if (tri_ids) {
        if (cap_ids < c->bvh_nids) return fail(c, RT_E_INVALID, "rt_download_bvh: id array too small");
        HIPCHK(c, hipMemcpyAsync(tri_ids, c->bvh_ids.p, (size_t)c->bvh_nids * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_set_uniforms(rt_ctx* c, const rt_uniform* u, const float* jitter)
{
    if (!c || !u) return RT_E_INVALID;
    if (u->resolution[0] == 0 || u->resolution[1] == 0) return fail(c, RT_E_INVALID, "rt_set_uniforms: zero resolution");
    // k_path packs a lane's pixel as x | y << 16
    if (u->resolution[0] > 65535u || u->resolution[1] > 65535u)
        return fail(c, RT_E_INVALID, "rt_set_uniforms: resolution above 65535");
    if (u->subdivision_level == 0 || u->subdivision_level > 10)
        return fail(c, RT_E_INVALID, "rt_set_uniforms: subdivision_level must be in [1,10] (uniform.rs:36)");
    if (!jitter && u->subdivision_level != 1)
        return fail(c, RT_E_INVALID, "rt_set_uniforms: jitter table required when subdivision_level > 1");
    if (int r = set_dev(c)) return r;
    c->u = *u;
    c->has_u = true;
    c->has_jitter = false;
    if (jitter) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const size_t bytes = (size_t)u->subdivision_level * u->subdivision_level * 2 * sizeof(float);
        if (int r = upload(c, c->jitter, jitter, bytes)) return r;
        c->has_jitter = true;
    }
    return RT_OK;
}

int rt_set_environment(rt_ctx* c, const float rgb[3])
{
    if (!c || !rgb) return RT_E_INVALID;
    memcpy(c->env, rgb, sizeof c->env);
    return RT_OK;
}

// The gather/unpack event triples (RT_OPT_KERNEL_TIMING, rt_gather_time): the
// next pooled event of the current call, recorded on stream s (nullptr: off).
// The first event of a triple reserves all three (a call records the other two
// only when the first was recorded, so the pool stays in whole triples).
static hipEvent_t gather_event(rt_ctx* c, hipStream_t s)
{
    if (!c->ktiming) return nullptr;
    if (c->gused % 3 == 0) {
        if (c->gused >= 3 * 4096) return nullptr;
        while (c->gev.size() < c->gused + 3) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            c->gev.push_back(e);
        }
    }
    hipEvent_t e = c->gev[c->gused];
    (void)hipEventRecord(e, s);
    c->gused++;
    return e;
}

// Launch the traversal kernel, bracketed by a pair of pooled events when
// kernel timing is on (rt_kernel_time).
static int launch_timed(rt_ctx* c, const rtk::DevScene& S, const rtk::DevLaunch& L, rt_mode mode, rt_traverse trav)
{
    const bool t = c->ktiming && c->kused + 2 <= 8192;
    if (t) {
        while (c->kev.size() < c->kused + 2) {
            hipEvent_t e;
            HIPCHK(c, hipEventCreate(&e));
            c->kev.push_back(e);
        }
        HIPCHK(c, hipEventRecord(c->kev[c->kused], c->stream));
    }
    int r = rtk::launch_render(S, L, mode, trav, c->detail, c->num_cus, c->waves_per_cu, c->stream);
    if (r) return fail(c, r, std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    if (t) {
        HIPCHK(c, hipEventRecord(c->kev[c->kused + 1], c->stream));
        c->kused += 2;
    }
    return RT_OK;
}

int rt_set_environment_map(rt_ctx* c, const uint8_t* rgba8, uint32_t width, uint32_t height)
{
    if (!c) return RT_E_INVALID;
    if (!rgba8) {
        c->env_tex.reset();
        c->env_w = c->env_h = 0;
        return RT_OK;
    }
    if (width == 0 || height == 0 || (uint64_t)width * height >= (1ull << 31))
        return fail(c, RT_E_INVALID, "rt_set_environment_map: bad texture size");
    if (int r = set_dev(c)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (int r = upload(c, c->env_tex, rgba8, (size_t)width * height * 4)) return r;
    c->env_w = width;
    c->env_h = height;
    return RT_OK;
}

// The device-resident scene as the kernels read it (rt_internal.h DevScene).
// The camera terms of the treelets for the uniforms' eye (certified culling,
// rt_bsp_build.hip launch_bsp_camera): recomputed when the eye moves.
static int ensure_hcam(rt_ctx* c)
{
    if (!c->has_bsp || !c->has_u || !cull_certified(c)) return RT_OK;
    const float* e = c->u.camera_pos;
    if (c->hcam_valid && memcmp(e, c->hcam_eye, sizeof c->hcam_eye) == 0) return RT_OK;
    if (!(std::isfinite(e[0]) && std::isfinite(e[1]) && std::isfinite(e[2]))) return RT_OK;
    HIPCHK(c, c->hcam_scratch.ensure((size_t)c->bsp_nnodes * 24));
    HIPCHK(c, c->bsp_sil.ensure(((size_t)c->bsp_nnodes + 1) * 16));
    HIPCHK(c, hipMemsetAsync(c->bsp_sil.p, 0, 16, c->stream));   // (slot 0: no node)
    if (rtk::launch_bsp_camera(c->bsp_ref_tree.as<uint32_t>(), c->bsp_nnodes, c->pos.as<float4>(), c->idx.as<uint4>(),
                               c->bsp_ids.as<uint32_t>(), c->bsp_nids, e, c->bsp_nodes.p, c->bsp_sil.as<uint32_t>(),
                               c->hcam_scratch.p, c->stream))
        return fail(c, RT_E_DEVICE, "BSP camera terms: launch failed");
    memcpy(c->hcam_eye, e, sizeof c->hcam_eye);
    c->hcam_valid = true;
    return RT_OK;
}

static rtk::DevScene dev_scene(const rt_ctx* c)
{
    rtk::DevScene S;
    memset(&S, 0, sizeof S);
    for (int k = 0; k < 3; k++) S.cam_eye[k] = c->hcam_valid ? c->hcam_eye[k] : NAN;
    S.pos = c->pos.as<float4>();
    S.nrm = c->nrm.as<float4>();
    S.tri_idx = c->idx.as<uint4>();
    S.mats = c->mats.as<rt_material>();
    S.lights = c->lights.as<uint32_t>();
    S.nverts = c->nverts;
    S.ntris = c->ntris;
    S.nmats = c->nmats;
    S.nlights = c->nlights;
    S.bsp_nodes = c->bsp_nodes.as<uint2>();
    S.bsp_recs = reinterpret_cast<const float4*>(c->bsp_nodes.as<uint8_t>() + c->bsp_rec_off);
    S.bsp_bytes = (uint32_t)c->bsp_nodes.n;
    S.bsp_rec_off = c->bsp_rec_off;
    S.bsp_ids = c->bsp_ids.as<uint32_t>();
    S.bsp_tm = c->bsp_tm.as<uint2>();
    S.bsp_sil = c->bsp_sil.as<uint4>();
    S.bsp_cull_mode = cull_in_use(c);
    S.bsp_div_checked = c->bsp_div_checked;
    S.bsp_depth = c->bsp_depth;
    memcpy(S.aabb, c->aabb, sizeof S.aabb);
    S.bvh_base = c->bvh_nodes.as<uint8_t>();
    S.bvh_bytes = (uint32_t)c->bvh_nodes.n;
    S.bvh_rec_off = c->bvh_rec_off;
    S.bvh_ids = c->bvh_ids.as<uint32_t>();
    S.bvh_nnodes = c->bvh_nnodes;
    // the culling margin as data (rt_internal.h DevScene, rt_kernels.hip bsp_box_miss)
    S.bsp_cull_gap = c->bsp_cull != RT_BSP_CULL_OFF ? 0x1p-18f : INFINITY;
    S.bsp_cull_emax = c->bsp_cull != RT_BSP_CULL_OFF ? FLT_MAX : INFINITY;
    // off: the fast formula's constants (k1 = 0 picks k_path's fast-margin
    // instantiation, launch_path); the +inf gap culls nothing either way
    if (!cull_certified(c)) {
        S.cull_k1 = 0.0f;
        S.cull_k3 = 0.0f;
        S.cull_ko = 0x1p-10f;
        S.bsp_margin = std::ldexp(c->bsp_scale, -10);
    } else {
        S.cull_k1 = 36.0f * 0x1p-24f;
        S.cull_k3 = 2.0f * 0x1p-24f;
        S.cull_ko = 0x1p-19f;
        S.bsp_margin = std::ldexp(c->bsp_scale, -19);
    }
    return S;
}

int rt_set_ray_capture(rt_ctx* c, float* rays_dev, uint32_t* flags_dev, uint64_t cap)
{
    if (!c || (rays_dev && !flags_dev)) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    if (rays_dev && !c->cap_count.p) HIPCHK(c, c->cap_count.alloc(8));
    if (rays_dev) HIPCHK(c, hipMemsetAsync(c->cap_count.p, 0, 8, c->stream));
    c->cap_rays = rays_dev;
    c->cap_flags = flags_dev;
    c->cap_max = rays_dev ? cap : 0;
    return RT_OK;
}

int rt_ray_capture_count(rt_ctx* c, uint64_t* n)
{
    if (!c || !n) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    *n = 0;
    if (!c->cap_count.p) return RT_OK;
    HIPCHK(c, hipMemcpyAsync(n, c->cap_count.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_trace_batch(rt_ctx* c, rt_traverse trav, const float* rays_dev, const uint32_t* flags_dev, uint32_t n,
                   uint32_t* hits_dev)
{
    if (!c) return RT_E_INVALID;
    if (n == 0) return RT_OK;
    if (!rays_dev || !hits_dev) return fail(c, RT_E_INVALID, "rt_trace_batch: rays and hits are required");
    // k_trace's shard heads hand out 64-ray blocks below a 2^28 cap: past 2^31 rays the
    // capped head would keep handing out the same block (and n + 63 overflows near 2^32)
    if (n >= (1u << 31)) return fail(c, RT_E_INVALID, "rt_trace_batch: n must be below 2^31");
    if (trav != RT_TRAVERSE_BSP) return fail(c, RT_E_UNSUPPORTED, "rt_trace_batch: the BSP walk only");
    if (!c->has_mesh || !c->has_bsp) return fail(c, RT_E_NOT_READY, "rt_trace_batch: no BSP uploaded");
    if (int r = set_dev(c)) return r;
    if (int r = ensure_hcam(c)) return r;
    const uint32_t T = c->shade_threshold >= 0 ? (uint32_t)c->shade_threshold & 0xFFu : 16u;
    const bool t = c->ktiming && c->kused + 2 <= 8192;
    if (t) {
        while (c->kev.size() < c->kused + 2) {
            hipEvent_t e;
            HIPCHK(c, hipEventCreate(&e));
            c->kev.push_back(e);
        }
        HIPCHK(c, hipEventRecord(c->kev[c->kused], c->stream));
    }
    const int r = rtk::launch_trace_batch(dev_scene(c), rays_dev, flags_dev, n, hits_dev, c->work.as<uint32_t>(),
                                          T < 64u ? T : 63u, c->num_cus, c->stream);
    if (r) return fail(c, r, std::string("rt_trace_batch: launch failed: ") + hipGetErrorString(hipGetLastError()));
    if (t) {
        HIPCHK(c, hipEventRecord(c->kev[c->kused + 1], c->stream));
        c->kused += 2;
    }
    return RT_OK;
}

int rt_trace_rays(rt_ctx* c, rt_traverse trav, const float* rays, const uint32_t* flags, uint32_t n, rt_ray_hit* hits)
{
    if (!c) return RT_E_INVALID;
    if (n == 0) return RT_OK;
    if (!rays || !hits) return fail(c, RT_E_INVALID, "rt_trace_rays: rays and hits are required");
    if (!c->has_mesh) return fail(c, RT_E_NOT_READY, "rt_trace_rays: no mesh uploaded");
    if (trav == RT_TRAVERSE_BSP && !c->has_bsp) return fail(c, RT_E_NOT_READY, "rt_trace_rays: no BSP uploaded");
    if (trav == RT_TRAVERSE_BVH && !c->has_bvh) return fail(c, RT_E_NOT_READY, "rt_trace_rays: no BVH uploaded");
    if (trav != RT_TRAVERSE_BSP && trav != RT_TRAVERSE_BVH)
        return fail(c, RT_E_UNSUPPORTED, "rt_trace_rays: traverse must be BSP or BVH");
    if (int r = set_dev(c)) return r;
    uint32_t* deep = nullptr;
    if (trav == RT_TRAVERSE_BVH) {
        const size_t need = rtk::bvh_deep_bytes(c->num_cus, 16);
        if (c->bvh_deep.n < need) HIPCHK(c, c->bvh_deep.alloc(need));
        deep = c->bvh_deep.as<uint32_t>();
    }
    if (trav == RT_TRAVERSE_BSP)
        if (int rr = ensure_hcam(c)) return rr;
    const int r = rtk::launch_query(dev_scene(c), trav, rays, flags, n, hits, deep, c->num_cus, c->stream);
    if (r) return fail(c, r, std::string("rt_trace_rays: launch failed: ") + hipGetErrorString(hipGetLastError()));
    return RT_OK;
}

// The shading threshold of a render (RT_OPT_SHADE_THRESHOLD, or the default per walk,
// shader and the culling kernel `cull` that runs; render_common has the measurements).
static uint32_t default_threshold(const rt_ctx* c, rt_mode mode, rt_traverse trav, uint32_t cull)
{
    if (c->shade_threshold >= 0) return (uint32_t)c->shade_threshold;
    if (trav == RT_TRAVERSE_BVH) return 4u;
    if (mode == RT_MODE_W7E3) return 24u;
    if (cull == RT_BSP_CULL_SILHOUETTE) return (1u << 16) | (32u << 8) | 24u;
    return cull_certified(c) ? (1u << 16) | (32u << 8) | 20u : (1u << 16) | (24u << 8) | 8u;
}

// RT_BSP_CULL_AUTO's probe.  The certified and the silhouette W9E1 kernels are both
// exact (the same frame bit for bit), so the choice between them moves only time: the
// silhouette bound gains 15 % on config 4's far grid of bunnies and loses 3-4 % on
// configs 3 and 5.  The probe costs no extra work: four of the
// renders' own launches, each of at least 2^20 samples, run certified, silhouette,
// certified, silhouette (a big render splits its first iterations into four such
// launches, 1/8 of it each at most; 1-spp frames of at least 2^20 pixels give one
// launch each, so a moving camera's frames finish the probe in four frames).  Their
// events are read without waiting, at a later render (probe_finish): until then the
// certified kernel runs.  The choice holds for the scene -- a new BSP, a change of the
// culling option, or an eye whose reach (farthest distance to the scene box) leaves
// [1/2, 2] of the reach it was made at starts a new probe; orbiting or small moves keep it.
static constexpr uint64_t PROBE_MIN_SAMPLES = 1ull << 20;
static constexpr float PROBE_MARGIN = 0.95f;   // the silhouette kernel's time must be below 0.95x

// the eye's farthest distance to the scene's box (|eye - centre| + half diagonal)
static float eye_reach(const rt_ctx* c)
{
    double d2 = 0.0, h2 = 0.0;
    for (int k = 0; k < 3; k++) {
        const double ctr = 0.5 * ((double)c->aabb[k] + c->aabb[k + 3]);
        const double half = 0.5 * ((double)c->aabb[k + 3] - c->aabb[k]);
        d2 += ((double)c->u.camera_pos[k] - ctr) * ((double)c->u.camera_pos[k] - ctr);
        h2 += half * half;
    }
    return (float)(std::sqrt(d2) + std::sqrt(h2));
}

// a finished probe's choice: read when its last event has completed (never waits)
static int probe_finish(rt_ctx* c)
{
    if (c->auto_cull || c->probe_n < 4) return RT_OK;
    const hipError_t q = hipEventQuery(c->auto_ev[7]);
    if (q == hipErrorNotReady) return RT_OK;
    HIPCHK(c, q);
    float best[2] = {INFINITY, INFINITY};
    for (int i = 0; i < 4; i++) {
        float t;
        HIPCHK(c, hipEventElapsedTime(&t, c->auto_ev[2 * i], c->auto_ev[2 * i + 1]));
        best[i & 1] = std::min(best[i & 1], (float)(t * (double)PROBE_MIN_SAMPLES / (double)c->probe_samples[i]));
    }
    c->auto_ms[0] = best[0];
    c->auto_ms[1] = best[1];
    // the silhouette kernel must win by 5 %: on config 3 the two probe within 0-4 % of each
    // other (the certified kernel 4-9 % faster over whole frames), on config 4 the silhouette
    // kernel wins by 8-12 % (profiles/r05/ab_auto.txt, the final bench lines' bsp_cull)
    c->auto_cull = best[1] < PROBE_MARGIN * best[0] ? RT_BSP_CULL_SILHOUETTE : RT_BSP_CULL_CERTIFIED;
    return RT_OK;
}

// the probe's part of a W9E1 BSP render under RT_BSP_CULL_AUTO, before its launches:
// finish a completed probe, and start over when the eye's reach moved out of range
static int probe_begin(rt_ctx* c)
{
    if (int r = probe_finish(c)) return r;
    if (c->auto_cull || c->probe_n) {
        const float reach = eye_reach(c);
        if (!(reach <= 2.0f * c->probe_reach && reach >= 0.5f * c->probe_reach)) {
            c->auto_cull = 0;
            c->probe_n = 0;
        }
    }
    return RT_OK;
}

// how many of a launch's n iterations (stride samples each, total in the whole render)
// become the probe's next timed launch, 0 for none
static uint32_t probe_take(const rt_ctx* c, uint32_t n, uint32_t total, uint32_t stride)
{
    if (c->auto_cull || c->probe_n >= 4 || stride == 0) return 0;
    const uint64_t need = (PROBE_MIN_SAMPLES + stride - 1) / stride;
    if (n < need) return 0;
    // (an eighth of the render each, at most 2^26 samples: a launch's fixed ~1.3-ms tail
    //  must stay small against the launch, or the two kernels' tails
    // decide the choice -- with 1/16 and 2^25, rank 0's share of a 4-rank config-3 split
    // probed the silhouette kernel 3.7 % faster in 3.6-ms launches, and it ran the frame
    // 8.6 % slower than the certified one, profiles/r06/final/bench_c3n4.json of fatbin
    // 104178909346469f)
    const uint64_t cap = std::max<uint64_t>(1, (1ull << 26) / stride);
    const uint64_t want = std::max<uint64_t>(need, std::min<uint64_t>(total / 8, cap));
    return (uint32_t)std::min<uint64_t>(n, want);
}

int rt_bsp_cull_in_use(rt_ctx* c, int* mode, float* probe_ms, uint32_t* probes)
{
    if (!c || !mode) return RT_E_INVALID;
    if (c->bsp_cull == RT_BSP_CULL_AUTO && c->probe_n == 4 && !c->auto_cull) {
        if (int r = set_dev_nojoin(c)) return r;   // (only the event query: no stream work)
        if (int r = probe_finish(c)) return r;
    }
    *mode = (int)cull_in_use(c);
    if (probe_ms) {
        const bool probed = c->bsp_cull == RT_BSP_CULL_AUTO && c->auto_cull != 0;
        probe_ms[0] = probed ? c->auto_ms[0] : 0.0f;
        probe_ms[1] = probed ? c->auto_ms[1] : 0.0f;
    }
    if (probes) {
        probes[0] = c->probes;
        probes[1] = c->probe_launches;
    }
    return RT_OK;
}

// a render launch; slot >= 0: the probe's launch `slot`, bracketed by its events
static int probe_launch(rt_ctx* c, const rtk::DevScene& S, const rtk::DevLaunch& L, rt_mode mode, rt_traverse trav,
                        int slot)
{
    if (slot < 0) return launch_timed(c, S, L, mode, trav);
    for (hipEvent_t& e : c->auto_ev)
        if (!e) HIPCHK(c, hipEventCreate(&e));
    if (slot == 0) {
        c->probes++;
        c->probe_reach = eye_reach(c);
    }
    HIPCHK(c, hipEventRecord(c->auto_ev[2 * slot], c->stream));
    if (int r = launch_timed(c, S, L, mode, trav)) return r;
    HIPCHK(c, hipEventRecord(c->auto_ev[2 * slot + 1], c->stream));
    c->probe_samples[slot] = (uint64_t)L.stride * L.spp;
    c->probe_n = (uint32_t)slot + 1;
    c->probe_launches++;
    return RT_OK;
}

static int render_common(rt_ctx* c, rt_mode mode, rt_traverse trav, rtk::DevLaunch& L, rt_ray_counts* counts)
{
    if (!c->has_u) return fail(c, RT_E_NOT_READY, "rt_render: uniforms not set");
    if (mode < RT_MODE_W1E6 || mode > RT_MODE_W9E3) return fail(c, RT_E_INVALID, "rt_render: bad mode");
    // W7E1/W7E2: progressive, folded inside k_direct (no per-iteration samples)
    const bool direct_prog = mode == RT_MODE_W7E1 || mode == RT_MODE_W7E2;
    // progressive path tracers: per-iteration samples, folded in order by k_fold
    const bool path = mode == RT_MODE_W7E3 || mode == RT_MODE_W9E1 || mode == RT_MODE_W8E1 || mode == RT_MODE_W8E2 ||
                      mode == RT_MODE_W8E3 || mode == RT_MODE_W9E2 || mode == RT_MODE_W9E3;
    if (mode == RT_MODE_W1E6) {
        if (trav != RT_TRAVERSE_NONE) return fail(c, RT_E_UNSUPPORTED, "W1E6 is analytic: traverse must be NONE");
    } else {
        if (!c->has_mesh) return fail(c, RT_E_NOT_READY, "rt_render: no mesh uploaded");
        if (trav == RT_TRAVERSE_BSP && !c->has_bsp) return fail(c, RT_E_NOT_READY, "rt_render: no BSP uploaded");
        if (trav == RT_TRAVERSE_BVH && !c->has_bvh) return fail(c, RT_E_NOT_READY, "rt_render: no BVH uploaded");
        if (trav == RT_TRAVERSE_NONE) return fail(c, RT_E_UNSUPPORTED, "mesh modes need BSP or BVH");
        if (path && mode != RT_MODE_W9E1 && mode != RT_MODE_W9E2 && mode != RT_MODE_W9E3 && c->nlights < 2)
            return fail(c, RT_E_INVALID, "W7E3/W8 sample area lights: the mesh has no emissive (illum 1) triangle");
        if ((mode == RT_MODE_W6E1 || mode == RT_MODE_PROJECT) && trav == RT_TRAVERSE_BSP && !c->has_bsp)
            return fail(c, RT_E_NOT_READY, "rt_render: W6E1/PROJECT need the BSP root AABB");
    }
    if (!L.accum) return fail(c, RT_E_INVALID, "rt_render: accum buffer required");
    // a path mode orders itself against a pending fold (double-buffered samples,
    // the fold stream); every other mode writes accum / ids on the context stream
    // itself, so a fold of an earlier path render still pending there is joined first
    if (int r = path ? set_dev_nojoin(c) : set_dev(c)) return r;
    if (int r = ensure_hcam(c)) return r;
    rtk::DevScene S = dev_scene(c);
    L.u = c->u;
    rtk::camera_basis(c->u, L.cam);
    L.jitter = c->has_jitter ? c->jitter.as<float>() : nullptr;
    memcpy(L.env, c->env, sizeof L.env);
    L.env_tex = c->env_w ? c->env_tex.as<uint32_t>() : nullptr;
    L.env_w = c->env_w;
    L.env_h = c->env_h;
    L.work_counter = c->work.as<uint32_t>();
    L.cap_rays = reinterpret_cast<float4*>(c->cap_rays);
    L.cap_flags = c->cap_flags;
    L.cap_count = c->cap_count.as<unsigned long long>();
    L.cap_max = c->cap_max;
    if (trav == RT_TRAVERSE_BVH) {
        const size_t need = rtk::bvh_deep_bytes(c->num_cus, c->waves_per_cu);
        if (c->bvh_deep.n < need) HIPCHK(c, c->bvh_deep.alloc(need));
        L.bvh_deep = c->bvh_deep.as<uint32_t>();
    }
    // default shading threshold per walk (BSP sweep 8 best;
    // BVH 2-4 best, 4695 vs 4604 Mrays/s at 8)
    // defaults per walk and shader (profiles/r02/ab_w7e3_shards.txt: W7E3's short
    // Cornell-box rays shade often, and refilling earlier pays there)
    // The BSP walk of the other modes chooses per wave between two thresholds (bit
    // 16: adaptive, k_path "Shading threshold"), the lower for walk-dominated waves,
    // the higher for test-dominated ones.  With the fast margin 8 and 24 (configs 4
    // and 5 test-dominated since subtree culling; fixed thresholds 12..48 on them: 24
    // best, profiles/r03/ab_T{hi,lo}_c{4,5}.txt).  The certified walk visits more
    // nodes and its rays take more trips, so finished lanes wait longer for the last
    // ones: 16 and 32 (profiles/r04/sweep_T.txt: config 3 fixed 16 +1.9 % over 8,
    // config 4 16..24 +3 %, config 5 32 +1.1 %); 20 and 32 since the cheaper
    // shadow-ray leaf tests of round 6 (profiles/r06/sweep_T.txt: config 3 +0.3..0.6 %
    // over 16, config 5 unchanged).
    // The silhouette kernel's camera rays take fewer, dearer trips: 24 and 32
    // (profiles/r05/sweep_T_c4s.txt: config 4 +1.2 % over 16 / 32).
    const bool sil = has_silhouette(c, mode, trav);
    S.bsp_cull_mode = cull_in_use(c, sil);
    L.shade_threshold = default_threshold(c, mode, trav, S.bsp_cull_mode);
    L.reserved0 = 0;
    L.counters = c->counters.as<unsigned long long>();
    HIPCHK(c, hipMemsetAsync(c->counters.p, 0, 32 * sizeof(unsigned long long), c->stream));
    if (L.nwork == 0 || (L.spp == 0 && (path || direct_prog))) {
        if (counts) return rt_last_counts(c, counts);
        return RT_OK;
    }
    if (path) {
        // passes of pass_spp iterations: k_path writes per-iteration samples,
        // k_fold applies the progressive average in order
        L.stride = L.tileset ? L.nwork * 64u : L.w * L.h;
        const uint64_t per_it = (uint64_t)L.stride * sizeof(float4);
        const uint64_t budget = c->sample_budget_mb << 20;
        uint32_t pass_spp = (uint32_t)std::min<uint64_t>(L.spp, std::max<uint64_t>(1, budget / per_it));
        const uint64_t need = per_it * pass_spp;
        const bool async = c->async_fold && c->fold_stream;
        if (c->samples.n < need) HIPCHK(c, c->samples.alloc(need));
        if (async && c->samples2.n < need) HIPCHK(c, c->samples2.alloc(need));
        L.samples = c->samples.as<float4>();
        // (a counting render, RT_OPT_DETAIL_COUNTERS, runs other kernels: it never probes)
        const bool autop = sil && c->bsp_cull == RT_BSP_CULL_AUTO && c->hcam_valid && !c->detail;
        if (autop)
            if (int r = probe_begin(c)) return r;
        if (async) {   // the folds follow the context stream's work up to here
            HIPCHK(c, hipEventRecord(c->ev_enter, c->stream));
            HIPCHK(c, hipStreamWaitEvent(c->fold_stream, c->ev_enter, 0));
        }
        const uint32_t first = L.first_iter, total = L.spp;
        for (uint32_t done = 0; done < total; done += L.spp) {
            L.first_iter = first + done;
            L.spp = std::min(pass_spp, total - done);
            // RT_BSP_CULL_AUTO: this launch may be one of the probe's four (probe_take)
            const uint32_t take = autop ? probe_take(c, L.spp, total, L.stride) : 0;
            int slot = -1;
            if (take) {
                slot = (int)c->probe_n;
                L.spp = take;
                S.bsp_cull_mode = (slot & 1) ? RT_BSP_CULL_SILHOUETTE : RT_BSP_CULL_CERTIFIED;
            } else {
                S.bsp_cull_mode = cull_in_use(c, sil);
            }
            L.shade_threshold = default_threshold(c, mode, trav, S.bsp_cull_mode);
            // work units (chunk, pixel slot) must stay below 2^31: widen chunks if needed
            uint32_t ch = std::max<uint32_t>(1, std::min(c->sample_chunk, L.spp));
            while ((uint64_t)L.nwork * 64u * ((L.spp + ch - 1) / ch) >= (1ull << 31)) ch *= 2;
            L.chunk = ch;
            L.unit_order = c->unit_order;
            L.nchunks = (L.spp + ch - 1) / ch;
            if (async) {   // alternate scratch buffers: wait for the fold that last read this one
                const uint32_t b = c->sbuf;
                c->sbuf ^= 1u;
                L.samples = (b ? c->samples2 : c->samples).as<float4>();
                HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_free[b], 0));
                HIPCHK(c, hipMemsetAsync(c->work.p, 0, 4096, c->stream));
                if (int r = probe_launch(c, S, L, mode, trav, slot)) return r;
                HIPCHK(c, hipEventRecord(c->ev_path, c->stream));
                HIPCHK(c, hipStreamWaitEvent(c->fold_stream, c->ev_path, 0));
                const int r = rtk::launch_fold(L, c->fold_stream);
                if (r) return fail(c, r, std::string("fold launch failed: ") + hipGetErrorString(hipGetLastError()));
                HIPCHK(c, hipEventRecord(c->ev_free[b], c->fold_stream));
                c->fold_pending = true;
                continue;
            }
            HIPCHK(c, hipMemsetAsync(c->work.p, 0, 4096, c->stream));
            if (int r = probe_launch(c, S, L, mode, trav, slot)) return r;
            const int r = rtk::launch_fold(L, c->stream);
            if (r) return fail(c, r, std::string("fold launch failed: ") + hipGetErrorString(hipGetLastError()));
        }
    } else {
        HIPCHK(c, hipMemsetAsync(c->work.p, 0, 4096, c->stream));
        if (int r = launch_timed(c, S, L, mode, trav)) return r;
    }
    if (counts) return rt_last_counts(c, counts);
    return RT_OK;
}

int rt_render(rt_ctx* c, rt_mode mode, rt_traverse trav, const rt_tile* region, uint32_t first_iter, uint32_t spp,
              float* accum, uint32_t* ids, rt_ray_counts* counts)
{
    if (!c || !region) return RT_E_INVALID;
    if (!c->has_u) return fail(c, RT_E_NOT_READY, "rt_render: uniforms not set");
    const uint32_t W = c->u.resolution[0], H = c->u.resolution[1];
    if ((uint64_t)region->x0 + region->w > W || (uint64_t)region->y0 + region->h > H)
        return fail(c, RT_E_INVALID, "rt_render: region outside uniforms.resolution");
    rtk::DevLaunch L;
    memset(&L, 0, sizeof L);
    L.tileset = 0;
    L.x0 = region->x0;
    L.y0 = region->y0;
    L.w = region->w;
    L.h = region->h;
    L.rank = 0;
    L.nranks = 1;
    L.tiles_x = (region->w + 7) / 8;
    L.tiles_y = (region->h + 7) / 8;
    L.nwork = L.tiles_x * L.tiles_y;
    L.first_iter = first_iter;
    L.spp = spp;
    L.accum = reinterpret_cast<float4*>(accum);
    L.ids = ids;
    return render_common(c, mode, trav, L, counts);
}

uint32_t rt_tileset_local_tiles(uint32_t width, uint32_t height, uint32_t nranks)
{
    if (nranks == 0) return 0;
    const uint64_t t = (uint64_t)((width + 7) / 8) * ((height + 7) / 8);
    return (uint32_t)((t + nranks - 1) / nranks);
}

int rt_render_tiles(rt_ctx* c, rt_mode mode, rt_traverse trav, const rt_tileset* ts, uint32_t first_iter,
                    uint32_t spp, float* accum, uint32_t* ids, rt_ray_counts* counts)
{
    if (!c || !ts) return RT_E_INVALID;
    if (!c->has_u) return fail(c, RT_E_NOT_READY, "rt_render_tiles: uniforms not set");
    if (ts->nranks == 0 || ts->rank >= ts->nranks) return fail(c, RT_E_INVALID, "rt_render_tiles: bad rank/nranks");
    const uint32_t W = c->u.resolution[0], H = c->u.resolution[1];
    rtk::DevLaunch L;
    memset(&L, 0, sizeof L);
    L.tileset = 1;
    L.x0 = 0;
    L.y0 = 0;
    L.w = W;
    L.h = H;
    L.rank = ts->rank;
    L.nranks = ts->nranks;
    L.tiles_x = (W + 7) / 8;
    L.tiles_y = (H + 7) / 8;
    L.nwork = rt_tileset_local_tiles(W, H, ts->nranks);
    L.first_iter = first_iter;
    L.spp = spp;
    L.accum = reinterpret_cast<float4*>(accum);
    L.ids = ids;
    return render_common(c, mode, trav, L, counts);
}

// The 255 thresholds of 8-bit sRGB codes: code k+1 starts where
// 255 * oetf(v) reaches k + 0.5 (oetf inverted in double, rounded up to the
// first float whose code is k + 1).
static void srgb_code_thresholds(float* t)
{
    for (int k = 0; k < 255; k++) {
        const double e = (k + 0.5) / 255.0;   // encoded value at the rounding midpoint
        const double v = e <= 0.04045 ? e / 12.92 : std::pow((e + 0.055) / 1.055, 2.4);
        float f = (float)v;
        auto code = [](float x) {
            const double xd = x;
            const double enc = xd <= 0.0031308 ? 12.92 * xd : 1.055 * std::pow(xd, 1.0 / 2.4) - 0.055;
            return (int)std::floor(enc * 255.0 + 0.5);
        };
        while (code(f) > k) f = std::nextafter(f, 0.0f);
        while (code(f) <= k) f = std::nextafter(f, 2.0f);
        t[k] = f;
    }
}

int rt_frame_rgba8(rt_ctx* c, const float* accum_rgba32f, uint32_t npix, uint8_t* frame_rgba8)
{
    if (!c || (!accum_rgba32f && npix) || (!frame_rgba8 && npix)) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    if (!c->srgb_thr.p) {
        float t[256];
        srgb_code_thresholds(t);
        t[255] = 0.0f;
        if (int r = upload(c, c->srgb_thr, t, sizeof t)) return r;
    }
    if (npix == 0) return RT_OK;
    if (rtk::launch_frame(reinterpret_cast<const float4*>(accum_rgba32f), npix, c->srgb_thr.as<float>(),
                          reinterpret_cast<uchar4*>(frame_rgba8), c->stream))
        return fail(c, RT_E_DEVICE, "rt_frame_rgba8: launch failed");
    return RT_OK;
}

int rt_unpack_tiles(rt_ctx* c, uint32_t width, uint32_t height, uint32_t nranks, const float* packed_accum,
                    const uint32_t* packed_ids, float* frame_accum, uint32_t* frame_ids)
{
    if (!c || nranks == 0) return RT_E_INVALID;
    if (int r = set_dev_nojoin(c)) return r;
    hipStream_t os;
    if (int r = out_stream(c, &os)) return r;
    const uint32_t lt = rt_tileset_local_tiles(width, height, nranks);
    const bool tm = gather_event(c, os) != nullptr;   // (no transfers: the first two events coincide)
    if (tm) gather_event(c, os);
    int r = rtk::launch_unpack(width, height, nranks, lt, reinterpret_cast<const float4*>(packed_accum), packed_ids,
                               reinterpret_cast<float4*>(frame_accum), frame_ids, os);
    if (r) return fail(c, r, "rt_unpack_tiles: launch failed");
    if (tm) gather_event(c, os);
    return RT_OK;
}

// ---- the tile gather over RCCL (rt.h "multi-GPU") ----------------------------
// RCCL is resolved at run time (dlopen of librccl.so.1): the library loads on
// hosts without it, and a process that already holds RCCL (PyTorch's) shares it.
extern "C++" {
namespace {
struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    std::string err;
};
const Rccl& rccl()
{
    static Rccl r = [] {
        Rccl x;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            x.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (x.h) break;
        }
        if (!x.h) {
            const char* e = dlerror();
            x.err = std::string("RCCL not found (librccl.so.1): ") + (e ? e : "");
            return x;
        }
        auto sym = [&](auto& f, const char* n) { f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(x.h, n)); };
        sym(x.get_unique_id, "ncclGetUniqueId");
        sym(x.comm_init_rank, "ncclCommInitRank");
        sym(x.comm_destroy, "ncclCommDestroy");
        sym(x.send, "ncclSend");
        sym(x.recv, "ncclRecv");
        sym(x.group_start, "ncclGroupStart");
        sym(x.group_end, "ncclGroupEnd");
        sym(x.error_string, "ncclGetErrorString");
        if (!x.get_unique_id || !x.comm_init_rank || !x.comm_destroy || !x.send || !x.recv || !x.group_start ||
            !x.group_end || !x.error_string)
            x.err = "RCCL lacks a symbol rt_comm needs";
        return x;
    }();
    return r;
}
std::string nccl_msg(const Rccl& R, ncclResult_t e) { return R.error_string ? R.error_string(e) : "RCCL error"; }
}  // namespace
}

int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES])
{
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RT_COMM_ID_BYTES");
    if (!id) return RT_E_INVALID;
    const Rccl& R = rccl();
    if (!R.err.empty()) return fail(nullptr, RT_E_UNSUPPORTED, "rt_comm_unique_id: " + R.err);
    ncclUniqueId u;
    if (ncclResult_t e = R.get_unique_id(&u)) return fail(nullptr, RT_E_DEVICE, "ncclGetUniqueId: " + nccl_msg(R, e));
    memcpy(id, &u, sizeof u);
    return RT_OK;
}

int rt_comm_init(rt_ctx* c, uint32_t nranks, uint32_t rank, const uint8_t id[RT_COMM_ID_BYTES])
{
    if (!c || !id || nranks == 0 || rank >= nranks || nranks > 4096) return RT_E_INVALID;
    if (c->comm) return fail(c, RT_E_INVALID, "rt_comm_init: the context already has a communicator");
    const Rccl& R = rccl();
    if (!R.err.empty()) return fail(c, RT_E_UNSUPPORTED, "rt_comm_init: " + R.err);
    if (int r = set_dev(c)) return r;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclComm_t comm = nullptr;
    if (ncclResult_t e = R.comm_init_rank(&comm, (int)nranks, u, (int)rank))
        return fail(c, RT_E_DEVICE, "ncclCommInitRank: " + nccl_msg(R, e));
    c->comm = comm;
    c->comm_nranks = nranks;
    c->comm_rank = rank;
    return RT_OK;
}

int rt_comm_destroy(rt_ctx* c)
{
    if (!c) return RT_E_INVALID;
    if (!c->comm) return RT_OK;
    const Rccl& R = rccl();
    (void)set_dev(c);   // joins a gather pending on the fold stream
    (void)hipStreamSynchronize(c->stream);
    ncclResult_t e = R.comm_destroy(c->comm);
    c->comm = nullptr;
    c->comm_nranks = c->comm_rank = 0;
    c->gather_accum.reset();
    c->gather_ids.reset();
    if (e) return fail(c, RT_E_DEVICE, "ncclCommDestroy: " + nccl_msg(R, e));
    return RT_OK;
}

int rt_gather_tiles(rt_ctx* c, uint32_t width, uint32_t height, const float* local_accum, const uint32_t* local_ids,
                    float* frame_accum, uint32_t* frame_ids)
{
    if (!c || !local_accum || width == 0 || height == 0) return RT_E_INVALID;
    if (!c->comm) return fail(c, RT_E_NOT_READY, "rt_gather_tiles: no communicator (rt_comm_init)");
    const uint32_t N = c->comm_nranks, me = c->comm_rank;
    const bool root = me == 0;
    if (root && !frame_accum) return fail(c, RT_E_INVALID, "rt_gather_tiles: rank 0 needs frame_accum");
    if (root && local_ids && !frame_ids) return fail(c, RT_E_INVALID, "rt_gather_tiles: rank 0 needs frame_ids");
    if (int r = set_dev_nojoin(c)) return r;
    hipStream_t os;   // the fold stream under RT_OPT_ASYNC_FOLD
    if (int r = out_stream(c, &os)) return r;
    const Rccl& R = rccl();
    const size_t px = (size_t)rt_tileset_local_tiles(width, height, N) * 64u;
    const bool tm = gather_event(c, os) != nullptr;   // transfers start (RT_OPT_KERNEL_TIMING)
    if (!root) {
        // one group: this rank's accumulation and ids to rank 0
        ncclResult_t e = R.group_start();
        if (!e) e = R.send(local_accum, px * 4, ncclFloat32, 0, c->comm, os);
        if (!e && local_ids) e = R.send(local_ids, px, ncclUint32, 0, c->comm, os);
        const ncclResult_t e2 = R.group_end();
        if (e || e2) return fail(c, RT_E_DEVICE, "rt_gather_tiles send: " + nccl_msg(R, e ? e : e2));
        if (tm) {   // sent; no unpack on this rank
            gather_event(c, os);
            gather_event(c, os);
        }
        return RT_OK;
    }
    // rank 0: every peer's packed tiles, rank-major beside its own (slot 0), in one group
    HIPCHK(c, c->gather_accum.ensure(px * 16 * N));
    if (local_ids) HIPCHK(c, c->gather_ids.ensure(px * 4 * N));
    float* ga = c->gather_accum.as<float>();
    uint32_t* gi = c->gather_ids.as<uint32_t>();
    HIPCHK(c, hipMemcpyAsync(ga, local_accum, px * 16, hipMemcpyDeviceToDevice, os));
    if (local_ids) HIPCHK(c, hipMemcpyAsync(gi, local_ids, px * 4, hipMemcpyDeviceToDevice, os));
    if (N > 1) {
        ncclResult_t e = R.group_start();
        for (uint32_t p = 1; p < N && !e; p++) {
            e = R.recv(ga + p * px * 4, px * 4, ncclFloat32, (int)p, c->comm, os);
            if (!e && local_ids) e = R.recv(gi + p * px, px, ncclUint32, (int)p, c->comm, os);
        }
        const ncclResult_t e2 = R.group_end();
        if (e || e2) return fail(c, RT_E_DEVICE, "rt_gather_tiles recv: " + nccl_msg(R, e ? e : e2));
    }
    if (tm) gather_event(c, os);   // received
    int r = rtk::launch_unpack(width, height, N, (uint32_t)(px / 64), reinterpret_cast<const float4*>(ga),
                               local_ids ? gi : nullptr, reinterpret_cast<float4*>(frame_accum),
                               local_ids ? frame_ids : nullptr, os);
    if (r) return fail(c, r, "rt_gather_tiles: unpack launch failed");
    if (tm) gather_event(c, os);   // unpacked
    return RT_OK;
}

int rt_gather_time(rt_ctx* c, int reset, double* transfer_ms, double* unpack_ms, uint32_t* calls)
{
    if (!c) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    double tx = 0.0, up = 0.0;
    for (size_t i = 0; i + 2 < c->gused; i += 3) {
        HIPCHK(c, hipEventSynchronize(c->gev[i + 2]));
        float a = 0.0f, b = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&a, c->gev[i], c->gev[i + 1]));
        HIPCHK(c, hipEventElapsedTime(&b, c->gev[i + 1], c->gev[i + 2]));
        tx += a;
        up += b;
    }
    if (transfer_ms) *transfer_ms = tx;
    if (unpack_ms) *unpack_ms = up;
    if (calls) *calls = (uint32_t)(c->gused / 3);
    if (reset) c->gused = 0;
    return RT_OK;
}

int rt_last_counts(rt_ctx* c, rt_ray_counts* counts)
{
    if (!c || !counts) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    unsigned long long h[32];
    static_assert(sizeof(rt_ray_counts) <= sizeof h, "counter buffer");
    HIPCHK(c, hipMemcpyAsync(h, c->counters.p, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint64_t* dst = reinterpret_cast<uint64_t*>(counts);
    for (size_t i = 0; i < sizeof(rt_ray_counts) / sizeof(uint64_t); i++) dst[i] = h[i];
    c->last = *counts;
    return RT_OK;
}

int rt_selftest_math(rt_ctx* c, uint32_t n, float lo, float hi, uint32_t* mismatches)
{
    if (!c || !mismatches || n == 0) return RT_E_INVALID;
    if (int r = set_dev(c)) return r;
    std::vector<float> in(n), hout((size_t)n * rtk::kMathOuts), dout((size_t)n * rtk::kMathOuts);
    uint32_t s = 12345u;
    for (uint32_t i = 0; i < n; i++) {
        s = s * 1664525u + 1013904223u;
        const float t = (float)i / (float)n;
        in[i] = lo + (hi - lo) * t + ((float)(s >> 8) * (1.0f / 16777216.0f) - 0.5f) * ((hi - lo) / (float)n);
    }
    rtk::host_math(in.data(), hout.data(), n);
    DevBuf din, dres;
    if (int r = upload(c, din, in.data(), in.size() * 4)) return r;
    HIPCHK(c, dres.alloc(dout.size() * 4));
    if (rtk::launch_selftest_math(din.as<float>(), dres.as<float>(), n, c->stream))
        return fail(c, RT_E_DEVICE, "rt_selftest_math: launch failed");
    HIPCHK(c, hipMemcpyAsync(dout.data(), dres.p, dout.size() * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint32_t bad = 0;
    for (size_t i = 0; i < dout.size(); i++) {
        uint32_t a, b;
        memcpy(&a, &hout[i], 4);
        memcpy(&b, &dout[i], 4);
        const bool both_nan = std::isnan(hout[i]) && std::isnan(dout[i]);
        if (a != b && !both_nan) bad++;
    }
    *mismatches = bad;
    return RT_OK;
}

int rt_upload_mesh_host(rt_ctx* c, const rt_mesh_host* m)
{
    if (!c || !m) return RT_E_INVALID;
    return rt_upload_mesh(c, m->pos.data(), m->nrm.data(), m->nverts(), m->idx.data(), m->ntris(), m->mats.data(),
                          (uint32_t)m->mats.size(), m->lights.data(), (uint32_t)m->lights.size());
}

int rt_upload_bsp_host(rt_ctx* c, const rt_bsp_host* b)
{
    if (!c || !b) return RT_E_INVALID;
    return rt_upload_bsp(c, b->aabb, b->tree.data(), b->planes.data(), (uint32_t)b->planes.size(), b->ids.data(),
                         (uint32_t)b->ids.size(), b->max_depth);
}

int rt_upload_bvh_host(rt_ctx* c, const rt_bvh_host* b)
{
    if (!c || !b) return RT_E_INVALID;
    return rt_upload_bvh(c, b->nodes.data(), (uint32_t)b->nodes.size(), b->tri_ids.data(), (uint32_t)b->tri_ids.size());
}

}  // extern "C"
