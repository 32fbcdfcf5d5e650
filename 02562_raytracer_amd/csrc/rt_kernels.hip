// rt_kernels.hip -- gfx950 (CDNA4) kernels for the per-pixel traversal + shading
// hot path of cakarsubasi/02562_raytracer (res/shaders/*.wgsl).
//
// Structure (DESIGN.md "Kernels"):
//   * persistent grid: every wave dequeues 8x8-pixel tiles from a global atomic
//     counter (one returning atomic per tile), so load balance does not depend
//     on launch order and one wave = one coherent screen tile;
//   * one lane = one pixel, running all `spp` progressive iterations of that
//     pixel in order (accumulation is sequential per pixel, w7e3.wgsl:261-271);
//   * "while-while" ray state machine with ONE traversal call site: each step
//     every live lane traces its current ray (camera / bounce closest-hit, or a
//     shadow any-hit) through the same BSP/BVH loop, then advances its path;
//     lanes never wait on a different ray type's code path;
//   * per-lane traversal stack in LDS (BSP: 8 B {far node, t} x MAX_LEVEL;
//     BVH: 4 B x 50), [level][thread] layout => conflict-free ds_read/write_b64;
//   * BSP nodes packed to 8 B (children implicit), triangles pre-transformed to
//     48-B records {v0, e0, e1, n} in treeIds order (one 3 x dwordx4 gather).
// Numerics: -ffp-contract=off, correctly rounded f32 div/sqrt, pinned
// transcendentals (include/rt_detmath.h) => bit-identical to the CPU oracle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_detmath.h"
#include "rt_internal.h"

namespace rtk {

// ------------------------------------------------------------------ f32 vector math
// Component formulas of the WGSL builtins, evaluated left to right.
struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 V(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 muls(f3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 divs(f3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ f3 neg(f3 a) { return V(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b)
{
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ f3 normalize(f3 a) { return divs(a, rt_det_sqrtf(dot(a, a))); }
__device__ __forceinline__ f3 ld3(const float4 v) { return V(v.x, v.y, v.z); }
__device__ __forceinline__ f3 ld3(const float* p) { return V(p[0], p[1], p[2]); }
__device__ __forceinline__ float comp(f3 a, uint32_t i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

#define RT_PI_F 3.14159265359f

// ------------------------------------------------------------------ PRNG (w7e3.wgsl:141-172)
__device__ __forceinline__ uint32_t tea16(uint32_t v0, uint32_t v1)
{
    uint32_t s0 = 0;
#pragma unroll
    for (int n = 0; n < 16; n++) {
        s0 += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
__device__ __forceinline__ uint32_t mcg31(uint32_t& prev)
{
    prev = (1977654935u * prev) & 0x7FFFFFFFu;
    return prev;
}
__device__ __forceinline__ float rnd(uint32_t& prev) { return (float)mcg31(prev) / (float)0x80000000u; }

// ------------------------------------------------------------------ counters
enum { C_SAMPLES, C_PRIMARY, C_SHADOW, C_BOUNCE, C_INTERIOR, C_LEAF, C_POPS, C_IDS, C_TESTS, C_ACCEPTS, C_N };

struct Counters {
    uint32_t v[C_N];
};

__device__ __forceinline__ void flush_counters(const Counters& c, unsigned long long* out, bool detail)
{
    const int n = detail ? C_N : 4;
    for (int i = 0; i < n; i++) {
        uint32_t x = c.v[i];
        unsigned long long s = x;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if ((threadIdx.x & 63u) == 0 && s) atomicAdd(out + i, s);
    }
}

// ------------------------------------------------------------------ camera (w7e3.wgsl:211-228)
struct Cam {
    f3 e, v, b1, b2;
    float d, aspect;
};
__device__ __forceinline__ Cam make_cam(const rt_uniform& u)
{
    Cam c;
    c.e = ld3(u.camera_pos);
    f3 p = ld3(u.camera_look_at), up = ld3(u.camera_up);
    c.v = normalize(sub(p, c.e));
    c.d = u.camera_constant;
    c.aspect = u.aspect_ratio;
    c.b1 = normalize(cross(c.v, up));
    c.b2 = cross(c.b1, c.v);
    return c;
}
__device__ __forceinline__ f3 cam_dir(const Cam& c, float ux, float uy, float jx, float jy)
{
    return normalize(add(add(muls(muls(c.b1, ux + jx), c.aspect), muls(c.b2, uy + jy)), muls(c.v, c.d)));
}

// ------------------------------------------------------------------ work mapping
struct Pix {
    uint32_t x, y, out;
    bool valid;
};
__device__ __forceinline__ Pix map_pixel(const DevLaunch& L, uint32_t work, uint32_t lane)
{
    Pix p;
    const uint32_t lx = lane & 7u, ly = lane >> 3;
    if (L.tileset == 0) {
        uint32_t tx = work % L.tiles_x, ty = work / L.tiles_x;
        uint32_t rx = tx * 8u + lx, ry = ty * 8u + ly;
        p.valid = rx < L.w && ry < L.h;
        p.x = L.x0 + rx;
        p.y = L.y0 + ry;
        p.out = ry * L.w + rx;
    } else {
        uint32_t t = work * L.nranks + L.rank;
        uint32_t tx = t % L.tiles_x, ty = t / L.tiles_x;
        p.x = tx * 8u + lx;
        p.y = ty * 8u + ly;
        p.valid = (t < L.tiles_x * L.tiles_y) && p.x < L.u.resolution[0] && p.y < L.u.resolution[1];
        p.out = work * 64u + lane;
    }
    return p;
}
__device__ __forceinline__ uint32_t fetch_work(uint32_t* ctr, uint32_t lane)
{
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(ctr, 1u);
    return __shfl(v, 0, 64);
}
__device__ __forceinline__ void pixel_uv(const rt_uniform& u, uint32_t x, uint32_t y, float& ux, float& uy)
{
    ux = ((float)x + 0.5f) / (float)u.resolution[0] - 0.5f;
    uy = 0.5f - ((float)y + 0.5f) / (float)u.resolution[1];
}

// ------------------------------------------------------------------ triangle test
// intersect_triangle_indexed (w7e3.wgsl:286-332) on a pre-transformed record:
// r0 = (v0.xyz, e0.x), r1 = (e0.yz, e1.xy), r2 = (e1.z, n.xyz).
__device__ __forceinline__ bool tri_test(const float4* recs, uint32_t k, f3 o, f3 w, float tmin, float tmax,
                                         float& dist, float& beta, float& gamma)
{
    const float4 r0 = recs[3u * k], r1 = recs[3u * k + 1u], r2 = recs[3u * k + 2u];
    const f3 v0 = V(r0.x, r0.y, r0.z), e0 = V(r0.w, r1.x, r1.y), e1 = V(r1.z, r1.w, r2.x);
    const f3 n = V(r2.y, r2.z, r2.w);
    const f3 ov = sub(v0, o);
    const f3 nom = cross(ov, w);
    const float denom = dot(w, n);
    if (rt_absf(denom) < 1e-10f) return false;
    beta = dot(nom, e1) / denom;
    gamma = -dot(nom, e0) / denom;
    dist = dot(ov, n) / denom;
    return !(beta < 0.0f || gamma < 0.0f || beta + gamma > 1.0f || dist > tmax || dist < tmin);
}

struct TraceOut {
    uint32_t k;   // record slot of the accepted triangle
    float beta, gamma, dist;
};

// ------------------------------------------------------------------ BSP traversal
// intersect_trimesh, bsp.wgsl:10-81.  The explicit stack keeps {far node, t};
// the tmax a pop restores is the t of the entry below it (or the ray's
// original tmax), which is exactly the value bsp.wgsl saves in branch_ray.y.
// anyhit: stop at the first accepted triangle (shadow rays only need the
// boolean; the walk up to that triangle is identical, so the result is too).
template <bool COUNT>
__device__ __forceinline__ bool trace_bsp(const DevScene& S, uint2* stk, const f3 o, const f3 d, float tmin,
                                          float tmax, const bool anyhit, TraceOut& out, Counters& c)
{
    const float tmax0 = tmax;
    uint32_t node = 0, lvl = 0;
    for (uint32_t guard = 0; guard < (1u << 24); guard++) {
        const uint2 n = S.bsp_nodes[node];
        const uint32_t axis = n.x & 3u;
        if (axis == 3u) {
            if (COUNT) c.v[C_LEAF]++;
            const uint32_t count = n.x >> 2, first = n.y;
            bool found = false;
            for (uint32_t j = 0; j < count; j++) {
                if (COUNT) {
                    c.v[C_IDS]++;
                    c.v[C_TESTS]++;
                }
                float dist, beta, gamma;
                if (tri_test(S.bsp_recs, first + j, o, d, tmin, tmax, dist, beta, gamma)) {
                    if (COUNT) c.v[C_ACCEPTS]++;
                    tmax = dist;
                    found = true;
                    out.k = first + j;
                    out.beta = beta;
                    out.gamma = gamma;
                    out.dist = dist;
                    if (anyhit) break;
                }
            }
            if (found) return true;
            if (lvl == 0) return false;
            lvl--;
            const uint2 e = stk[lvl * 256u];
            node = e.x;
            tmin = __uint_as_float(e.y);
            tmax = lvl ? __uint_as_float(stk[(lvl - 1u) * 256u].y) : tmax0;
            continue;
        }
        if (COUNT) c.v[C_INTERIOR]++;
        const float ad = comp(d, axis), ao = comp(o, axis);
        const uint32_t left = 2u * node + 1u;
        const uint32_t near_node = ad >= 0.0f ? left : left + 1u;
        const uint32_t far_node = ad >= 0.0f ? left + 1u : left;
        const float denom = rt_absf(ad) < 1.0e-8f ? 1.0e-8f : ad;
        const float t = (__uint_as_float(n.y) - ao) / denom;
        if (t > tmax) {
            node = near_node;
        } else if (t < tmin) {
            node = far_node;
        } else {
            stk[lvl * 256u] = make_uint2(far_node, __float_as_uint(t));
            lvl++;
            tmax = t;
            node = near_node;
        }
    }
    return false;
}

// ------------------------------------------------------------------ BVH traversal
// intersect_bvh + intersect_bb2, bvh.wgsl:154-191 / 16-83: slab test in axis
// order y, x, z on [0, 1e27] (ray interval ignored), right child popped first,
// 1000-pop cap, WGSL index clamping of the 50-entry stack.
__device__ __forceinline__ bool bb2(const f3 inv, const f3 o, const float4 a, const float4 b)
{
    float t0 = 0.0f, t1 = 1e27f;
    const f3 nr = mul(sub(V(a.x, a.y, a.z), o), inv);
    const f3 fr = mul(sub(V(b.x, b.y, b.z), o), inv);
    float tn = nr.y, tf = fr.y;
    if (tn > tf) { float s = tn; tn = tf; tf = s; }
    if (tn > t0) t0 = tn;
    if (tf < t1) t1 = tf;
    if (t0 > t1) return false;
    tn = nr.x; tf = fr.x;
    if (tn > tf) { float s = tn; tn = tf; tf = s; }
    if (tn > t0) t0 = tn;
    if (tf < t1) t1 = tf;
    if (t0 > t1) return false;
    tn = nr.z; tf = fr.z;
    if (tn > tf) { float s = tn; tn = tf; tf = s; }
    if (tn > t0) t0 = tn;
    if (tf < t1) t1 = tf;
    return !(t0 > t1);
}

template <bool COUNT>
__device__ __forceinline__ bool trace_bvh(const DevScene& S, uint32_t* stk, const f3 o, const f3 d, float tmin,
                                          float tmax, const bool anyhit, TraceOut& out, Counters& c)
{
    const f3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    uint32_t top = 0;
    stk[0] = 0u;
    top = 1;
    bool found = false;
    for (uint32_t pops = 0; pops < 1000u && top > 0u; pops++) {
        top--;
        const uint32_t cur = stk[(top < 50u ? top : 49u) * 256u];
        if (COUNT) c.v[C_POPS]++;
        const float4 a = S.bvh_nodes[2u * cur], b = S.bvh_nodes[2u * cur + 1u];
        if (bb2(inv, o, a, b)) {
            const uint32_t off = __float_as_uint(a.w), np = __float_as_uint(b.w);
            if (np > 0u) {
                for (uint32_t i = 0; i < np; i++) {
                    if (COUNT) {
                        c.v[C_IDS]++;
                        c.v[C_TESTS]++;
                    }
                    float dist, beta, gamma;
                    if (tri_test(S.bvh_recs, off + i, o, d, tmin, tmax, dist, beta, gamma)) {
                        if (COUNT) c.v[C_ACCEPTS]++;
                        tmax = dist;
                        found = true;
                        out.k = off + i;
                        out.beta = beta;
                        out.gamma = gamma;
                        out.dist = dist;
                        if (anyhit) return true;
                    }
                }
            } else {
                stk[(top < 50u ? top : 49u) * 256u] = cur + 1u;
                top++;
                stk[(top < 50u ? top : 49u) * 256u] = off;
                top++;
            }
        }
    }
    return found;
}

template <int TRAV, bool COUNT>
__device__ __forceinline__ bool trace(const DevScene& S, void* stk, const f3 o, const f3 d, float tmin, float tmax,
                                      bool anyhit, TraceOut& out, Counters& c)
{
    if (TRAV == RT_TRAVERSE_BVH)
        return trace_bvh<COUNT>(S, reinterpret_cast<uint32_t*>(stk), o, d, tmin, tmax, anyhit, out, c);
    return trace_bsp<COUNT>(S, reinterpret_cast<uint2*>(stk), o, d, tmin, tmax, anyhit, out, c);
}

// Hit record of the accepted triangle (the values intersect_triangle_indexed
// writes on its last accept): tri id, position, interpolated normal, material.
struct HitRec {
    uint32_t tri, material;
    f3 pos, nrm;
};
template <int TRAV>
__device__ __forceinline__ HitRec resolve(const DevScene& S, const TraceOut& t, const f3 o, const f3 d,
                                          bool face_normals)
{
    HitRec h;
    const uint32_t* ids = TRAV == RT_TRAVERSE_BVH ? S.bvh_ids : S.bsp_ids;
    const float4* recs = TRAV == RT_TRAVERSE_BVH ? S.bvh_recs : S.bsp_recs;
    h.tri = ids[t.k];
    const uint4 ix = S.tri_idx[h.tri];
    h.pos = add(o, muls(d, t.dist));
    f3 n0, n1, n2;
    if (face_normals) {
        const float4 r2 = recs[3u * t.k + 2u];
        n0 = n1 = n2 = V(r2.y, r2.z, r2.w);
    } else {
        n0 = ld3(S.nrm[ix.x]);
        n1 = ld3(S.nrm[ix.y]);
        n2 = ld3(S.nrm[ix.z]);
    }
    h.nrm = normalize(add(add(muls(n0, 1.0f - t.beta - t.gamma), muls(n1, t.beta)), muls(n2, t.gamma)));
    h.material = ix.w;
    return h;
}

__device__ __forceinline__ const rt_material& mat_of(const DevScene& S, uint32_t m)
{
    return S.mats[m < S.nmats ? m : S.nmats - 1u];   // naga Restrict bounds policy
}

// ------------------------------------------------------------------ path-tracer pieces
__device__ __forceinline__ f3 rotate_to_normal(f3 normal, f3 v)   // w7e3.wgsl:181-189
{
    const float signbit = rt_signf(normal.z + 1.0e-16f);
    const float a = -1.0f / (1.0f + rt_absf(normal.z));
    const float b = normal.x * normal.y * a;
    const f3 c0 = V(1.0f + normal.x * normal.x * a, b, -signbit * normal.x);
    const f3 c1 = V(signbit * b, signbit * (1.0f + normal.y * normal.y * a), -normal.y);
    return add(add(muls(c0, v.x), muls(c1, v.y)), muls(normal, v.z));
}

// setup_indirect (w7e3.wgsl:472-489): new direction about normalize(normal)
__device__ __forceinline__ f3 indirect_dir(f3 hn, uint32_t& rng)
{
    const f3 normal = normalize(hn);
    const float xi1 = rnd(rng);
    const float xi2 = rnd(rng);
    const float thet = rt_det_acosf(rt_det_sqrtf(1.0f - xi1));
    const float phi = 2.0f * RT_PI_F * xi2;
    const float st = rt_det_sinf(thet), ct = rt_det_cosf(thet);
    const f3 tang = V(st * rt_det_cosf(phi), st * rt_det_sinf(phi), ct);
    return rotate_to_normal(normal, tang);
}

struct Light {
    f3 l_i, w_i;
    float dist;
};
// sample_area_light, w7e3.wgsl:362-389
__device__ __forceinline__ Light sample_area_light(const DevScene& S, f3 pos, uint32_t idx, uint32_t& rng)
{
    const uint32_t li = S.lights[idx < S.nlights ? idx : S.nlights - 1u];
    const uint4 tri = S.tri_idx[li < S.ntris ? li : S.ntris - 1u];
    const f3 v0 = ld3(S.pos[tri.x]), v1 = ld3(S.pos[tri.y]), v2 = ld3(S.pos[tri.z]);
    const f3 cr = cross(sub(v0, v1), sub(v0, v2));
    const float area = 0.5f * rt_det_sqrtf(dot(cr, cr));
    const f3 l_e = ld3(mat_of(S, tri.w).ambient);
    const float psi1 = rt_det_sqrtf(rnd(rng));
    const float psi2 = rnd(rng);
    const float alpha = 1.0f - psi1;
    const float beta = (1.0f - psi2) * psi1;
    const float gamma = psi2 * psi1;
    const f3 normal = normalize(cross(sub(v0, v1), sub(v0, v2)));
    const f3 sampled = add(add(muls(v0, alpha), muls(v1, beta)), muls(v2, gamma));
    const f3 ld = sub(sampled, pos);
    const float cos_l = rt_maxf(dot(normalize(neg(ld)), normal), 0.0f);
    const float distance = rt_det_sqrtf(dot(ld, ld));
    Light L;
    L.l_i = divs(muls(muls(l_e, area), cos_l), distance * distance);
    L.w_i = normalize(ld);
    L.dist = distance;
    return L;
}

enum { PH_NEW = 0, PH_CLOSEST = 1, PH_SHADOW = 2 };

// ------------------------------------------------------------------ W7E3 / W9E1 path kernel
template <int MODE, int TRAV, bool COUNT>
__global__ void __launch_bounds__(256) k_path(DevScene S, DevLaunch L)
{
    extern __shared__ uint2 lds_stack[];
    void* stk = TRAV == RT_TRAVERSE_BVH ? (void*)(reinterpret_cast<uint32_t*>(lds_stack) + threadIdx.x)
                                        : (void*)(lds_stack + threadIdx.x);
    constexpr bool W9 = MODE == RT_MODE_W9E1;
    const float ETA = W9 ? 0.0001f : 0.01f;
    const uint32_t lane = threadIdx.x & 63u;
    const Cam cam = make_cam(L.u);
    const float fH = (float)L.u.resolution[1];
    const uint32_t light_tris = S.nlights - 1u;
    const uint32_t sel = W9 ? L.u.selection1 : 0u;
    Counters cnt;
#pragma unroll
    for (int i = 0; i < C_N; i++) cnt.v[i] = 0;

    for (;;) {
        const uint32_t work = fetch_work(L.work_counter, lane);
        if (work >= L.nwork) break;
        const Pix px = map_pixel(L, work, lane);
        bool alive = px.valid && L.spp > 0u;
        uint32_t it = L.first_iter;
        const uint32_t it_end = L.first_iter + L.spp;
        float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
        if (alive && L.first_iter > 0u) {
            const float4 pa = L.accum[px.out];
            a0 = pa.x;
            a1 = pa.y;
            a2 = pa.z;
        }
        uint32_t prim = 0xFFFFFFFFu, rng = 0, phase = PH_NEW, bounce = 0;
        bool emit = true, survive = false;
        f3 res = V(0, 0, 0), fac = V(1, 1, 1);
        f3 ro = V(0, 0, 0), rd = V(0, 0, 1);
        float rtmin = 0.0f, rtmax = 0.0f, prob = 1.0f;
        f3 hpos = V(0, 0, 0), hnrm = V(0, 0, 1), dvf = V(0, 0, 0), zf = V(0, 0, 0), amb = V(0, 0, 0);

        while (__ballot(alive)) {
            if (alive && phase == PH_NEW) {
                // fs_main prologue, w7e3.wgsl:236-248
                const uint32_t launch_idx = px.y * L.u.resolution[0] + px.x;
                rng = tea16(launch_idx, it);
                float jx = rnd(rng);
                float jy = rnd(rng);
                jx = jx / fH;
                jy = jy / fH;
                float ux, uy;
                pixel_uv(L.u, px.x, px.y, ux, uy);
                rd = cam_dir(cam, ux, uy, jx, jy);
                ro = cam.e;
                rtmin = ETA;
                rtmax = 5000.0f;
                res = V(0, 0, 0);
                fac = V(1, 1, 1);
                emit = true;
                bounce = 0;
                prim = 0xFFFFFFFFu;
                phase = PH_CLOSEST;
                cnt.v[C_SAMPLES]++;
                cnt.v[C_PRIMARY]++;
            }
            TraceOut tr;
            bool hit = false;
            if (alive) hit = trace<TRAV, COUNT>(S, stk, ro, rd, rtmin, rtmax, phase == PH_SHADOW, tr, cnt);
            if (!alive) continue;

            bool sample_done = false;
            if (phase == PH_CLOSEST) {
                if (hit) {
                    const HitRec h = resolve<TRAV>(S, tr, ro, rd, !W9);
                    if (bounce == 0) prim = h.tri;
                    const rt_material& m = mat_of(S, h.material);
                    if (sel == 0u) {
                        // lambertian (w7e3.wgsl:427-470 / w9e1.wgsl:428-470) up to the shadow ray
                        const f3 brdf = divs(ld3(m.diffuse), RT_PI_F);
                        const f3 emission = ld3(m.ambient);
                        Light Lt;
                        if (W9) {
                            Lt.l_i = V(0, 0, 0);   // light_init(), w9e1.wgsl:67-73
                            Lt.w_i = V(0.0f, 1.0f, 0.0f);
                            Lt.dist = 999999.0f;
                        } else {
                            const uint32_t ri = mcg31(rng);
                            const uint32_t idx = ri % light_tris + 1u;
                            Lt = sample_area_light(S, h.pos, idx, rng);
                        }
                        f3 dv = mul(muls(brdf, rt_satf(dot(h.nrm, Lt.w_i))), Lt.l_i);
                        if (!W9) dv = muls(dv, (float)light_tris);
                        amb = emit ? (W9 ? mul(emission, fac) : emission) : V(0, 0, 0);
                        dvf = mul(dv, fac);
                        zf = mul(V(0, 0, 0), fac);
                        fac = mul(fac, muls(brdf, RT_PI_F));
                        prob = (brdf.x + brdf.y + brdf.z) / 3.0f;
                        survive = rnd(rng) < prob;
                        hpos = h.pos;
                        hnrm = h.nrm;
                        // shadow ray (ray_init + tmin/tmax override)
                        ro = h.pos;
                        rd = Lt.w_i;
                        rtmin = ETA;
                        rtmax = Lt.dist - ETA;
                        phase = PH_SHADOW;
                        cnt.v[C_SHADOW]++;
                    } else if (sel == 2u) {
                        // mirror (w9e1.wgsl:491-504): reflect, offset origin, emit = true
                        const f3 n = h.nrm;
                        rd = sub(rd, muls(n, 2.0f * dot(n, rd)));
                        ro = add(h.pos, muls(n, ETA));
                        rtmin = ETA;
                        rtmax = 5000.0f;
                        emit = true;
                        if (bounce + 1u < 50u) {
                            bounce++;
                            cnt.v[C_BOUNCE]++;
                        } else {
                            sample_done = true;
                        }
                    } else {
                        f3 col;
                        if (sel == 5u) col = muls(add(h.nrm, V(1.0f, 1.0f, 1.0f)), 0.5f);
                        else if (sel == 6u) col = add(ld3(m.diffuse), ld3(m.ambient));
                        else col = V(0.7f, 0.0f, 0.7f);
                        res = add(res, col);
                        sample_done = true;
                    }
                } else {
                    // miss: background (w7e3) / environment_map(dir) * factor (w9e1.wgsl:264-265)
                    res = add(res, W9 ? mul(V(L.env[0], L.env[1], L.env[2]), fac) : V(0, 0, 0));
                    sample_done = true;
                }
            } else {   // PH_SHADOW finished: rest of lambertian
                res = add(res, add(hit ? zf : dvf, amb));
                if (survive && bounce + 1u < 50u) {
                    rd = indirect_dir(hnrm, rng);
                    ro = hpos;
                    rtmin = ETA;
                    rtmax = 5000.0f;
                    emit = false;
                    fac = divs(fac, prob);
                    bounce++;
                    phase = PH_CLOSEST;
                    cnt.v[C_BOUNCE]++;
                } else {
                    sample_done = true;
                }
            }
            if (sample_done) {
                // accumulation, w7e3.wgsl:261-271
                const float fi = (float)it, fi1 = (float)(it + 1u);
                a0 = rt_max0f((res.x + a0 * fi) / fi1);
                a1 = rt_max0f((res.y + a1 * fi) / fi1);
                a2 = rt_max0f((res.z + a2 * fi) / fi1);
                it++;
                if (it < it_end) {
                    phase = PH_NEW;
                } else {
                    L.accum[px.out] = make_float4(a0, a1, a2, 1.0f);
                    if (L.ids) L.ids[px.out] = prim;
                    alive = false;
                }
            }
        }
    }
    flush_counters(cnt, L.counters, COUNT);
}

// ------------------------------------------------------------------ W6E1 / PROJECT kernel
// fs_main of w6e1.wgsl:152-185 / project.wgsl:152-185 (primary rays, root
// AABB clip, directional-light Lambertian, mirror bounces up to MAX_DEPTH 10).
__device__ __forceinline__ bool intersect_min_max(const float* aabb, const f3 o, const f3 d, float& rtmin,
                                                  float& rtmax)
{
    float tmin = 1.0e32f, tmax = -1.0e32f;
#pragma unroll
    for (uint32_t i = 0; i < 3; i++) {
        const float di = comp(d, i), oi = comp(o, i);
        if (rt_absf(di) > 1.0e-8f) {
            const float p1 = (aabb[i] - oi) / di;
            const float p2 = (aabb[3 + i] - oi) / di;
            tmin = rt_minf(tmin, rt_minf(p1, p2));
            tmax = rt_maxf(tmax, rt_maxf(p1, p2));
        }
    }
    if (tmin > tmax || tmin > rtmax || tmax < rtmin) return false;
    rtmin = rt_maxf(tmin - 1.0e-4f, rtmin);
    rtmax = rt_minf(tmax + 1.0e-4f, rtmax);
    return true;
}

template <int TRAV, bool COUNT>
__global__ void __launch_bounds__(256) k_primary(DevScene S, DevLaunch L, int project)
{
    extern __shared__ uint2 lds_stack[];
    void* stk = TRAV == RT_TRAVERSE_BVH ? (void*)(reinterpret_cast<uint32_t*>(lds_stack) + threadIdx.x)
                                        : (void*)(lds_stack + threadIdx.x);
    const float ETA = 0.00001f;
    const uint32_t lane = threadIdx.x & 63u;
    const Cam cam = make_cam(L.u);
    const uint32_t subdiv = L.u.subdivision_level;
    const uint32_t nsamp = subdiv * subdiv;
    const uint32_t sel = L.u.selection1;
    const f3 bg = V(0.1f, 0.3f, 0.6f);
    Counters cnt;
#pragma unroll
    for (int i = 0; i < C_N; i++) cnt.v[i] = 0;

    for (;;) {
        const uint32_t work = fetch_work(L.work_counter, lane);
        if (work >= L.nwork) break;
        const Pix px = map_pixel(L, work, lane);
        bool alive = px.valid;
        float ux, uy;
        pixel_uv(L.u, px.x, px.y, ux, uy);
        uint32_t sample = 0, bounce = 0, prim = 0xFFFFFFFFu, phase = PH_NEW;
        f3 res = V(0, 0, 0), ro = cam.e, rd = V(0, 0, 1);
        float rtmin = 0.0f, rtmax = 0.0f;
        if (alive) cnt.v[C_SAMPLES]++;
        while (__ballot(alive)) {
            bool pixel_done = false;
            if (alive && phase == PH_NEW) {
                const float jx = L.jitter ? L.jitter[2u * sample] : 0.0f;
                const float jy = L.jitter ? L.jitter[2u * sample + 1u] : 0.0f;
                rd = cam_dir(cam, ux, uy, jx, jy);
                ro = cam.e;
                rtmin = ETA;
                rtmax = 100000.0f;
                bounce = 0;
                phase = PH_CLOSEST;
                cnt.v[C_PRIMARY]++;
                // aabb.wgsl:8-31 for BSP scenes; bvh.wgsl:197-200 makes it a no-op for BVH scenes
                if (TRAV == RT_TRAVERSE_BSP && !intersect_min_max(S.aabb, ro, rd, rtmin, rtmax)) {
                    res = bg;   // result = bgcolor.rgb; break (leaves the sample loop)
                    pixel_done = true;
                }
            }
            TraceOut tr;
            bool hit = false;
            const bool tracing = alive && !pixel_done;
            if (tracing) hit = trace<TRAV, COUNT>(S, stk, ro, rd, rtmin, rtmax, false, tr, cnt);
            if (tracing) {
                bool sample_done = false;
                if (hit) {
                    const HitRec h = resolve<TRAV>(S, tr, ro, rd, false);
                    if (bounce == 0u && sample + 1u == nsamp) prim = h.tri;
                    const rt_material& m = mat_of(S, h.material);
                    if (sel == 0u) {
                        // lambertian, w6e1.wgsl:279-310 / project.wgsl:279-306
                        const f3 w_i = neg(normalize(V(-1.0f, -1.0f, -1.0f)));
                        const f3 l_i = muls(V(RT_PI_F, RT_PI_F, RT_PI_F), 1.0f);
                        const float dist = 1.0f;
                        const float dd = dot(h.nrm, w_i);
                        f3 dfc = V(dd, dd, dd);
                        dfc = divs(dfc, dist * dist);
                        dfc = mul(dfc, l_i);
                        dfc = divs(dfc, RT_PI_F);
                        const f3 diffuse = add(V(0, 0, 0), mul(ld3(m.diffuse), dfc));
                        f3 col;
                        if (project) col = add(diffuse, muls(ld3(m.ambient), 0.1f));
                        else col = add(muls(diffuse, 0.9f), muls(ld3(m.ambient), 0.1f));
                        res = add(res, col);
                        sample_done = true;
                    } else if (sel == 2u) {
                        const f3 n = h.nrm;
                        rd = sub(rd, muls(n, 2.0f * dot(n, rd)));
                        ro = add(h.pos, muls(n, ETA));
                        rtmin = ETA;
                        rtmax = 100000.0f;
                        if (bounce + 1u < 10u) {
                            bounce++;
                            cnt.v[C_BOUNCE]++;
                        } else {
                            sample_done = true;
                        }
                    } else {
                        f3 col;
                        if (sel == 5u) col = muls(add(h.nrm, V(1.0f, 1.0f, 1.0f)), 0.5f);
                        else if (sel == 6u) col = add(ld3(m.diffuse), ld3(m.ambient));
                        else col = V(0.7f, 0.0f, 0.7f);
                        res = add(res, col);
                        sample_done = true;
                    }
                } else {
                    res = add(res, bg);
                    sample_done = true;
                }
                if (sample_done) {
                    sample++;
                    if (sample < nsamp) phase = PH_NEW;
                    else pixel_done = true;
                }
            }
            if (alive && pixel_done) {
                const float multiplier = 1.0f / (float)nsamp;
                res = muls(res, multiplier);
                L.accum[px.out] = make_float4(res.x, res.y, res.z, 1.0f);
                if (L.ids) L.ids[px.out] = prim;
                alive = false;
            }
        }
    }
    flush_counters(cnt, L.counters, COUNT);
}

// ------------------------------------------------------------------ W1E6 analytic kernel
// res/shaders/w1e6.wgsl: triangle + sphere + plane, point light, no mesh.
__device__ __forceinline__ bool w1_triangle(f3 o, f3 w, float tmin, float& tmax, f3 a, f3 b, f3 c, f3& pos,
                                            f3& nrm)
{
    const f3 e0 = sub(b, a), e1 = sub(c, a), ov = sub(a, o);
    const f3 normal = cross(e0, e1);
    const f3 nom = cross(ov, w);
    const float denom = dot(w, normal);
    if (rt_absf(denom) < 1e-6f) return false;
    const float beta = dot(nom, e1) / denom;
    const float gamma = -dot(nom, e0) / denom;
    const float distance = dot(ov, normal) / denom;
    if (beta < 0.0f || gamma < 0.0f || beta + gamma > 1.0f || distance > tmax || distance < tmin) return false;
    tmax = distance;
    pos = add(o, muls(w, distance));
    nrm = normalize(normal);
    return true;
}
__device__ __forceinline__ bool w1_sphere(f3 o, f3 w, float tmin, float& tmax, f3 center, float radius, f3& pos,
                                          f3& nrm)
{
    const f3 oc = sub(o, center);
    const float a = dot(w, w);
    const float b2 = dot(oc, w);
    const float c = dot(oc, oc) - radius * radius;
    const float disc = b2 * b2 - a * c;
    if (disc < 0.0f) return false;
    const float ds = rt_det_sqrtf(disc);
    float root = (-b2 - ds) / a;
    if (root < tmin || root > tmax) {
        root = (-b2 + ds) / a;
        if (root < tmin || root > tmax) return false;
    }
    tmax = root;
    pos = add(o, muls(w, root));
    nrm = normalize(sub(pos, center));
    return true;
}
__device__ __forceinline__ bool w1_plane(f3 o, f3 w, float tmin, float& tmax, f3 normal, f3 position, f3& pos,
                                         f3& nrm)
{
    const float distance = dot(sub(position, o), normal) / dot(w, normal);
    if (distance < tmin || distance > tmax) return false;
    tmax = distance;
    pos = add(o, muls(w, distance));
    nrm = normal;
    return true;
}

__global__ void __launch_bounds__(256) k_w1e6(DevLaunch L)
{
    const uint32_t lane = threadIdx.x & 63u;
    const Cam cam = make_cam(L.u);
    Counters cnt;
#pragma unroll
    for (int i = 0; i < C_N; i++) cnt.v[i] = 0;
    for (;;) {
        const uint32_t work = fetch_work(L.work_counter, lane);
        if (work >= L.nwork) break;
        const Pix px = map_pixel(L, work, lane);
        if (!px.valid) continue;
        cnt.v[C_SAMPLES]++;
        cnt.v[C_PRIMARY]++;
        float ux, uy;
        pixel_uv(L.u, px.x, px.y, ux, uy);
        const f3 w = normalize(add(add(muls(muls(cam.b1, ux), cam.aspect), muls(cam.b2, uy)), muls(cam.v, cam.d)));
        const f3 o = cam.e;
        float tmax = 5000.0f;
        const float tmin = 0.00001f;
        f3 pos = V(0, 0, 0), nrm = V(0, 0, 0), base = V(0, 0, 0);
        bool any = false;
        uint32_t which = 0xFFFFFFFFu;
        if (w1_triangle(o, w, tmin, tmax, V(0.2f, 0.1f, 0.9f), V(-0.2f, 0.1f, -0.1f), V(-0.2f, 0.1f, 0.9f), pos,
                        nrm)) {
            any = true;
            base = V(0.4f, 0.3f, 0.2f);
            which = 0;
        }
        if (w1_sphere(o, w, tmin, tmax, V(0.0f, 0.5f, 0.0f), 0.3f, pos, nrm)) {
            any = true;
            base = V(0.0f, 0.0f, 0.0f);
            which = 1;
        }
        if (w1_plane(o, w, tmin, tmax, V(0.0f, 1.0f, 0.0f), V(0.0f, 0.0f, 0.0f), pos, nrm)) {
            any = true;
            base = V(0.1f, 0.7f, 0.0f);
            which = 2;
        }
        f3 result;
        if (any) {
            // lambertian + sample_point_light, w1e6.wgsl:239-284
            const f3 intensity = muls(V(RT_PI_F, RT_PI_F, RT_PI_F), 5.0f);
            const f3 dir = sub(V(0.0f, 1.2f, 0.0f), pos);
            const float dist = dot(dir, dir);
            const f3 l_i = divs(intensity, dist * dist);
            const float dd = dot(nrm, dir);
            f3 dfc = V(dd, dd, dd);
            dfc = mul(dfc, l_i);
            dfc = muls(dfc, (1.0f - 0.0f) / RT_PI_F);
            const f3 diffuse = mul(base, dfc);
            result = add(V(0, 0, 0), add(muls(diffuse, 0.9f), muls(base, 0.1f)));
        } else {
            result = add(V(0, 0, 0), V(0.1f, 0.3f, 0.6f));
        }
        L.accum[px.out] = make_float4(result.x, result.y, result.z, 1.0f);
        if (L.ids) L.ids[px.out] = which;
    }
    flush_counters(cnt, L.counters, false);
}

// ------------------------------------------------------------------ tile unpack
// packed (rank-major all-gather output): [nranks][local_tiles][64] -> row-major frame
__global__ void __launch_bounds__(256) k_unpack(uint32_t W, uint32_t H, uint32_t nranks, uint32_t local_tiles,
                                                const float4* pa, const uint32_t* pi, float4* fa, uint32_t* fi)
{
    const uint32_t tiles_x = (W + 7u) / 8u, tiles_y = (H + 7u) / 8u;
    const uint64_t total = (uint64_t)tiles_x * tiles_y * 64u;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t t = (uint32_t)(g >> 6), lane = (uint32_t)(g & 63u);
        const uint32_t x = (t % tiles_x) * 8u + (lane & 7u), y = (t / tiles_x) * 8u + (lane >> 3);
        if (x >= W || y >= H) continue;
        const uint32_t rank = t % nranks, l = t / nranks;
        const uint64_t src = ((uint64_t)rank * local_tiles + l) * 64u + lane;
        const uint64_t dst = (uint64_t)y * W + x;
        if (pa && fa) fa[dst] = pa[src];
        if (pi && fi) fi[dst] = pi[src];
    }
}

// ------------------------------------------------------------------ math self test
__host__ __device__ inline void math_eval(float x, float* o)
{
    o[0] = rt_det_sqrtf(x < 0.0f ? -x : x);
    o[1] = 1.0f / (x == 0.0f ? 1.0f : x);
    o[2] = rt_det_sinf(x * 6.2831855f);
    o[3] = rt_det_cosf(x * 6.2831855f);
    o[4] = rt_det_acosf(x - __builtin_floorf(x));
    o[5] = (x * 3.0f + 1.0f) / (x - 7.0f);
    o[6] = (float)(uint32_t)(x * 1000.0f) / (float)0x80000000u;
    o[7] = rt_det_acosf(rt_det_sqrtf(1.0f - (x - __builtin_floorf(x))));
}
__global__ void k_selftest_math(const float* in, float* out, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) math_eval(in[i], out + (size_t)i * kMathOuts);
}
void host_math(const float* in, float* out, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) math_eval(in[i], out + (size_t)i * kMathOuts);
}

// ------------------------------------------------------------------ launchers
static int grid_for(int num_cus, int waves_per_cu)
{
    int wpc = waves_per_cu > 0 ? waves_per_cu : 16;
    int blocks = num_cus * wpc / 4;   // 256-thread blocks = 4 waves
    return blocks > 0 ? blocks : 1;
}

template <int MODE, int TRAV, bool COUNT>
static void launch_path(const DevScene& s, const DevLaunch& l, int grid, size_t lds, hipStream_t st)
{
    hipLaunchKernelGGL((k_path<MODE, TRAV, COUNT>), dim3(grid), dim3(256), lds, st, s, l);
}
template <int TRAV, bool COUNT>
static void launch_primary(const DevScene& s, const DevLaunch& l, int project, int grid, size_t lds, hipStream_t st)
{
    hipLaunchKernelGGL((k_primary<TRAV, COUNT>), dim3(grid), dim3(256), lds, st, s, l, project);
}

int launch_render(const DevScene& s, const DevLaunch& l, rt_mode mode, rt_traverse trav, bool detail, int num_cus,
                  int waves_per_cu, hipStream_t stream)
{
    const int grid = grid_for(num_cus, waves_per_cu);
    const size_t lds = trav == RT_TRAVERSE_BVH ? (size_t)50 * 256 * 4 : (size_t)(s.bsp_depth ? s.bsp_depth : 1) * 256 * 8;
    if (mode == RT_MODE_W1E6) {
        hipLaunchKernelGGL(k_w1e6, dim3(grid), dim3(256), 0, stream, l);
        return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
    }
    const bool bvh = trav == RT_TRAVERSE_BVH;
    switch (mode) {
    case RT_MODE_W7E3:
        if (bvh) detail ? launch_path<RT_MODE_W7E3, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W7E3, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_path<RT_MODE_W7E3, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_path<RT_MODE_W7E3, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W9E1:
        if (bvh) detail ? launch_path<RT_MODE_W9E1, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W9E1, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_path<RT_MODE_W9E1, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_path<RT_MODE_W9E1, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W6E1:
    case RT_MODE_PROJECT: {
        const int project = mode == RT_MODE_PROJECT;
        if (bvh) detail ? launch_primary<RT_TRAVERSE_BVH, true>(s, l, project, grid, lds, stream)
                        : launch_primary<RT_TRAVERSE_BVH, false>(s, l, project, grid, lds, stream);
        else detail ? launch_primary<RT_TRAVERSE_BSP, true>(s, l, project, grid, lds, stream)
                    : launch_primary<RT_TRAVERSE_BSP, false>(s, l, project, grid, lds, stream);
        break;
    }
    default:
        return RT_E_UNSUPPORTED;
    }
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

int launch_unpack(uint32_t width, uint32_t height, uint32_t nranks, uint32_t local_tiles, const float4* packed_accum,
                  const uint32_t* packed_ids, float4* frame_accum, uint32_t* frame_ids, hipStream_t stream)
{
    const uint64_t total = (uint64_t)((width + 7) / 8) * ((height + 7) / 8) * 64u;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_unpack, dim3((uint32_t)blocks), dim3(256), 0, stream, width, height, nranks, local_tiles,
                       packed_accum, packed_ids, frame_accum, frame_ids);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

int launch_selftest_math(const float* in, float* out, uint32_t n, hipStream_t stream)
{
    hipLaunchKernelGGL(k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, stream, in, out, n);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

}  // namespace rtk
