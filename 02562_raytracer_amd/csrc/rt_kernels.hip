// rt_kernels.hip -- gfx950 (CDNA4) kernels for the per-pixel traversal + shading
// hot path of cakarsubasi/02562_raytracer (res/shaders/*.wgsl).
//
// Structure of the path tracers' k_path:
//   * persistent grid (num_CUs x waves_per_CU waves, capped by LDS and by the
//     register budget) over WORK UNITS of one (pixel, iteration) pair: the
//     iterations of a pixel are independent (the PRNG seed is tea16(pixel,
//     iteration)), so a unit traces one sample and writes its radiance and
//     primary-hit id as a 16-B record to samples[pixel][iteration];
//   * k_fold then applies the progressive average of w7e3.wgsl:261-271 to every
//     pixel in iteration order -- bit-identical to the reference's spp
//     sequential render() calls;
//   * units come from 8 work shards, one per XCD (HW_REG_XCC_ID), each owning
//     every 8th block of 64 consecutive units, with its queue head in its own
//     128-B line; a wave refill is one atomic, and ballot + mbcnt hand the
//     slots to the idle lanes (active-lane compaction); pixel-major unit order
//     gives a refill's lanes the iterations of one pixel (coherent rays);
//   * ray state machine with ONE traversal call site: each trip every tracing
//     lane advances its ray (camera / bounce closest-hit, or a shadow any-hit)
//     by one 96-B load: a treelet (its subtree's content box, tested first:
//     subtree culling, then three BSP levels walked), or a leaf's triangle
//     records (two tests per trip); lanes whose ray ended wait and
//     shade together once few lanes still trace (shading threshold, chosen
//     per wave from its leaf share), so no lane waits for the slowest ray;
//   * per-lane traversal stack in LDS, [level][thread] (conflict-free):
//     BSP: a bit trail in a register + one 4-B tmax per depth;
//     BVH: 16 entries in LDS, the rest of the 50 in a per-lane global region;
//   * BSP treelets and triangle records ({v0, e0, e1, n}, 48 B, in treeIds
//     order) share one buffer resource; out-of-range reads return 0.
// Numerics: -ffp-contract=off, correctly rounded f32 div/sqrt, pinned
// transcendentals (include/rt_detmath.h) => bit-identical to the CPU oracle.
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

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

// The lane's index in its wave, recomputed where used (volatile: never hoisted
// into a long-lived register, which at 8 waves/SIMD would be spilled).
__device__ __forceinline__ uint32_t lane_v()
{
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// IEEE-mode v_max / v_min of quiet-NaN-or-number operands.  fmaxf / fminf of
// a value the compiler cannot prove canonical (a loop-carried tmin / tmax, a
// kernel argument) get a canonicalising v_max_f32 x, x first -- only a
// signalling NaN would need it, and no value of the walks is one (every NaN
// here is produced by arithmetic or is a quiet constant).  The instruction
// drops a quiet NaN operand exactly as fmaxf / fminf do.  (bsp_box_miss: three
// such v_max per walking trip.)
__device__ __forceinline__ float qmax(float a, float b)
{
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float qmin(float a, float b)
{
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float qmax3(float a, float b, float c)
{
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float qmin3(float a, float b, float c)
{
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// min(x, s) with s a uniform (SGPR) operand
__device__ __forceinline__ float qmin_s(float s, float x)
{
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "s"(s), "v"(x));
    return r;
}
// 96 * m (a treelet's byte offset) as two full-rate shifts-and-adds: the
// compiler's v_mul_lo_u32 is a quarter-rate instruction, and m can exceed the
// 24 bits of v_mul_u32_u24 (heap indices up to 2^25 at max_depth 24)
__device__ __forceinline__ uint32_t times96(uint32_t m)
{
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 1, %1\n\tv_lshlrev_b32 %0, 5, %0" : "=&v"(r) : "v"(m));
    return r;
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 as_f4(v4u q)
{
    return make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w));
}

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
enum { C_SAMPLES, C_PRIMARY, C_SHADOW, C_BOUNCE, C_INTERIOR, C_LEAF, C_POPS, C_IDS, C_TESTS, C_ACCEPTS,
       C_TRIPS, C_LANE_STEPS, C_LEAF_LANE_STEPS, C_NODE_TRIPS, C_LEAF_TRIPS, C_EXACT_TESTS, C_EXACT_NODES,
       C_SHADE_PASSES, C_SHADE_LANES, C_TRAV_CYC64, C_SHADE_CYC64, C_MEMWAIT_CYC64, C_CULLS, C_N };

struct Counters {
    uint32_t v[C_N];
};

__device__ __forceinline__ void flush_counters(const Counters& c, unsigned long long* out, bool detail)
{
    const int n = detail ? (int)C_N : 4;
    for (int i = 0; i < n; i++) {
        uint32_t x = c.v[i];
        unsigned long long s = x;
        if (i == C_TRAV_CYC64 || i == C_SHADE_CYC64 || i == C_MEMWAIT_CYC64)
            s <<= 6;   // wave cycles, accumulated in units of 64
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
// The basis v = normalize(p - e), b1 = normalize(cross(v, u)), b2 = cross(b1, v)
// is loop-invariant: rt_api.cpp evaluates it once on the host with the same
// IEEE operations (no contraction) and passes it as kernel arguments (SGPRs).
__device__ __forceinline__ Cam make_cam(const DevLaunch& L)
{
    Cam c;
    c.e = ld3(L.cam + 0);
    c.v = ld3(L.cam + 3);
    c.b1 = ld3(L.cam + 6);
    c.b2 = ld3(L.cam + 9);
    c.d = L.cam[12];
    c.aspect = L.cam[13];
    return c;
}
// Kernel arguments made opaque where a sample starts or a lane is refilled:
// the values derived from them (the camera products, float resolutions,
// integer-division reciprocals) are then recomputed there from SGPRs instead
// of being hoisted out of the persistent loop into VGPRs that live across the
// trip loop and are spilled (k_path at 8 waves/SIMD has 64 VGPRs).
__device__ __forceinline__ uint32_t sopaque(uint32_t x)
{
    asm volatile("" : "+s"(x));
    return x;
}
__device__ __forceinline__ float sopaque(float x)
{
    asm volatile("" : "+s"(x));
    return x;
}
__device__ __forceinline__ Cam make_cam_opaque(const DevLaunch& L)
{
    Cam c = make_cam(L);
    c.v = V(sopaque(c.v.x), sopaque(c.v.y), sopaque(c.v.z));
    c.b1 = V(sopaque(c.b1.x), sopaque(c.b1.y), sopaque(c.b1.z));
    c.b2 = V(sopaque(c.b2.x), sopaque(c.b2.y), sopaque(c.b2.z));
    c.d = sopaque(c.d);
    c.aspect = sopaque(c.aspect);
    return c;
}
// The kernel argument blocks of k_path(DevScene, DevLaunch), re-read from
// the kernarg segment through an opaque pointer where k_path shades and
// refills: the fields used there are then scalar loads in that phase instead
// of SGPRs (and VGPR lanes holding SGPR spills) kept across the trip loop.
// (Taking the address of the parameters themselves would copy them to
// scratch.)  The explicit arguments are laid out in order at their natural
// alignment.
// Every GPU parity test reads both blocks through these offsets (a wrong one
// would change every frame).
static_assert(std::is_standard_layout<DevScene>::value && std::is_trivially_copyable<DevScene>::value, "DevScene");
static_assert(std::is_standard_layout<DevLaunch>::value && std::is_trivially_copyable<DevLaunch>::value, "DevLaunch");
constexpr size_t KARG_S = 0;
constexpr size_t KARG_L = (sizeof(DevScene) + alignof(DevLaunch) - 1) & ~(alignof(DevLaunch) - 1);
template <class T>
__device__ __forceinline__ const T& kreload(size_t off)
{
    typedef __attribute__((address_space(4))) const char KC;
    KC* p = (KC*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const T*)(p + off);   // generic; the address-space inference restores the scalar loads
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
// The tile rows' rotation is ty mod 8 (tiling.tile_of_seq)
__device__ __forceinline__ Pix map_pixel(const DevLaunch& L, uint32_t work, uint32_t lane)
{
    Pix p;
    const uint32_t lx = lane & 7u, ly = lane >> 3;
    const uint32_t tiles_x = sopaque(L.tiles_x);   // see make_cam_opaque
    if (L.tileset == 0) {
        uint32_t tx = work % tiles_x, ty = work / tiles_x;
        uint32_t rx = tx * 8u + lx, ry = ty * 8u + ly;
        p.valid = rx < L.w && ry < L.h;
        p.x = L.x0 + rx;
        p.y = L.y0 + ry;
        p.out = ry * L.w + rx;
    } else {
        // sequence position s = work * nranks + rank; row ty = s / tiles_x, the
        // row rotated by ty mod 8 (tiling.tile_of_seq): rank r owns the diagonal
        // columns tx = r + ty (mod nranks) when nranks divides 8 and tiles_x
        // (1080p: 240 tile columns); frames under 8 tiles wide are not rotated
        uint32_t t = work * L.nranks + L.rank;
        uint32_t ty = t / tiles_x, tx = t - ty * tiles_x + (tiles_x >= 8u ? (ty & 7u) : 0u);
        tx = tx >= tiles_x ? tx - tiles_x : tx;
        p.x = tx * 8u + lx;
        p.y = ty * 8u + ly;
        p.valid = (t < L.tiles_x * L.tiles_y) && p.x < L.u.resolution[0] && p.y < L.u.resolution[1];
        p.out = work * 64u + lane;
    }
    return p;
}
// map_pixel's output index recomputed from the pixel (k_path keeps only the
// pixel across the trip loop): region mode ry * w + rx; tileset mode the
// packed slot work * 64 + lane of tile t = work * nranks + rank.
__device__ __forceinline__ uint32_t pixel_out(const DevLaunch& L, uint32_t x, uint32_t y)
{
    if (L.tileset == 0) return (y - L.y0) * L.w + (x - L.x0);
    const uint32_t ty = y >> 3, tx = x >> 3, r = L.tiles_x >= 8u ? (ty & 7u) : 0u;
    const uint32_t t = ty * L.tiles_x + (tx >= r ? tx - r : tx + L.tiles_x - r);   // map_pixel's s
    return (t - L.rank) / L.nranks * 64u + ((y & 7u) << 3) + (x & 7u);
}
// The work shard of this wave: the XCD it runs on (HW_REG_XCC_ID, hwreg 20,
// bits 3:0; 0-7 on MI355X), and with RT_SHARD_LG > 3 also the low bits of its
// CU id within the XCD (HW_REG_HW_ID, hwreg 4, bits 11:8).  Any value is
// correct, only the atomic spread changes.
#ifndef RT_SHARD_LG
#define RT_SHARD_LG 3
#endif
__device__ __forceinline__ uint32_t shard_of_wave()
{
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | ((3 - 1) << 11)) & 7u;
    if (RT_SHARD_LG <= 3) return xcc;
    const uint32_t cu = ((uint32_t)__builtin_amdgcn_s_getreg(4 | (8 << 6) | ((4 - 1) << 11))) & 15u;
    constexpr uint32_t SUB = RT_SHARD_LG > 3 ? RT_SHARD_LG - 3 : 0;
    return (xcc << SUB) | (cu & ((1u << SUB) - 1u));
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
//
// Exact fast rejection: the accept predicate is a pure function of the
// correctly rounded quotients beta = a/denom, gamma = b/denom, dist = c/denom,
// so a quotient is only divided out when its sign/range is not already
// certain.  With 1e-10 <= |denom| <= 2^60, r = v_rcp_f32(denom) is a normal
// number within 1 ulp of 1/denom, so a*r carries the quotient's sign and is
// within 2^-22 relative of it: a*r < -2^-100 makes a/denom a negative number of
// magnitude > 2^-101, far from the 2^-150 underflow threshold, so RN(a/denom) < 0
// (an infinite a*r means an infinite quotient of the same sign; NaN compares
// false and falls back to the division).  The dist range test uses the same r
// with a 2^-20 relative margin, which bounds |RN(c*r) - RN(c/denom)|.
// Result of a triangle test: 0 reject, 1 accept, 2 the exact quotients pass
// but the distance lies within the margin of an inexact ray bound (the
// caller resolves the bound exactly).  exact_bounds: tmin and tmax are the
// shader's values (the BSP walk keeps approximate pushed t values, see
// bsp_decide).
// CULL: the back-face culling test of w9e3.wgsl:328 (|denom| < 5e-5 or
// denom > 0 rejects) in place of |denom| < 1e-10.
// BARY false (the walks' trip loops): the barycentrics are
// not returned, and a candidate whose approximate quotients already settle
// every condition of the accept predicate (beta and gamma non-negative by the
// sign of a*r and b*r, their sum below 1 and the distance inside [tmin, tmax]
// by the same margins as the rejections) is accepted after dividing out only
// dist, which becomes tmax; beta and gamma are derived where the hit is shaded
// (bary_of: the same operations on the same record, so the same bits).  Only
// an unsettled candidate divides all three quotients.
// VERT: the ray direction is exactly (0, 1, 0) (W9E1's shadow rays,
// light_init, w9e1.wgsl:67-73, :442-446).  Then cross(ov, w) is (-ov.z, +-0,
// ov.x) and dot(w, n) is n.y exactly -- each product with 0 is a zero, each
// with 1 the other operand, and adding a zero changes nothing but the sign of
// a zero -- so a and b are one product pair and one add each, and the cross
// product and the denominator cost nothing: 14 arithmetic instructions
// instead of 32.  Every value equals the general form's except possibly the
// sign of a zero a, b (or denom, which is then rejected by its magnitude):
// the predicate below compares them with < / > only, and the sign-bit shortcut
// of a sure accept falls back to the exact quotients, whose comparisons do not
// see it either, so the accept decision and dist are the general form's.
template <bool FAST, bool COUNT = false, bool CULL = false, bool BARY = true, bool VERT = false>
__device__ __forceinline__ bool tri_math(const float4 r0, const float4 r1, const float4 r2, f3 o, f3 w, float tmin,
                                         float tmax, float& dist, float& beta, float& gamma, Counters* cn = nullptr,
                                         bool vert = false)
{
    const f3 v0 = V(r0.x, r0.y, r0.z), e0 = V(r0.w, r1.x, r1.y), e1 = V(r1.z, r1.w, r2.x);
    const f3 n = V(r2.y, r2.z, r2.w);
    const f3 ov = sub(v0, o);
    float denom, a, b;
    if (VERT && vert) {
        denom = n.y;
        a = (-ov.z) * e1.x + ov.x * e1.z;
        b = -((-ov.z) * e0.x + ov.x * e0.z);
    } else {
        const f3 nom = cross(ov, w);
        denom = dot(w, n);
        a = dot(nom, e1);
        b = -dot(nom, e0);
    }
    const float c = dot(ov, n);
    bool reject = CULL ? ((rt_absf(denom) < 0.00005f) | (denom > 0.0f)) : rt_absf(denom) < 1e-10f;
    float tq = 0.0f, m = 0.0f, qa = 0.0f, qb = 0.0f, ms = 0.0f;
    bool inr = false;
    if (FAST) {
        // certain rejections, each implying the exact predicate below rejects:
        // a sign (beta < 0 / gamma < 0), the distance range, or
        // RN(beta + gamma) > 1 (needs beta + gamma > 1 + 2^-24: margin 2^-22)
        const float r = __builtin_amdgcn_rcpf(denom);
        tq = c * r;
        m = __builtin_fmaf(rt_absf(tq), 0x1p-20f, 1e-30f);   // the product is exact: = mul + add
        qa = a * r;
        qb = b * r;
        ms = (rt_absf(qa) + rt_absf(qb)) * 0x1p-20f;
        inr = rt_absf(denom) <= 0x1p60f;
        reject = reject | (inr & ((qa < -0x1p-100f) | (qb < -0x1p-100f) | (tq - m > tmax) | (tq + m < tmin) |
                                  (qa + qb - ms > 1.0f + 0x1p-22f)));
    }
    if (reject) return false;
    if (COUNT) cn->v[C_EXACT_TESTS]++;
    dist = c / denom;
    if (FAST && !BARY) {
        // certain accepts (decided only for the candidates that survive): the
        // sign of a*r is the sign of a/denom (so a clear sign bit means
        // RN(a/denom) is +0 or positive, never < 0); the sum and the range with
        // the margins above, on the other side
        const bool sure = inr & !(__float_as_uint(qa) >> 31) & !(__float_as_uint(qb) >> 31) &
                          (qa + qb + ms < 1.0f - 0x1p-22f) & (tq - m >= tmin) & (tq + m <= tmax);
        if (sure) return true;
    }
    beta = a / denom;
    gamma = b / denom;
    return !((beta < 0.0f) | (gamma < 0.0f) | (beta + gamma > 1.0f) | (dist > tmax) | (dist < tmin));
}
// beta and gamma of the accepted record at byte offset k of the walk's buffer
// for the ray (o, w): intersect_triangle's a / denom and b / denom with the
// operations of tri_math (the trip loops do not keep them)
template <int TRAV>
__device__ __forceinline__ void bary_of(const DevScene& S, uint32_t k, const f3 o, const f3 w, float& beta,
                                        float& gamma)
{
    const uint8_t* base = TRAV == RT_TRAVERSE_BVH ? S.bvh_base : reinterpret_cast<const uint8_t*>(S.bsp_nodes);
    const float4* rp = reinterpret_cast<const float4*>(base + k);
    const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
    const f3 v0 = V(r0.x, r0.y, r0.z), e0 = V(r0.w, r1.x, r1.y), e1 = V(r1.z, r1.w, r2.x);
    const f3 n = V(r2.y, r2.z, r2.w);
    const f3 ov = sub(v0, o);
    const f3 nom = cross(ov, w);
    const float denom = dot(w, n);
    const float a = dot(nom, e1);
    const float b = -dot(nom, e0);
    beta = a / denom;
    gamma = b / denom;
}
struct TraceOut {
    uint32_t k;   // record slot of the accepted triangle
    float beta, gamma, dist;
};

// Per-lane traversal state (kept in registers across the persistent loop).
// The accepted hit's distance is tmax (every accept sets tmax = dist, and
// neither walk raises tmax again after its last accept).
struct Trav {
    uint32_t node;   // BSP: 1-based heap index of the current node   BVH: stack top
    uint32_t lvl;    // BSP: bit trail (bit d = pending far child pushed at depth d)   BVH: pops so far
    uint32_t leaf_k, leaf_end;   // triangle slots of the leaf being tested (empty when equal)
    float tmin, tmax;
    bool found;
    uint32_t hit_k;
    float beta, gamma;
    uint32_t tos;    // BVH: cached top-of-stack value (node byte offset)
    uint32_t tos2;   // BVH: cached second entry (valid while node >= 2)
};

__device__ __forceinline__ void trav_init(Trav& t, float tmin, float tmax)
{
    t.node = 1;
    t.lvl = 0;
    t.leaf_k = t.leaf_end = 0;
    t.tmin = tmin;
    t.tmax = tmax;
    t.found = false;
}
__device__ __forceinline__ TraceOut trav_out(const Trav& t) { return TraceOut{t.hit_k, t.beta, t.gamma, t.tmax}; }

// ------------------------------------------------------------------ tested-triangle log
// The walks report each triangle they test (its record's byte offset) to a LOG:
// NoLog (every render kernel) compiles to nothing; the ray-query kernel
// (k_query) hashes the tested ids in order (FNV-1a over little-endian u32, as
// tests/golden/gen_js_walk.js hashes the reference walk's tests).
struct NoLog {
    __device__ __forceinline__ void tested(uint32_t) {}
};
struct FnvLog {
    const uint32_t* ids;   // record slot -> triangle id (treeIds / bvh_triangles)
    uint32_t rec_off;      // byte offset of record slot 0 in the walk's buffer
    uint32_t n, h, last;
    __device__ __forceinline__ void tested(uint32_t k)
    {
        const uint32_t id = ids[(k - rec_off) / 48u];
#pragma unroll
        for (int b = 0; b < 4; b++) h = (h ^ ((id >> (8 * b)) & 0xFFu)) * 0x01000193u;
        n++;
        last = id;
    }
};

// ------------------------------------------------------------------ BSP traversal
// intersect_trimesh, bsp.wgsl:10-81, as a per-lane state machine: each call
// visits at most one node and tests at most one triangle ("if-if"), so a wave
// trip never serialises behind the longest leaf of any lane.  Returns true
// when the ray is finished (t.found = hit).
//
// Stack as a bit trail.  Nodes are numbered 1-based in heap order (children
// 2M, 2M+1; the device array has one pad node in front, so node M is at
// [M]).  Every pending stack entry of bsp.wgsl is an ancestor of the current
// node at which the walk pushed its far child, so an entry is fully described
// by its depth d: bit d of `lvl` marks it, the far child is the sibling of
// the current node's ancestor at depth d+1, ((M >> (depth(M)-d-1)) ^ 1), and
// one float is stored -- in LDS, indexed by depth ([depth][thread], 4 B): the
// tmax at the push, which is what bsp.wgsl saves in branch_ray.y and its pop
// restores.  The other saved value, branch_ray.x = t, needs no slot: the push
// sets tmax = t, tmax only changes on push, pop, and on an accept (after
// which the walk ends), and every entry pushed above this one restores the
// tmax it saw, so when this entry is popped the current tmax is its t, bit
// for bit.  A pop is one LDS read.
// anyhit: stop at the first accepted triangle -- shadow rays use only the
// boolean, and the walk up to that triangle is identical, so it is too.
// Interior nodes: the exact t = RN((plane - o)/denom) is only derived when the
// approximate t (x * RN(1/denom), 2^-20 margin) cannot decide near/far.
// m >= 1 always (a zero argument would be undefined: no clamp instruction)
__device__ __forceinline__ uint32_t heap_depth(uint32_t m) { return 31u - (uint32_t)__builtin_clz(m); }

__device__ __forceinline__ bool bsp_pop(const float* stk, Trav& t)
{
    if (t.lvl == 0) return true;   // `branch_lvl == 0u` -> return false (miss)
    const uint32_t d = heap_depth(t.lvl);
    t.lvl ^= 1u << d;
    t.node = (t.node >> (heap_depth(t.node) - d - 1u)) ^ 1u;
    t.tmin = t.tmax;       // = the entry's t (see above)
    t.tmax = stk[d * 256u];
    return false;
}


// One interior-node decision of bsp.wgsl:54-78 at node m (data n, depth dep).
// Returns the next node.  Branch-free except for the exact division, which
// only lanes whose approximate t cannot decide near/far take.  The push
// stores the current tmax into the depth-dep slot unconditionally: no pending
// entry lives at a depth >= depth(m) (they are all ancestors of m), so the
// store is dead unless the trail bit is set.
// The walk derives the trail slot of its first level once per trip and the next
// levels' slots as constant offsets from it (ds_write immediate offsets; `stk` is
// this level's slot), and sets the trail bit with one shift-or.  Every decision
// divides out the exact t (the wave runs the exact path in nearly every trip
// anyway: 28 % of decisions need it), with no approximate test first.
// chk (wave-uniform, k_path's per-check choice): some lane's ray, or the scene's planes
// (rt_bsp_build.hip k_plane_range), may put x outside the range where rt_div_by_recip
// is exact.  Without it every x is 0 or inside the range (x = +-0 gives a zero, whose
// sign may differ from x / denom's for -0: t values are only compared, and every
// comparison sees +0 == -0, tests/native/fastdiv_check.c), so the per-lane test and its
// fallback branch are skipped: a scalar
// branch instead of three VALU and about five scalar instructions per decision, and
// scalar issue costs the trip as much as vector issue does (profiles/r06/ab_chk.txt;
// two instantiations of the whole trip group instead, one per value, ran 5 % slower:
// twice the code and more spills)
template <bool COUNT>
__device__ __forceinline__ uint32_t bsp_decide(float* stk, const uint2 n, uint32_t m, uint32_t dep, const f3 o,
                                               const f3 d, const f3 inv, Trav& t, Counters& c, float lo, float& hi,
                                               uint32_t chk = 1u)
{
    if (COUNT) c.v[C_INTERIOR]++;
    const uint32_t axis = n.x & 3u;
    const float ao = comp(o, axis), iv = comp(inv, axis);
    const uint32_t near_node = 2u * m + (__float_as_uint(iv) >> 31);   // see bsp_inv1
    const float x = __uint_as_float(n.y) - ao;
#ifndef RT_DBG_VERT
    if (COUNT) c.v[C_EXACT_NODES]++;
#endif
    const float ad = comp(d, axis);
    const float denom = rt_absf(ad) < 1.0e-8f ? 1.0e-8f : ad;
    // RN(x / denom) from the per-ray RN(1/denom) (include/rt_detmath.h); the IEEE
    // division outside its operand range or for a NaN-flagged axis
    float tt = rt_div_by_recip(x, denom, iv);
    if (chk != 0u) {
        if (!(rt_div_by_recip_ok(x) & (iv == iv))) {
            asm volatile("");   // keep the rare IEEE division behind its branch (no if-conversion)
            tt = x / denom;
        }
    }
    // against [lo, hi]: the ray interval, clipped to the treelet root's content
    // box (bsp_box_miss); a plane beyond it leaves one side hitless
    const bool cnear = tt > hi;
    const bool gofar = (!cnear) & (tt < lo);
    const bool push = (!cnear) & !(tt < lo);
    stk[0] = t.tmax;   // the tmax its pop restores
    t.lvl |= (uint32_t)push << dep;
    t.tmax = push ? tt : t.tmax;
    hi = push ? tt : hi;
    return gofar ? near_node ^ 1u : near_node;
}

// One trip of a lane through intersect_trimesh (bsp.wgsl:10-81).  Every lane
// issues the same five 16-B loads at one base offset, before any decision
// (one memory round trip per trip):
//   * a lane inside a leaf tests its 48-B record (and the next one, below);
//   * a lane walking nodes reads the 96-B treelet of its node m
//     (rt_bsp_build.hip k_bsp_repack: m's content box | nodes m | 2m, 2m+1 |
//     4m..4m+3), tests the content box (bsp_walk) and walks up to three
//     levels with no further load.
// Treelets and records share one buffer resource (out-of-range reads are 0).
// A walk that reaches a leaf starts its triangle range (tested from the next
// trip on); an empty leaf, or a leaf tested without a hit, pops.  Leaf ranges
// (leaf_k, leaf_end, hit_k) are byte offsets of records in that buffer.
// A second triangle test of a leaf in the same trip (BSP walk).  A leaf
// lane's trip loads 96 B at its record (the treelet size): the 48-B record it
// tests and the whole next one (`nx`, `r1`, `r2`; records of a leaf are 48 B
// apart).  The next record is tested in order, after the first one's accept
// has narrowed tmax, exactly as one test per trip would.  A walk that stops at
// its first hit (anyhit) stops here too.
// Two tests per trip take the per-trip costs (the check, the walking half of
// the wave, the pop) off the leaf work: config 3 +2.9 %, config 4 +12 %,
// config 5 (32-triangle leaves) +20 % (profiles/r02/ab_lt2.txt); three or more
// per trip, or the same for the BVH walk (leaves of at most 4), were slower
// (ab_lt.txt).  (With 80-B treelets the second record's last 16 B took one
// more round trip; loading them with the trip's loads was no faster then,
// profiles/r03/ab_pre_c*.txt.  The 96-B treelets of the certified culling load
// them anyway.)
template <bool COUNT, bool CULL, class LOG, bool VERT = false>
__device__ __forceinline__ void leaf_test_next(const __amdgpu_buffer_rsrc_t rs, const v4u nx, const v4u r1, const v4u q5,
                                               const f3 o, const f3 d, bool anyhit, Trav& t, Counters& c, LOG& lg,
                                               bool vert)
{
    if ((t.leaf_k != t.leaf_end) & !(anyhit & t.found)) {
        // the trip's 96-B load holds this whole record (nx, r1, r2 = q5)
        const v4u r2 = q5;
        lg.tested(t.leaf_k);
        if (COUNT) {
            c.v[C_IDS]++;
            c.v[C_TESTS]++;
        }
        float dist, beta, gamma;
        if (tri_math<true, COUNT, CULL, false, VERT>(as_f4(nx), as_f4(r1), as_f4(r2), o, d, t.tmin, t.tmax, dist,
                                                             beta, gamma, &c, vert)) {
            if (COUNT) c.v[C_ACCEPTS]++;
            t.tmax = dist;
            t.found = true;
            // an any-hit walk keeps the hit it started from (k_path redraws from
            // it); selects, not a branch (no exec-mask work in the trip)
            t.hit_k = anyhit ? t.hit_k : t.leaf_k;
        }
        t.leaf_k += 48u;
    }
}

// The leaf half of a BSP trip: test the record in q0..q2 and the next one,
// whose 48 B are q3..q5.
template <bool COUNT, bool CULL, class LOG, bool VERT = false>
__device__ __forceinline__ void bsp_leaf_tests(const __amdgpu_buffer_rsrc_t rs, const v4u q0, const v4u q1, const v4u q2,
                                               const v4u q3, const v4u q4, const v4u q5, const f3 o, const f3 d, bool anyhit, Trav& t,
                                               Counters& c, bool& done, bool& pop, LOG& lg, bool vert = false)
{
    lg.tested(t.leaf_k);
    if (COUNT) {
        c.v[C_IDS]++;
        c.v[C_TESTS]++;
    }
    float dist, beta, gamma;
    if (tri_math<true, COUNT, CULL, false, VERT>(as_f4(q0), as_f4(q1), as_f4(q2), o, d, t.tmin, t.tmax, dist, beta,
                                                         gamma, &c, vert)) {
        if (COUNT) c.v[C_ACCEPTS]++;
        t.tmax = dist;
        t.found = true;
        t.hit_k = anyhit ? t.hit_k : t.leaf_k;
    }
    t.leaf_k += 48u;
    leaf_test_next<COUNT, CULL, LOG, VERT>(rs, q3, q4, q5, o, d, anyhit, t, c, lg, vert);
    const bool leaf_done = (t.leaf_k == t.leaf_end) | (anyhit & t.found);
    done = leaf_done & t.found;   // a leaf with an accepted triangle ends the walk
    pop = leaf_done & !t.found;
}

// Subtree culling (RT_OPT_BSP_CULL, DESIGN.md section 4 "Subtree culling"): a
// trip that starts at node M first tests the ray interval [tmin, tmax] against
// M's content box -- the union of the bounding boxes of the triangles M's
// leaves reference -- grown by a margin m.  If the interval misses it by a
// clear gap, no triangle of the subtree can be accepted inside the interval,
// so the reference's walk of that subtree (bsp.wgsl:10-81: every leaf tested
// without a hit, every pending entry pushed inside it popped again) ends where
// the next pop starts: the walk pops at once.  Which triangle is hit, and
// where, does not change; only hitless work is skipped.
// The margin (DESIGN.md section 4 "Certified culling"):
//   m = D1 * (k1 * w1 / max(F, 2 Dlb - 20u w1) + k3) + max(|o|inf * ko, dscene)
// with D1 >= |v0 - o|_1 for every point v0 of the box, w1 = |w|_1, F = 1e-10 /
// E2 and 2 Dlb a lower bound of |w . n*| / E2 over the subtree's normals from
// the treelet's normal box (q5: centre and radius of n* / E2); for a camera ray
// also G |w|inf, G precomputed per treelet from how far the eye is from its
// triangles' planes (q5.x's high half, k_treelet_hcam).  Certified mode (k1 = 36u, k3 = 2u, ko and
// dscene 2^-19 of the magnitudes): m bounds the L-inf distance from the box of
// every point o + dist*w where intersect_triangle (w7e3.wgsl:286-332) can
// accept one of the subtree's triangles -- its f32 rounding, including
// |denom| >= 1e-10 at grazing angles -- so the cull is exact for every ray.
// Fast mode (k1 = k3 = 0, ko and dscene 2^-10): the round-3 margin, not a bound.
// Axes whose direction component is below the shader's 1e-8 cut (bsp_inv1):
//  * exactly zero (+-0; inv is +1e8 = RN(1/1e-8)): every point o + dist*w of the
//    ray has that coordinate o_a exactly, so the slab is a yes/no test of o_a
//    against the grown box -- inv * inf makes its products +-inf (o_a outside:
//    both ends of the slab at +inf or at -inf, the interval is empty; inside:
//    -inf..+inf, no constraint).  An infinite end culls against the gap
//    tolerance's cap S.bsp_cull_emax (FLT_MAX; +inf with culling off).  W9E1's
//    shadow rays (0, 1, 0) (w9e1.wgsl:442-446) are the common case.  On the grown
//    box's face itself (RN(dl - m) == 0 or RN(dh + m) == 0) that end's product is
//    0 x inf = NaN, fminf / fmaxf take the other end (+-inf) and the subtree is
//    culled: the closed face counts as outside, and so may o_a within the two
//    roundings of dl - m (a few ulps of the coordinates) inside it.  That is exact
//    because the certified margin carries slack beyond its bound: its 2u D1 and
//    2^-19 max(|o|inf, scene) terms exceed the proven L-inf distance of any
//    accepted hit point from its triangle's box by far more than those ulps, so no
//    point within them of the grown face can be an accept.  (The fast margin is
//    not a bound either way.);
//  * nonzero, |w_a| <= 1e-8 (inv is the NaN flag): constrains nothing, the NaN
//    drops out of fminf / fmaxf.
// The trip's decisions also use the interval clipped to the box (bsp_walk;
// DESIGN.md section 4 "Subtree culling").
// The gap factor `gap` is DevScene.bsp_cull_gap: 2^-18, or +inf with culling
// off (no gap exceeds an infinite threshold; 0 x inf = NaN compares false).
// Off is data, not a branch on a uniform flag: a uniform bool kept as a lane
// mask across the walk loops was reused under a wider exec mask by the
// compiler (k_direct's shadow walk culled in the lanes that had been inactive
// where the mask was computed; tests/test_gpu_cull.py caught it).  The mode
// is data for the same reason (DevScene cull_k1 / cull_k3 / cull_ko).
__device__ __forceinline__ float h2f(uint32_t bits) { return (float)__builtin_bit_cast(_Float16, (uint16_t)bits); }
// CM 0: the fast margin's formula alone, m = max(|o|inf ko, dscene), for a
// context whose culling is not certified (the host picks k_path's
// instantiation, so the fast and off modes do not pay for the certified terms;
// off keeps the +inf gap factor either way).  The generic (CM 1) form
// evaluates every mode from its data constants.
// CM: the margin formula -- 0 the fast margin's alone, 1 certified (the generic
// form every mode's data evaluates), 2 certified with the silhouette bound of
// camera rays (RT_BSP_CULL_SILHOUETTE, q6 = the node's DevScene.bsp_sil entry)
template <int CM = 1>
__device__ __forceinline__ bool bsp_box_miss(const DevScene& S, const v4u q0, const v4u q1, const v4u q5, const v4u q6,
                                             const f3 o, const f3 w, const f3 inv, float tmin, float tmax, float& lo,
                                             float& hi)
{
    constexpr bool FULL = CM >= 1;
    const float oo[3] = {o.x, o.y, o.z}, iv[3] = {inv.x, inv.y, inv.z};
    // vectors from the origin to the box's faces; D1 bounds |v0 - o|_1 over the box
    float dl[3], dh[3], D1 = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        dl[a] = __uint_as_float(a == 0 ? q0.x : (a == 1 ? q0.y : q0.z)) - oo[a];
        dh[a] = __uint_as_float(a == 0 ? q0.w : (a == 1 ? q1.x : q1.y)) - oo[a];
        if (FULL) D1 += __builtin_fmaxf(rt_absf(dl[a]), rt_absf(dh[a]));
    }
    const float mo = __builtin_fmaxf(__builtin_fmaxf(rt_absf(o.x), rt_absf(o.y)), rt_absf(o.z));
    float m = __builtin_fmaxf(mo * S.cull_ko, S.bsp_margin);
    if constexpr (FULL) {
        // (the compiler keeps w1's products and the origin term in registers across
        // the trip loop; recomputing them every trip, through an opaque asm, was
        // 2.5 % slower: profiles/r04/ab_opq.txt)
        const float w1 = rt_absf(w.x) + rt_absf(w.y) + rt_absf(w.z);
        // |w . n*| / E2 >= 2 Dlb over the normal box, stored as centre c and
        // radius r (f16): the box's minimum of |w . x| is |w . c| - |w| . r
        // (fused multiply-adds of f16 and f32 operands: v_fma_mix_f32)
        // (the first terms as fma(x, y, 0): one v_fma_mix_f32 each, no conversion; only
        // the sign of a zero product can differ, and |w . c| and |w| . r do not see it)
        const float wc = __builtin_fmaf(w.z, h2f(q5.z & 0xFFFFu),
                                        __builtin_fmaf(w.y, h2f(q5.y >> 16), __builtin_fmaf(w.x, h2f(q5.y & 0xFFFFu), 0.0f)));
        const float wr = __builtin_fmaf(rt_absf(w.z), h2f(q5.w >> 16),
                                        __builtin_fmaf(rt_absf(w.y), h2f(q5.w & 0xFFFFu),
                                                       __builtin_fmaf(rt_absf(w.x), h2f(q5.z >> 16), 0.0f)));
        const float dlb2 = rt_absf(wc) - wr;
        float den = __uint_as_float(q5.x << 16);
        den = __builtin_fmaxf(den, dlb2 - (20.0f * 0x1p-24f) * w1);
        // a camera ray (its origin is the eye the treelets' camera terms are for):
        // |denom| / E_T^2 >= G |w|inf, G (f16) precomputed per treelet for the eye
        // (k_treelet_hcam; DESIGN.md section 4 "Certified culling", the camera bound)
        const bool cam = (o.x == S.cam_eye[0]) & (o.y == S.cam_eye[1]) & (o.z == S.cam_eye[2]);
        const float winf = __builtin_fmaxf(__builtin_fmaxf(rt_absf(w.x), rt_absf(w.y)), rt_absf(w.z));
        const float dcam = __builtin_fmaf(winf, h2f(q5.x >> 16), 0.0f);   // G: f16 in the high half
        float dc = dcam;
        if constexpr (CM == 2) {
            // RT_BSP_CULL_SILHOUETTE: the subtree's two triangles of smallest camera
            // term are bounded per ray by their own normals x = n*/E_t^2 (f16, q6; NaN
            // slots drop out of the minimum), the rest by G_x (q6.w): |denom| / E_t^2
            // >= min(|w . x| - 2^-9 |w|1, G_x |w|inf) (k_treelet_hcam)
            const float x0 = __builtin_fmaf(w.z, h2f(q6.y & 0xFFFFu), __builtin_fmaf(w.y, h2f(q6.x >> 16),
                                                                                     __builtin_fmaf(w.x, h2f(q6.x & 0xFFFFu), 0.0f)));
            const float x1 = __builtin_fmaf(w.z, h2f(q6.z >> 16), __builtin_fmaf(w.y, h2f(q6.z & 0xFFFFu),
                                                                                __builtin_fmaf(w.x, h2f(q6.y >> 16), 0.0f)));
            const float dx = __builtin_fmaf(-0x1p-9f, w1, __builtin_fminf(rt_absf(x0), rt_absf(x1)));
            dc = __builtin_fmaxf(dcam, __builtin_fminf(dx, __builtin_fmaf(winf, h2f(q6.w & 0xFFFFu), 0.0f)));
        }
        den = __builtin_fmaxf(den, cam ? dc : 0.0f);
        // (fused: fewer roundings than the proof's constants allow for)
        m = __builtin_fmaf(D1, __builtin_fmaf(S.cull_k1 * w1, __builtin_amdgcn_rcpf(den), S.cull_k3), m);
    }
    float mn[3], mx[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float ib = rt_absf(iv[a]) < 1e8f ? iv[a] : iv[a] * __builtin_inff();   // +1e8: a zero component
        const float t1 = (dl[a] - m) * ib, t2 = (dh[a] + m) * ib;
        mn[a] = __builtin_fminf(t1, t2);
        mx[a] = __builtin_fmaxf(t1, t2);
    }
    // max(tmin, mn...) / min(tmax, mx...) in the order fmaxf / fminf would take
    // them (qmax: no canonicalising instruction for the loop-carried tmin / tmax)
    const float tn = qmax(qmax3(tmin, mn[0], mn[1]), mn[2]);
    const float tf = qmin(qmin3(tmax, mx[0], mx[1]), mx[2]);
    // a clear gap: the rounding of the slab products cannot close it
    // (capped: an infinite slab end from a zero direction component must still
    // show a gap; a finite product cannot reach the cap)
    const float e = qmin_s(S.bsp_cull_emax, (rt_absf(tn) + rt_absf(tf)) * S.bsp_cull_gap);
    // the interval the subtree's content can be hit in, widened by the same
    // tolerance (culling off: e = inf or NaN, lo = tmin, hi = tmax)
    lo = qmax(tmin, tn - e);
    hi = qmin(tmax, tf + e);
    // an empty subtree's content box is +inf / -inf (its slabs are NaN, never a
    // gap): culled outright, except with culling off (e = inf or NaN)
    return (tn - tf > e) | (__uint_as_float(q0.x) - __uint_as_float(q0.w) > e);
}

// The walking half of a BSP trip: node m (level 0), a child (level 1), a
// grandchild (level 2) from the 96-B treelet in q0..q5 (rt_internal.h:
// {box | box, node M | 2M, 2M+1 | 4M, 4M+1 | 4M+2, 4M+3 | certification data}).  Returns true when
// the walk reached a non-empty leaf (its range is set, its tests start next
// trip); an empty leaf, or a subtree culled by its content box, sets pop.
// (Testing the first record of a leaf in the trip that reaches it -- one more
// round trip -- was slower: config 4 -3.7 %, config 5 -11 %, profiles/r02/ab_et1.txt.)
template <bool COUNT, int CM = 1>
__device__ __forceinline__ bool bsp_walk(const DevScene& S, float* stk, const v4u q0, const v4u q1, const v4u q2,
                                         const v4u q3, const v4u q4, const v4u q5, const v4u q6, const f3 o, const f3 d,
                                         const f3 inv, Trav& t, Counters& c, bool& pop, uint32_t chk = 1u)
{
    uint32_t m = t.node;
    float lo = t.tmin, hi = t.tmax;   // the decisions' interval: [tmin, tmax] clipped to the box
    float blo, bhi;
    if (bsp_box_miss<CM>(S, q0, q1, q5, q6, o, d, inv, t.tmin, t.tmax, blo, bhi)) {
        if (COUNT) c.v[C_CULLS]++;
        pop = true;
        return false;
    }
    lo = blo;
    hi = bhi;
    const uint32_t dep = heap_depth(m);
    uint2 n = make_uint2(q1.z, q1.w);
    bool leaf = (n.x & 3u) == 3u;
    if (!leaf) {
        // the trail slot of this level
        float* const s0 = stk + dep * 256u;
        m = bsp_decide<COUNT>(s0, n, m, dep, o, d, inv, t, c, lo, hi, chk);
        n = (m & 1u) ? make_uint2(q2.z, q2.w) : make_uint2(q2.x, q2.y);
        leaf = (n.x & 3u) == 3u;
        if (!leaf) {
            m = bsp_decide<COUNT>(s0 + 256, n, m, dep + 1u, o, d, inv, t, c, lo, hi, chk);
            const v4u g = (m & 2u) ? q4 : q3;
            n = (m & 1u) ? make_uint2(g.z, g.w) : make_uint2(g.x, g.y);
            leaf = (n.x & 3u) == 3u;
            if (!leaf) m = bsp_decide<COUNT>(s0 + 512, n, m, dep + 2u, o, d, inv, t, c, lo, hi, chk);
        }
    }
    t.node = m;
    if (leaf) {
        if (COUNT) c.v[C_LEAF]++;
        t.leaf_k = n.y;
        t.leaf_end = n.y + (n.x >> 2);   // 48 * count
        pop = (n.x >> 2) == 0u;
    }
    return leaf & !pop;
}

template <bool COUNT, bool CULL, class LOG, int CM = 1, bool VSH = false>
__device__ __forceinline__ bool bsp_step_log(const DevScene& S, float* stk, const f3 o, const f3 d, const f3 inv,
                                             bool anyhit, Trav& t, Counters& c, LOG& lg, uint32_t chk = 1u)
{
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)S.bsp_nodes, (short)0, (int)S.bsp_bytes, 0x00020000);
    const bool in_leaf = t.leaf_k != t.leaf_end;
    // a leaf lane: its next 96 B of records (two whole records); a walking
    // lane: the 96-B treelet of its node
    static_assert(BSP_TREELET_BYTES == 96, "times96");
    const uint32_t base = in_leaf ? t.leaf_k : times96(t.node);
    uint64_t tw = COUNT ? __builtin_amdgcn_s_memtime() : 0;
    v4u q0 = __builtin_amdgcn_raw_buffer_load_b128(rs, base, 0, 0);
    v4u q1 = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16u, 0, 0);
    v4u q2 = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 32u, 0, 0);
    v4u q3 = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 48u, 0, 0);
    v4u q4 = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 64u, 0, 0);
    v4u q5 = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 80u, 0, 0);
    // (RT_BSP_CULL_SILHOUETTE: a seventh, the node's silhouette data, from its own
    // array; a leaf lane's is unused)
    v4u q6 = {0u, 0u, 0u, 0u};
    // keep the loads together (the compiler would sink the later ones
    // into the level-2 branch: a second round trip)
    if constexpr (CM == 2) {
        const __amdgpu_buffer_rsrc_t rs6 = __builtin_amdgcn_make_buffer_rsrc(
            (void*)S.bsp_sil, (short)0, (int)((S.bsp_bytes / BSP_TREELET_BYTES) * 16u), 0x00020000);
        // only a walking camera ray uses it: every other lane's offset lies past the
        // array, so its load returns zeros without a memory access (zeros give
        // dc = dcam, and a non-camera ray ignores dc) -- the secondary rays of a
        // large scene do not stream the array
        const bool cam = (o.x == S.cam_eye[0]) & (o.y == S.cam_eye[1]) & (o.z == S.cam_eye[2]);
        const uint32_t off6 = (!in_leaf & cam) ? t.node * 16u : 0x80000000u;
        q6 = __builtin_amdgcn_raw_buffer_load_b128(rs6, off6, 0, 0);
        asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6));
    } else {
        asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5));
    }
    if (COUNT) {   // diagnostics: cycles from issuing the loads to their data
        tw = __builtin_amdgcn_s_memtime() - tw;
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x & 63u))
            c.v[C_MEMWAIT_CYC64] += (uint32_t)(tw >> 6);
    }
    bool done = false, pop = false;
    if (in_leaf) {
        // VSH (W9E1): every any-hit ray is a shadow ray of direction (0, 1, 0).  When
        // all of the wave's leaf lanes hold one, the wave takes the tests' VERT form
        // (a uniform branch on a ballot of the any-hit flag; a ballot taken once per
        // check instead, outside the trips, measured slower: profiles/r06/ab_vsh.txt)
        bsp_leaf_tests<COUNT, CULL, LOG, VSH>(rs, q0, q1, q2, q3, q4, q5, o, d, anyhit, t, c, done, pop, lg,
                                              VSH && __ballot(!anyhit) == 0);
    }
    else bsp_walk<COUNT, CM>(S, stk, q0, q1, q2, q3, q4, q5, q6, o, d, inv, t, c, pop, chk);
    if (pop) done = bsp_pop(stk, t);
    return done;
}
template <bool COUNT, bool CULL = false, int CM = 1, bool VSH = false>
__device__ __forceinline__ bool bsp_step(const DevScene& S, float* stk, const f3 o, const f3 d, const f3 inv,
                                         bool anyhit, Trav& t, Counters& c, uint32_t chk = 1u)
{
    NoLog lg;
    return bsp_step_log<COUNT, CULL, NoLog, CM, VSH>(S, stk, o, d, inv, anyhit, t, c, lg, chk);
}

// RN(1/denom) per axis (denom as bsp.wgsl:63): the approximate interior-node
// test multiplies by it, and the exact t is derived from it (rt_div_by_recip).
// Its sign bit also carries the near-child choice (`dir[axis] >= 0` -> left,
// bsp.wgsl:54-60): the two disagree only when dir[axis] is a negative value
// of magnitude < 1e-8 (denom is +1e-8 there) or NaN; those components get a
// negative NaN, which sends every decision on that axis to the exact path
// (NaN compares false) with the right near child.
// +1e8 marks an exactly zero component for the subtree cull (bsp_box_miss): every
// other component of magnitude <= 1e-8 (whose reciprocal would also be +-1e8)
// gets the NaN flag with its near child in the sign bit; the exact path divides
// by the same denominator, so its decisions do not change.
__device__ __forceinline__ float bsp_inv1(float ad)
{
    const float r = 1.0f / (rt_absf(ad) < 1.0e-8f ? 1.0e-8f : ad);   // RN(1/denom): rt_div_by_recip's reciprocal
    const bool near_right = !(ad >= 0.0f);
    const bool tiny = (rt_absf(ad) <= 1.0e-8f) & (ad != 0.0f);
    return ((near_right && !(__float_as_uint(r) >> 31)) || tiny)
               ? __uint_as_float(near_right ? 0xFFC00000u : 0x7FC00000u)
               : r;
}
__device__ __forceinline__ f3 bsp_inv(const f3 d) { return V(bsp_inv1(d.x), bsp_inv1(d.y), bsp_inv1(d.z)); }

// ------------------------------------------------------------------ BVH traversal
// intersect_bvh + intersect_bb2, bvh.wgsl:154-191 / 16-83: slab test in axis
// order y, x, z on [0, 1e27] (ray interval ignored), right child popped first,
// 1000-pop cap, WGSL index clamping of the 50-entry stack.  One pop per call.
// The same predicate without control flow: the swaps and bound updates are
// selects with the shader's comparisons (NaN compares false, as its ifs do).
// The early `return false` after an axis needs no flag: t0 only grows and t1
// only shrinks (neither can become NaN), so t0 > t1 once means t0 > t1 at the end.
__device__ __forceinline__ void bb2_axis(float tn, float tf, float& t0, float& t1)
{
    const bool sw = tn > tf;
    const float lo = sw ? tf : tn, hi = sw ? tn : tf;
    t0 = lo > t0 ? lo : t0;
    t1 = hi < t1 ? hi : t1;
}
__device__ __forceinline__ bool bb2(const f3 inv, const f3 o, const float4 a, const float4 b)
{
    float t0 = 0.0f, t1 = 1e27f;
    const f3 nr = mul(sub(V(a.x, a.y, a.z), o), inv);
    const f3 fr = mul(sub(V(b.x, b.y, b.z), o), inv);
    bb2_axis(nr.y, fr.y, t0, t1);
    bb2_axis(nr.x, fr.x, t0, t1);
    bb2_axis(nr.z, fr.z, t0, t1);
    return !(t0 > t1);
}

// BVH stack split: entries [0, K) in LDS ([slot][thread], 4 B), entries [K, 50)
// in a per-lane global region ([slot - K][lane] across the grid) -- a walk
// deeper than K is rare, and the LDS share drops from 50 to K entries, which
// lets the BVH kernels run 8 waves/SIMD like the BSP ones.
#ifndef RT_BVH_LDS_ENTRIES
#define RT_BVH_LDS_ENTRIES 16
#endif
struct BvhDeep {
    uint32_t* p;        // this lane's first deep entry (entry j at p[j * stride])
    uint32_t stride;    // lanes in the grid
};
__device__ __forceinline__ void bvh_st(uint32_t* stk, const BvhDeep& dp, uint32_t i, uint32_t v)
{
    if (i < RT_BVH_LDS_ENTRIES) stk[i * 256u + lane_v()] = v;
    else dp.p[(size_t)(i - RT_BVH_LDS_ENTRIES) * dp.stride] = v;
}
__device__ __forceinline__ uint32_t bvh_ld(const uint32_t* stk, const BvhDeep& dp, uint32_t i)
{
    return i < RT_BVH_LDS_ENTRIES ? stk[i * 256u + lane_v()] : dp.p[(size_t)(i - RT_BVH_LDS_ENTRIES) * dp.stride];
}

__device__ __forceinline__ void bvh_init(Trav& t, float tmin, float tmax)
{
    trav_init(t, tmin, tmax);
    t.node = 1;     // top: stack_push_node(0u)
    t.lvl = 0;      // pops
    t.tos = 0u;     // the root's byte offset, cached top of stack
    t.tos2 = 0u;    // second entry (none yet: its speculative load reads the root again)
}

// Stack slot of entry i under WGSL index clamping (bvh.wgsl:134-137: node_stack[50]).
__device__ __forceinline__ uint32_t bvh_slot(uint32_t i) { return i < 50u ? i : 49u; }

// One trip of a lane through intersect_bvh (bvh.wgsl:154-191), one memory
// round trip: a lane inside a leaf tests one triangle (its 48-B record), a
// lane between leaves pops one node (32-B record) and slab-tests it.  The
// stack holds node byte offsets in LDS ([slot][thread], slot = min(i, 49):
// WGSL index clamping) with its top value cached in a register (t.tos), so a
// pop needs no LDS read before the node load; the next top is read from LDS
// for the following trip.  Device node records (rt_api.cpp rt_upload_bvh):
// {min.xyz, w0}{max.xyz, w1}, interior w0 = byte offset of the right child
// (the left child is the next record), w1 = 0; leaf w0 = byte offset of its
// first triangle record, w1 = 48 * n_prims.
template <bool COUNT, bool CULL, class LOG>
__device__ __forceinline__ bool bvh_step_log(const DevScene& S, uint32_t* stk, const BvhDeep& dp, const f3 o,
                                             const f3 d, const f3 inv, bool anyhit, Trav& t, Counters& c, LOG& lg)
{
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)S.bvh_base, (short)0, (int)S.bvh_bytes, 0x00020000);
    const bool in_leaf = t.leaf_k != t.leaf_end;
    // a walking lane loads the records of the top two stack entries: when the
    // first misses, the second is the next pop and is handled in the same trip
    const uint32_t base = in_leaf ? t.leaf_k : t.tos;
    const uint32_t base2 = in_leaf ? t.leaf_k + 32u : t.tos2;
    v4u q0 = __builtin_amdgcn_raw_buffer_load_b128(rs, base, 0, 0);
    v4u q1 = __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16u, 0, 0);
    v4u q2 = __builtin_amdgcn_raw_buffer_load_b128(rs, base2, 0, 0);
    v4u q3 = __builtin_amdgcn_raw_buffer_load_b128(rs, base2 + 16u, 0, 0);
    asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3));
    if (in_leaf) {
        lg.tested(t.leaf_k);
        if (COUNT) {
            c.v[C_IDS]++;
            c.v[C_TESTS]++;
        }
        float dist, beta, gamma;
        // the BVH walk never narrows the ray interval: both bounds are exact
        if (tri_math<true, COUNT, CULL, false>(as_f4(q0), as_f4(q1), as_f4(q2), o, d, t.tmin, t.tmax, dist,
                                                       beta, gamma, &c)) {
            if (COUNT) c.v[C_ACCEPTS]++;
            t.tmax = dist;
            t.found = true;
            // an any-hit walk keeps the hit it started from (k_path redraws from
            // it); selects, not a branch (no exec-mask work in the trip)
            t.hit_k = anyhit ? t.hit_k : t.leaf_k;
        }
        t.leaf_k += 48u;
        if (anyhit & t.found) return true;
    } else {
        // Stack invariant: tos = entry node-1, tos2 = entry node-2 (clamped
        // slots), so both reads the reference does after a push are exact.
        // Box tests have no side effect (the slab test ignores the ray
        // interval), so testing the second entry early changes nothing; it is
        // only acted on when it is the reference's next pop (the first missed)
        // and the 1000-pop cap still allows that pop.
        if (COUNT) c.v[C_POPS]++;
        t.lvl++;
        t.node--;
        uint32_t top = t.tos;
        bool hit = bb2(inv, o, as_f4(q0), as_f4(q1));
        uint32_t w0 = q0.w, w1 = q1.w;
        bool reload = false;   // the new top must come from the stack
        if (!hit & (t.node != 0u) & (t.lvl < 1000u)) {
            if (COUNT) c.v[C_POPS]++;
            t.lvl++;
            t.node--;
            top = t.tos2;
            hit = bb2(inv, o, as_f4(q2), as_f4(q3));
            w0 = q2.w;
            w1 = q3.w;
            reload = true;
        }
        if (hit & (w1 != 0u)) {   // leaf: its triangles from the next trip on
            t.leaf_k = w0;
            t.leaf_end = w0 + w1;
        }
        if (hit & (w1 == 0u)) {   // interior: push left (top + 1), then right
            const uint32_t n = t.node;
            bvh_st(stk, dp, bvh_slot(n), top + 32u);
            bvh_st(stk, dp, bvh_slot(n + 1u), w0);
            t.node = n + 2u;
            t.tos = w0;
            t.tos2 = n >= 49u ? w0 : top + 32u;   // both pushes land in slot 49 from n = 49 on
        } else {
            if (t.node != 0u) t.tos = reload ? bvh_ld(stk, dp, bvh_slot(t.node - 1u)) : t.tos2;
            if (t.node >= 2u) t.tos2 = bvh_ld(stk, dp, bvh_slot(t.node - 2u));
        }
    }
    return (t.leaf_k == t.leaf_end) & ((t.lvl >= 1000u) | (t.node == 0u));
}
template <bool COUNT, bool CULL = false>
__device__ __forceinline__ bool bvh_step(const DevScene& S, uint32_t* stk, const BvhDeep& dp, const f3 o, const f3 d,
                                         const f3 inv, bool anyhit, Trav& t, Counters& c)
{
    NoLog lg;
    return bvh_step_log<COUNT, CULL>(S, stk, dp, o, d, inv, anyhit, t, c, lg);
}

// The 1/d of bvh.wgsl:155 (exact division: it feeds the slab test directly).
__device__ __forceinline__ f3 bvh_inv(const f3 d) { return V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); }

template <int TRAV>
__device__ __forceinline__ f3 trav_inv(const f3 d)
{
    return TRAV == RT_TRAVERSE_BVH ? bvh_inv(d) : bsp_inv(d);
}
template <int TRAV>
__device__ __forceinline__ void trav_start(Trav& t, void* stk, float tmin, float tmax)
{
    if (TRAV == RT_TRAVERSE_BVH) bvh_init(t, tmin, tmax);
    else trav_init(t, tmin, tmax);
}
template <int TRAV, bool COUNT, bool CULL = false, int CM = 1, bool VSH = false>
__device__ __forceinline__ bool trav_step(const DevScene& S, void* stk, const BvhDeep& dp, const f3 o, const f3 d,
                                          const f3 inv, bool anyhit, Trav& t, Counters& c, uint32_t chk = 1u)
{
    if (TRAV == RT_TRAVERSE_BVH)
        return bvh_step<COUNT, CULL>(S, reinterpret_cast<uint32_t*>(stk), dp, o, d, inv, anyhit, t, c);
    return bsp_step<COUNT, CULL, CM, VSH>(S, reinterpret_cast<float*>(stk), o, d, inv, anyhit, t, c, chk);
}

// Whole traversal of one ray (used by the primary-ray kernel).
template <int TRAV, bool COUNT>
__device__ __forceinline__ bool trace(const DevScene& S, void* stk, const BvhDeep& dp, const f3 o, const f3 d,
                                      float tmin, float tmax, bool anyhit, TraceOut& out, Counters& c)
{
    Trav t;
    t.hit_k = 0;   // an any-hit walk leaves the hit record alone
    t.beta = t.gamma = 0.0f;
    trav_start<TRAV>(t, stk, tmin, tmax);
    const f3 inv = trav_inv<TRAV>(d);
    for (uint32_t guard = 0; guard < (1u << 24); guard++)
        if (trav_step<TRAV, COUNT>(S, stk, dp, o, d, inv, anyhit, t, c)) break;
    if (t.found && !anyhit) bary_of<TRAV>(S, t.hit_k, o, d, t.beta, t.gamma);
    out = trav_out(t);
    return t.found;
}

// Hit record of the accepted triangle (the values intersect_triangle_indexed
// writes on its last accept): tri id, position, interpolated normal, material.
struct HitRec {
    uint32_t tri, material;
    f3 pos, nrm;
};
// ETA_W: w9e3.wgsl:343 adds ETA (1e-4) to each interpolation weight
template <int TRAV, bool ETA_W = false>
__device__ __forceinline__ HitRec resolve(const DevScene& S, const TraceOut& t, const f3 o, const f3 d,
                                          bool face_normals)
{
    HitRec h;
    // t.k is the record's byte offset in the node+record buffer of the traversal
    const uint8_t* base = TRAV == RT_TRAVERSE_BVH ? S.bvh_base : reinterpret_cast<const uint8_t*>(S.bsp_nodes);
    const uint32_t slot = (t.k - (TRAV == RT_TRAVERSE_BVH ? S.bvh_rec_off : S.bsp_rec_off)) / 48u;
    const float4* r2p = reinterpret_cast<const float4*>(base + t.k + 32u);
    uint4 ix;
    if (TRAV == RT_TRAVERSE_BSP) {
        // {triangle id, material} of the slot in one load (DevScene.bsp_tm); the
        // vertex indices only where vertex normals are interpolated
        const uint2 tm = S.bsp_tm[slot];
        h.tri = tm.x;
        ix.w = tm.y;
        if (!face_normals) ix = S.tri_idx[h.tri];
    } else {
        h.tri = S.bvh_ids[slot];
        ix = S.tri_idx[h.tri];
    }
    h.pos = add(o, muls(d, t.dist));
    f3 n0, n1, n2;
    if (face_normals) {
        const float4 r2 = *r2p;
        n0 = n1 = n2 = V(r2.y, r2.z, r2.w);
    } else {
        n0 = ld3(S.nrm[ix.x]);
        n1 = ld3(S.nrm[ix.y]);
        n2 = ld3(S.nrm[ix.z]);
    }
    if (ETA_W)
        h.nrm = normalize(add(add(muls(n0, 1.0f - t.beta - t.gamma + 0.0001f), muls(n1, t.beta + 0.0001f)),
                              muls(n2, t.gamma + 0.0001f)));
    else
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
// Persistent "while-while" megakernel with per-lane work regeneration:
//   * a lane owns one work unit at a time -- one iteration of one pixel (or
//     RT_OPT_SAMPLE_CHUNK consecutive ones) -- and writes that iteration's
//     16-B sample record; an idle lane takes the next unit from its XCD's work
//     shard (wave-aggregated: one atomic per refill, slots handed out with
//     ballot + mbcnt prefix ranks, so idle lanes are compacted onto new work);
//   * traversal phase: each loop trip advances every tracing lane by one BSP
//     treelet (three levels) or two triangle tests / one BVH pop; lanes whose
//     ray finished wait;
//   * shading phase: entered when at most `shade_threshold` lanes are still
//     tracing (or none): the finished lanes shade, set up their next ray
//     (shadow, bounce or the next sample) and rejoin; lanes still mid-ray keep
//     their traversal state, so no lane waits for the slowest ray of the wave.
// The per-pixel arithmetic is exactly fs_main (w7e3.wgsl:233-272 /
// w9e1.wgsl:244-284): the lambertian continuation after the shadow ray only
// needs the two possible contributions (visible / blocked), the RR decision
// and the next direction, all computed with the same operations in the same
// PRNG order before the shadow ray is traced.
// Occupancy target (waves per SIMD): the register budget the compiler fits the
// path kernel into (8 -> <= 64 VGPRs; the traversal loop keeps everything in
// registers except the hit record of an accept, and the spills sit in the
// shading code).  Measured at 256 spp: 5 waves 2744, 6: 2897, 7: 3029,
// 8: 3084 Mrays/s.
// BVH instantiations: 8 waves/SIMD (64 VGPRs).  Round 1 measured 7 best
// (3007 Mrays/s vs 2712 at 8); with the SLP-free build and four steps per
// check 8 wins: 5792 vs 5667 (7) and 5511 (6) (profiles/r02/ab_waves2.txt)
#ifndef RT_BVH_WAVES_PER_EU
#define RT_BVH_WAVES_PER_EU 8
#endif
// W7E3 (config 2): its area-light shading keeps more state than W9E1's.  At 8
// waves/SIMD (64 VGPRs) it spilled 272 B per lane and moved 103 GB per config-2
// launch through L2 for 1 GB of sample records; at 5 (96 VGPRs) 76 B and 10 GB,
// and the frame is 3.5 % faster: 4528 vs 4375 Mrays/s (profiles/r02/ab_w7e3_waves.txt).
// With the round-2 spill cuts and per-XCD work shards, 7 waves (72 VGPRs, 52 B of
// scratch per lane) is the best: 8500 vs 7866 (5) and 8205 (8) Mrays/s
// (profiles/r02/ab_w7e3_shards.txt)
#ifndef RT_W7E3_WAVES_PER_EU
#define RT_W7E3_WAVES_PER_EU 7
#endif
// traversal steps per shading-threshold check in k_path's trip loop
// (profiles/r02/ab_tpc2.txt: 2 vs 1 = config 3 +1.4%, BVH +2.6%, config 2 +0.6%;
// ab_tpc34.txt: 4 vs 2 = config 3 +1.9%, BVH +1.0%, 3 vs 2 config 2 +0.4%;
// ab_tpc8.txt: 8 vs 4 = config 3 +1.2%, config 4 +1.1%, BVH -1.2%)
#ifndef RT_TRIPS_PER_CHECK
#define RT_TRIPS_PER_CHECK 8
#endif
#ifndef RT_BVH_TRIPS_PER_CHECK
#define RT_BVH_TRIPS_PER_CHECK 4
#endif
#ifndef RT_PATH_WAVES_PER_EU
#define RT_PATH_WAVES_PER_EU 8
#endif
// intersect_sphere (w1e6.wgsl / w8e1.wgsl:352-376): closest root in [tmin, tmax]
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
// The two balls of intersect_scene_bsp (w8e1.wgsl:244-262), in its order: the
// mirror ball, then the glass ball on the interval the first leaves.  id 0:
// none, 1: mirror, 2: transparent (ior1_over_ior2 1.5).  The kernel tests them
// when a ray starts (their nearest hit bounds the mesh walk, as r.tmax does in
// the shader) and again when a ray that found no triangle is shaded.
struct W8Ball {
    uint32_t id;
    float t;
    f3 pos, nrm;
};
__device__ __forceinline__ W8Ball w8_balls(f3 o, f3 w, float tmin, float tmax)
{
    W8Ball b;
    b.id = 0;
    b.t = tmax;
    b.pos = b.nrm = V(0, 0, 0);
    if (w1_sphere(o, w, tmin, b.t, V(420.0f, 90.0f, 370.0f), 90.0f, b.pos, b.nrm)) b.id = 1;
    if (w1_sphere(o, w, tmin, b.t, V(130.0f, 90.0f, 250.0f), 90.0f, b.pos, b.nrm)) b.id = 2;
    return b;
}

// intersect_plane (w9e2.wgsl:388-404): the holdout plane through the origin
// with normal (0, 1, 0), in the shader's arithmetic
__device__ __forceinline__ bool w9_plane(f3 o, f3 w, float tmin, float& tmax)
{
    const f3 n = V(0.0f, 1.0f, 0.0f);
    const float distance = dot(sub(V(0.0f, 0.0f, 0.0f), o), n) / dot(w, n);
    if (distance < tmin || distance > tmax) return false;
    tmax = distance;
    return true;
}

// sample_directional_light (w9e3.wgsl:405-414): the sun, L = 10, from -normalize(1, -0.35, 0)
__device__ __forceinline__ Light sun_light()
{
    Light L;
    L.l_i = V(10.0f, 10.0f, 10.0f);
    L.w_i = neg(normalize(V(1.0f, -0.35f, 0.0f)));
    L.dist = 999999.0f;
    return L;
}

// tmax of a closest-hit ray [ETA, 5000] from o along w: the analytic objects
// the shader tests before intersect_trimesh bound the mesh walk (r.tmax)
template <int MODE>
__device__ __forceinline__ float ray_tmax(f3 o, f3 w, float eta)
{
    float tm = 5000.0f;
    if (MODE == RT_MODE_W8E1 || MODE == RT_MODE_W8E2 || MODE == RT_MODE_W8E3) tm = w8_balls(o, w, eta, 5000.0f).t;
    if (MODE == RT_MODE_W9E2 || MODE == RT_MODE_W9E3) w9_plane(o, w, eta, tm);
    return tm;
}

// environment_map(dir) of the W9 modes (w9e1.wgsl:232-239; w9e2.wgsl:234-246
// decodes RGBE): the texture if one is set, else the constant environment
template <int MODE>
__device__ __forceinline__ f3 env_at(const DevLaunch& L, const f3 env, const f3 d)
{
    f3 e = env;
    if (L.env_tex) {
        float rgb[3];
        const uint32_t w = sopaque(L.env_w), h = sopaque(L.env_h);   // see make_cam_opaque
        if (MODE == RT_MODE_W9E2) rt_det_env_sample_rgbe(L.env_tex, w, h, d.x, d.y, d.z, rgb);
        else rt_det_env_sample(L.env_tex, w, h, d.x, d.y, d.z, rgb);
        e = V(rgb[0], rgb[1], rgb[2]);
    }
    return e;
}

// Shading of a ball hit (shade(), w8e1.wgsl:379-404): mirror (id 1,
// w8e1.wgsl:437-445 / w8e2.wgsl:509-522) or transparent (id 2,
// w8e1.wgsl:447-490 / w8e2.wgsl:524-569 / w8e3.wgsl: absorption on exit).
// Replaces the ray (ro, rd) and updates factor/emit; adds what the shader
// returns (0, or error_shader()) to res.  Returns true when the sample goes on
// with the new ray.  Under total internal reflection w_t carries sqrt of a
// negative number (NaN), as in the shader; the walks and the oracle follow
// IEEE comparison semantics for it.
template <int MODE>
__device__ __forceinline__ bool w8_ball_shade(const W8Ball& b, f3& ro, f3& rd, f3& fac, bool& emit, f3& res,
                                              uint32_t& rng, float ETA)
{
    constexpr bool E1 = MODE == RT_MODE_W8E1, E2 = MODE == RT_MODE_W8E2, E3 = MODE == RT_MODE_W8E3;
    f3 n = b.nrm;
    bool go = true, reflect_ray = true;
    if (b.id == 2u) {
        const f3 w_i = neg(normalize(rd));
        const f3 normal = normalize(n);
        f3 out_n;
        float ior = 1.5f, cos_i = dot(w_i, normal), tp = 0.0f;
        const bool entering = cos_i < 0.0f;
        f3 T_r = V(1.0f, 1.0f, 1.0f);
        if (entering) {
            cos_i = dot(w_i, neg(normal));
            out_n = neg(normal);
        } else {
            ior = 1.0f / ior;
            out_n = normal;
            if (E3) {   // T_r = exp(-rho_t * s), s = length(position - origin) / 100
                const f3 dd = sub(b.pos, ro);
                const float sd = rt_det_sqrtf(dot(dd, dd)) / 100.0f;
                const f3 nr = neg(V(0.5f, 0.2f, 0.2f));
                T_r = V(rt_det_expf(nr.x * sd), rt_det_expf(nr.y * sd), rt_det_expf(nr.z * sd));
                tp = (T_r.x + T_r.y + T_r.z) / 3.0f;
                if (tp < 0.0f || tp > 1.0f) {
                    res = add(res, V(0.7f, 0.0f, 0.7f));   // error_shader; has_hit ends the sample
                    return false;
                }
            }
        }
        const float cos_t2 = (1.0f - (ior * ior) * (1.0f - cos_i * cos_i));
        float refl = 1.0f;
        if (!(cos_t2 < 0.0f)) {   // fresnel_r, w8e2.wgsl:202-212
            const float ct = rt_det_sqrtf(cos_t2);
            const float ii = ior * cos_i, tt = 1.0f * ct, ti = 1.0f * cos_i, it2 = ior * ct;
            const float r1 = (ii - tt) / (ii + tt), r2 = (ti - it2) / (ti + it2);
            refl = 0.5f * (r1 * r1 + r2 * r2);
            if (E1) refl = rt_satf(refl);
        }
        const f3 tangent = sub(muls(out_n, cos_i), w_i);
        rd = sub(muls(tangent, ior), muls(E1 ? out_n : normalize(out_n), rt_det_sqrtf(cos_t2)));
        ro = b.pos;
        if (!E1) emit = true;
        const float step = rnd(rng);
        reflect_ray = step < refl;
        if (reflect_ray) {
            n = out_n;
        } else if (E2) {
            fac = divs(fac, 1.0f - refl);
        } else if (E3 && !entering) {
            if (step < refl + tp) fac = divs(mul(fac, T_r), refl + tp);
            else go = false;   // absorbed
        }
    }
    if (reflect_ray) {
        rd = sub(rd, muls(n, 2.0f * dot(n, rd)));   // reflect
        ro = E1 ? b.pos : add(b.pos, muls(n, ETA));
        if (!E1) emit = true;
    }
    res = add(res, V(0, 0, 0));   // result += shade() (= vec3(0)); keeps -0 + 0 semantics
    return go;
}

// W9E1 with uniforms.selection1 == 7 (the transparent shader) runs as its own
// instantiation: its shading code in the default kernel raises the register
// pressure enough to spill inside the traversal loop.
constexpr int MODE_W9E1_TRANSPARENT = 100 + RT_MODE_W9E1;

// CM: the BSP walk's margin formula (bsp_box_miss): 1, the generic form every
// culling mode runs correctly with; 0, the fast margin's alone (launch_path picks
// it for W9E1 / W7E3 when the context's culling is not certified); 2, the certified
// form with the silhouette bound (RT_BSP_CULL_SILHOUETTE, W9E1)
// Ray capture of the counting instantiation (DevLaunch.cap_*, rt_set_ray_capture):
// the ray a walk is about to trace, appended in issue order.  Compiles to
// nothing in the timed instantiations.
template <bool COUNT>
__device__ __forceinline__ void capture_ray(const DevLaunch& L, const f3 o, const f3 d, float tmin, float tmax,
                                            bool anyhit)
{
    if constexpr (COUNT) {
        if (L.cap_rays) {
            const unsigned long long i = atomicAdd(L.cap_count, 1ull);
            if (i < L.cap_max) {
                L.cap_rays[2 * i] = make_float4(o.x, o.y, o.z, d.x);
                L.cap_rays[2 * i + 1] = make_float4(d.y, d.z, tmin, tmax);
                L.cap_flags[i] = anyhit ? 1u : 0u;
            }
        }
    }
}

template <int MODE, int TRAV, bool COUNT, int CM = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    TRAV == RT_TRAVERSE_BVH ? RT_BVH_WAVES_PER_EU : MODE == RT_MODE_W7E3 ? RT_W7E3_WAVES_PER_EU : RT_PATH_WAVES_PER_EU,
    8)))
k_path(DevScene S, DevLaunch L)
{
    extern __shared__ uint32_t lds_stack[];   // [level][thread], 4 B entries
#ifdef RT_DBG_WAVE_TIMES
    // diagnostic builds only (tools/wave_times.py): each wave's start and end on the
    // 100-MHz real-time clock, into the ray-capture buffer
    const uint64_t dbg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    // BSP: the lane's column of the [level][thread] stack.  BVH: the wave's
    // column (uniform); a lane adds lane_v() at each access, so no per-lane
    // address stays live across the loop (at 7 waves/SIMD it was spilled;
    // 3008 -> 3604 Mrays/s).  The BSP loop keeps its address in a register
    // (measured 3178 vs 2959 with lane_v).
    void* stk = TRAV == RT_TRAVERSE_BVH ? lds_stack + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u)
                                        : lds_stack + threadIdx.x;
    const BvhDeep dp{TRAV == RT_TRAVERSE_BVH ? L.bvh_deep + (size_t)blockIdx.x * 256u + threadIdx.x : nullptr,
                     gridDim.x * 256u};
    // W9E2: W9E1 + the holdout plane y = 0 (ambient-occlusion ray, environment
    // seen through it) and an RGBE environment; one instantiation for all its shaders
    constexpr bool W9E2 = MODE == RT_MODE_W9E2;
    // W9E3: the holdout plane shaded by an ambient-occlusion ray and a sun ray,
    // a sun-lit lambertian, back-face culled triangles, transparent at selection 3
    constexpr bool W9E3 = MODE == RT_MODE_W9E3;
    constexpr bool PLANE = W9E2 || W9E3;
    constexpr bool W9 = MODE == RT_MODE_W9E1 || MODE == MODE_W9E1_TRANSPARENT || W9E2 || W9E3;
    constexpr bool XT = MODE == MODE_W9E1_TRANSPARENT || W9E2 || W9E3;
    constexpr uint32_t TSEL = W9E3 ? 3u : 7u;   // the transparent shader's selection value
    // W8E1/W8E2/W8E3: the Cornell box with its two analytic balls; W8E1 lights
    // directly only (10 segments), W8E2/W8E3 path trace with a firefly clamp
    constexpr bool W8 = MODE == RT_MODE_W8E1 || MODE == RT_MODE_W8E2 || MODE == RT_MODE_W8E3;
    constexpr bool W8E1 = MODE == RT_MODE_W8E1;
    constexpr bool W8E3 = MODE == RT_MODE_W8E3;
    constexpr bool CLAMP = W8 && !W8E1;
    constexpr bool FAC_AMB = W9 || W8E3;   // ambient = emission * factor
    constexpr uint32_t MAXD = W8E1 ? 10u : 50u;
    // the shading phase's issue priority (W7E3's short Cornell-box rays shade often:
    // +0.9 % at 2, profiles/r04/ab_shade_prio.txt; neutral on W9E1's configs)
    constexpr int SPRIO = MODE == RT_MODE_W7E3 ? 2 : 0;
    // W9E1 draws the next bounce direction after the shadow walk, from the hit
    // the any-hit walk left in the traversal state (resolve() again): the shadow
    // walk draws no random numbers, so the PRNG sequence is the reference's, and
    // the direction (3 floats) need not be kept across the walk
    constexpr bool REDRAW = MODE == RT_MODE_W9E1 || MODE == MODE_W9E1_TRANSPARENT;
    // W9E1: every shadow ray is light_init's (0, 1, 0) (the lambertian branch
    // below); the BSP walk's leaf tests take their VERT form in the trips whose
    // leaf lanes all hold one (W9E2 / W9E3 also send other any-hit rays)
    constexpr bool VSH = REDRAW && TRAV == RT_TRAVERSE_BSP;
    const float ETA = W9 ? 0.0001f : 0.01f;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t T = L.shade_threshold;
    Counters cnt;
#pragma unroll
    for (int i = 0; i < C_N; i++) cnt.v[i] = 0;

    // lane state: ST_IDLE (no pixel), ST_TRACE (a ray in flight), ST_SHADE (ray done, waiting to shade)
    enum : uint32_t { ST_IDLE = 0, ST_TRACE = 1, ST_SHADE = 2 };
    uint32_t st = ST_IDLE;
    bool exhausted = L.spp == 0u, shadow = false, emit = true, survive = false, ao = false, hblk = false;
    uint32_t hph = 0;   // W9E3 holdout: 1 = occlusion ray in flight, 2 = sun ray in flight
    // pxy: the pixel as x | y << 16 (the host keeps the resolution below 2^16)
    uint32_t pxy = 0, it = 0, prim = 0xFFFFFFFFu, rng = 0, bounce = 0;
    f3 res = V(0, 0, 0), fac = V(1, 1, 1), ro = V(0, 0, 0), rd = V(0, 0, 1), inv = V(0, 0, 0);
    f3 ndir = V(0, 0, 1), cu = V(0, 0, 0), cb = V(0, 0, 0);
    Trav tr;
    trav_init(tr, 0.0f, 0.0f);


    // fs_main prologue for iteration `it` of the lane's pixel (w7e3.wgsl:236-248)
    auto start_sample = [&](const DevLaunch& L) {
        const uint32_t px = pxy & 0xFFFFu, py = pxy >> 16;
        rt_uniform u;
        u.resolution[0] = sopaque(L.u.resolution[0]);
        u.resolution[1] = sopaque(L.u.resolution[1]);
        const float fH = (float)u.resolution[1];
        const Cam cam = make_cam_opaque(L);
        rng = tea16(py * u.resolution[0] + px, it);
        float jx = rnd(rng);
        float jy = rnd(rng);
        jx = jx / fH;
        jy = jy / fH;
        float ux, uy;
        pixel_uv(u, px, py, ux, uy);
        rd = cam_dir(cam, ux, uy, jx, jy);
        ro = cam.e;
        res = V(0, 0, 0);
        fac = V(1, 1, 1);
        emit = true;
        bounce = 0;
        prim = 0xFFFFFFFFu;
        shadow = false;
        inv = trav_inv<TRAV>(rd);
        trav_start<TRAV>(tr, stk, ETA, ray_tmax<MODE>(ro, rd, ETA));
        capture_ray<COUNT>(L, ro, rd, ETA, ray_tmax<MODE>(ro, rd, ETA), false);
        st = ST_TRACE;
        ao = false;
        hph = 0;
        cnt.v[C_SAMPLES]++;
        cnt.v[C_PRIMARY]++;
    };

    // Shading threshold.  L.shade_threshold bit 16 set: chosen by the wave
    // between T_lo (bits 0-7) and T_hi (bits 8-15) from the share of its
    // tracing lanes that sit in a leaf (testing triangles), counted at every
    // check.  A test-dominated walk (long leaves: config 5's 32-triangle
    // leaves; with subtree culling config 4's bunny grid too, 0.73-0.75 of the
    // tracing lanes in a leaf) has long, uneven per-lane tails, so finished
    // lanes are refilled early (T_hi); a walk-dominated one (config 3: 0.34)
    // keeps the refills together (T_lo) for the coherence of the pixel-major
    // units.
    // (T_hi once the leaf share of the tracing lanes reaches NUM/DEN: 1/2 since
    // subtree culling, which made config 4's walk 0.75 and config 5's 0.73 leaf
    // tests; at 3/4 config 5 ran 2708 vs 2886 Mrays/s at 128 spp, config 4 3521
    // vs 3559, configs 2 and 3 unchanged; profiles/r03/ab_ls_c*.txt)
#ifndef RT_THI_SHARE_NUM
#define RT_THI_SHARE_NUM 1
#define RT_THI_SHARE_DEN 2
#endif
    int32_t leaf_score = 0;   // sum of DEN * leaf lanes - NUM * tracing lanes over the checks (wave-uniform)
    uint64_t tstamp = COUNT ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
        // ---- traversal phase: every tracing lane advances its ray by one node
        //      visit / triangle test per trip, until enough lanes wait to shade
        for (;;) {
            const uint64_t trm = __ballot(st == ST_TRACE);
            const uint64_t wtm = __ballot(st == ST_SHADE);
            uint32_t Te = T & 0xFFu;
            if (TRAV == RT_TRAVERSE_BSP && (T >> 16)) {   // (the host asks for it on the BSP walk only)
                const int32_t lf = __popcll(__ballot((st == ST_TRACE) & (tr.leaf_k != tr.leaf_end)));
                leaf_score += RT_THI_SHARE_DEN * lf - RT_THI_SHARE_NUM * (int32_t)__popcll(trm);
                leaf_score = leaf_score < -(1 << 24) ? -(1 << 24) : leaf_score > (1 << 24) ? (1 << 24) : leaf_score;
                Te = leaf_score >= 0 ? (T >> 8) & 0xFFu : T & 0xFFu;
            }
            if (!(trm != 0 && (wtm == 0 || Te >= 64u || (uint32_t)__popcll(trm) > Te))) break;
            if (COUNT) {
                const bool leafst = tr.leaf_k != tr.leaf_end;
                const uint64_t nm = __ballot(st == ST_TRACE && !leafst);
                const uint64_t lm = __ballot(st == ST_TRACE && leafst);
                if (st == ST_TRACE) {
                    cnt.v[C_LANE_STEPS]++;
                    if (leafst) cnt.v[C_LEAF_LANE_STEPS]++;
                }
#ifdef RT_DBG_VERT
                // diagnostic build only: trips whose leaf (walking) lanes are all shadow rays
                // (C_POPS, unused by the BSP walk; C_EXACT_NODES, whose per-decision count is
                // C_INTERIOR's)
                const uint64_t lms = __ballot(st == ST_TRACE && leafst && !shadow);
                const uint64_t nms = __ballot(st == ST_TRACE && !leafst && !shadow);
                if (lane == 0) {
                    cnt.v[C_POPS] += (lm != 0) & (lms == 0);
                    cnt.v[C_EXACT_NODES] += (nm != 0) & (nms == 0);
                }
#endif
                if (lane == 0) {
                    cnt.v[C_TRIPS]++;
                    cnt.v[C_NODE_TRIPS] += nm != 0;
                    cnt.v[C_LEAF_TRIPS] += lm != 0;
                }
            }
            // the plane divisions' range check (bsp_decide): kept for the next trips when
            // the scene's planes need it or a tracing lane's ray has a direction component
            // of magnitude <= 1e-8 other than 0 (a NaN in inv) or an origin coordinate
            // outside {0} U [2^-76, 2^99] in magnitude; no lane starts a new ray before the
            // next check
            uint32_t chk = 1u;
            if (TRAV == RT_TRAVERSE_BSP) {
                const float ax = rt_absf(ro.x), ay = rt_absf(ro.y), az = rt_absf(ro.z);
                const float isum = inv.x + inv.y + inv.z;   // |inv| <= 1e8: NaN only from a flag
                const bool odd = (isum != isum) | (((ax < 0x1p-76f) & (ax != 0.0f)) | (ax > 0x1p99f)) |
                                 (((ay < 0x1p-76f) & (ay != 0.0f)) | (ay > 0x1p99f)) |
                                 (((az < 0x1p-76f) & (az != 0.0f)) | (az > 0x1p99f));
                // (readfirstlane: a wave-uniform scalar)
                chk = __builtin_amdgcn_readfirstlane((S.bsp_div_checked != 0u || __ballot((st == ST_TRACE) & odd) != 0) ? 1u : 0u);
            }
            const bool go = st == ST_TRACE;
            if (go) {
                if (trav_step<TRAV, COUNT, W9E3, CM, VSH>(S, stk, dp, ro, rd, inv, shadow, tr, cnt, chk)) st = ST_SHADE;
            }
            // further steps before the next check: the check (two ballots, a
            // popcount, the compares) is SALU work, and the SALU is a per-CU
            // limit here; the counting build checks every trip
#pragma unroll
            for (int k = 1; k < (COUNT ? 1 : TRAV == RT_TRAVERSE_BVH ? RT_BVH_TRIPS_PER_CHECK : RT_TRIPS_PER_CHECK); ++k) {
                if (st == ST_TRACE) {
                    if (trav_step<TRAV, COUNT, W9E3, CM, VSH>(S, stk, dp, ro, rd, inv, shadow, tr, cnt, chk)) st = ST_SHADE;
                }
            }
        }
        if (COUNT) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            if (lane == 0) {
                cnt.v[C_TRAV_CYC64] += (uint32_t)((now - tstamp) >> 6);
                cnt.v[C_SHADE_PASSES]++;
            }
            if (st == ST_SHADE) cnt.v[C_SHADE_LANES]++;
            tstamp = now;
        }
        {
        // (SPRIO raises the wave's issue priority for its shading and refill phase,
        // so lanes are refilled sooner while the other waves trace)
        if (SPRIO) __builtin_amdgcn_s_setprio(SPRIO);
        // the shading and refill phases read the kernel arguments afresh (kreload)
        const DevScene& Sk = kreload<DevScene>(KARG_S);
        const DevLaunch& Lk = kreload<DevLaunch>(KARG_L);
        const DevScene& S = Sk;
        const DevLaunch& L = Lk;
        const uint32_t light_tris = S.nlights - 1u;
        const uint32_t sel = W9 ? L.u.selection1 : 0u;
        const uint32_t it_end = L.first_iter + L.spp;
        const uint32_t pslots = L.nwork * 64u;            // pixel slots
        const uint32_t nslots = pslots * L.nchunks;       // work units (host keeps this < 2^31)
        const f3 env = V(L.env[0], L.env[1], L.env[2]);
        // ---- shading phase
        if (st == ST_SHADE) {
            bool sample_done = false;
            if (!shadow) {
                if (tr.found) {
                    // the hit's barycentrics, kept in tr across a shadow walk (REDRAW)
                    bary_of<TRAV>(S, tr.hit_k, ro, rd, tr.beta, tr.gamma);
                    const HitRec h = resolve<TRAV, W9E3>(S, trav_out(tr), ro, rd, !W9);
                    if (bounce == 0) prim = h.tri;
                    const rt_material& m = mat_of(S, h.material);
                    if (sel == 0u) {
                        // lambertian (w7e3.wgsl:427-470 / w9e1.wgsl:428-470)
                        const f3 brdf = divs(ld3(m.diffuse), RT_PI_F);
                        const f3 emission = ld3(m.ambient);
                        Light Lt;
                        if (W9E3) {
                            Lt = sun_light();   // sample_directional_light, w9e3.wgsl:405-414
                        } else if (W9) {
                            Lt.l_i = V(0, 0, 0);   // light_init(), w9e1.wgsl:67-73
                            Lt.w_i = V(0.0f, 1.0f, 0.0f);
                            Lt.dist = 999999.0f;
                        } else {
                            const uint32_t ri = mcg31(rng);
                            Lt = sample_area_light(S, h.pos, ri % light_tris + 1u, rng);
                        }
                        f3 dv = mul(muls(brdf, rt_satf(dot(h.nrm, Lt.w_i))), Lt.l_i);
                        if (!W9) dv = muls(dv, (float)light_tris);
                        const f3 amb = emit ? (FAC_AMB ? mul(emission, fac) : emission) : V(0, 0, 0);
                        cu = add(mul(dv, fac), amb);             // not blocked: diffuse*factor + ambient
                        // blocked: vec3(0)*factor + ambient (w8e3.wgsl: vec3(0) + ambient)
                        cb = add(W8E3 ? V(0, 0, 0) : mul(V(0, 0, 0), fac), amb);
                        if (CLAMP) {   // min(shade(), firefly_clamp), w8e2.wgsl:265
                            cu = V(rt_minf(cu.x, 100.0f), rt_minf(cu.y, 100.0f), rt_minf(cu.z, 100.0f));
                            cb = V(rt_minf(cb.x, 100.0f), rt_minf(cb.y, 100.0f), rt_minf(cb.z, 100.0f));
                        }
                        // both outcomes' sums now (the same additions the shadow
                        // result would select): res carries the unblocked one and cb
                        // the blocked one across the shadow walk, 3 floats fewer
                        cb = add(res, cb);
                        res = add(res, cu);
                        fac = mul(fac, muls(brdf, RT_PI_F));
                        const float prob = (brdf.x + brdf.y + brdf.z) / 3.0f;
                        survive = !W8E1 && rnd(rng) < prob;   // w8e1.wgsl: direct light only
                        if (survive && bounce + 1u < MAXD) {
                            if (!REDRAW) ndir = indirect_dir(h.nrm, rng);   // setup_indirect (:472-489)
                            fac = divs(fac, prob);
                        }
                        // shadow ray (ray_init + tmin/tmax override, :442-449)
                        ro = h.pos;
                        rd = Lt.w_i;
                        inv = trav_inv<TRAV>(rd);
                        shadow = true;
                        st = ST_TRACE;
                        cnt.v[C_SHADOW]++;
                        float tpl = Lt.dist - ETA;
                        if ((W8 && w8_balls(ro, rd, ETA, Lt.dist - ETA).id != 0u) ||
                            (PLANE && w9_plane(ro, rd, ETA, tpl))) {
                            tr.found = true;   // a ball / the plane blocks the light: no mesh walk
                            st = ST_SHADE;
                        } else {
                            trav_start<TRAV>(tr, stk, ETA, Lt.dist - ETA);
                            capture_ray<COUNT>(L, ro, rd, ETA, Lt.dist - ETA, true);
                        }
                    } else if (sel == 2u || (XT && sel == TSEL)) {
                        f3 n = h.nrm;
                        bool reflect_ray = true;
                        if (XT && sel == TSEL) {
                            // transparent (w9e1.wgsl:505-558); hit_record_init: ior1_over_ior2 1.0,
                            // extinction (1,1,1).  The refracted ray replaces r before the mirror
                            // branch reflects it (as the shader does).
                            const f3 w_i = neg(normalize(rd));
                            const f3 normal = normalize(h.nrm);
                            const f3 ext = V(1.0f, 1.0f, 1.0f);
                            f3 out_n;
                            // W9E3's intersect_scene_bsp sets ior1_over_ior2 = 1.5 on mesh hits
                            float ior = W9E3 ? 1.5f : 1.0f, cos_i = dot(w_i, normal), absorption = 0.0f;
                            if (cos_i < 0.0f) {
                                cos_i = dot(w_i, neg(normal));
                                out_n = neg(normal);
                            } else {
                                ior = 1.0f / ior;
                                out_n = normal;
                                const f3 dd = sub(h.pos, ro);
                                const float sd = rt_det_sqrtf(dot(dd, dd));
                                const f3 nr = neg(ext);
                                const f3 tr = V(rt_det_expf(nr.x * sd), rt_det_expf(nr.y * sd), rt_det_expf(nr.z * sd));
                                absorption = 1.0f - (tr.x + tr.y + tr.z) / 3.0f;
                            }
                            const float cos_t2 = (1.0f - (ior * ior) * (1.0f - cos_i * cos_i));
                            float refl = 1.0f;
                            if (!(cos_t2 < 0.0f)) {   // fresnel_r, w9e1.wgsl:191-201
                                const float ct = rt_det_sqrtf(cos_t2);
                                const float ii = ior * cos_i, tt = 1.0f * ct, ti = 1.0f * cos_i, it2 = ior * ct;
                                const float r1 = (ii - tt) / (ii + tt), r2 = (ti - it2) / (ti + it2);
                                refl = 0.5f * (r1 * r1 + r2 * r2);
                            }
                            const f3 tangent = sub(muls(out_n, cos_i), w_i);
                            rd = sub(muls(tangent, ior), muls(normalize(out_n), rt_det_sqrtf(cos_t2)));
                            ro = h.pos;
                            reflect_ray = rnd(rng) < refl;
                            if (reflect_ray) {
                                n = out_n;
                            } else if (rnd(rng) < absorption) {
                                fac = mul(fac, divs(ext, absorption));
                            }
                        }
                        if (reflect_ray) {
                            // mirror (w9e1.wgsl:491-504): reflect, offset origin
                            rd = sub(rd, muls(n, 2.0f * dot(n, rd)));
                            ro = add(h.pos, muls(n, ETA));
                        }
                        emit = true;
                        if (bounce + 1u < 50u) {
                            bounce++;
                            inv = trav_inv<TRAV>(rd);
                            trav_start<TRAV>(tr, stk, ETA, ray_tmax<MODE>(ro, rd, ETA));
                            capture_ray<COUNT>(L, ro, rd, ETA, ray_tmax<MODE>(ro, rd, ETA), false);
                            st = ST_TRACE;
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
                    W8Ball ball;
                    ball.id = 0u;
                    if (W8) ball = w8_balls(ro, rd, ETA, 5000.0f);
                    if (W8 && ball.id != 0u) {
                        if (w8_ball_shade<MODE>(ball, ro, rd, fac, emit, res, rng, ETA) && bounce + 1u < MAXD) {
                            bounce++;
                            inv = trav_inv<TRAV>(rd);
                            trav_start<TRAV>(tr, stk, ETA, ray_tmax<MODE>(ro, rd, ETA));
                            st = ST_TRACE;
                            cnt.v[C_BOUNCE]++;
                        } else {
                            sample_done = true;
                        }
                    } else {
                        float tpl = 5000.0f;
                        if (W9E3 && w9_plane(ro, rd, ETA, tpl)) {
                            // holdout_shader (w9e3.wgsl:490-517): environment * factor, less 0.5
                            // for an occluded cosine ray and 0.5 for a blocked sun ray; both
                            // through intersect_scene_bsp (plane + mesh)
                            cu = mul(env_at<MODE>(L, env, rd), fac);
                            ro = add(ro, muls(rd, tpl));   // ray_at
                            rd = indirect_dir(V(0.0f, 1.0f, 0.0f), rng);
                            inv = trav_inv<TRAV>(rd);
                            shadow = true;
                            hph = 1;
                            st = ST_TRACE;
                            cnt.v[C_SHADOW]++;
                            float tp2 = 5000.0f;
                            if (w9_plane(ro, rd, ETA, tp2)) {
                                tr.found = true;
                                st = ST_SHADE;
                            } else {
                                trav_start<TRAV>(tr, stk, ETA, 5000.0f);
                            }
                        } else if (W9E2 && w9_plane(ro, rd, ETA, tpl)) {
                            // holdout_shader (w9e2.wgsl:514-537): an any-hit ambient-occlusion
                            // ray about the plane normal; unoccluded, the environment behind
                            ndir = rd;
                            ro = add(ro, muls(rd, tpl));   // ray_at
                            rd = indirect_dir(V(0.0f, 1.0f, 0.0f), rng);
                            inv = trav_inv<TRAV>(rd);
                            trav_start<TRAV>(tr, stk, ETA, 5000.0f);
                            shadow = true;
                            ao = true;
                            st = ST_TRACE;
                            cnt.v[C_SHADOW]++;
                        } else {
                            // miss: background (w7e3, w8e*) / environment_map(dir) * factor (w9e1.wgsl:264-265)
                            res = add(res, W9 ? mul(env_at<MODE>(L, env, rd), fac) : (W8E1 ? V(0.1f, 0.3f, 0.6f) : V(0, 0, 0)));
                            sample_done = true;
                        }
                    }
                }
            } else if (W9E3 && hph == 1u) {
                // occlusion ray finished: the sun ray from the same plane point
                hblk = tr.found;
                rd = sun_light().w_i;
                inv = trav_inv<TRAV>(rd);
                hph = 2;
                st = ST_TRACE;
                cnt.v[C_SHADOW]++;
                float tp2 = 5000.0f;
                if (w9_plane(ro, rd, ETA, tp2)) {
                    tr.found = true;
                    st = ST_SHADE;
                } else {
                    trav_start<TRAV>(tr, stk, ETA, 5000.0f);
                }
            } else if (W9E3 && hph == 2u) {
                float contribution = 1.0f;
                if (hblk) contribution -= 0.5f;
                if (tr.found) contribution -= 0.5f;
                res = add(res, muls(cu, contribution));
                sample_done = true;
            } else if (W9E2 && ao) {
                // ambient-occlusion ray finished: occluded adds vec3(0); the sample ends
                res = add(res, tr.found ? V(0, 0, 0) : mul(env_at<MODE>(L, env, ndir), fac));
                sample_done = true;
            } else {
                // shadow ray finished: rest of lambertian, then the bounce
                if (tr.found) res = cb;
                if (survive && bounce + 1u < MAXD) {
                    if (REDRAW) rd = indirect_dir(resolve<TRAV>(S, trav_out(tr), ro, rd, !W9).nrm, rng);
                    else rd = ndir;   // origin = hit position, already in ro
                    inv = trav_inv<TRAV>(rd);
                    trav_start<TRAV>(tr, stk, ETA, ray_tmax<MODE>(ro, rd, ETA));
                    capture_ray<COUNT>(L, ro, rd, ETA, ray_tmax<MODE>(ro, rd, ETA), false);
                    emit = false;
                    bounce++;
                    shadow = false;
                    st = ST_TRACE;
                    cnt.v[C_BOUNCE]++;
                } else {
                    sample_done = true;
                }
            }
            if (sample_done) {
                // this iteration's `result` (+ primary id); k_fold accumulates in
                // iteration order (w7e3.wgsl:261-271).  Streaming store: keep the
                // scene, not the samples, in L2/MALL.
                const uint32_t out = pixel_out(L, pxy & 0xFFFFu, pxy >> 16);
                // record layout follows the unit order: pixel-major units keep a
                // pixel's iterations together ([pixel][iteration]), so the lanes of a
                // refill (one pixel, consecutive iterations) write whole lines
                const uint32_t ip = it - L.first_iter;
                const size_t ri = L.unit_order ? (size_t)out * L.spp + ip : (size_t)ip * L.stride + out;
                v4f* sp = reinterpret_cast<v4f*>(L.samples + ri);
                const v4f sv = {res.x, res.y, res.z, __uint_as_float(prim)};
                __builtin_nontemporal_store(sv, sp);
                it++;
                // the unit's end, from its chunk (it - 1 lies in it)
                const uint32_t ue = L.first_iter + ((it - 1u - L.first_iter) / L.chunk + 1u) * L.chunk;
                if (it < (ue < it_end ? ue : it_end)) start_sample(L);
                else st = ST_IDLE;
            }
        }
        // ---- refill idle lanes with new pixels (ballot + mbcnt compaction).
        //      The slots are dealt to 8 shards, one per XCD, each with its own
        //      queue head in its own 128-B line, so the refills of 256 CUs do not
        //      all meet on one atomic: a shard owns every 8th block of 64
        //      consecutive slots (a refill's worth, so a refill still hands out
        //      neighbouring units).  The shard is the XCD id read from the
        //      hardware at each refill; the shards' blocks interleave over the
        //      frame, so they drain together; a wave whose home shard is drained
        //      moves on to the next ones (restarting from home at each refill), so
        //      every slot is handed out whatever XCDs the waves land on.  One
        //      global queue cost config 2 (short Cornell-box rays, many refills)
        //      39 % of its frame; interleaving single slots instead of blocks cost
        //      config 4 at 16 spp 13 % (profiles/r02/ab_shards.txt).
#ifndef RT_BSP_SHARDS_LG
#define RT_BSP_SHARDS_LG RT_SHARD_LG
#endif
        constexpr uint32_t LGSH = TRAV == RT_TRAVERSE_BVH ? RT_SHARD_LG : RT_BSP_SHARDS_LG;
        uint32_t shard = LGSH ? shard_of_wave() : 0u;
        uint32_t tried = 0;
        for (;;) {
            const uint64_t need = __ballot(st == ST_IDLE && !exhausted);
            if (need == 0) break;
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)need) - 1u;
            uint32_t base = 0;
            if (lane == leader) {
                const uint32_t head = atomicAdd(L.work_counter + shard * 32u, (uint32_t)__popcll(need));
                // a drained shard's head keeps growing with every futile draw:
                // clamp it so the slot below cannot wrap (nslots < 2^31)
                base = LGSH == 0u ? head : head < (1u << 28) ? head : (1u << 28);
            }
            base = __shfl(base, (int)leader, 64);
            bool ran_out = false;
            if (st == ST_IDLE && !exhausted) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                // position h of the shard's sequence; the shard owns every
                // 2^LGSH-th block of 64 consecutive slots, so one refill still hands
                // out neighbouring units (pixel-major: the iterations of one pixel)
                const uint32_t h = base + rank;
                const uint32_t slot = LGSH == 0u ? h : ((((h >> 6) << LGSH) + shard) << 6) | (h & 63u);
                if (slot >= nslots) {
                    if (LGSH == 0u) exhausted = true;
                    else ran_out = true;
                } else {
                    // chunk-major (unit_order 0): a refill hands out neighbouring
                    // pixels at the same iteration; pixel-major (1): the iterations
                    // of one pixel side by side
                    uint32_t ch, ps;
                    const uint32_t psl = sopaque(L.nwork) * 64u, nch = sopaque(L.nchunks);
                    if (L.unit_order == 0u) {
                        ch = slot / psl;
                        ps = slot - ch * psl;
                    } else {
                        ps = slot / nch;
                        ch = slot - ps * nch;
                    }
                    const Pix p = map_pixel(L, ps >> 6, ps & 63u);
                    if (p.valid) {
                        pxy = p.x | p.y << 16;
                        it = L.first_iter + ch * L.chunk;
                        start_sample(L);
                    }
                }
            }
            if (LGSH != 0u && __ballot(ran_out) != 0) {   // this shard is drained (its head only grows)
                shard = (shard + 1u) & ((1u << LGSH) - 1u);
                if (++tried == (1u << LGSH)) exhausted = true;
            }
        }
        }
        if (COUNT) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            if (lane == 0) cnt.v[C_SHADE_CYC64] += (uint32_t)((now - tstamp) >> 6);
            tstamp = now;
        }
        if (SPRIO) __builtin_amdgcn_s_setprio(0);
        if (__ballot(st != ST_IDLE) == 0) break;
    }
    flush_counters(cnt, L.counters, COUNT);
#ifdef RT_DBG_WAVE_TIMES
    if (!COUNT && L.cap_rays && (threadIdx.x & 63u) == 0u) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | ((4 - 1) << 11));
        L.cap_rays[blockIdx.x * 4u + (threadIdx.x >> 6)] =
            make_float4(__uint_as_float((uint32_t)dbg_t0), __uint_as_float((uint32_t)(dbg_t0 >> 32)),
                        __uint_as_float((uint32_t)t1), __uint_as_float(xcc & 0xFu));
    }
#endif
}

// ------------------------------------------------------------------ progressive fold
// The accumulation of fs_main (w7e3.wgsl:261-271 / w9e1.wgsl:272-283), applied
// for iterations first_iter .. first_iter+spp-1 in order to each output pixel:
// accum = max(vec4((result + prev*it)/(it+1), 1), 0) with prev the stored
// accumulation (read when first_iter > 0, as the RenderSource texture).  One
// thread per pixel.  Chunk-major units write samples as [iteration][pixel] (a
// wave reads 1 KiB contiguous per iteration); pixel-major units (the default)
// as [pixel][iteration], so k_path's 16-B records land in whole lines and a
// thread here streams its own pixel's records.  ids = primary hit of the last
// iteration.
__global__ void __launch_bounds__(256) k_fold(DevLaunch L)
{
    const uint32_t nout = L.tileset ? L.nwork * 64u : L.w * L.h;
    for (uint32_t o = blockIdx.x * blockDim.x + threadIdx.x; o < nout; o += gridDim.x * blockDim.x) {
        if (L.tileset && !map_pixel(L, o >> 6, o & 63u).valid) continue;
        float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
        if (L.first_iter > 0u) {
            const float4 pa = L.accum[o];
            a0 = pa.x;
            a1 = pa.y;
            a2 = pa.z;
        }
        v4f r = {0.0f, 0.0f, 0.0f, 0.0f};
        auto fold1 = [&](const v4f x, uint32_t i) {
            const uint32_t it = L.first_iter + i;
            const float fi = (float)it, fi1 = (float)(it + 1u);
            a0 = rt_max0f((x.x + a0 * fi) / fi1);
            a1 = rt_max0f((x.y + a1 * fi) / fi1);
            a2 = rt_max0f((x.z + a2 * fi) / fi1);
        };
        uint32_t i = 0;
        if (L.unit_order) {
            // [pixel][iteration]: the thread's own records are contiguous; eight
            // (128 B) are loaded together, so each line is fetched once while the
            // wave's 64 threads stream 64 lines side by side
            const v4f* sp = reinterpret_cast<const v4f*>(L.samples + (size_t)o * L.spp);
#ifndef RT_FOLD_BATCH
#define RT_FOLD_BATCH 8
#endif
            for (; i + RT_FOLD_BATCH <= L.spp; i += RT_FOLD_BATCH) {
                v4f q[RT_FOLD_BATCH];
#pragma unroll
                for (int k = 0; k < RT_FOLD_BATCH; k++) q[k] = sp[i + k];
#pragma unroll
                for (int k = 0; k < RT_FOLD_BATCH; k++) fold1(q[k], i + k);
                r = q[RT_FOLD_BATCH - 1];
            }
            for (; i < L.spp; i++) {
                r = sp[i];
                fold1(r, i);
            }
        } else {
            // [iteration][pixel]: a wave reads 1 KiB contiguous per iteration
            const v4f* sp = reinterpret_cast<const v4f*>(L.samples + o);
            for (; i < L.spp; i++) {
                r = __builtin_nontemporal_load(sp + (size_t)i * L.stride);
                fold1(r, i);
            }
        }
        L.accum[o] = make_float4(a0, a1, a2, 1.0f);
        if (L.ids && L.spp) L.ids[o] = __float_as_uint(r.w);
    }
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
    extern __shared__ uint32_t lds_stack[];   // [level][thread], 4 B entries
    // BSP: the lane's column of the [level][thread] stack.  BVH: the wave's
    // column (uniform); a lane adds lane_v() at each access, so no per-lane
    // address stays live across the loop (at 7 waves/SIMD it was spilled;
    // 3008 -> 3604 Mrays/s).  The BSP loop keeps its address in a register
    // (measured 3178 vs 2959 with lane_v).
    void* stk = TRAV == RT_TRAVERSE_BVH ? lds_stack + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u)
                                        : lds_stack + threadIdx.x;
    const BvhDeep dp{TRAV == RT_TRAVERSE_BVH ? L.bvh_deep + (size_t)blockIdx.x * 256u + threadIdx.x : nullptr,
                     gridDim.x * 256u};
    const float ETA = 0.00001f;
    const uint32_t lane = threadIdx.x & 63u;
    const Cam cam = make_cam(L);
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
            if (tracing) hit = trace<TRAV, COUNT>(S, stk, dp, ro, rd, rtmin, rtmax, false, tr, cnt);
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

// ------------------------------------------------------------------ ray queries
// rt_trace_rays: one walk per ray with the render kernels' own step functions
// (bsp_step / bvh_step, with the culling mode's margin formula CM): intersect_trimesh (bsp.wgsl:10-81) or intersect_bvh
// (bvh.wgsl:154-191) for a closest-hit ray, the any-hit walk of the shadow
// rays (flags bit 0; bsp.wgsl:83-155 stops at the first accept) otherwise.
// One ray per lane, grid-stride; the tested triangles are hashed in order.
template <int TRAV, int CM = 1>
__global__ void __launch_bounds__(256) k_query(DevScene S, const float* rays, const uint32_t* flags, uint32_t n,
                                               rt_ray_hit* out, uint32_t* bvh_deep)
{
    extern __shared__ uint32_t lds_stack[];
    void* stk = TRAV == RT_TRAVERSE_BVH ? lds_stack + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u)
                                        : lds_stack + threadIdx.x;
    const BvhDeep dp{TRAV == RT_TRAVERSE_BVH ? bvh_deep + (size_t)blockIdx.x * 256u + threadIdx.x : nullptr,
                     gridDim.x * 256u};
    Counters cnt;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; __ballot(i < n); i += gridDim.x * 256u) {
        if (i >= n) continue;   // lanes past the end idle (the walk's LDS columns are per lane)
        const float* r = rays + 8 * (size_t)i;
        const f3 o = V(r[0], r[1], r[2]), d = V(r[3], r[4], r[5]);
        const bool anyhit = flags && (flags[i] & 1u);
        FnvLog lg{TRAV == RT_TRAVERSE_BVH ? S.bvh_ids : S.bsp_ids,
                  TRAV == RT_TRAVERSE_BVH ? S.bvh_rec_off : S.bsp_rec_off, 0u, 0x811c9dc5u, 0xFFFFFFFFu};
        Trav t;
        t.hit_k = 0;
        t.beta = t.gamma = 0.0f;
        trav_start<TRAV>(t, stk, r[6], r[7]);
        const f3 inv = trav_inv<TRAV>(d);
        for (uint32_t guard = 0; guard < (1u << 24); guard++) {
            const bool done = TRAV == RT_TRAVERSE_BVH
                                  ? bvh_step_log<false, false>(S, reinterpret_cast<uint32_t*>(stk), dp, o, d, inv,
                                                               anyhit, t, cnt, lg)
                                  : bsp_step_log<false, false, FnvLog, CM>(S, reinterpret_cast<float*>(stk), o, d, inv,
                                                                           anyhit, t, cnt, lg);
            if (done) break;
        }
        rt_ray_hit h;
        // an any-hit walk keeps no hit record: its accept is the last tested triangle
        const uint32_t slot = (t.hit_k - (TRAV == RT_TRAVERSE_BVH ? S.bvh_rec_off : S.bsp_rec_off)) / 48u;
        h.tri = !t.found ? 0xFFFFFFFFu : anyhit ? lg.last : (TRAV == RT_TRAVERSE_BVH ? S.bvh_ids : S.bsp_ids)[slot];
        h.dist = t.found ? t.tmax : 0.0f;
        if (t.found && !anyhit) bary_of<TRAV>(S, t.hit_k, o, d, t.beta, t.gamma);
        h.beta = t.found && !anyhit ? t.beta : 0.0f;
        h.gamma = t.found && !anyhit ? t.gamma : 0.0f;
        h.ntested = lg.n;
        h.tested_fnv = lg.h;
        h.tmin = t.tmin;
        h.tmax = t.tmax;
        out[i] = h;
    }
}

// ------------------------------------------------------------------ batch trace
// rt_trace_batch: the trace stage of a wavefront renderer -- device-resident
// rays in, one hit record per ray out, no shading state.  A persistent grid
// like k_path's (8 waves per SIMD, the BSP trail in LDS, refills by ballot +
// mbcnt from 8 per-XCD shards of 64-ray blocks, eight steps per check) whose
// lanes hold only the walk: o, w, the reciprocals, the interval and the trail
// state.  Finished lanes wait until at most T lanes of the wave still trace,
// then refill together (k_path's shading threshold, without the shading).
// Rays: 32 B {o.xyz, w.xyz, tmin, tmax} (rt_trace_rays' layout), flags bit 0 =
// any-hit (the shadow walk).  Hits: {record byte offset of the accepted triangle (closest hit) or
// 0xFFFFFFFE (any-hit: blocked), 0xFFFFFFFF on a miss | dist bits}.
// DESIGN.md section 4 "Outside the megakernel": the price of a wavefront split.
template <int CM>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_PATH_WAVES_PER_EU, 8)))
k_trace(DevScene S, const float4* rays, const uint32_t* flags, uint32_t n, uint2* hits, uint32_t* work,
        uint32_t T)
{
    extern __shared__ uint32_t lds_stack[];
    float* stk = reinterpret_cast<float*>(lds_stack) + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    Counters cnt;
    bool busy = false, anyhit = false, exhausted = n == 0u;
    uint32_t ri = 0;
    f3 o = V(0, 0, 0), d = V(0, 0, 1), inv = V(0, 0, 0);
    Trav tr;
    trav_init(tr, 0.0f, 0.0f);
    const uint32_t nblk = (n + 63u) >> 6;   // 64-ray blocks, dealt to the shards round-robin
    for (;;) {
        // ---- refill the idle lanes (one atomic per wave and refill)
        uint32_t shard = shard_of_wave(), tried = 0;
        for (;;) {
            const uint64_t need = __ballot(!busy && !exhausted);
            if (need == 0) break;
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)need) - 1u;
            uint32_t base = 0;
            if (lane == leader) {
                const uint32_t head = atomicAdd(work + shard * 32u, (uint32_t)__popcll(need));
                base = head < (1u << 28) ? head : (1u << 28);
            }
            base = __shfl(base, (int)leader, 64);
            bool ran_out = false;
            if (!busy && !exhausted) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint32_t h = base + rank;
                const uint32_t blk = ((h >> 6) << RT_SHARD_LG) + shard;
                const uint32_t i = (blk << 6) | (h & 63u);
                if (blk >= nblk) {
                    ran_out = true;
                } else if (i < n) {
                    const float4 a = rays[2 * (size_t)i], b = rays[2 * (size_t)i + 1];   // o.xyz w.x | w.yz tmin tmax
                    o = V(a.x, a.y, a.z);
                    d = V(a.w, b.x, b.y);
                    anyhit = flags && (flags[i] & 1u);
                    inv = bsp_inv(d);
                    trav_start<RT_TRAVERSE_BSP>(tr, stk, b.z, b.w);
                    ri = i;
                    busy = true;
                }
            }
            if (__ballot(ran_out) != 0) {   // this shard is drained (its head only grows)
                shard = (shard + 1u) & ((1u << RT_SHARD_LG) - 1u);
                if (++tried == (1u << RT_SHARD_LG)) exhausted = true;
            }
        }
        if (__ballot(busy) == 0) break;
        // ---- trace until at most T lanes are busy (every lane, once the rays ran out)
        for (;;) {
            const uint64_t bm = __ballot(busy);
            if (bm == 0 || (!exhausted && (uint32_t)__popcll(bm) <= T)) break;
#pragma unroll
            for (int k = 0; k < RT_TRIPS_PER_CHECK; ++k) {
                if (busy && bsp_step<false, false, CM>(S, stk, o, d, inv, anyhit, tr, cnt)) {
                    busy = false;
                    const uint32_t hk = !tr.found ? 0xFFFFFFFFu : anyhit ? 0xFFFFFFFEu : tr.hit_k;
                    hits[ri] = make_uint2(hk, __float_as_uint(tr.tmax));
                }
            }
        }
    }
}

// ------------------------------------------------------------------ W6E2 / W7E1 / W7E2 kernel
// The Cornell-box direct-lighting worksheet shaders (w6e2.wgsl, w7e1.wgsl,
// w7e2.wgsl): the shader is always LAMBERTIAN, so a sample is one closest-hit
// ray plus one any-hit shadow ray per area-light triangle, and ends.  One
// lane per pixel (a trip-free walk per ray, as k_primary): these scenes have
// 36 triangles.  W6E2 averages subdiv^2 jittered samples (no progression);
// W7E1/W7E2 run iterations first_iter.. in order and fold each into the
// accumulation as fs_main does, without the max(., 0) of W7E3.
template <int MODE>
__device__ __forceinline__ Light direct_light(const DevScene& S, f3 pos, uint32_t idx, uint32_t& rng)
{
    // sample_area_light: w6e2.wgsl:245-262, w7e1.wgsl:327-346 (centre, no 1/d^2),
    // w7e2.wgsl:327-354 (random point, 1/d^2); cos_l unclamped in all three
    const uint32_t li = S.lights[idx < S.nlights ? idx : S.nlights - 1u];
    const uint4 tri = S.tri_idx[li < S.ntris ? li : S.ntris - 1u];
    const f3 v0 = ld3(S.pos[tri.x]), v1 = ld3(S.pos[tri.y]), v2 = ld3(S.pos[tri.z]);
    const f3 cr = cross(sub(v0, v1), sub(v0, v2));
    const float area = 0.5f * rt_det_sqrtf(dot(cr, cr));
    const f3 l_e = ld3(mat_of(S, tri.w).ambient);
    f3 point;
    if (MODE == RT_MODE_W7E2) {
        const float psi1 = rt_det_sqrtf(rnd(rng));
        const float psi2 = rnd(rng);
        const float alpha = 1.0f - psi1;
        const float beta = (1.0f - psi2) * psi1;
        const float gamma = psi2 * psi1;
        point = add(add(muls(v0, alpha), muls(v1, beta)), muls(v2, gamma));
    } else {
        point = divs(add(add(v0, v1), v2), 3.0f);
    }
    const f3 normal = normalize(cross(sub(v0, v1), sub(v0, v2)));
    const f3 ld = sub(point, pos);
    const float cos_l = dot(normalize(neg(ld)), normal);
    const float distance = rt_det_sqrtf(dot(ld, ld));
    Light L;
    L.l_i = muls(muls(l_e, area), cos_l);
    // W6E3 (w6e3.wgsl:298-318): the centre, with 1/d^2
    if (MODE == RT_MODE_W7E2 || MODE == RT_MODE_W6E3) L.l_i = divs(L.l_i, distance * distance);
    L.w_i = normalize(ld);
    L.dist = distance;
    return L;
}

template <int MODE, int TRAV, bool COUNT>
__device__ __forceinline__ f3 direct_sample(const DevScene& S, void* stk, const BvhDeep& dp, const f3 ro,
                                            const f3 rd, uint32_t& rng, uint32_t& prim, Counters& cnt)
{
    constexpr bool W6 = MODE == RT_MODE_W6E2, E2 = MODE == RT_MODE_W7E2;
    const float ETA = W6 ? 0.00001f : 0.001f;
    cnt.v[C_PRIMARY]++;
    TraceOut tr;
    if (!trace<TRAV, COUNT>(S, stk, dp, ro, rd, ETA, 5000.0f, false, tr, cnt))
        return W6 ? V(0.1f, 0.3f, 0.6f) : V(0.0f, 0.0f, 0.0f);   // result += bgcolor.rgb
    const HitRec h = resolve<TRAV>(S, tr, ro, rd, true);
    prim = h.tri;
    // lambertian: w6e2.wgsl:297-322 / w7e1.wgsl:385-410 / w7e2.wgsl:392-417
    const rt_material& m = mat_of(S, h.material);
    const f3 bdrf = ld3(m.diffuse);
    f3 diffuse = V(0, 0, 0);
    for (uint32_t idx = 1; idx < S.nlights; idx++) {
        const Light Lt = direct_light<MODE>(S, h.pos, idx, rng);
        const f3 so = E2 ? h.pos : add(h.pos, muls(muls(h.nrm, ETA), W6 ? 10.0f : 100.0f));
        const float stmax = E2 ? Lt.dist - ETA : Lt.dist - ETA * 1000.0f;
        cnt.v[C_SHADOW]++;
        TraceOut sh;
        if (trace<TRAV, COUNT>(S, stk, dp, so, Lt.w_i, ETA, stmax, true, sh, cnt)) continue;   // blocked
        const float dd = dot(h.nrm, Lt.w_i);
        if (E2) {
            diffuse = add(diffuse, divs(mul(mul(bdrf, V(dd, dd, dd)), Lt.l_i), RT_PI_F));
        } else {   // light_diffuse_contribution
            f3 c = divs(V(dd, dd, dd), Lt.dist * Lt.dist);
            c = mul(c, Lt.l_i);
            c = divs(c, RT_PI_F);
            diffuse = add(diffuse, mul(bdrf, c));
        }
    }
    if (E2) return add(diffuse, ld3(m.ambient));
    const f3 ambient = add(ld3(m.ambient), muls(ld3(m.diffuse), 0.1f));
    return add(muls(diffuse, 0.9f), muls(ambient, 0.1f));   // diffuse_and_ambient
}

// One sample of w6e3.wgsl's fs_main (:166-192): up to MAX_DEPTH 10 segments
// through intersect_scene_bsp (mirror ball, glossy ball with ior 1.5, then the
// mesh, :196-216).  Lambertian ends the sample; the mirror reflects from the
// hit point; glossy adds the Phong lobe over all lights and refracts
// (transmit), or ends with error_shader() under total internal reflection.
// `result` is fs_main's running sum over all samples and segments (the
// shader adds every segment's shade() to it in order).
template <int TRAV, bool COUNT>
__device__ __forceinline__ void w6e3_sample(const DevScene& S, const DevLaunch& L, void* stk, const BvhDeep& dp,
                                            f3 ro, f3 rd, uint32_t& prim, Counters& cnt, f3& result)
{
    const float ETA = 0.001f;
    uint32_t rng = 0;
    cnt.v[C_PRIMARY]++;
    for (int i = 0; i < 10; i++) {
        if (i > 0) cnt.v[C_BOUNCE]++;
        const W8Ball b = w8_balls(ro, rd, ETA, 5000.0f);
        TraceOut tr;
        if (trace<TRAV, COUNT>(S, stk, dp, ro, rd, ETA, b.t, false, tr, cnt)) {
            // lambertian, w6e3.wgsl:354-379
            const HitRec h = resolve<TRAV>(S, tr, ro, rd, true);
            if (i == 0) prim = h.tri;
            const rt_material& m = mat_of(S, h.material);
            const f3 bdrf = ld3(m.diffuse);
            f3 diffuse = V(0, 0, 0);
            for (uint32_t idx = 1; idx < S.nlights; idx++) {
                const Light Lt = direct_light<RT_MODE_W6E3>(S, h.pos, idx, rng);
                cnt.v[C_SHADOW]++;
                if (w8_balls(h.pos, Lt.w_i, ETA, Lt.dist - ETA).id != 0u) continue;   // a ball blocks
                TraceOut sh;
                if (trace<TRAV, COUNT>(S, stk, dp, h.pos, Lt.w_i, ETA, Lt.dist - ETA, true, sh, cnt)) continue;
                const float dd = dot(h.nrm, Lt.w_i);
                diffuse = add(diffuse, divs(mul(mul(bdrf, V(dd, dd, dd)), Lt.l_i), RT_PI_F));
            }
            result = add(result, add(diffuse, ld3(m.ambient)));
            break;
        }
        if (b.id == 1u) {
            // mirror, w6e3.wgsl:381-389: origin at the hit point
            rd = sub(rd, muls(b.nrm, 2.0f * dot(b.nrm, rd)));
            ro = b.pos;
            result = add(result, V(0, 0, 0));
            continue;
        }
        if (b.id == 2u) {
            // glossy = phong + transmit, w6e3.wgsl:391-457
            const f3 normal = b.nrm, position = b.pos;
            const float coeff = 0.9f * (42.0f + 2.0f) / (2.0f * RT_PI_F);
            const f3 w_o = normalize(sub(V(L.u.camera_pos[0], L.u.camera_pos[1], L.u.camera_pos[2]), position));
            f3 phong_total = V(0, 0, 0);
            for (uint32_t idx = 1; idx < S.nlights; idx++) {
                const Light Lt = direct_light<RT_MODE_W6E3>(S, position, idx, rng);
                const f3 nw = neg(Lt.w_i);
                const f3 w_r = normalize(sub(nw, muls(normal, 2.0f * dot(normal, nw))));
                const float dd = rt_satf(dot(normal, Lt.w_i));
                const f3 dif = divs(mul(V(dd, dd, dd), Lt.l_i), RT_PI_F);
                phong_total = add(phong_total, muls(dif, rt_det_powf(rt_satf(dot(w_o, w_r)), 42.0f)));
            }
            const f3 ph = muls(phong_total, coeff);
            // transmit
            const f3 w_i = neg(normalize(rd));
            const f3 n2 = normalize(normal);
            float ior = 1.5f;
            const float cos_i = dot(w_i, n2);
            f3 out_n;
            if (cos_i < 0.0f) {
                out_n = neg(n2);
            } else {
                ior = 1.0f / ior;
                out_n = n2;
            }
            const float cos_t2 = (1.0f - (ior * ior) * (1.0f - cos_i * cos_i));
            if (cos_t2 < 0.0f) {   // error_shader(); has_hit stays set
                result = add(result, add(ph, V(0.7f, 0.0f, 0.7f)));
                break;
            }
            const f3 tangent = sub(muls(n2, cos_i), w_i);
            rd = sub(muls(tangent, ior), muls(out_n, rt_det_sqrtf(cos_t2)));
            ro = position;
            result = add(result, add(ph, V(0, 0, 0)));
            continue;
        }
        result = add(result, V(0, 0, 0));   // BACKGROUND_COLOR (0, 0, 0)
        break;
    }
}

template <int MODE, int TRAV, bool COUNT>
__global__ void __launch_bounds__(256) k_direct(DevScene S, DevLaunch L)
{
    extern __shared__ uint32_t lds_stack[];
    void* stk = TRAV == RT_TRAVERSE_BVH ? lds_stack + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u)
                                        : lds_stack + threadIdx.x;
    const BvhDeep dp{TRAV == RT_TRAVERSE_BVH ? L.bvh_deep + (size_t)blockIdx.x * 256u + threadIdx.x : nullptr,
                     gridDim.x * 256u};
    const uint32_t lane = threadIdx.x & 63u;
    const Cam cam = make_cam(L);
    Counters cnt;
#pragma unroll
    for (int i = 0; i < C_N; i++) cnt.v[i] = 0;
    for (;;) {
        const uint32_t work = fetch_work(L.work_counter, lane);
        if (work >= L.nwork) break;
        const Pix px = map_pixel(L, work, lane);
        if (!px.valid) continue;
        float ux, uy;
        pixel_uv(L.u, px.x, px.y, ux, uy);
        uint32_t prim = 0xFFFFFFFFu;
        if (MODE == RT_MODE_W6E2 || MODE == RT_MODE_W6E3) {
            // fs_main, w6e2.wgsl:160-186 / w6e3.wgsl:166-192
            const uint32_t subdiv = L.u.subdivision_level, nsamp = subdiv * subdiv;
            f3 res = V(0, 0, 0);
            uint32_t rng = 0;
            cnt.v[C_SAMPLES]++;
            for (uint32_t s = 0; s < nsamp; s++) {
                const float jx = L.jitter ? L.jitter[2u * s] : 0.0f;
                const float jy = L.jitter ? L.jitter[2u * s + 1u] : 0.0f;
                uint32_t p = 0xFFFFFFFFu;
                const f3 rd0 = cam_dir(cam, ux, uy, jx, jy);
                if (MODE == RT_MODE_W6E3) w6e3_sample<TRAV, COUNT>(S, L, stk, dp, cam.e, rd0, p, cnt, res);
                else res = add(res, direct_sample<MODE, TRAV, COUNT>(S, stk, dp, cam.e, rd0, rng, p, cnt));
                if (s + 1u == nsamp) prim = p;
            }
            res = muls(res, 1.0f / (float)nsamp);
            L.accum[px.out] = make_float4(res.x, res.y, res.z, 1.0f);
        } else {
            // fs_main, w7e1.wgsl:202-236: iterations in order, folded as the shader does
            float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
            if (L.first_iter > 0u) {
                const float4 pa = L.accum[px.out];
                a0 = pa.x;
                a1 = pa.y;
                a2 = pa.z;
            }
            const float fH = (float)L.u.resolution[1];
            for (uint32_t k = 0; k < L.spp; k++) {
                const uint32_t it = L.first_iter + k;
                uint32_t rng = tea16(px.y * L.u.resolution[0] + px.x, it);
                float jx = rnd(rng);
                float jy = rnd(rng);
                jx = jx / fH;
                jy = jy / fH;
                cnt.v[C_SAMPLES]++;
                prim = 0xFFFFFFFFu;
                const f3 r = direct_sample<MODE, TRAV, COUNT>(S, stk, dp, cam.e, cam_dir(cam, ux, uy, jx, jy), rng, prim,
                                                              cnt);
                const float fi = (float)it, fi1 = (float)(it + 1u);
                a0 = (r.x + a0 * fi) / fi1;
                a1 = (r.y + a1 * fi) / fi1;
                a2 = (r.z + a2 * fi) / fi1;
            }
            L.accum[px.out] = make_float4(a0, a1, a2, 1.0f);
        }
        if (L.ids) L.ids[px.out] = prim;
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
    const Cam cam = make_cam(L);
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
        // t: the sequence position (map_pixel: rows rotated by their index mod 8)
        const uint32_t t = (uint32_t)(g >> 6), lane = (uint32_t)(g & 63u);
        const uint32_t ty = t / tiles_x;
        uint32_t tx = t - ty * tiles_x + (tiles_x >= 8u ? (ty & 7u) : 0u);
        tx = tx >= tiles_x ? tx - tiles_x : tx;
        const uint32_t x = tx * 8u + (lane & 7u), y = ty * 8u + (lane >> 3);
        if (x >= W || y >= H) continue;
        const uint32_t rank = t % nranks, l = t / nranks;
        const uint64_t src = ((uint64_t)rank * local_tiles + l) * 64u + lane;
        const uint64_t dst = (uint64_t)y * W + x;
        if (pa && fa) fa[dst] = pa[src];
        if (pi && fi) fi[dst] = pi[src];
    }
}

// ------------------------------------------------------------------ display frame
// fs_main's frame output (w7e3.wgsl:261-271, w9e1.wgsl:272-283):
// saturate(pow(accum, 1.5)), written to the sRGB surface (render_state.rs:
// 108-115, is_srgb()), i.e. encoded to 8-bit sRGB by the presentation engine.
// Pinned choices (the display path is outside the parity contract, SURVEY.md
// 8(a) a13): pow(x, 1.5) = x * sqrt(x); the 8-bit sRGB code is the exact
// rounding of 255 * srgb_oetf(v), found by counting the 255 code thresholds
// (computed on the host in double precision) that v reaches.
__global__ void __launch_bounds__(256) k_frame(const float4* accum, uint32_t npix, const float* thr, uchar4* out)
{
    __shared__ float t[256];
    t[threadIdx.x] = threadIdx.x < 255u ? thr[threadIdx.x] : 3.0e38f;
    __syncthreads();
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < npix; i += gridDim.x * 256u) {
        const float4 a = accum[i];
        const float c[3] = {a.x, a.y, a.z};
        unsigned char q[3];
        for (int k = 0; k < 3; k++) {
            const float x = c[k] > 0.0f ? c[k] : 0.0f;
            float v = x * rt_det_sqrtf(x);            // pow(x, 1.5)
            v = v < 1.0f ? v : 1.0f;                  // saturate
            uint32_t lo = 0, hi = 255;                // code = #thresholds <= v
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (t[mid] <= v) lo = mid + 1u;
                else hi = mid;
            }
            q[k] = (unsigned char)lo;
        }
        out[i] = make_uchar4(q[0], q[1], q[2], 255);
    }
}

int launch_frame(const float4* accum, uint32_t npix, const float* thr, uchar4* out, hipStream_t stream)
{
    uint64_t blocks = ((uint64_t)npix + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_frame, dim3((uint32_t)blocks), dim3(256), 0, stream, accum, npix, thr, out);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
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
    o[6] = (float)(uint32_t)((x < 0.0f ? -x : x) * 1000.0f) / (float)0x80000000u;
    o[7] = rt_det_acosf(rt_det_sqrtf(1.0f - (x - __builtin_floorf(x))));
    const float dd = 0.13f + (x < 0.0f ? -x : x) * 0.2f, xx = x * 37.1f + 0.3f;   // the BSP walk's fast exact division
    o[8] = rt_div_by_recip(xx, dd, 1.0f / dd);
    o[9] = xx / dd;
    o[10] = rt_det_atan2f(x, 1.3f - x * 0.9f);   // environment_map's atan2 (w9e1.wgsl:236)
    o[11] = rt_det_atanf(x * 5.0f);
    o[12] = rt_det_expf(x * 30.0f);    // over- and underflow at |x| > 2.96 / 3.47
    o[13] = rt_det_exp2f(x * 40.0f);   // the RGBE decode's pow(2, e) (w9e2.wgsl:244); subnormal below -126
    o[14] = rt_det_powf(rt_satf(x * 0.3f + 0.5f), 42.0f);   // the phong lobe pow(saturate(.), 42) (w6e3.wgsl:418)
    o[15] = rt_det_log2f(x < 0.0f ? -x * 1e-30f : x * 1e30f);
}
__global__ void k_selftest_math(const float* in, float* out, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) math_eval(in[i], out + (size_t)i * kMathOuts);
}
void camera_basis(const rt_uniform& u, float cam[14])
{
    auto nrm = [](float& x, float& y, float& z) {
        const float l = rt_det_sqrtf(x * x + y * y + z * z);
        x = x / l;
        y = y / l;
        z = z / l;
    };
    const float* e = u.camera_pos;
    float v[3] = {u.camera_look_at[0] - e[0], u.camera_look_at[1] - e[1], u.camera_look_at[2] - e[2]};
    nrm(v[0], v[1], v[2]);
    const float* up = u.camera_up;
    float b1[3] = {v[1] * up[2] - v[2] * up[1], v[2] * up[0] - v[0] * up[2], v[0] * up[1] - v[1] * up[0]};
    nrm(b1[0], b1[1], b1[2]);
    const float b2[3] = {b1[1] * v[2] - b1[2] * v[1], b1[2] * v[0] - b1[0] * v[2], b1[0] * v[1] - b1[1] * v[0]};
    for (int i = 0; i < 3; i++) {
        cam[i] = e[i];
        cam[3 + i] = v[i];
        cam[6 + i] = b1[i];
        cam[9 + i] = b2[i];
    }
    cam[12] = u.camera_constant;
    cam[13] = u.aspect_ratio;
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

size_t bvh_deep_bytes(int num_cus, int waves_per_cu)
{
    return (size_t)grid_for(num_cus, waves_per_cu) * 256u * (50u - RT_BVH_LDS_ENTRIES) * 4u;
}

template <int MODE, int TRAV, bool COUNT>
static void launch_path(const DevScene& s, const DevLaunch& l, int grid, size_t lds, hipStream_t st)
{
    // W9E1's and W7E3's BSP walks (configs 2-5) have a fast-margin instantiation: a context whose
    // culling is not certified (cull_k1 = 0: fast, or off with its +inf gap) skips the
    // certified terms (round 3's trip).  The other modes run the generic formula.
    if constexpr ((MODE == RT_MODE_W9E1 || MODE == RT_MODE_W7E3) && TRAV == RT_TRAVERSE_BSP) {
        if (s.cull_k1 == 0.0f) {
            hipLaunchKernelGGL((k_path<MODE, TRAV, COUNT, 0>), dim3(grid), dim3(256), lds, st, s, l);
            return;
        }
    }
    if constexpr (MODE == RT_MODE_W9E1 && TRAV == RT_TRAVERSE_BSP) {
        if (s.bsp_cull_mode == RT_BSP_CULL_SILHOUETTE) {
            hipLaunchKernelGGL((k_path<MODE, TRAV, COUNT, 2>), dim3(grid), dim3(256), lds, st, s, l);
            return;
        }
    }
    hipLaunchKernelGGL((k_path<MODE, TRAV, COUNT>), dim3(grid), dim3(256), lds, st, s, l);
}
template <int MODE, int TRAV, bool COUNT>
static void launch_direct(const DevScene& s, const DevLaunch& l, int grid, size_t lds, hipStream_t st)
{
    hipLaunchKernelGGL((k_direct<MODE, TRAV, COUNT>), dim3(grid), dim3(256), lds, st, s, l);
}
template <int TRAV, bool COUNT>
static void launch_primary(const DevScene& s, const DevLaunch& l, int project, int grid, size_t lds, hipStream_t st)
{
    hipLaunchKernelGGL((k_primary<TRAV, COUNT>), dim3(grid), dim3(256), lds, st, s, l, project);
}

int launch_render(const DevScene& s, const DevLaunch& l, rt_mode mode, rt_traverse trav, bool detail, int num_cus,
                  int waves_per_cu, hipStream_t stream)
{
    const size_t lds = trav == RT_TRAVERSE_BVH ? (size_t)RT_BVH_LDS_ENTRIES * 256 * 4
                                               : (size_t)(s.bsp_depth ? s.bsp_depth : 1) * 256 * 4;
    // a persistent grid larger than what fits at once (160 KiB LDS per CU)
    // would only add blocks that start after the queue ran dry
    const int lds_waves = 4 * (int)((160u * 1024u) / (lds ? lds : 1));
    // and by the register budget k_path is fitted to (waves per SIMD x 4 SIMDs)
    const int reg_waves = 4 * (trav == RT_TRAVERSE_BVH    ? RT_BVH_WAVES_PER_EU
                               : mode == RT_MODE_W7E3 ? RT_W7E3_WAVES_PER_EU
                                                      : RT_PATH_WAVES_PER_EU);
    const int grid = grid_for(num_cus, std::min(std::min(waves_per_cu > 0 ? waves_per_cu : 16, reg_waves),
                                                std::max(4, lds_waves)));
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
        if (l.u.selection1 == 7u) {
            if (bvh) detail ? launch_path<MODE_W9E1_TRANSPARENT, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                            : launch_path<MODE_W9E1_TRANSPARENT, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
            else detail ? launch_path<MODE_W9E1_TRANSPARENT, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                        : launch_path<MODE_W9E1_TRANSPARENT, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        } else {
            if (bvh) detail ? launch_path<RT_MODE_W9E1, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                            : launch_path<RT_MODE_W9E1, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
            else detail ? launch_path<RT_MODE_W9E1, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W9E1, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        }
        break;
    case RT_MODE_W9E3:
        if (bvh) detail ? launch_path<RT_MODE_W9E3, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W9E3, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_path<RT_MODE_W9E3, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_path<RT_MODE_W9E3, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W9E2:
        if (bvh) detail ? launch_path<RT_MODE_W9E2, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W9E2, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_path<RT_MODE_W9E2, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_path<RT_MODE_W9E2, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W8E1:
        if (bvh) detail ? launch_path<RT_MODE_W8E1, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W8E1, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_path<RT_MODE_W8E1, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_path<RT_MODE_W8E1, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W8E2:
        if (bvh) detail ? launch_path<RT_MODE_W8E2, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W8E2, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_path<RT_MODE_W8E2, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_path<RT_MODE_W8E2, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W8E3:
        if (bvh) detail ? launch_path<RT_MODE_W8E3, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_path<RT_MODE_W8E3, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_path<RT_MODE_W8E3, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_path<RT_MODE_W8E3, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W6E2:
        if (bvh) detail ? launch_direct<RT_MODE_W6E2, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_direct<RT_MODE_W6E2, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_direct<RT_MODE_W6E2, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_direct<RT_MODE_W6E2, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W6E3:
        if (bvh) detail ? launch_direct<RT_MODE_W6E3, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_direct<RT_MODE_W6E3, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_direct<RT_MODE_W6E3, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_direct<RT_MODE_W6E3, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W7E1:
        if (bvh) detail ? launch_direct<RT_MODE_W7E1, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_direct<RT_MODE_W7E1, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_direct<RT_MODE_W7E1, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_direct<RT_MODE_W7E1, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
        break;
    case RT_MODE_W7E2:
        if (bvh) detail ? launch_direct<RT_MODE_W7E2, RT_TRAVERSE_BVH, true>(s, l, grid, lds, stream)
                        : launch_direct<RT_MODE_W7E2, RT_TRAVERSE_BVH, false>(s, l, grid, lds, stream);
        else detail ? launch_direct<RT_MODE_W7E2, RT_TRAVERSE_BSP, true>(s, l, grid, lds, stream)
                    : launch_direct<RT_MODE_W7E2, RT_TRAVERSE_BSP, false>(s, l, grid, lds, stream);
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

int launch_query(const DevScene& s, rt_traverse trav, const float* rays, const uint32_t* flags, uint32_t n,
                 rt_ray_hit* out, uint32_t* bvh_deep, int num_cus, hipStream_t stream)
{
    const size_t lds = trav == RT_TRAVERSE_BVH ? (size_t)RT_BVH_LDS_ENTRIES * 256 * 4
                                               : (size_t)(s.bsp_depth ? s.bsp_depth : 1) * 256 * 4;
    uint32_t blocks = (n + 255u) / 256u;
    const uint32_t cap = (uint32_t)grid_for(num_cus, 16);
    if (blocks > cap) blocks = cap;
    if (blocks == 0) return 0;
    if (trav == RT_TRAVERSE_BVH)
        hipLaunchKernelGGL(k_query<RT_TRAVERSE_BVH>, dim3(blocks), dim3(256), lds, stream, s, rays, flags, n, out,
                           bvh_deep);
    else if (s.cull_k1 == 0.0f)   // the culling mode's formula, as the render kernels pick it (launch_path)
        hipLaunchKernelGGL((k_query<RT_TRAVERSE_BSP, 0>), dim3(blocks), dim3(256), lds, stream, s, rays, flags, n, out,
                           bvh_deep);
    else if (s.bsp_cull_mode == RT_BSP_CULL_SILHOUETTE)
        hipLaunchKernelGGL((k_query<RT_TRAVERSE_BSP, 2>), dim3(blocks), dim3(256), lds, stream, s, rays, flags, n, out,
                           bvh_deep);
    else
        hipLaunchKernelGGL((k_query<RT_TRAVERSE_BSP, 1>), dim3(blocks), dim3(256), lds, stream, s, rays, flags, n, out,
                           bvh_deep);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

int launch_trace_batch(const DevScene& s, const float* rays, const uint32_t* flags, uint32_t n, uint32_t* hits,
                       uint32_t* work, uint32_t threshold, int num_cus, hipStream_t stream)
{
    const size_t lds = (size_t)(s.bsp_depth ? s.bsp_depth : 1) * 256 * 4;
    const int lds_waves = 4 * (int)((160u * 1024u) / lds);
    const int grid = grid_for(num_cus, std::min(4 * RT_PATH_WAVES_PER_EU, std::max(4, lds_waves)));
    if (hipMemsetAsync(work, 0, 8 * 128, stream) != hipSuccess) return RT_E_DEVICE;
    const float4* r = reinterpret_cast<const float4*>(rays);
    uint2* h = reinterpret_cast<uint2*>(hits);
    if (s.cull_k1 == 0.0f)
        hipLaunchKernelGGL(k_trace<0>, dim3(grid), dim3(256), lds, stream, s, r, flags, n, h, work, threshold);
    else if (s.bsp_cull_mode == RT_BSP_CULL_SILHOUETTE)
        hipLaunchKernelGGL(k_trace<2>, dim3(grid), dim3(256), lds, stream, s, r, flags, n, h, work, threshold);
    else
        hipLaunchKernelGGL(k_trace<1>, dim3(grid), dim3(256), lds, stream, s, r, flags, n, h, work, threshold);
    return hipGetLastError() == hipSuccess ? 0 : RT_E_DEVICE;
}

int launch_fold(const DevLaunch& l, hipStream_t stream)
{
    const uint64_t nout = l.tileset ? (uint64_t)l.nwork * 64u : (uint64_t)l.w * l.h;
    uint64_t blocks = (nout + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_fold, dim3((uint32_t)blocks), dim3(256), 0, stream, l);
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
