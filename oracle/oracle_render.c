/*
 * oracle_render.c -- TEST INFRASTRUCTURE (see oracle.h header).
 *
 * Scalar f32 restatement of the per-pixel fragment shaders:
 *   res/shaders/bsp.wgsl   intersect_trimesh            :10-81
 *   res/shaders/aabb.wgsl  intersect_min_max            :8-31
 *   res/shaders/bvh.wgsl   intersect_bvh / intersect_bb2 :154-191 / :16-83
 *   res/shaders/w7e3.wgsl  fs_main, PRNG, lambertian, sample_area_light,
 *                          setup_indirect, rotate_to_normal, triangle test
 *   res/shaders/w9e1.wgsl  fs_main, lambertian (dummy light), environment escape
 *   res/shaders/w6e1.wgsl, project.wgsl  fs_main, lambertian (directional light)
 *   res/shaders/w1e6.wgsl  analytic scene
 * WGSL evaluates left to right and never contracts; compile with
 * -ffp-contract=off.  Vector helpers below are the component formulas the
 * shader builtins denote (dot = (x*x'+y*y')+z*z', normalize = v/sqrt(dot)).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "../include/rt_detmath.h"

typedef struct { float x, y, z; } v3;

static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static v3 muls(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static v3 divs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static v3 neg(v3 a) { return V(-a.x, -a.y, -a.z); }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 cross(v3 a, v3 b)
{
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static v3 normalize(v3 a) { return divs(a, rt_det_sqrtf(dot(a, a))); }
static float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static v3 load3(const float* p) { return V(p[0], p[1], p[2]); }

#define PI_F 3.14159265359f

typedef struct { v3 direction, origin; float tmax, tmin; } Ray;

typedef struct {
    int has_hit;
    float dist;
    v3 position, normal, factor;
    int emit;
    uint32_t material, tri;
    uint32_t shader;
} Hit;

typedef struct {
    const or_scene* s;
    const or_uniform* u;
    const float* jitter;
    int mode, trav;
    or_counts c;
    uint32_t* log;       /* or_trace_query: triangle ids in test order (NULL: off) */
    uint32_t log_cap, log_n;
    float* rlog;         /* or_render_raylog: every traced ray, 8 floats (NULL: off) */
    uint32_t rlog_cap, rlog_n;
} Ctx;

/* ------------------------------------------------------------ PRNG (w7e3.wgsl:141-172) */
static uint32_t tea16(uint32_t v0, uint32_t v1)
{
    uint32_t s0 = 0;
    for (int n = 0; n < 16; n++) {
        s0 += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
static uint32_t mcg31(uint32_t* prev)
{
    *prev = (1977654935u * *prev) & 0x7FFFFFFFu;
    return *prev;
}
static float rnd(uint32_t* prev) { return (float)mcg31(prev) / (float)0x80000000u; }

/* ------------------------------------------------------------ triangle test
 * intersect_triangle_indexed, w7e3.wgsl:286-332 / w9e1.wgsl:297-339 /
 * project.wgsl:193-235.  face_normals: W7E3 uses n0=n1=n2=cross(e0,e1). */
static int tri_test(Ctx* C, Ray* r, Hit* h, uint32_t v, int face_normals)
{
    const or_scene* s = C->s;
    C->c.tri_tests++;
    if (C->log) {
        if (C->log_n < C->log_cap) C->log[C->log_n] = v;
        C->log_n++;
    }
    const uint32_t* ix = s->idx + 4 * (size_t)v;
    v3 v0 = load3(s->pos + 4 * (size_t)ix[0]);
    v3 v1 = load3(s->pos + 4 * (size_t)ix[1]);
    v3 v2 = load3(s->pos + 4 * (size_t)ix[2]);
    Ray ray = *r;
    v3 w_i = ray.direction, o = ray.origin;
    v3 e0 = sub(v1, v0), e1 = sub(v2, v0), o_to_v0 = sub(v0, o);
    v3 normal = cross(e0, e1);
    v3 nom = cross(o_to_v0, w_i);
    float denom = dot(w_i, normal);
    if (C->mode == OR_MODE_W9E3) {   /* w9e3.wgsl:328: back faces and grazing hits rejected */
        if (rt_absf(denom) < 0.00005f || denom > 0.0f) return 0;
    } else if (rt_absf(denom) < 1e-10f) {
        return 0;
    }
    float beta = dot(nom, e1) / denom;
    float gamma = -dot(nom, e0) / denom;
    float distance = dot(o_to_v0, normal) / denom;
    if (beta < 0.0f || gamma < 0.0f || beta + gamma > 1.0f || distance > ray.tmax || distance < ray.tmin)
        return 0;
    C->c.tri_accepts++;
    v3 n0, n1, n2;
    if (face_normals) {
        n0 = n1 = n2 = normal;
    } else {
        n0 = load3(s->nrm + 4 * (size_t)ix[0]);
        n1 = load3(s->nrm + 4 * (size_t)ix[1]);
        n2 = load3(s->nrm + 4 * (size_t)ix[2]);
    }
    r->tmax = distance;
    h->dist = distance;
    h->position = add(o, muls(w_i, distance));   /* ray_at */
    if (C->mode == OR_MODE_W9E3)   /* w9e3.wgsl:343: ETA (1e-4) on every weight */
        h->normal = normalize(add(add(muls(n0, 1.0f - beta - gamma + 0.0001f), muls(n1, beta + 0.0001f)),
                                  muls(n2, gamma + 0.0001f)));
    else
        h->normal = normalize(add(add(muls(n0, 1.0f - beta - gamma), muls(n1, beta)), muls(n2, gamma)));
    h->material = ix[3];
    h->tri = v;
    return 1;
}

/* ------------------------------------------------------------ BSP, bsp.wgsl:10-81 */
static int trace_bsp(Ctx* C, Ray* r, Hit* h, int face_normals)
{
    const or_scene* s = C->s;
    const uint32_t MAX_LEVEL = s->max_depth;
    uint32_t branch_node[2 * 32];
    float branch_ray[2 * 32];
    uint32_t branch_lvl = 0, near_node = 0, far_node = 0, node = 0;
    float t = 0.0f;
    for (uint32_t i = 0; i <= MAX_LEVEL; i++) {
        const uint32_t* tn = s->tree + 4 * (size_t)node;
        uint32_t axis_leaf = tn[0] & 3u;
        if (axis_leaf == 3u) {
            C->c.node_leaf++;
            uint32_t count = tn[0] >> 2, first = tn[1];
            int found = 0;
            for (uint32_t j = 0; j < count; j++) {
                C->c.ids_read++;
                uint32_t obj = s->ids[first + j];
                if (tri_test(C, r, h, obj, face_normals)) {
                    r->tmax = h->dist;
                    found = 1;
                }
            }
            if (found) return 1;
            if (branch_lvl == 0) return 0;
            branch_lvl--;
            i = branch_node[2 * branch_lvl];
            node = branch_node[2 * branch_lvl + 1];
            r->tmin = branch_ray[2 * branch_lvl];
            r->tmax = branch_ray[2 * branch_lvl + 1];
            continue;
        }
        C->c.node_interior++;
        float axis_direction = comp(r->direction, (int)axis_leaf);
        float axis_origin = comp(r->origin, (int)axis_leaf);
        if (axis_direction >= 0.0f) {
            near_node = tn[2];
            far_node = tn[3];
        } else {
            near_node = tn[3];
            far_node = tn[2];
        }
        float node_plane = s->planes[node];
        float denom = rt_absf(axis_direction) < 1.0e-8f ? 1.0e-8f : axis_direction;
        t = (node_plane - axis_origin) / denom;
        if (t > r->tmax) {
            node = near_node;
        } else if (t < r->tmin) {
            node = far_node;
        } else {
            branch_node[2 * branch_lvl] = i;
            branch_node[2 * branch_lvl + 1] = far_node;
            branch_ray[2 * branch_lvl] = t;
            branch_ray[2 * branch_lvl + 1] = r->tmax;
            branch_lvl++;
            r->tmax = t;
            node = near_node;
        }
    }
    return 0;
}

/* ------------------------------------------------------------ BVH, bvh.wgsl:16-83, 154-191 */
static int intersect_bb2(v3 inv, v3 o, const or_gpu_node* b)
{
    float t0 = 0.0f, t1 = 1e27f;
    v3 nr = mul(sub(load3(b->min), o), inv);
    v3 fr = mul(sub(load3(b->max), o), inv);
    const int order[3] = {1, 0, 2};   /* y, x, z */
    for (int k = 0; k < 3; k++) {
        float tn = comp(nr, order[k]), tf = comp(fr, order[k]);
        if (tn > tf) {
            float tmp = tn;
            tn = tf;
            tf = tmp;
        }
        if (tn > t0) t0 = tn;
        if (tf < t1) t1 = tf;
        if (t0 > t1) return 0;
    }
    return 1;
}

static int trace_bvh(Ctx* C, Ray* r, Hit* h, int face_normals)
{
    const or_scene* s = C->s;
    v3 inv = V(1.0f / r->direction.x, 1.0f / r->direction.y, 1.0f / r->direction.z);
    v3 orig = r->origin;
    uint32_t stack[50];
    uint32_t top = 0;
    int found = 0;
    /* stack_push_node: WGSL clamps an out-of-range index to the last element */
    stack[top < 50 ? top : 49] = 0;
    top++;
    for (uint32_t depth = 0; depth < 1000u; depth++) {
        if (top == 0) break;
        top--;
        uint32_t cur = stack[top < 50 ? top : 49];
        C->c.bvh_pops++;
        const or_gpu_node* n = &s->bvh_nodes[cur];
        if (intersect_bb2(inv, orig, n)) {
            uint32_t off = n->offset_ptr;
            if (n->n_prims > 0) {
                for (uint32_t i = 0; i < n->n_prims; i++) {
                    C->c.ids_read++;
                    uint32_t obj = s->bvh_ids[off + i];
                    if (tri_test(C, r, h, obj, face_normals)) {
                        r->tmax = h->dist;
                        found = 1;
                    }
                }
            } else {
                stack[top < 50 ? top : 49] = cur + 1;
                top++;
                stack[top < 50 ? top : 49] = off;
                top++;
            }
        }
    }
    return found;
}

static int trace(Ctx* C, Ray* r, Hit* h, int face_normals)
{
    if (C->rlog) {   /* or_render_raylog: the ray as the walk receives it */
        if (C->rlog_n < C->rlog_cap) {
            float* q = C->rlog + 8 * (size_t)C->rlog_n;
            q[0] = r->origin.x; q[1] = r->origin.y; q[2] = r->origin.z;
            q[3] = r->direction.x; q[4] = r->direction.y; q[5] = r->direction.z;
            q[6] = r->tmin; q[7] = r->tmax;
        }
        C->rlog_n++;
    }
    return C->trav == OR_TRAV_BVH ? trace_bvh(C, r, h, face_normals) : trace_bsp(C, r, h, face_normals);
}

/* ------------------------------------------------------------ camera (w7e3.wgsl:211-228) */
typedef struct { v3 e, v, b1, b2; float d, aspect; } Cam;

static Cam make_cam(const or_uniform* u)
{
    Cam c;
    c.e = load3(u->camera_pos);
    v3 p = load3(u->camera_look_at), up = load3(u->camera_up);
    c.v = normalize(sub(p, c.e));
    c.d = u->camera_constant;
    c.aspect = u->aspect_ratio;
    c.b1 = normalize(cross(c.v, up));
    c.b2 = cross(c.b1, c.v);
    return c;
}
static v3 cam_dir(const Cam* c, float ux, float uy, float jx, float jy)
{
    /* normalize(b1 * (uv.x + j_x) * aspect + b2 * (uv.y + j_y) + v*d) */
    return normalize(add(add(muls(muls(c->b1, ux + jx), c->aspect), muls(c->b2, uy + jy)), muls(c->v, c->d)));
}
static void pixel_uv(const or_uniform* u, uint32_t x, uint32_t y, float* ux, float* uy)
{
    /* uv = coords * 0.5 with coords the NDC of the pixel centre (vs_main + rasteriser) */
    *ux = ((float)x + 0.5f) / (float)u->resolution[0] - 0.5f;
    *uy = 0.5f - ((float)y + 0.5f) / (float)u->resolution[1];
}

static const or_material* mat_of(const or_scene* s, uint32_t m)
{
    /* WGSL runtime-array index is clamped to the last element (naga Restrict) */
    return &s->mats[m < s->nmats ? m : s->nmats - 1];
}

/* ------------------------------------------------------------ W7E3 / W9E1 */

static v3 rotate_to_normal(v3 normal, v3 v)   /* w7e3.wgsl:181-189 */
{
    float signbit = rt_signf(normal.z + 1.0e-16f);
    float a = -1.0f / (1.0f + rt_absf(normal.z));
    float b = normal.x * normal.y * a;
    v3 c0 = V(1.0f + normal.x * normal.x * a, b, -signbit * normal.x);
    v3 c1 = V(signbit * b, signbit * (1.0f + normal.y * normal.y * a), -normal.y);
    return add(add(muls(c0, v.x), muls(c1, v.y)), muls(normal, v.z));
}

static void setup_indirect(Ray* r, Hit* h, uint32_t* t, float eta)   /* w7e3.wgsl:472-489 */
{
    v3 normal = normalize(h->normal);
    float xi1 = rnd(t);
    float xi2 = rnd(t);
    float thet = rt_det_acosf(rt_det_sqrtf(1.0f - xi1));
    float phi = 2.0f * PI_F * xi2;
    float st = rt_det_sinf(thet), ct = rt_det_cosf(thet);
    v3 tang = V(st * rt_det_cosf(phi), st * rt_det_sinf(phi), ct);   /* spherical_direction */
    r->direction = rotate_to_normal(normal, tang);
    r->origin = h->position;
    r->tmin = eta;
    r->tmax = 5000.0f;
    h->has_hit = 0;
    h->emit = 0;
}

static float triangle_area(v3 v0, v3 v1, v3 v2)   /* w7e3.wgsl:133-138 */
{
    v3 cr = cross(sub(v0, v1), sub(v0, v2));
    return 0.5f * rt_det_sqrtf(dot(cr, cr));
}

typedef struct { v3 l_i, w_i; float dist; } Light;

static Light sample_area_light(const or_scene* s, v3 pos, uint32_t idx, uint32_t* rand)
{
    /* w7e3.wgsl:362-389 */
    uint32_t li = s->lights[idx < s->nlights ? idx : s->nlights - 1];
    const uint32_t* tri = s->idx + 4 * (size_t)(li < s->ntris ? li : s->ntris - 1);
    v3 v0 = load3(s->pos + 4 * (size_t)tri[0]);
    v3 v1 = load3(s->pos + 4 * (size_t)tri[1]);
    v3 v2 = load3(s->pos + 4 * (size_t)tri[2]);
    float area = triangle_area(v0, v1, v2);
    v3 l_e = load3(mat_of(s, tri[3])->ambient);
    float psi1 = rt_det_sqrtf(rnd(rand));
    float psi2 = rnd(rand);
    float alpha = 1.0f - psi1;
    float beta = (1.0f - psi2) * psi1;
    float gamma = psi2 * psi1;
    v3 normal = normalize(cross(sub(v0, v1), sub(v0, v2)));
    v3 sampled = add(add(muls(v0, alpha), muls(v1, beta)), muls(v2, gamma));
    v3 ld = sub(sampled, pos);
    float cos_l = rt_maxf(dot(normalize(neg(ld)), normal), 0.0f);
    float distance = rt_det_sqrtf(dot(ld, ld));
    Light L;
    L.l_i = divs(muls(muls(l_e, area), cos_l), distance * distance);
    L.w_i = normalize(ld);
    L.dist = distance;
    return L;
}

static v3 shade_w7e3(Ctx* C, Ray* r, Hit* h, uint32_t* t)
{
    /* shade (:391-425) -> lambertian (:427-470) */
    const or_scene* s = C->s;
    const float ETA = 0.01f;
    h->has_hit = 1;
    const or_material* m = mat_of(s, h->material);
    v3 brdf = divs(load3(m->diffuse), PI_F);
    v3 emission = load3(m->ambient);
    v3 diffuse = V(0, 0, 0), ambient = V(0, 0, 0);
    v3 normal = h->normal;
    uint32_t light_tris = s->nlights - 1u;
    uint32_t ri = mcg31(t);
    uint32_t idx = (light_tris ? ri % light_tris : 0u) + 1u;
    Light L = sample_area_light(s, h->position, idx, t);
    Ray sr;
    sr.direction = L.w_i;
    sr.origin = h->position;
    sr.tmax = L.dist - ETA;
    sr.tmin = ETA;
    Hit hi;
    memset(&hi, 0, sizeof hi);
    C->c.shadow++;
    int blocked = trace(C, &sr, &hi, 1);
    if (!blocked)
        diffuse = muls(mul(muls(brdf, rt_satf(dot(normal, L.w_i))), L.l_i), (float)light_tris);
    if (h->emit) ambient = emission;
    diffuse = mul(diffuse, h->factor);
    h->factor = mul(h->factor, muls(brdf, PI_F));
    float prob = (brdf.x + brdf.y + brdf.z) / 3.0f;
    float step = rnd(t);
    if (step < prob) {
        setup_indirect(r, h, t, ETA);
        h->factor = divs(h->factor, prob);
    }
    return add(diffuse, ambient);
}

/* ------------------------------------------------------------ W9E2 additions
 * res/shaders/w9e2.wgsl: the holdout plane y = 0 tested before the mesh, its
 * ambient-occlusion shader, and the RGBE environment decode. */
#define SH_HOLDOUT 8u

static v3 env_lookup(Ctx* C, v3 d)   /* environment_map, w9e1.wgsl:232-239 / w9e2.wgsl:234-246 */
{
    v3 e = load3(C->s->env);
    if (C->s->env_tex) {
        float rgb[3];
        if (C->mode == OR_MODE_W9E2)
            rt_det_env_sample_rgbe(C->s->env_tex, C->s->env_w, C->s->env_h, d.x, d.y, d.z, rgb);
        else
            rt_det_env_sample(C->s->env_tex, C->s->env_w, C->s->env_h, d.x, d.y, d.z, rgb);
        e = V(rgb[0], rgb[1], rgb[2]);
    }
    return e;
}

static int intersect_plane_w9e2(Ray* r, Hit* h)   /* intersect_plane, w9e2.wgsl:388-404 */
{
    v3 normal = V(0.0f, 1.0f, 0.0f), position = V(0.0f, 0.0f, 0.0f);
    float distance = dot(sub(position, r->origin), normal) / dot(r->direction, normal);
    if (distance < r->tmin || distance > r->tmax) return 0;
    r->tmax = distance;
    h->dist = distance;
    h->position = add(r->origin, muls(r->direction, distance));
    h->normal = normal;
    return 1;
}

static int intersect_scene_w9e2(Ctx* C, Ray* r, Hit* h)   /* intersect_scene_bsp, w9e2.wgsl:290-304 */
{
    int has_hit = 0;
    if (intersect_plane_w9e2(r, h)) {
        h->shader = SH_HOLDOUT;
        has_hit = 1;
    }
    if (trace(C, r, h, 0)) {
        h->shader = C->u->selection1;
        has_hit = 1;
    }
    return has_hit;
}

static v3 holdout_w9e2(Ctx* C, Ray* r, Hit* h, uint32_t* t)   /* holdout_shader, w9e2.wgsl:514-537 */
{
    const float ETA = 0.0001f;
    Ray ao;
    Hit hi;
    memset(&hi, 0, sizeof hi);
    v3 normal = normalize(h->normal);
    float xi1 = rnd(t);
    float xi2 = rnd(t);
    float thet = rt_det_acosf(rt_det_sqrtf(1.0f - xi1));
    float phi = 2.0f * PI_F * xi2;
    float st = rt_det_sinf(thet), ct = rt_det_cosf(thet);
    v3 tang = V(st * rt_det_cosf(phi), st * rt_det_sinf(phi), ct);
    ao.direction = rotate_to_normal(normal, tang);
    ao.origin = h->position;
    ao.tmin = ETA;
    ao.tmax = 5000.0f;
    C->c.shadow++;
    /* intersect_trimesh_immediate_return (bsp.wgsl:83-155): the same walk as
     * intersect_trimesh up to its first accepted triangle, so the same boolean */
    if (trace(C, &ao, &hi, 0)) return V(0, 0, 0);
    h->has_hit = 1;
    return mul(env_lookup(C, r->direction), h->factor);
}

static Light sun_light_w9e3(void)   /* sample_directional_light, w9e3.wgsl:405-414 */
{
    Light L;
    L.l_i = V(10.0f, 10.0f, 10.0f);
    L.w_i = neg(normalize(V(1.0f, -0.35f, 0.0f)));
    L.dist = 999999.0f;
    return L;
}

static v3 holdout_w9e3(Ctx* C, Ray* r, Hit* h, uint32_t* t)   /* holdout_shader, w9e3.wgsl:490-517 */
{
    const float ETA = 0.0001f;
    float contribution = 1.0f;
    v3 normal = normalize(h->normal);
    float xi1 = rnd(t);
    float xi2 = rnd(t);
    float thet = rt_det_acosf(rt_det_sqrtf(1.0f - xi1));
    float phi = 2.0f * PI_F * xi2;
    float st = rt_det_sinf(thet), ct = rt_det_cosf(thet);
    v3 tang = V(st * rt_det_cosf(phi), st * rt_det_sinf(phi), ct);
    v3 direct_dir = rotate_to_normal(normal, tang);
    v3 color = mul(env_lookup(C, r->direction), h->factor);
    Hit hi;
    memset(&hi, 0, sizeof hi);
    Ray ray;
    ray.direction = direct_dir;   /* ray_init */
    ray.origin = h->position;
    ray.tmax = 5000.0f;
    ray.tmin = ETA;
    C->c.shadow++;
    if (intersect_scene_w9e2(C, &ray, &hi)) contribution -= 0.5f;
    Light L = sun_light_w9e3();
    ray.direction = L.w_i;
    ray.origin = h->position;
    ray.tmax = 5000.0f;
    ray.tmin = ETA;
    C->c.shadow++;
    if (intersect_scene_w9e2(C, &ray, &hi)) contribution -= 0.5f;
    h->has_hit = 1;
    return muls(color, contribution);
}

static v3 shade_w9e1(Ctx* C, Ray* r, Hit* h, uint32_t* t)
{
    /* shade (w9e1.wgsl) with selection1; lambertian with light_init() (:428-470) */
    const or_scene* s = C->s;
    const float ETA = 0.0001f;
    h->has_hit = 1;
    if (C->mode == OR_MODE_W9E2 && h->shader == SH_HOLDOUT) return holdout_w9e2(C, r, h, t);
    if (C->mode == OR_MODE_W9E3 && h->shader == SH_HOLDOUT) return holdout_w9e3(C, r, h, t);
    const or_material* m = mat_of(s, h->material);
    uint32_t selc = C->u->selection1;
    if (C->mode == OR_MODE_W9E3) selc = selc == 3u ? 7u : (selc == 7u ? 0xFFu : selc);   /* transparent is case 3 */
    switch (selc) {
    case 0: {
        v3 brdf = divs(load3(m->diffuse), PI_F);
        v3 emission = load3(m->ambient);
        v3 diffuse = V(0, 0, 0), ambient = V(0, 0, 0);
        v3 normal = h->normal;
        Light L;   /* light_init(), w9e1.wgsl:67-73 */
        L.l_i = V(0, 0, 0);
        L.w_i = V(0.0f, 1.0f, 0.0f);
        L.dist = 999999.0f;
        if (C->mode == OR_MODE_W9E3) L = sun_light_w9e3();
        Ray sr;
        sr.direction = L.w_i;
        sr.origin = h->position;
        sr.tmax = L.dist - ETA;
        sr.tmin = ETA;
        Hit hi;
        memset(&hi, 0, sizeof hi);
        C->c.shadow++;
        int blocked = (C->mode == OR_MODE_W9E2 || C->mode == OR_MODE_W9E3) ? intersect_scene_w9e2(C, &sr, &hi)
                                                                          : trace(C, &sr, &hi, 0);
        if (!blocked) diffuse = mul(muls(brdf, rt_satf(dot(normal, L.w_i))), L.l_i);
        if (h->emit) ambient = mul(emission, h->factor);
        diffuse = mul(diffuse, h->factor);
        h->factor = mul(h->factor, muls(brdf, PI_F));
        float prob = (brdf.x + brdf.y + brdf.z) / 3.0f;
        float step = rnd(t);
        if (step < prob) {
            setup_indirect(r, h, t, ETA);
            h->factor = divs(h->factor, prob);
        }
        return add(diffuse, ambient);
    }
    case 2: {   /* mirror, w9e1.wgsl:491-504 (+ emit = true) */
        v3 n = h->normal, d = r->direction;
        v3 rd = sub(d, muls(n, 2.0f * dot(n, d)));   /* reflect(e1, e2) = e1 - 2 dot(e2,e1) e2 */
        r->origin = add(h->position, muls(n, ETA));
        r->direction = rd;
        r->tmax = 5000.0f;
        r->tmin = ETA;
        h->has_hit = 0;
        h->emit = 1;
        return V(0, 0, 0);
    }
    case 5:
        return muls(add(h->normal, V(1.0f, 1.0f, 1.0f)), 0.5f);
    case 6:
        return add(load3(m->diffuse), load3(m->ambient));
    case 7: {   /* transparent, w9e1.wgsl:505-558; hit_record_init: ior1_over_ior2 1.0, extinction (1,1,1) */
        v3 w_i = neg(normalize(r->direction));
        v3 normal = normalize(h->normal);
        v3 out_normal;
        float ior = C->mode == OR_MODE_W9E3 ? 1.5f : 1.0f;   /* W9E3 sets ior1_over_ior2 = 1.5 on mesh hits */
        float cos_i = dot(w_i, normal);
        float absorption = 0.0f;
        v3 extinction = V(1.0f, 1.0f, 1.0f);
        if (cos_i < 0.0f) {
            cos_i = dot(w_i, neg(normal));
            out_normal = neg(normal);
        } else {
            ior = 1.0f / ior;
            out_normal = normal;
            v3 dd = sub(h->position, r->origin);
            float sd = rt_det_sqrtf(dot(dd, dd));                     /* length() */
            v3 nr = neg(extinction);
            v3 tr = V(rt_det_expf(nr.x * sd), rt_det_expf(nr.y * sd), rt_det_expf(nr.z * sd));
            absorption = 1.0f - (tr.x + tr.y + tr.z) / 3.0f;
        }
        float cos_t2 = (1.0f - (ior * ior) * (1.0f - cos_i * cos_i));
        float refl;
        if (cos_t2 < 0.0f) {
            refl = 1.0f;
        } else {   /* fresnel_r, w9e1.wgsl:191-201 */
            float ct = rt_det_sqrtf(cos_t2);
            float ii = ior * cos_i, tt = 1.0f * ct, ti = 1.0f * cos_i, it = ior * ct;
            float r1 = (ii - tt) / (ii + tt), r2 = (ti - it) / (ti + it);
            refl = 0.5f * (r1 * r1 + r2 * r2);
        }
        v3 tangent = sub(muls(out_normal, cos_i), w_i);
        v3 w_t = sub(muls(tangent, ior), muls(normalize(out_normal), rt_det_sqrtf(cos_t2)));
        r->direction = w_t;            /* ray_init(w_t, position) */
        r->origin = h->position;
        r->tmax = 5000.0f;
        r->tmin = ETA;
        h->has_hit = 0;
        h->emit = 1;
        float step = rnd(t);
        if (step < refl) {             /* mirror(r, hit) with hit.normal = out_normal */
            h->normal = out_normal;
            v3 n = h->normal, d = r->direction;
            v3 rd = sub(d, muls(n, 2.0f * dot(n, d)));
            r->origin = add(h->position, muls(n, ETA));
            r->direction = rd;
            r->tmax = 5000.0f;
            r->tmin = ETA;
            return V(0, 0, 0);
        }
        float step1 = rnd(t);
        if (step1 < absorption) h->factor = mul(h->factor, divs(extinction, absorption));
        return V(0, 0, 0);
    }
    default:
        return V(0.7f, 0.0f, 0.7f);
    }
}

/* ------------------------------------------------------------ W8E1 / W8E2 / W8E3
 * Cornell box with two analytic balls (res/shaders/w8e1.wgsl, w8e2.wgsl,
 * w8e3.wgsl).  Rays that turn NaN (sqrt of a negative cos_t^2 under total
 * internal reflection, reflected) follow IEEE comparison semantics
 * throughout, as the kernel does. */
enum { SH_LAMBERTIAN = 0, SH_MIRROR = 2, SH_TRANSPARENT = 7 };

static int intersect_sphere(Ray* r, Hit* h, v3 center, float radius)   /* w8e1.wgsl:352-376 */
{
    v3 oc = sub(r->origin, center);
    float a = dot(r->direction, r->direction);
    float b_over_2 = dot(oc, r->direction);
    float c = dot(oc, oc) - radius * radius;
    float discriminant = b_over_2 * b_over_2 - a * c;
    if (discriminant < 0.0f) return 0;
    float disc_sqrt = rt_det_sqrtf(discriminant);
    float root = (-b_over_2 - disc_sqrt) / a;
    if (root < r->tmin || root > r->tmax) {
        root = (-b_over_2 + disc_sqrt) / a;
        if (root < r->tmin || root > r->tmax) return 0;
    }
    r->tmax = root;
    h->dist = root;
    h->position = add(r->origin, muls(r->direction, root));   /* ray_at */
    h->normal = normalize(sub(h->position, center));
    return 1;
}

static int intersect_scene_w8(Ctx* C, Ray* r, Hit* h)   /* intersect_scene_bsp, w8e1.wgsl:244-262 */
{
    int has_hit = 0;
    if (intersect_sphere(r, h, V(420.0f, 90.0f, 370.0f), 90.0f)) {
        h->shader = SH_MIRROR;
        has_hit = 1;
    }
    if (intersect_sphere(r, h, V(130.0f, 90.0f, 250.0f), 90.0f)) {
        h->shader = SH_TRANSPARENT;   /* ior1_over_ior2 1.5; W8E3: extinction (0.5, 0.2, 0.2) */
        has_hit = 1;
    }
    if (trace(C, r, h, 1)) {
        h->shader = SH_LAMBERTIAN;
        has_hit = 1;
    }
    return has_hit;
}

static v3 lambertian_w8(Ctx* C, Ray* r, Hit* h, uint32_t* t)
{
    /* w8e1.wgsl:406-435; w8e2.wgsl:444-489 adds factor, Russian roulette and
     * setup_indirect; w8e3.wgsl scales diffuse and ambient by factor in place */
    const or_scene* s = C->s;
    const float ETA = 0.01f;
    const int e3 = C->mode == OR_MODE_W8E3;
    const or_material* m = mat_of(s, h->material);
    v3 brdf = divs(load3(m->diffuse), PI_F);
    v3 emission = load3(m->ambient);
    v3 diffuse = V(0, 0, 0), ambient = V(0, 0, 0);
    v3 normal = h->normal;
    uint32_t light_tris = s->nlights - 1u;
    uint32_t ri = mcg31(t);
    uint32_t idx = (light_tris ? ri % light_tris : 0u) + 1u;
    Light L = sample_area_light(s, h->position, idx, t);
    Ray sr;
    sr.direction = L.w_i;
    sr.origin = h->position;
    sr.tmax = L.dist - ETA;
    sr.tmin = ETA;
    Hit hi;
    memset(&hi, 0, sizeof hi);
    C->c.shadow++;
    int blocked = intersect_scene_w8(C, &sr, &hi);
    if (!blocked) {
        diffuse = muls(mul(muls(brdf, rt_satf(dot(normal, L.w_i))), L.l_i), (float)light_tris);
        if (e3) diffuse = mul(diffuse, h->factor);
    }
    if (h->emit) ambient = e3 ? mul(emission, h->factor) : emission;
    if (C->mode == OR_MODE_W8E1) return add(diffuse, ambient);
    if (!e3) diffuse = mul(diffuse, h->factor);
    h->factor = mul(h->factor, muls(brdf, PI_F));
    float prob = (brdf.x + brdf.y + brdf.z) / 3.0f;
    float step = rnd(t);
    if (step < prob) {
        setup_indirect(r, h, t, ETA);
        h->factor = divs(h->factor, prob);
    }
    return add(diffuse, ambient);
}

static v3 mirror_w8(Ctx* C, Ray* r, Hit* h)   /* w8e1.wgsl:437-445 / w8e2.wgsl:509-522 */
{
    const float ETA = 0.01f;
    v3 n = h->normal, d = r->direction;
    r->direction = sub(d, muls(n, 2.0f * dot(n, d)));   /* reflect */
    r->origin = C->mode == OR_MODE_W8E1 ? h->position : add(h->position, muls(n, ETA));
    r->tmax = 5000.0f;
    r->tmin = ETA;
    h->has_hit = 0;
    if (C->mode != OR_MODE_W8E1) h->emit = 1;
    return V(0, 0, 0);
}

static float fresnel_r(float cos_i, float cos_t, float ni_over_nt)   /* w8e2.wgsl:202-212 */
{
    float ii = ni_over_nt * cos_i, tt = 1.0f * cos_t, ti = 1.0f * cos_i, it = ni_over_nt * cos_t;
    float r1 = (ii - tt) / (ii + tt), r2 = (ti - it) / (ti + it);
    return 0.5f * (r1 * r1 + r2 * r2);
}

static v3 transparent_w8(Ctx* C, Ray* r, Hit* h, uint32_t* t)
{
    /* w8e1.wgsl:447-490, w8e2.wgsl:524-569, w8e3.wgsl (absorption on exit) */
    const float ETA = 0.01f;
    const int mode = C->mode;
    v3 w_i = neg(normalize(r->direction));
    v3 normal = normalize(h->normal);
    v3 out_normal;
    float ior = 1.5f;
    float cos_i = dot(w_i, normal);
    int entering = cos_i < 0.0f;
    v3 T_r = V(1.0f, 1.0f, 1.0f);
    float tprob = 0.0f;
    if (entering) {
        cos_i = dot(w_i, neg(normal));
        out_normal = neg(normal);
    } else {
        ior = 1.0f / ior;
        out_normal = normal;
        if (mode == OR_MODE_W8E3) {
            v3 dd = sub(h->position, r->origin);
            float sd = rt_det_sqrtf(dot(dd, dd)) / 100.0f;
            v3 nr = neg(V(0.5f, 0.2f, 0.2f));
            T_r = V(rt_det_expf(nr.x * sd), rt_det_expf(nr.y * sd), rt_det_expf(nr.z * sd));
            tprob = (T_r.x + T_r.y + T_r.z) / 3.0f;
            if (tprob < 0.0f || tprob > 1.0f) return V(0.7f, 0.0f, 0.7f);   /* error_shader */
        }
    }
    float cos_t2 = (1.0f - (ior * ior) * (1.0f - cos_i * cos_i));
    float refl;
    if (cos_t2 < 0.0f) {
        refl = 1.0f;
    } else {
        refl = fresnel_r(cos_i, rt_det_sqrtf(cos_t2), ior);
        if (mode == OR_MODE_W8E1) refl = rt_satf(refl);
    }
    v3 tangent = sub(muls(out_normal, cos_i), w_i);
    v3 on = mode == OR_MODE_W8E1 ? out_normal : normalize(out_normal);
    v3 w_t = sub(muls(tangent, ior), muls(on, rt_det_sqrtf(cos_t2)));
    r->direction = w_t;   /* ray_init(w_t, position) */
    r->origin = h->position;
    r->tmax = 5000.0f;
    r->tmin = ETA;
    h->has_hit = 0;
    if (mode != OR_MODE_W8E1) h->emit = 1;
    float step = rnd(t);
    if (step < refl) {
        h->normal = out_normal;
        return mirror_w8(C, r, h);
    }
    if (mode == OR_MODE_W8E2) {
        h->factor = divs(h->factor, 1.0f - refl);
    } else if (mode == OR_MODE_W8E3 && !entering) {
        if (step < refl + tprob) h->factor = divs(mul(h->factor, T_r), refl + tprob);
        else h->has_hit = 1;   /* absorbed */
    }
    return V(0, 0, 0);
}

static void sample_w8(Ctx* C, const Cam* cam, uint32_t x, uint32_t y, uint32_t it, float out[3], uint32_t* prim)
{
    /* fs_main, w8e1.wgsl:207-241 / w8e2.wgsl:246-281 */
    const or_uniform* u = C->u;
    const int e1 = C->mode == OR_MODE_W8E1;
    const float ETA = 0.01f;
    const v3 bg = e1 ? V(0.1f, 0.3f, 0.6f) : V(0.0f, 0.0f, 0.0f);
    const int max_depth = e1 ? 10 : 50;
    uint32_t t = tea16(y * u->resolution[0] + x, it);
    float jx = rnd(&t);
    float jy = rnd(&t);
    jx = jx / (float)u->resolution[1];
    jy = jy / (float)u->resolution[1];
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    Ray r;
    r.direction = cam_dir(cam, ux, uy, jx, jy);
    r.origin = cam->e;
    r.tmax = 5000.0f;
    r.tmin = ETA;
    Hit h;
    memset(&h, 0, sizeof h);
    h.factor = V(1, 1, 1);
    h.emit = 1;
    v3 result = V(0, 0, 0);
    *prim = 0xFFFFFFFFu;
    C->c.primary++;
    for (int i = 0; i < max_depth; i++) {
        if (i > 0) C->c.bounce++;
        if (intersect_scene_w8(C, &r, &h)) {
            if (i == 0 && h.shader == SH_LAMBERTIAN) *prim = h.tri;
            h.has_hit = 1;   /* shade() */
            v3 c;
            if (h.shader == SH_LAMBERTIAN) c = lambertian_w8(C, &r, &h, &t);
            else if (h.shader == SH_MIRROR) c = mirror_w8(C, &r, &h);
            else c = transparent_w8(C, &r, &h, &t);
            if (!e1) c = V(rt_minf(c.x, 100.0f), rt_minf(c.y, 100.0f), rt_minf(c.z, 100.0f));   /* firefly clamp */
            result = add(result, c);
        } else {
            result = add(result, bg);
            break;
        }
        if (h.has_hit) break;
    }
    out[0] = result.x;
    out[1] = result.y;
    out[2] = result.z;
}

static void sample_path(Ctx* C, const Cam* cam, uint32_t x, uint32_t y, uint32_t it, float out[3],
                        uint32_t* prim)
{
    const or_uniform* u = C->u;
    int w9 = C->mode == OR_MODE_W9E1 || C->mode == OR_MODE_W9E2 || C->mode == OR_MODE_W9E3;
    int plane = C->mode == OR_MODE_W9E2 || C->mode == OR_MODE_W9E3;
    float eta = w9 ? 0.0001f : 0.01f;
    uint32_t launch_idx = y * u->resolution[0] + x;
    uint32_t t = tea16(launch_idx, it);
    float jx = rnd(&t);
    float jy = rnd(&t);
    jx = jx / (float)u->resolution[1];
    jy = jy / (float)u->resolution[1];
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    Ray r;
    r.direction = cam_dir(cam, ux, uy, jx, jy);
    r.origin = cam->e;
    r.tmax = 5000.0f;
    r.tmin = eta;
    Hit h;
    memset(&h, 0, sizeof h);
    h.factor = V(1, 1, 1);
    h.emit = 1;
    v3 result = V(0, 0, 0);
    *prim = 0xFFFFFFFFu;
    C->c.primary++;
    for (int i = 0; i < 50; i++) {
        if (i > 0) C->c.bounce++;
        int hit = plane ? intersect_scene_w9e2(C, &r, &h) : trace(C, &r, &h, !w9);
        if (hit) {
            if (i == 0 && !(plane && h.shader == SH_HOLDOUT)) *prim = h.tri;
            result = add(result, w9 ? shade_w9e1(C, &r, &h, &t) : shade_w7e3(C, &r, &h, &t));
        } else {
            if (w9)   /* environment_map(r.direction) * hit.factor, w9e1.wgsl:264-265 */
                result = add(result, mul(env_lookup(C, r.direction), h.factor));
            /* W7E3: + BACKGROUND_COLOR (0,0,0) */
            else result = add(result, V(0, 0, 0));
            break;
        }
        if (h.has_hit) break;
    }
    out[0] = result.x;
    out[1] = result.y;
    out[2] = result.z;
}

/* ------------------------------------------------------------ W6E1 / PROJECT */

static int intersect_min_max(const float* aabb, Ray* r)   /* aabb.wgsl:8-31 */
{
    float tmin = 1.0e32f, tmax = -1.0e32f;
    for (int i = 0; i < 3; i++) {
        float d = comp(r->direction, i), o = comp(r->origin, i);
        if (rt_absf(d) > 1.0e-8f) {
            float p1 = (aabb[i] - o) / d;
            float p2 = (aabb[4 + i] - o) / d;
            float pmin = rt_minf(p1, p2), pmax = rt_maxf(p1, p2);
            tmin = rt_minf(tmin, pmin);
            tmax = rt_maxf(tmax, pmax);
        }
    }
    if (tmin > tmax || tmin > r->tmax || tmax < r->tmin) return 0;
    r->tmin = rt_maxf(tmin - 1.0e-4f, r->tmin);
    r->tmax = rt_minf(tmax + 1.0e-4f, r->tmax);
    return 1;
}

static v3 shade_w6e1(Ctx* C, Ray* r, Hit* h)
{
    /* shade (w6e1.wgsl:250-277) */
    const or_scene* s = C->s;
    const float ETA = 0.00001f;
    h->has_hit = 1;
    const or_material* m = mat_of(s, h->material);
    switch (h->shader) {
    case 0: {   /* lambertian :279-298 (project.wgsl: ambient*0.1, diffuse+ambient) */
        v3 bdrf = load3(m->diffuse);
        v3 normal = h->normal;
        /* sample_directional_light :237-248 */
        v3 w_i = neg(normalize(V(-1.0f, -1.0f, -1.0f)));
        v3 l_i = muls(V(PI_F, PI_F, PI_F), 1.0f);
        float dist = 1.0f;
        /* light_diffuse_contribution :300-306 */
        float dd = dot(normal, w_i);
        v3 dfc = V(dd, dd, dd);
        dfc = divs(dfc, dist * dist);
        dfc = mul(dfc, l_i);
        dfc = divs(dfc, PI_F);
        v3 diffuse = add(V(0, 0, 0), mul(bdrf, dfc));
        if (C->mode == OR_MODE_PROJECT) {
            v3 ambient = muls(load3(m->ambient), 0.1f);
            return add(diffuse, ambient);
        }
        v3 ambient = load3(m->ambient);
        return add(muls(diffuse, 0.9f), muls(ambient, 0.1f));
    }
    case 2: {   /* mirror :312-326 */
        v3 n = h->normal, d = r->direction;
        v3 rd = sub(d, muls(n, 2.0f * dot(n, d)));
        r->direction = rd;
        r->origin = add(h->position, muls(n, ETA));
        r->tmax = 100000.0f;
        r->tmin = ETA;
        h->has_hit = 0;
        return V(0, 0, 0);
    }
    case 5:
        return muls(add(h->normal, V(1.0f, 1.0f, 1.0f)), 0.5f);
    case 6:
        return add(load3(m->diffuse), load3(m->ambient));
    default:
        return V(0.7f, 0.0f, 0.7f);
    }
}

static void sample_w6e1(Ctx* C, const Cam* cam, uint32_t x, uint32_t y, float out[3], uint32_t* prim)
{
    /* fs_main, w6e1.wgsl:152-185 / project.wgsl:152-185 */
    const or_uniform* u = C->u;
    const float ETA = 0.00001f;
    v3 bg = V(0.1f, 0.3f, 0.6f);
    uint32_t subdiv = u->subdivision_level;
    v3 result = V(0, 0, 0);
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    *prim = 0xFFFFFFFFu;
    for (uint32_t sample = 0; sample < subdiv * subdiv; sample++) {
        float jx = C->jitter ? C->jitter[2 * sample] : 0.0f;
        float jy = C->jitter ? C->jitter[2 * sample + 1] : 0.0f;
        Ray r;
        r.direction = cam_dir(cam, ux, uy, jx, jy);
        r.origin = cam->e;
        r.tmax = 100000.0f;
        r.tmin = ETA;
        Hit h;
        memset(&h, 0, sizeof h);
        h.shader = 255;
        C->c.primary++;
        /* bvh.wgsl:197-200 replaces intersect_min_max by `return true` */
        if (C->trav == OR_TRAV_BSP && !intersect_min_max(C->s->aabb, &r)) {
            result = bg;
            break;
        }
        for (int i = 0; i < 10; i++) {
            if (i > 0) C->c.bounce++;
            h.shader = u->selection1;   /* intersect_scene_bsp :187-191 */
            if (trace(C, &r, &h, 0)) {
                if (i == 0 && sample + 1 == subdiv * subdiv) *prim = h.tri;
                result = add(result, shade_w6e1(C, &r, &h));
            } else {
                result = add(result, bg);
                break;
            }
            if (h.has_hit) break;
        }
    }
    float multiplier = 1.0f / (float)(subdiv * subdiv);
    result = muls(result, multiplier);
    out[0] = result.x;
    out[1] = result.y;
    out[2] = result.z;
}

/* ------------------------------------------------------------ W6E2 / W7E1 / W7E2
 * Cornell-box direct lighting (res/shaders/w6e2.wgsl, w7e1.wgsl, w7e2.wgsl):
 * one closest-hit ray per sample, then a shadow ray to every area-light
 * triangle; W6E2 takes subdiv^2 jittered samples, W7E1/W7E2 are progressive. */
static Light area_light_direct(Ctx* C, v3 pos, uint32_t idx, uint32_t* t)
{
    /* sample_area_light: w6e2.wgsl:245-262 / w7e1.wgsl:327-346 (triangle
     * centre, l_i without 1/d^2) and w7e2.wgsl:327-354 (random point, 1/d^2);
     * cos_l is not clamped in any of the three */
    const or_scene* s = C->s;
    uint32_t li = s->lights[idx < s->nlights ? idx : s->nlights - 1];
    const uint32_t* tri = s->idx + 4 * (size_t)(li < s->ntris ? li : s->ntris - 1);
    v3 v0 = load3(s->pos + 4 * (size_t)tri[0]);
    v3 v1 = load3(s->pos + 4 * (size_t)tri[1]);
    v3 v2 = load3(s->pos + 4 * (size_t)tri[2]);
    float area = triangle_area(v0, v1, v2);
    v3 l_e = load3(mat_of(s, tri[3])->ambient);
    v3 point;
    if (C->mode == OR_MODE_W7E2) {
        float psi1 = rt_det_sqrtf(rnd(t));
        float psi2 = rnd(t);
        float alpha = 1.0f - psi1;
        float beta = (1.0f - psi2) * psi1;
        float gamma = psi2 * psi1;
        point = add(add(muls(v0, alpha), muls(v1, beta)), muls(v2, gamma));
    } else {
        point = divs(add(add(v0, v1), v2), 3.0f);
    }
    v3 normal = normalize(cross(sub(v0, v1), sub(v0, v2)));
    v3 ld = sub(point, pos);
    float cos_l = dot(normalize(neg(ld)), normal);
    float distance = rt_det_sqrtf(dot(ld, ld));
    Light L;
    L.l_i = muls(muls(l_e, area), cos_l);
    if (C->mode == OR_MODE_W7E2 || C->mode == OR_MODE_W6E3) L.l_i = divs(L.l_i, distance * distance);
    L.w_i = normalize(ld);
    L.dist = distance;
    return L;
}

static v3 lambertian_direct(Ctx* C, Hit* h, uint32_t* t)
{
    /* w6e2.wgsl:297-322 / w7e1.wgsl:385-410 / w7e2.wgsl:392-417 */
    const or_scene* s = C->s;
    const int e2 = C->mode == OR_MODE_W7E2;
    const float ETA = C->mode == OR_MODE_W6E2 ? 0.00001f : 0.001f;
    const float off = C->mode == OR_MODE_W6E2 ? 10.0f : 100.0f;
    v3 normal = h->normal, position = h->position;
    const or_material* m = mat_of(s, h->material);
    v3 bdrf = load3(m->diffuse);
    v3 diffuse = V(0, 0, 0);
    for (uint32_t idx = 1; idx < s->nlights; idx++) {
        Light L = area_light_direct(C, position, idx, t);
        Ray sr;
        sr.direction = L.w_i;
        sr.origin = e2 ? position : add(position, muls(muls(normal, ETA), off));
        sr.tmin = ETA;
        sr.tmax = e2 ? L.dist - ETA : L.dist - ETA * 1000.0f;
        Hit hi;
        memset(&hi, 0, sizeof hi);
        C->c.shadow++;
        if (trace(C, &sr, &hi, 1)) continue;   /* blocked */
        float dd = dot(normal, L.w_i);
        if (e2) {
            diffuse = add(diffuse, divs(mul(mul(bdrf, V(dd, dd, dd)), L.l_i), PI_F));
        } else {   /* light_diffuse_contribution */
            v3 c = divs(V(dd, dd, dd), L.dist * L.dist);
            c = mul(c, L.l_i);
            c = divs(c, PI_F);
            diffuse = add(diffuse, mul(bdrf, c));
        }
    }
    if (e2) return add(diffuse, load3(m->ambient));
    v3 ambient = add(load3(m->ambient), muls(load3(m->diffuse), 0.1f));
    return add(muls(diffuse, 0.9f), muls(ambient, 0.1f));   /* diffuse_and_ambient */
}

static v3 trace_direct(Ctx* C, Ray* r, uint32_t* t, uint32_t* prim, int record_prim)
{
    /* one sample of fs_main: the shader is always LAMBERTIAN, which ends the
     * bounce loop (has_hit) */
    v3 bg = C->mode == OR_MODE_W6E2 ? V(0.1f, 0.3f, 0.6f) : V(0.0f, 0.0f, 0.0f);
    Hit h;
    memset(&h, 0, sizeof h);
    C->c.primary++;
    if (!trace(C, r, &h, 1)) return bg;
    if (record_prim) *prim = h.tri;
    return lambertian_direct(C, &h, t);
}

static void sample_w6e2(Ctx* C, const Cam* cam, uint32_t x, uint32_t y, float out[3], uint32_t* prim)
{
    /* fs_main, w6e2.wgsl:160-186: subdiv^2 jittered samples, averaged */
    const or_uniform* u = C->u;
    uint32_t subdiv = u->subdivision_level;
    v3 result = V(0, 0, 0);
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    *prim = 0xFFFFFFFFu;
    for (uint32_t sample = 0; sample < subdiv * subdiv; sample++) {
        float jx = C->jitter ? C->jitter[2 * sample] : 0.0f;
        float jy = C->jitter ? C->jitter[2 * sample + 1] : 0.0f;
        Ray r;
        r.direction = cam_dir(cam, ux, uy, jx, jy);
        r.origin = cam->e;
        r.tmax = 5000.0f;
        r.tmin = 0.00001f;
        result = add(result, trace_direct(C, &r, NULL, prim, sample + 1 == subdiv * subdiv));
    }
    result = muls(result, 1.0f / (float)(subdiv * subdiv));
    out[0] = result.x;
    out[1] = result.y;
    out[2] = result.z;
}

static void sample_w7_direct(Ctx* C, const Cam* cam, uint32_t x, uint32_t y, uint32_t it, float out[3],
                             uint32_t* prim)
{
    /* fs_main, w7e1.wgsl:202-236 / w7e2.wgsl: TEA-seeded jitter, one sample */
    const or_uniform* u = C->u;
    uint32_t t = tea16(y * u->resolution[0] + x, it);
    float jx = rnd(&t);
    float jy = rnd(&t);
    jx = jx / (float)u->resolution[1];
    jy = jy / (float)u->resolution[1];
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    Ray r;
    r.direction = cam_dir(cam, ux, uy, jx, jy);
    r.origin = cam->e;
    r.tmax = 5000.0f;
    r.tmin = 0.001f;
    *prim = 0xFFFFFFFFu;
    v3 res = trace_direct(C, &r, &t, prim, 1);
    out[0] = res.x;
    out[1] = res.y;
    out[2] = res.z;
}

/* ------------------------------------------------------------ W6E3
 * res/shaders/w6e3.wgsl: W6E2's scene loop over the Cornell box with the two
 * balls of intersect_scene_bsp (:196-216): mirror, glossy (phong + transmit,
 * ior 1.5), lambertian mesh with 1/d^2 centre lights. */
static int intersect_scene_w6e3(Ctx* C, Ray* r, Hit* h)
{
    int has_hit = 0;
    if (intersect_sphere(r, h, V(420.0f, 90.0f, 370.0f), 90.0f)) {
        h->shader = 2;
        has_hit = 1;
    }
    if (intersect_sphere(r, h, V(130.0f, 90.0f, 250.0f), 90.0f)) {
        h->shader = 4;   /* GLOSSY, ior1_over_ior2 = 1.5 */
        has_hit = 1;
    }
    if (trace(C, r, h, 1)) {
        h->shader = 0;
        has_hit = 1;
    }
    return has_hit;
}

static v3 shade_w6e3(Ctx* C, Ray* r, Hit* h)
{
    const or_scene* s = C->s;
    const float ETA = 0.001f;
    h->has_hit = 1;
    if (h->shader == 0) {   /* lambertian, :354-379 */
        v3 normal = h->normal;
        const or_material* m = mat_of(s, h->material);
        v3 bdrf = load3(m->diffuse);
        v3 diffuse = V(0, 0, 0);
        for (uint32_t idx = 1; idx < s->nlights; idx++) {
            Light L = area_light_direct(C, h->position, idx, NULL);
            Ray sr;
            sr.direction = L.w_i;
            sr.origin = h->position;
            sr.tmax = L.dist - ETA;
            sr.tmin = ETA;
            Hit hi;
            memset(&hi, 0, sizeof hi);
            C->c.shadow++;
            if (intersect_scene_w6e3(C, &sr, &hi)) continue;
            float dd = dot(normal, L.w_i);
            diffuse = add(diffuse, divs(mul(mul(bdrf, V(dd, dd, dd)), L.l_i), PI_F));
        }
        return add(diffuse, load3(m->ambient));
    }
    if (h->shader == 2) {   /* mirror, :381-389 */
        v3 n = h->normal, d = r->direction;
        r->direction = sub(d, muls(n, 2.0f * dot(n, d)));
        r->origin = h->position;
        r->tmax = 5000.0f;
        r->tmin = ETA;
        h->has_hit = 0;
        return V(0, 0, 0);
    }
    /* glossy = phong + transmit, :391-457 */
    v3 normal = h->normal, position = h->position;
    float coeff = 0.9f * (42.0f + 2.0f) / (2.0f * PI_F);
    v3 w_o = normalize(sub(load3(C->u->camera_pos), position));
    v3 phong_total = V(0, 0, 0);
    for (uint32_t idx = 1; idx < s->nlights; idx++) {
        Light L = area_light_direct(C, position, idx, NULL);
        v3 nw = neg(L.w_i);
        v3 w_r = normalize(sub(nw, muls(normal, 2.0f * dot(normal, nw))));
        float dd = rt_satf(dot(normal, L.w_i));
        v3 dif = divs(mul(V(dd, dd, dd), L.l_i), PI_F);
        phong_total = add(phong_total, muls(dif, rt_det_powf(rt_satf(dot(w_o, w_r)), 42.0f)));
    }
    v3 ph = muls(phong_total, coeff);
    v3 w_i = neg(normalize(r->direction));
    v3 n2 = normalize(h->normal);
    float ior = 1.5f;
    float cos_i = dot(w_i, n2);
    v3 out_n;
    if (cos_i < 0.0f) {
        out_n = neg(n2);
    } else {
        ior = 1.0f / ior;
        out_n = n2;
    }
    float cos_t2 = (1.0f - (ior * ior) * (1.0f - cos_i * cos_i));
    if (cos_t2 < 0.0f) return add(ph, V(0.7f, 0.0f, 0.7f));   /* error_shader, has_hit stays */
    v3 tangent = sub(muls(n2, cos_i), w_i);
    r->direction = sub(muls(tangent, ior), muls(out_n, rt_det_sqrtf(cos_t2)));
    r->origin = position;
    r->tmax = 5000.0f;
    r->tmin = ETA;
    h->has_hit = 0;
    return add(ph, V(0, 0, 0));
}

static void sample_w6e3(Ctx* C, const Cam* cam, uint32_t x, uint32_t y, float out[3], uint32_t* prim)
{
    /* fs_main, w6e3.wgsl:166-192 */
    const or_uniform* u = C->u;
    uint32_t subdiv = u->subdivision_level;
    v3 result = V(0, 0, 0);
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    *prim = 0xFFFFFFFFu;
    for (uint32_t sample = 0; sample < subdiv * subdiv; sample++) {
        float jx = C->jitter ? C->jitter[2 * sample] : 0.0f;
        float jy = C->jitter ? C->jitter[2 * sample + 1] : 0.0f;
        Ray r;
        r.direction = cam_dir(cam, ux, uy, jx, jy);
        r.origin = cam->e;
        r.tmax = 5000.0f;
        r.tmin = 0.001f;
        Hit h;
        memset(&h, 0, sizeof h);
        C->c.primary++;
        for (int i = 0; i < 10; i++) {
            if (i > 0) C->c.bounce++;
            if (intersect_scene_w6e3(C, &r, &h)) {
                if (i == 0 && sample + 1 == subdiv * subdiv && h.shader == 0) *prim = h.tri;
                result = add(result, shade_w6e3(C, &r, &h));
            } else {
                result = add(result, V(0.0f, 0.0f, 0.0f));
                break;
            }
            if (h.has_hit) break;
        }
    }
    result = muls(result, 1.0f / (float)(subdiv * subdiv));
    out[0] = result.x;
    out[1] = result.y;
    out[2] = result.z;
}

/* ------------------------------------------------------------ W1E6 */

static int w1_triangle(Ray* r, Hit* h, v3 a, v3 b, v3 c)   /* w1e6.wgsl:179-209 */
{
    Ray ray = *r;
    v3 w_i = ray.direction, o = ray.origin;
    v3 e0 = sub(b, a), e1 = sub(c, a), o_to_v0 = sub(a, o);
    v3 normal = cross(e0, e1);
    v3 nom = cross(o_to_v0, w_i);
    float denom = dot(w_i, normal);
    if (rt_absf(denom) < 1e-6f) return 0;
    float beta = dot(nom, e1) / denom;
    float gamma = -dot(nom, e0) / denom;
    float distance = dot(o_to_v0, normal) / denom;
    if (beta < 0.0f || gamma < 0.0f || beta + gamma > 1.0f || distance > ray.tmax || distance < ray.tmin)
        return 0;
    r->tmax = distance;
    h->dist = distance;
    h->position = add(o, muls(w_i, distance));
    h->normal = normalize(normal);
    return 1;
}
static int w1_sphere(Ray* r, Hit* h, v3 center, float radius)   /* :211-237 */
{
    Ray ray = *r;
    v3 oc = sub(ray.origin, center);
    float a = dot(ray.direction, ray.direction);
    float b_over_2 = dot(oc, ray.direction);
    float c = dot(oc, oc) - radius * radius;
    float disc = b_over_2 * b_over_2 - a * c;
    if (disc < 0.0f) return 0;
    float ds = rt_det_sqrtf(disc);
    float root = (-b_over_2 - ds) / a;
    if (root < ray.tmin || root > ray.tmax) {
        root = (-b_over_2 + ds) / a;
        if (root < ray.tmin || root > ray.tmax) return 0;
    }
    r->tmax = root;
    h->dist = root;
    v3 pos = add(ray.origin, muls(ray.direction, root));
    h->position = pos;
    h->normal = normalize(sub(pos, center));
    return 1;
}
static int w1_plane(Ray* r, Hit* h, v3 normal, v3 position)   /* :164-177 */
{
    Ray ray = *r;
    float distance = dot(sub(position, ray.origin), normal) / dot(ray.direction, normal);
    if (distance < ray.tmin || distance > ray.tmax) return 0;
    r->tmax = distance;
    h->dist = distance;
    h->position = add(ray.origin, muls(ray.direction, distance));
    h->normal = normal;
    return 1;
}

static void sample_w1e6(Ctx* C, const Cam* cam, uint32_t x, uint32_t y, float out[3], uint32_t* prim)
{
    const or_uniform* u = C->u;
    v3 bg = V(0.1f, 0.3f, 0.6f);
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    Ray r;
    /* get_camera_ray (:98-113): normalize(b1 * uv.x * aspect + b2 * uv.y + v*d) */
    r.direction = normalize(add(add(muls(muls(cam->b1, ux), cam->aspect), muls(cam->b2, uy)), muls(cam->v, cam->d)));
    r.origin = cam->e;
    r.tmax = 5000.0f;
    r.tmin = 0.00001f;
    Hit h;
    memset(&h, 0, sizeof h);
    v3 base = V(0, 0, 0);
    v3 result = V(0, 0, 0);
    *prim = 0xFFFFFFFFu;
    C->c.primary++;
    for (int i = 0; i < 10; i++) {
        int any = 0;
        uint32_t which = 0xFFFFFFFFu;
        if (w1_triangle(&r, &h, V(0.2f, 0.1f, 0.9f), V(-0.2f, 0.1f, -0.1f), V(-0.2f, 0.1f, 0.9f))) {
            any = 1; base = V(0.4f, 0.3f, 0.2f); which = 0;
        }
        if (w1_sphere(&r, &h, V(0.0f, 0.5f, 0.0f), 0.3f)) {
            any = 1; base = V(0.0f, 0.0f, 0.0f); which = 1;
        }
        if (w1_plane(&r, &h, V(0.0f, 1.0f, 0.0f), V(0.0f, 0.0f, 0.0f))) {
            any = 1; base = V(0.1f, 0.7f, 0.0f); which = 2;
        }
        if (any) {
            if (i == 0) *prim = which;
            /* shade -> lambertian (:254-284) with sample_point_light (:239-252) */
            h.has_hit = 1;
            v3 light_pos = V(0.0f, 1.2f, 0.0f);
            v3 intensity = muls(V(PI_F, PI_F, PI_F), 5.0f);
            v3 dir = sub(light_pos, h.position);
            float dist = dot(dir, dir);
            v3 l_i = divs(intensity, dist * dist);
            v3 w_i = dir;
            float dd = dot(h.normal, w_i);
            v3 dfc = V(dd, dd, dd);
            dfc = mul(dfc, l_i);
            dfc = muls(dfc, (1.0f - 0.0f) / PI_F);
            v3 diffuse = mul(base, dfc);
            result = add(result, add(muls(diffuse, 0.9f), muls(base, 0.1f)));
        } else {
            result = add(result, bg);
            break;
        }
        if (h.has_hit) break;
    }
    out[0] = result.x;
    out[1] = result.y;
    out[2] = result.z;
}

/* ------------------------------------------------------------ driver */

typedef struct {
    const or_scene* s;
    const or_uniform* u;
    const float* jitter;
    int mode, trav;
    uint32_t x0, y0, w, h, first_iter, spp;
    float* accum;
    uint32_t* ids;
    volatile uint32_t next_row;
    pthread_mutex_t mu;
    or_counts total;
    float* rlog;         /* single-threaded ray log (or_render_raylog) */
    uint32_t rlog_cap, rlog_n;
} Job;

static void render_row(Job* J, Ctx* C, const Cam* cam, uint32_t ry)
{
    uint32_t y = J->y0 + ry;
    for (uint32_t rx = 0; rx < J->w; rx++) {
        uint32_t x = J->x0 + rx;
        size_t o = (size_t)ry * J->w + rx;
        float* acc = J->accum + 4 * o;
        uint32_t prim = 0xFFFFFFFFu;
        if (J->mode == OR_MODE_W7E3 || J->mode == OR_MODE_W9E1 || J->mode == OR_MODE_W9E3 ||
            (J->mode >= OR_MODE_W8E1 && J->mode != OR_MODE_W6E2 && J->mode != OR_MODE_W6E3)) {
            /* progressive */
            const int clamp0 = J->mode != OR_MODE_W7E1 && J->mode != OR_MODE_W7E2;   /* w7e1.wgsl:229-235: no max */
            float a[3] = {acc[0], acc[1], acc[2]};
            if (J->first_iter == 0) a[0] = a[1] = a[2] = 0.0f;
            for (uint32_t k = 0; k < J->spp; k++) {
                uint32_t it = J->first_iter + k;
                float res[3];
                C->c.samples++;
                if (J->mode >= OR_MODE_W8E1 && J->mode <= OR_MODE_W8E3) sample_w8(C, cam, x, y, it, res, &prim);
                else if (J->mode == OR_MODE_W7E1 || J->mode == OR_MODE_W7E2) sample_w7_direct(C, cam, x, y, it, res, &prim);
                else sample_path(C, cam, x, y, it, res, &prim);
                /* fs_main accumulation, w7e3.wgsl:261-271 */
                for (int c = 0; c < 3; c++) {
                    float curr_sum = a[c] * (float)it;
                    float ac = (res[c] + curr_sum) / (float)(it + 1u);
                    a[c] = clamp0 ? rt_max0f(ac) : ac;
                }
            }
            acc[0] = a[0]; acc[1] = a[1]; acc[2] = a[2]; acc[3] = 1.0f;
        } else {
            float res[3];
            C->c.samples++;
            if (J->mode == OR_MODE_W1E6) sample_w1e6(C, cam, x, y, res, &prim);
            else if (J->mode == OR_MODE_W6E2) sample_w6e2(C, cam, x, y, res, &prim);
            else if (J->mode == OR_MODE_W6E3) sample_w6e3(C, cam, x, y, res, &prim);
            else sample_w6e1(C, cam, x, y, res, &prim);
            acc[0] = res[0]; acc[1] = res[1]; acc[2] = res[2]; acc[3] = 1.0f;
        }
        if (J->ids) J->ids[o] = prim;
    }
}

static void* worker(void* arg)
{
    Job* J = (Job*)arg;
    Ctx C;
    memset(&C, 0, sizeof C);
    C.s = J->s;
    C.u = J->u;
    C.jitter = J->jitter;
    C.mode = J->mode;
    C.trav = J->trav;
    C.rlog = J->rlog;
    C.rlog_cap = J->rlog_cap;
    Cam cam = make_cam(J->u);
    for (;;) {
        uint32_t ry = __sync_fetch_and_add(&J->next_row, 1u);
        if (ry >= J->h) break;
        render_row(J, &C, &cam, ry);
    }
    J->rlog_n = C.rlog_n;
    pthread_mutex_lock(&J->mu);
    uint64_t* d = (uint64_t*)&J->total;
    const uint64_t* sC = (const uint64_t*)&C.c;
    for (size_t i = 0; i < sizeof(or_counts) / sizeof(uint64_t); i++) d[i] += sC[i];
    pthread_mutex_unlock(&J->mu);
    return NULL;
}

static int render_job(const or_scene* s, const or_uniform* u, const float* jitter, int mode, int trav,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t first_iter, uint32_t spp,
                      float* accum, uint32_t* ids, or_counts* counts, int nthreads, float* rlog, uint32_t rlog_cap,
                      uint32_t* rlog_n);

int or_render(const or_scene* s, const or_uniform* u, const float* jitter, int mode, int trav,
              uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t first_iter, uint32_t spp,
              float* accum, uint32_t* ids, or_counts* counts, int nthreads)
{
    return render_job(s, u, jitter, mode, trav, x0, y0, w, h, first_iter, spp, accum, ids, counts, nthreads, NULL, 0,
                      NULL);
}

/* or_render on one thread, logging every ray trace() receives (origin,
 * direction, tmin, tmax) in trace order: the primary, shadow and bounce rays
 * of the shaders as the walk sees them (tests/golden/gen_js_walk2.py) */
int or_render_raylog(const or_scene* s, const or_uniform* u, int mode, int trav, uint32_t x0, uint32_t y0, uint32_t w,
                     uint32_t h, uint32_t first_iter, uint32_t spp, float* accum, uint32_t* ids, float* rays,
                     uint32_t cap, uint32_t* nrays)
{
    return render_job(s, u, NULL, mode, trav, x0, y0, w, h, first_iter, spp, accum, ids, NULL, 1, rays, cap, nrays);
}

static int render_job(const or_scene* s, const or_uniform* u, const float* jitter, int mode, int trav,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t first_iter, uint32_t spp,
                      float* accum, uint32_t* ids, or_counts* counts, int nthreads, float* rlog, uint32_t rlog_cap,
                      uint32_t* rlog_n)
{
    if (mode < 0 || mode > OR_MODE_W9E3) return -1;
    if (mode != OR_MODE_W1E6) {
        if (!s || !s->nmats) return -1;
        if (trav == OR_TRAV_BSP && (!s->tree || !s->planes)) return -1;
        if (trav == OR_TRAV_BVH && !s->bvh_nodes) return -1;
        if (trav == OR_TRAV_NONE) return -1;
        if ((mode == OR_MODE_W7E3 || (mode >= OR_MODE_W8E1 && mode <= OR_MODE_W8E3)) && s->nlights < 2) return -1;
    }
    if (x0 + w > u->resolution[0] || y0 + h > u->resolution[1]) return -1;
    Job J;
    memset(&J, 0, sizeof J);
    J.s = s; J.u = u; J.jitter = jitter; J.mode = mode; J.trav = trav;
    J.x0 = x0; J.y0 = y0; J.w = w; J.h = h; J.first_iter = first_iter; J.spp = spp;
    J.accum = accum; J.ids = ids;
    J.rlog = rlog; J.rlog_cap = rlog_cap;
    pthread_mutex_init(&J.mu, NULL);
    if (rlog) nthreads = 1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, worker, &J);
    worker(&J);
    for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&J.mu);
    if (counts) *counts = J.total;
    if (rlog_n) *rlog_n = J.rlog_n;
    return 0;
}

int or_trace_one(const or_scene* s, int trav, int face_normals, const float o[3], const float d[3],
                 float tmin, float tmax, uint32_t* tri, float* dist)
{
    Ctx C;
    memset(&C, 0, sizeof C);
    C.s = s;
    C.trav = trav;
    Ray r;
    r.origin = load3(o);
    r.direction = load3(d);
    r.tmin = tmin;
    r.tmax = tmax;
    Hit h;
    memset(&h, 0, sizeof h);
    int hit = trace(&C, &r, &h, face_normals);
    *tri = hit ? h.tri : 0xFFFFFFFFu;
    *dist = hit ? h.dist : 0.0f;
    return hit;
}

/* or_trace_one over n rays (8 floats each: origin, direction, tmin, tmax) on
 * nthreads threads: closest hit (triangle id or 0xFFFFFFFF, distance) */
typedef struct {
    const or_scene* s;
    int trav;
    uint32_t n, nth, k;
    const float* rays;
    uint32_t* tri;
    float* dist;
} ManyJob;
static void* many_worker(void* p)
{
    ManyJob* J = (ManyJob*)p;
    const uint32_t k = __atomic_fetch_add(&J->k, 1u, __ATOMIC_RELAXED);
    for (uint32_t i = k; i < J->n; i += J->nth) {
        const float* q = J->rays + 8 * (size_t)i;
        or_trace_one(J->s, J->trav, 1, q, q + 3, q[6], q[7], J->tri + i, J->dist + i);
    }
    return NULL;
}
int or_trace_many(const or_scene* s, int trav, uint32_t n, const float* rays, uint32_t* tri, float* dist, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    ManyJob J = {s, trav, n, (uint32_t)nthreads, 0u, rays, tri, dist};
    pthread_t th[256];
    for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, many_worker, &J);
    many_worker(&J);
    for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
    return 0;
}

void or_camera_ray(const or_uniform* u, uint32_t x, uint32_t y, float jx, float jy, float o[3], float d[3])
{
    Cam cam = make_cam(u);
    float ux, uy;
    pixel_uv(u, x, y, &ux, &uy);
    v3 dir = cam_dir(&cam, ux, uy, jx, jy);
    o[0] = cam.e.x;
    o[1] = cam.e.y;
    o[2] = cam.e.z;
    d[0] = dir.x;
    d[1] = dir.y;
    d[2] = dir.z;
}

int or_trace_query(const or_scene* s, int trav, int clip, const float o[3], const float d[3], float tmin,
                   float tmax, uint32_t* tri, float* dist, float* out_tmin, float* out_tmax, uint32_t* tested,
                   uint32_t cap, uint32_t* ntested)
{
    Ctx C;
    memset(&C, 0, sizeof C);
    C.s = s;
    C.trav = trav;
    C.log = tested;
    C.log_cap = tested ? cap : 0;
    Ray r;
    r.origin = load3(o);
    r.direction = load3(d);
    r.tmin = tmin;
    r.tmax = tmax;
    Hit h;
    memset(&h, 0, sizeof h);
    int hit = 0, clipped = 0;
    if (clip && !intersect_min_max(s->aabb, &r)) clipped = 1;   /* w6e1.wgsl:165-168: the sample ends */
    if (!clipped) hit = trace(&C, &r, &h, 1);
    *tri = hit ? h.tri : 0xFFFFFFFFu;
    *dist = hit ? h.dist : 0.0f;
    *out_tmin = r.tmin;
    *out_tmax = r.tmax;
    if (ntested) *ntested = C.log_n;
    return clipped ? -1 : hit;
}

int or_trace_brute(const or_scene* s, const float o[3], const float d[3], float tmin, float tmax,
                   uint32_t* tri, float* dist)
{
    Ctx C;
    memset(&C, 0, sizeof C);
    C.s = s;
    Ray r;
    r.origin = load3(o);
    r.direction = load3(d);
    r.tmin = tmin;
    r.tmax = tmax;
    Hit h;
    memset(&h, 0, sizeof h);
    int found = 0;
    for (uint32_t t = 0; t < s->ntris; t++)
        if (tri_test(&C, &r, &h, t, 1)) found = 1;
    *tri = found ? h.tri : 0xFFFFFFFFu;
    *dist = found ? h.dist : 0.0f;
    return found;
}

float or_det_sinf(float x) { return rt_det_sinf(x); }
float or_det_cosf(float x) { return rt_det_cosf(x); }
float or_det_acosf(float x) { return rt_det_acosf(x); }
