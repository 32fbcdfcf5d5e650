/* walk_sim.c -- trip-count model of k_path's BSP walk,
 * for pricing walk changes on the CPU before building them.  Test/tool code:
 * not part of the product.
 *
 * Replays bsp.wgsl:10-81 (the oracle's trace_bsp) per ray in f32 and counts
 * the trips the kernel's per-lane state machine needs (bsp_step: a walking
 * trip reads one 64-B treelet and decides up to three levels; a leaf trip
 * tests up to two triangles; an empty leaf or a leaf without a hit pops at
 * the end of its trip), under variants of the walk:
 *   v0  the committed walk;
 *   v1  + "skip empty near child": a push whose near child is an empty leaf
 *       would pop straight back (tmin = t, tmax unchanged, node = far), so the
 *       walk goes to the far child at once, in the same trip;
 *   v2  + "skip empty far child": a pending entry whose far child is an empty
 *       leaf is popped past (its pop would only reach that leaf and pop again),
 *       in the same trip as the pop that reaches it.
 * All variants return the same hit (checked per ray against v0).
 * Build: gcc -O2 -ffp-contract=off -shared -fPIC -o walk_sim.so walk_sim.c */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

typedef struct { float x, y, z; } v3;
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 cross(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

typedef struct {
    const uint32_t* tree;   /* nnodes x 4 (reference layout, 0-based, children 2i+1, 2i+2) */
    const float* planes;
    const uint32_t* ids;
    const float* pos;       /* float4 */
    const uint32_t* idx;    /* uint4 */
} Scene;

static int tri(const Scene* s, uint32_t v, v3 o, v3 w, float tmin, float tmax, float* dist)
{
    const uint32_t* ix = s->idx + 4 * (size_t)v;
    v3 v0 = V(s->pos[4 * ix[0]], s->pos[4 * ix[0] + 1], s->pos[4 * ix[0] + 2]);
    v3 v1 = V(s->pos[4 * ix[1]], s->pos[4 * ix[1] + 1], s->pos[4 * ix[1] + 2]);
    v3 v2 = V(s->pos[4 * ix[2]], s->pos[4 * ix[2] + 1], s->pos[4 * ix[2] + 2]);
    v3 e0 = sub(v1, v0), e1 = sub(v2, v0), ov = sub(v0, o);
    v3 n = cross(e0, e1), nom = cross(ov, w);
    float den = dot(w, n);
    if (fabsf(den) < 1e-10f) return 0;
    float b = dot(nom, e1) / den, g = -dot(nom, e0) / den, d = dot(ov, n) / den;
    if (b < 0.0f || g < 0.0f || b + g > 1.0f || d > tmax || d < tmin) return 0;
    *dist = d;
    return 1;
}

int g_levels = 3;
static uint32_t depth_of(uint32_t n0);
static const float* g_boxes = 0;
int g_root_only = 0;
int g_cull_every = 0;
int g_clip = 0;
int g_chunk = 0, g_chunk_min = 0, g_chunk_free = 0;
float g_chunk_margin = 0;
void walk_sim_chunk(int c, int mn, int fr, float mg) { g_chunk = c; g_chunk_min = mn; g_chunk_free = fr; g_chunk_margin = mg; }
void walk_sim_clip(int c) { g_clip = c; }
void walk_sim_cull_every(int c) { g_cull_every = c; }
double g_bad[256];
int g_bad_n = 0;
int walk_sim_bad(double* out) { for (int i = 0; i < 4 * g_bad_n; i++) out[i] = g_bad[i]; return g_bad_n; }
double g_cull[32], g_cull_leaf;
void walk_sim_culls(double* out) { for (int i = 0; i < 32; i++) out[i] = g_cull[i]; out[32] = g_cull_leaf; }
void walk_sim_root_only(int r) { g_root_only = r; }
/* WALK_AXIS: 1 (default) an axis with |d| < 1e-8 culls on the origin's coordinate
 * against the grown box (option (a)); 0 it constrains nothing (round 4's kernel) */
int g_axis = 1;
void walk_sim_axis(int a) { g_axis = a; }   /* nnodes x 6: content box (min.xyz, max.xyz) of each node's subtree, or NULL */
void walk_sim_boxes(const float* b) { g_boxes = b; }
static float g_tn, g_tf;   /* the ray interval clipped to the last tested box */
/* WALK_SPEC: the speculative exact cull.  The walk culls when the
 * certified margin proves it *or* the fast margin (2^-10 of max(|o|inf, scene)) culls,
 * and decides against the intersection of the two clipped intervals; a ray is flagged
 * when a cull or a near-/far-only decision rested on the fast margin alone (the
 * certified test would not have made it).  An unflagged ray's walk made only proven
 * decisions (its hit is the reference's); a flagged ray is re-walked certified. */
int g_spec = 0, g_spec_flag = 0;
static float g_tn_c = -INFINITY, g_tf_c = INFINITY;   /* the certified interval of the last box test */
void walk_sim_spec(int sp) { g_spec = sp; }
double g_spec_stat[8];   /* flagged rays, spec-only culls, spec-only clip decisions, proven culls, rewalk trips */
void walk_sim_spec_stats(double* o) { for (int i = 0; i < 8; i++) o[i] = g_spec_stat[i]; }
/* WALK_CERT: the certified margin (DESIGN.md section 4 "Certified culling"):
 * g_cert[node*7] = E2 (max over the subtree's triangles of max(|e0|inf, |e1|inf)^2),
 * +1..3 / +4..6 = the box of n* / (2 E2) over them (lower / upper) */
static const double* g_cert = 0;
static double g_cert_mag = 0;
static int g_cert_floor_only = 0;
void walk_sim_cert(const double* c, double mag, int floor_only) { g_cert = c; g_cert_mag = mag; g_cert_floor_only = floor_only; }
double g_cert_margin_sum = 0, g_cert_margin_n = 0;
double walk_sim_cert_mean(void) { return g_cert_margin_n ? g_cert_margin_sum / g_cert_margin_n : 0; }
static int g_cert_is_floor = 0;
/* WALK_CAM: per node min over the subtree's triangles of |(v0 - E) . n*| / E_T^2 for the
 * camera eye E (camera rays start at E: the accept point must then be near the plane of
 * the triangle *and* the eye off it, which bounds |denom| below) */
static const double* g_hcam = 0;
/* WALK_SHADOW: per node min over the subtree's triangles of |n*_y| / E_T^2 (option (b):
 * the W9E1 shadow direction (0, 1, 0) is fixed, so |w . n*| is known per treelet) */
static const double* g_hy = 0;
void walk_sim_hy(const double* h) { g_hy = h; }
static v3 g_eye;
void walk_sim_cam(const double* h, float ex, float ey, float ez) { g_hcam = h; g_eye = V(ex, ey, ez); }
double g_lost[4];
void walk_sim_lost(double* o) { for (int i = 0; i < 4; i++) o[i] = g_lost[i]; }
/* WALK_CAMX=k: the camera term over each subtree with its k triangles of smallest H
 * (the eye's distance from their planes) left out; a camera-ray cull that only those
 * triangles prevent tests them directly with the ray's interval (a second load and
 * up to k tests) and culls when none is accepted -- exact by the same argument */
static const Scene* g_scene = 0;
static int g_camx = 0, g_use_hx = 0, g_camx_bound = 0;
void walk_sim_camx_bound(int b) { g_camx_bound = b; }
static double* g_hx = 0;     /* per node: the (k+1)-th smallest H of the subtree */
static uint32_t* g_xt = 0;   /* per node: its k excluded triangles (~0u: none) */
static const uint32_t* g_tree_x = 0;
static const uint32_t* g_ids_x = 0;
static const double* g_htri = 0;
double g_camx_stat[4];   /* culls won, excluded-triangle tests, won culls refused by an accept, checks */
void walk_sim_camx_stats(double* o) { for (int i = 0; i < 4; i++) o[i] = g_camx_stat[i]; }
#define CAMX_MAX 8
typedef struct { int n; double h[CAMX_MAX + 1]; uint32_t t[CAMX_MAX + 1]; } XList;
static void xl_add(XList* l, double h, uint32_t t, int cap)
{
    for (int i = 0; i < l->n; i++) if (l->t[i] == t) return;
    int i;
    if (l->n < cap) i = l->n++;
    else if (h >= l->h[cap - 1]) return;
    else i = cap - 1;
    l->h[i] = h; l->t[i] = t;
    while (i > 0 && l->h[i] < l->h[i - 1]) {
        double th = l->h[i]; l->h[i] = l->h[i - 1]; l->h[i - 1] = th;
        uint32_t tt = l->t[i]; l->t[i] = l->t[i - 1]; l->t[i - 1] = tt;
        i--;
    }
}
static XList camx_rec(uint32_t node, uint32_t nnodes)
{
    XList l; l.n = 0;
    const int cap = g_camx + 1;
    if (node >= nnodes) return l;
    const uint32_t* tn = g_tree_x + 4 * (size_t)node;
    if ((tn[0] & 3u) == 3u) {
        for (uint32_t j = 0; j < (tn[0] >> 2); j++) xl_add(&l, g_htri[g_ids_x[tn[1] + j]], g_ids_x[tn[1] + j], cap);
    } else {
        XList a = camx_rec(2 * node + 1, nnodes), b = camx_rec(2 * node + 2, nnodes);
        for (int i = 0; i < a.n; i++) xl_add(&l, a.h[i], a.t[i], cap);
        for (int i = 0; i < b.n; i++) xl_add(&l, b.h[i], b.t[i], cap);
    }
    g_hx[node] = l.n > g_camx ? l.h[g_camx] : INFINITY;
    for (int i = 0; i < g_camx; i++) g_xt[(size_t)node * CAMX_MAX + i] = i < l.n ? l.t[i] : ~0u;
    return l;
}
void walk_sim_camx(const uint32_t* tree, const uint32_t* ids, uint32_t nnodes, const double* htri, int k)
{
    g_camx = k > CAMX_MAX ? CAMX_MAX : k;
    g_tree_x = tree; g_ids_x = ids; g_htri = htri;
    g_hx = (double*)malloc(sizeof(double) * nnodes);
    g_xt = (uint32_t*)malloc(sizeof(uint32_t) * CAMX_MAX * (size_t)nnodes);
    camx_rec(0, nnodes);
}
static double cert_margin_c(const double* c, v3 o, v3 d, const float* b);
static double cert_margin(uint32_t node, v3 o, v3 d, const float* b) { return cert_margin_c(g_cert + 7 * (size_t)node, o, d, b); }
static double cert_margin_c(const double* c, v3 o, v3 d, const float* b)
{
    const double u = 0x1p-24;
    double E2 = c[0];
    double w1 = fabs(d.x) + fabs(d.y) + fabs(d.z);
    double d1 = 0;
    for (int k = 0; k < 3; k++) {
        double a = fabs(b[k] - comp(o, k)), e = fabs(b[3 + k] - comp(o, k));
        d1 += a > e ? a : e;
    }
    double lo = 0, hi = 0;
    for (int k = 0; k < 3; k++) {
        double p = comp(d, k) * c[1 + k], q = comp(d, k) * c[4 + k];
        lo += p < q ? p : q;
        hi += p < q ? q : p;
    }
    double dlb = lo > 0 ? lo : (hi < 0 ? -hi : 0);
    static int nocone = -1;
    if (nocone < 0) { const char* e = getenv("WALK_NOCONE"); nocone = e ? atoi(e) : 0; }
    if (nocone) dlb = 0;
    double den = 2 * dlb - 32 * u * w1;
    double fl = 1e-10 / E2;
    if (g_cert_floor_only || den < fl) den = fl;
    if (g_hcam && o.x == g_eye.x && o.y == g_eye.y && o.z == g_eye.z) {
        /* camera ray: den >= winf (Hmin - 128u D1) / Dinf (rt_bsp_build.hip k_treelet_hcam) */
        double Dinf = 0, winf = fmax(fmax(fabs(d.x), fabs(d.y)), fabs(d.z));
        for (int k = 0; k < 3; k++) {
            double a = fabs(b[k] - comp(o, k)), e = fabs(b[3 + k] - comp(o, k));
            Dinf = fmax(Dinf, fmax(a, e));
        }
        const size_t nd = c - g_cert >= 0 && (c - g_cert) % 7 == 0 ? (c - g_cert) / 7 : 0;
        double H = (g_use_hx || g_camx_bound) ? g_hx[nd] : g_hcam[nd];
        double dc = winf * (H - 128 * u * d1) / Dinf;
        if (g_camx_bound && g_camx) {
            /* the excluded triangles' own |w . n*| / E_T^2, per ray (their normals stored
             * in the treelet): the camera bound holds for the rest of the subtree */
            for (int j = 0; j < g_camx; j++) {
                uint32_t t = g_xt[nd * CAMX_MAX + j];
                if (t == ~0u) continue;
                const uint32_t* ix = g_scene->idx + 4 * (size_t)t;
                v3 p0 = V(g_scene->pos[4 * ix[0]], g_scene->pos[4 * ix[0] + 1], g_scene->pos[4 * ix[0] + 2]);
                v3 p1 = V(g_scene->pos[4 * ix[1]], g_scene->pos[4 * ix[1] + 1], g_scene->pos[4 * ix[1] + 2]);
                v3 p2 = V(g_scene->pos[4 * ix[2]], g_scene->pos[4 * ix[2] + 1], g_scene->pos[4 * ix[2] + 2]);
                v3 e0 = sub(p1, p0), e1 = sub(p2, p0);
                double nn[3] = {(double)e0.y * e1.z - (double)e0.z * e1.y, (double)e0.z * e1.x - (double)e0.x * e1.z,
                                (double)e0.x * e1.y - (double)e0.y * e1.x};
                double wn = fabs(d.x * nn[0] + d.y * nn[1] + d.z * nn[2]) / E2 - 24 * u * w1;
                if (wn < dc) dc = wn;
            }
        }
        if (dc > den) den = dc;
    }
    if (g_hy && d.x == 0.0f && d.y == 1.0f && d.z == 0.0f) {
        const double hy = g_hy[(c - g_cert) / 7] - 20 * u;
        if (hy > den) den = hy;
    }
    if (g_cert_floor_only == 2) return 1e30;
    g_cert_is_floor = den == fl;
    double om = fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z));
    static double kscale = -1;
    if (kscale < 0) { const char* e = getenv("WALK_CERT_K"); kscale = e ? atof(e) : 1.0; }
    return kscale * 34 * u * d1 * w1 / den + 2 * u * d1 + 0x1p-20 * (om + g_cert_mag);
}
/* WALK_CELLS: n x 6 doubles, the box of the cells of the subtree's non-empty
 * leaves (the cells are the half-space intersections along the path: +-inf
 * where unbounded) -- every accept of the reference walk in the subtree lies
 * in one of them on every axis with |d| >= 1e-8 */
static const double* g_cells = 0;
void walk_sim_cells(const double* c) { g_cells = c; }
static int cell_clip(uint32_t node, v3 o, v3 d, double* t0p, double* t1p)
{
    const double* b = g_cells + 6 * (size_t)node;
    double om = fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z));
    double m = 0x1p-20 * (om + g_cert_mag);
    double t0 = *t0p, t1 = *t1p;
    for (int k = 0; k < 3; k++) {
        double dk = comp(d, k), ok = comp(o, k);
        if (!(fabs(dk) >= 1e-8)) continue;
        double a = (b[k] - m - ok) / dk, cc = (b[3 + k] + m - ok) / dk;
        if (a > cc) { double x = a; a = cc; cc = x; }
        if (a > t0) t0 = a;
        if (cc < t1) t1 = cc;
    }
    *t0p = t0;
    *t1p = t1;
    return t0 > t1 + (fabs(t0) + fabs(t1)) * 0x1p-18;
}
static int box_miss(uint32_t node, v3 o, v3 d, float tmin, float tmax)
{
    const float* b = g_boxes + 6 * (size_t)node;
    if (g_cells && b[0] <= b[3]) {
        double c0 = tmin, c1 = tmax;
        if (cell_clip(node, o, d, &c0, &c1)) return 1;
        tmin = (float)c0 > tmin ? (float)c0 : tmin;   /* approximately: the model only counts trips */
        tmax = (float)c1 < tmax ? (float)c1 : tmax;
    }
    if (g_cert && b[0] <= b[3]) {
        double m = cert_margin(node, o, d, b);
        g_cert_margin_sum += m; g_cert_margin_n += 1;
        double t0 = tmin, t1 = tmax;
        for (int k = 0; k < 3; k++) {
            double dk = comp(d, k), ok = comp(o, k);
            if (fabs(dk) < 1e-8) { if (g_axis && dk == 0.0f && (ok < b[k] - m || ok > b[3 + k] + m)) return 1; continue; }
            double a = (b[k] - m - ok) / dk, cc = (b[3 + k] + m - ok) / dk;
            if (a > cc) { double x = a; a = cc; cc = x; }
            if (a > t0) t0 = a;
            if (cc < t1) t1 = cc;
        }
        g_tn = (float)t0;
        g_tf = (float)t1;
        int miss = t0 > t1 + (fabs(t0) + fabs(t1)) * 0x1p-18;
        if (!miss && g_camx && !g_camx_bound && g_hcam && o.x == g_eye.x && o.y == g_eye.y && o.z == g_eye.z && isfinite(g_hx[node])) {
            g_use_hx = 1;
            const double m2 = cert_margin(node, o, d, b);
            g_use_hx = 0;
            double a0 = tmin, a1 = tmax;
            for (int k = 0; k < 3; k++) {
                double dk = comp(d, k), ok = comp(o, k);
                if (fabs(dk) < 1e-8) { if (g_axis && dk == 0.0f && (ok < b[k] - m2 || ok > b[3 + k] + m2)) { a0 = 1; a1 = 0; } continue; }
                double a = (b[k] - m2 - ok) / dk, cc = (b[3 + k] + m2 - ok) / dk;
                if (a > cc) { double x = a; a = cc; cc = x; }
                if (a > a0) a0 = a;
                if (cc < a1) a1 = cc;
            }
            g_camx_stat[3] += 1;
            if (a0 > a1 + (fabs(a0) + fabs(a1)) * 0x1p-18) {
                int acc = 0;
                for (int j = 0; j < g_camx; j++) {
                    uint32_t t = g_xt[(size_t)node * CAMX_MAX + j];
                    if (t == ~0u) continue;
                    float dd;
                    g_camx_stat[1] += 1;
                    if (tri(g_scene, t, o, d, tmin, tmax, &dd)) { acc = 1; break; }
                }
                if (!acc) { g_camx_stat[0] += 1; return 1; }
                g_camx_stat[2] += 1;
            }
        }
        if (g_spec) {
            /* the fast margin's cull and interval beside the certified ones */
            double om = fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z));
            double mf = fmax(om, g_cert_mag) * 0x1p-10;
            double a0 = tmin, a1 = tmax;
            int fmiss = 0;
            for (int k = 0; k < 3; k++) {
                double dk = comp(d, k), ok = comp(o, k);
                if (fabs(dk) < 1e-8) { if (g_axis && dk == 0.0f && (ok < b[k] - mf || ok > b[3 + k] + mf)) fmiss = 1; continue; }
                double a = (b[k] - mf - ok) / dk, cc = (b[3 + k] + mf - ok) / dk;
                if (a > cc) { double x = a; a = cc; cc = x; }
                if (a > a0) a0 = a;
                if (cc < a1) a1 = cc;
            }
            fmiss = fmiss || a0 > a1 + (fabs(a0) + fabs(a1)) * 0x1p-18;
            g_tn_c = (float)t0;
            g_tf_c = (float)t1;
            if (miss) { g_spec_stat[3] += 1; return 1; }
            if (fmiss) { g_spec_stat[1] += 1; g_spec_flag = 1; return 1; }
            g_tn = (float)(a0 > t0 ? a0 : t0);
            g_tf = (float)(a1 < t1 ? a1 : t1);
            return 0;
        }
        if (!miss) {
            /* would the fast margin (2^-10 of max(|o|, scene)) have culled? */
            double om = fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z));
            double mf = fmax(om, g_cert_mag) * 0x1p-10;
            double a0 = tmin, a1 = tmax;
            for (int k = 0; k < 3; k++) {
                double dk = comp(d, k), ok = comp(o, k);
                if (fabs(dk) < 1e-8) continue;
                double a = (b[k] - mf - ok) / dk, cc = (b[3 + k] + mf - ok) / dk;
                if (a > cc) { double x = a; a = cc; cc = x; }
                if (a > a0) a0 = a;
                if (cc < a1) a1 = cc;
            }
            if (a0 > a1) g_lost[g_cert_is_floor] += 1;
        }
        return miss;
    }
    g_tn = tmin;
    g_tf = tmax;
    if (b[0] > b[3]) return 1;   /* empty subtree */
    float t0 = tmin, t1 = tmax;
    for (int k = 0; k < 3; k++) {
        float dk = comp(d, k), ok = comp(o, k);
        if (dk == 0.0f) { if (ok < b[k] || ok > b[3 + k]) return 1; continue; }
        float a = (b[k] - ok) / dk, c = (b[3 + k] - ok) / dk;
        if (a > c) { float x = a; a = c; c = x; }
        if (a > t0) t0 = a;
        if (c < t1) t1 = c;
    }
    g_tn = t0;
    g_tf = t1;
    return t0 > t1;
}
void walk_sim_levels(int l) { g_levels = l; }
static int is_empty_leaf(const Scene* s, uint32_t node) { return (s->tree[4 * node] & 3u) == 3u && (s->tree[4 * node] >> 2) == 0; }
static uint32_t depth_of(uint32_t n0) { uint32_t m = n0 + 1, d = 0; while (m > 1) { m >>= 1; d++; } return d; }

/* stats[variant][k]: 0 walk trips, 1 leaf trips, 2 interior decisions, 3 leaf visits,
 * 4 empty leaf visits, 5 tests, 6 pushes, 7 pops, 8 hits, 9 mismatches vs v0 */
enum { S_WT, S_LT, S_DEC, S_LEAF, S_EMPTY, S_TEST, S_PUSH, S_POP, S_HIT, S_BAD, S_BOXT, S_N };

/* WALK_TRACE: the trip sequence of every ray's v4 walk (0 walking trip, 1 leaf trip),
 * concatenated in ray order, with each ray's start offset (tools/two_ray_price.py) */
static uint8_t* g_trace = 0;
static uint64_t g_trace_cap = 0, g_trace_n = 0;
static uint64_t* g_trace_off = 0;
static int g_trace_on = 0;
void walk_sim_trace(uint8_t* buf, uint64_t cap, uint64_t* off) { g_trace = buf; g_trace_cap = cap; g_trace_off = off; g_trace_n = 0; }
uint64_t walk_sim_trace_len(void) { return g_trace_n; }
static void trace_put(int kind) { if (g_trace_on && g_trace_n < g_trace_cap) g_trace[g_trace_n++] = (uint8_t)kind; }

static int walk(const Scene* s, int var, v3 o, v3 d, float tmin, float tmax, int anyhit, float* hd, uint32_t* htri,
                double* st)
{
    uint32_t stk_node[64], stk_dep[64], stk_skip[64];
    float stk_t[64], stk_tmax[64];
    int sp = 0;
    uint32_t node = 0;
    int found = 0;
    for (;;) {
        /* one walking trip from `node`: up to three levels */
        st[S_WT] += 1;
        if (var == 4) trace_put(0);
        int lv = 0, reached_leaf = 0, do_pop = 0;
        float ctn = -INFINITY, ctf = INFINITY;   /* v4 + WALK_CLIP: decisions against the box's interval */
        static int box_every = -1;
        if (box_every < 0) { const char* e = getenv("WALK_BOX_EVERY"); box_every = e ? atoi(e) : 1; }
        const int test_box = box_every <= 1 || ((depth_of(node) / 3) % (uint32_t)box_every) == 0;
        if (var >= 3 && g_boxes && test_box) st[S_BOXT] += 1;
        if (var >= 3 && g_boxes && test_box && (node == 0 || !g_root_only) && box_miss(node, o, d, tmin, tmax)) {
            do_pop = 1;   /* v3: the subtree's content misses the ray interval */
            g_cull[depth_of(node) < 32 ? depth_of(node) : 31] += 1;
            g_cull_leaf += (s->tree[4 * node] & 3u) == 3u;
            lv = g_levels;
        } else if (var == 4 && g_boxes && g_clip && test_box) {
            ctn = g_tn;
            ctf = g_tf;
        }
        while (lv < g_levels) {
            if (var == 4 && g_cull_every && lv > 0 && box_miss(node, o, d, tmin, tmax)) {
                do_pop = 1;   /* v4 + WALK_CULL_EVERY: a child's content box too (boxes of every treelet level) */
                g_cull[depth_of(node) < 32 ? depth_of(node) : 31] += 1;
                break;
            }
            const uint32_t* tn = s->tree + 4 * (size_t)node;
            uint32_t ax = tn[0] & 3u;
            if (ax == 3u) {
                st[S_LEAF] += 1;
                uint32_t cnt = tn[0] >> 2, first = tn[1];
                if (cnt == 0) {
                    st[S_EMPTY] += 1;
                    do_pop = 1;
                } else {
                    /* leaf trips: two tests per trip */
                    uint32_t j = 0;
                    while (j < cnt) {
                        if (var == 4 && g_chunk && j % (uint32_t)g_chunk == 0 && cnt > (uint32_t)g_chunk_min) {
                            /* v4 + WALK_CHUNK: a header trip tests the box of the next
                             * g_chunk records (in leaf order) and skips them on a miss */
                            uint32_t e = j + (uint32_t)g_chunk < cnt ? j + (uint32_t)g_chunk : cnt;
                            float bb[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
                            for (uint32_t q = j; q < e; q++) {
                                const uint32_t* ix = s->idx + 4 * (size_t)s->ids[first + q];
                                for (int vv = 0; vv < 3; vv++)
                                    for (int a = 0; a < 3; a++) {
                                        float x = s->pos[4 * ix[vv] + a];
                                        if (x < bb[a]) bb[a] = x;
                                        if (x > bb[3 + a]) bb[3 + a] = x;
                                    }
                            }
                            st[S_LT] += g_chunk_free ? 0 : 1;
                            int miss;
                            if (g_cert) {
                                /* the run's certification data, as the repack would store it */
                                double c7[7] = {0, INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
                                for (uint32_t q = j; q < e; q++) {
                                    const uint32_t* ix = s->idx + 4 * (size_t)s->ids[first + q];
                                    v3 p0 = V(s->pos[4 * ix[0]], s->pos[4 * ix[0] + 1], s->pos[4 * ix[0] + 2]);
                                    v3 p1 = V(s->pos[4 * ix[1]], s->pos[4 * ix[1] + 1], s->pos[4 * ix[1] + 2]);
                                    v3 p2 = V(s->pos[4 * ix[2]], s->pos[4 * ix[2] + 1], s->pos[4 * ix[2] + 2]);
                                    v3 e0 = sub(p1, p0), e1 = sub(p2, p0);
                                    double nn[3] = {(double)e0.y * e1.z - (double)e0.z * e1.y, (double)e0.z * e1.x - (double)e0.x * e1.z,
                                                    (double)e0.x * e1.y - (double)e0.y * e1.x};
                                    double E = fmax(fmax(fmax(fabs(e0.x), fabs(e0.y)), fabs(e0.z)), fmax(fmax(fabs(e1.x), fabs(e1.y)), fabs(e1.z)));
                                    if (E * E > c7[0]) c7[0] = E * E;
                                    for (int a = 0; a < 3; a++) {
                                        if (nn[a] < c7[1 + a]) c7[1 + a] = nn[a];
                                        if (nn[a] > c7[4 + a]) c7[4 + a] = nn[a];
                                    }
                                }
                                if (c7[0] > 0)
                                    for (int a = 1; a < 7; a++) c7[a] /= c7[0];
                                else
                                    for (int a = 1; a < 7; a++) c7[a] = 0, c7[0] = 1;
                                double m = cert_margin_c(c7, o, d, bb);
                                double t0 = tmin, t1 = tmax;
                                for (int k = 0; k < 3; k++) {
                                    double dk = comp(d, k), ok = comp(o, k);
                                    if (fabs(dk) < 1e-8) continue;
                                    double a = (bb[k] - m - ok) / dk, cc = (bb[3 + k] + m - ok) / dk;
                                    if (a > cc) { double x = a; a = cc; cc = x; }
                                    if (a > t0) t0 = a;
                                    if (cc < t1) t1 = cc;
                                }
                                miss = t0 > t1 + (fabs(t0) + fabs(t1)) * 0x1p-18;
                            } else {
                                for (int a = 0; a < 3; a++) { bb[a] -= g_chunk_margin; bb[3 + a] += g_chunk_margin; }
                                const float* sv = g_boxes;
                                g_boxes = bb;
                                miss = box_miss(0, o, d, tmin, tmax);
                                g_boxes = sv;
                            }
                            if (miss) { j = e; continue; }
                        }
                        st[S_LT] += 1;
                        if (var == 4) trace_put(1);
                        for (int k = 0; k < 2 && j < cnt; k++, j++) {
                            float dd;
                            st[S_TEST] += 1;
                            if (tri(s, s->ids[first + j], o, d, tmin, tmax, &dd)) {
                                tmax = dd;
                                *hd = dd;
                                *htri = s->ids[first + j];
                                found = 1;
                                if (anyhit) { j = cnt; break; }
                            }
                        }
                    }
                    if (found) { st[S_HIT] += 1; return 1; }
                    do_pop = 1;
                }
                reached_leaf = 1;
                break;
            }
            st[S_DEC] += 1;
            float ad = comp(d, (int)ax), ao = comp(o, (int)ax);
            uint32_t nearn = ad >= 0.0f ? tn[2] : tn[3], farn = ad >= 0.0f ? tn[3] : tn[2];
            float den = fabsf(ad) < 1.0e-8f ? 1.0e-8f : ad;
            float t = (s->planes[node] - ao) / den;
            if (t > tmax || t > ctf) {
                if (g_spec && !(t > tmax) && !(t > g_tf_c)) { g_spec_flag = 1; g_spec_stat[2] += 1; }
                node = nearn;
            } else if (t < tmin || t < ctn) {
                if (g_spec && !(t < tmin) && !(t < g_tn_c)) { g_spec_flag = 1; g_spec_stat[2] += 1; }
                node = farn;
            } else if ((var == 1 || var == 2 || var == 3) && is_empty_leaf(s, nearn)) {
                /* push + visit the empty near leaf + pop, folded: the counted
                 * leaf visit and pop of v0 are skipped */
                tmin = t;
                node = farn;
            } else {
                st[S_PUSH] += 1;
                stk_node[sp] = farn;
                stk_dep[sp] = depth_of(node);
                stk_skip[sp] = (var == 2 || var == 3) && is_empty_leaf(s, farn);
                stk_t[sp] = t;
                stk_tmax[sp] = tmax;
                sp++;
                tmax = t;
                node = nearn;
            }
            lv++;
        }
        if (!reached_leaf && !do_pop) continue;   /* next trip from the node three levels down */
        if (do_pop) {
            /* pop (v2: past entries whose far child is an empty leaf) */
            for (;;) {
                if (sp == 0) return 0;
                sp--;
                st[S_POP] += 1;
                node = stk_node[sp];
                tmin = stk_t[sp];
                tmax = stk_tmax[sp];
                if (!stk_skip[sp]) break;
                st[S_LEAF] += 1;   /* the reference visits that empty leaf */
                st[S_EMPTY] += 1;
            }
        }
    }
}

/* rays: n x 8 floats (o.xyz, d.xyz, tmin, tmax), flags: n (bit 0 anyhit).
 * out: 3 x S_N doubles (per variant) */
int walk_sim(const uint32_t* tree, const float* planes, const uint32_t* ids, const float* pos, const uint32_t* idx,
             const float* rays, const uint32_t* flags, uint32_t n, double* out)
{
    Scene s = {tree, planes, ids, pos, idx};
    g_scene = &s;
    memset(out, 0, sizeof(double) * 5 * S_N);
    for (uint32_t i = 0; i < n; i++) {
        const float* r = rays + 8 * (size_t)i;
        v3 o = V(r[0], r[1], r[2]), d = V(r[3], r[4], r[5]);
        float h0 = -1, hv;
        uint32_t t0 = ~0u, tv;
        int f0 = walk(&s, 0, o, d, r[6], r[7], flags[i] & 1, &h0, &t0, out);
        for (int v = 1; v < (g_boxes ? 5 : 3); v++) {
            hv = -1;
            tv = ~0u;
            g_spec_flag = 0;
            g_tn_c = -INFINITY;
            g_tf_c = INFINITY;
            if (v == 4 && g_trace) { g_trace_off[i] = g_trace_n; g_trace_on = 1; }
            int fv = walk(&s, v, o, d, r[6], r[7], flags[i] & 1, &hv, &tv, out + v * S_N);
            g_trace_on = 0;
            if (v == 4 && g_spec && g_spec_flag) {
                /* the re-walk of a flagged ray: certified only (its trips go to rewalk) */
                double st2[S_N];
                memset(st2, 0, sizeof st2);
                g_spec = 0;
                hv = -1;
                tv = ~0u;
                fv = walk(&s, v, o, d, r[6], r[7], flags[i] & 1, &hv, &tv, st2);
                g_spec = 1;
                g_spec_stat[0] += 1;
                g_spec_stat[4] += st2[S_WT] + st2[S_LT];
                g_spec_stat[5] += st2[S_TEST];
            }
            if (fv != f0 || (f0 && (hv != h0 || tv != t0))) {
                out[v * S_N + S_BAD] += 1;
                if (g_bad_n < 64) {
                    g_bad[g_bad_n * 4] = (double)i;
                    g_bad[g_bad_n * 4 + 1] = (double)v;
                    g_bad[g_bad_n * 4 + 2] = f0 ? (double)t0 : -1.0;
                    g_bad[g_bad_n * 4 + 3] = fv ? (double)tv : -1.0;
                    g_bad_n++;
                }
            }
        }
    }
    return 0;
}

/* Compact-trail model: the trail's pending
 * entries in push order, K slots per lane in LDS as a ring (entry p in slot
 * p mod K, written on push only), an entry overwritten by a later push is "lost"
 * and must be recomputed when popped (its value is the t of the entry below it,
 * (plane - o)/d at an ancestor: a node load and an exact division).  Per ray and
 * K in ks[0..nk): out[k*4 + 0] pushes, +1 pushes that overwrite a pending entry,
 * +2 pops, +3 pops of lost entries.  Closest-hit walk of v0 (anyhit per flags). */
int trail_sim(const uint32_t* tree, const float* planes, const uint32_t* ids, const float* pos, const uint32_t* idx,
              const float* rays, const uint32_t* flags, uint32_t n, const uint32_t* ks, uint32_t nk, double* out)
{
    Scene s = {tree, planes, ids, pos, idx};
    memset(out, 0, sizeof(double) * 4 * nk);
    for (uint32_t i = 0; i < n; i++) {
        const float* r = rays + 8 * (size_t)i;
        v3 o = V(r[0], r[1], r[2]), d = V(r[3], r[4], r[5]);
        float tmin = r[6], tmax = r[7];
        int anyhit = flags[i] & 1;
        uint32_t stk_node[64];
        float stk_t[64], stk_tmax[64];
        int owner[16][64];
        for (uint32_t k = 0; k < nk; k++)
            for (int q = 0; q < 64; q++) owner[k][q] = -1;
        int sp = 0;
        uint32_t node = 0;
        for (;;) {
            const uint32_t* tn = s.tree + 4 * (size_t)node;
            uint32_t ax = tn[0] & 3u;
            if (ax == 3u) {
                uint32_t cnt = tn[0] >> 2, first = tn[1];
                int found = 0;
                for (uint32_t j = 0; j < cnt; j++) {
                    float dd;
                    if (tri(&s, s.ids[first + j], o, d, tmin, tmax, &dd)) {
                        tmax = dd;
                        found = 1;
                        if (anyhit) break;
                    }
                }
                if (found || sp == 0) break;
                sp--;
                for (uint32_t k = 0; k < nk; k++) {
                    out[4 * k + 2] += 1;
                    if (owner[k][sp % ks[k]] != sp) out[4 * k + 3] += 1;
                }
                node = stk_node[sp];
                tmin = stk_t[sp];
                tmax = stk_tmax[sp];
                continue;
            }
            float ad = comp(d, (int)ax), ao = comp(o, (int)ax);
            uint32_t nearn = ad >= 0.0f ? tn[2] : tn[3], farn = ad >= 0.0f ? tn[3] : tn[2];
            float den = fabsf(ad) < 1.0e-8f ? 1.0e-8f : ad;
            float t = (s.planes[node] - ao) / den;
            if (t > tmax) {
                node = nearn;
            } else if (t < tmin) {
                node = farn;
            } else {
                for (uint32_t k = 0; k < nk; k++) {
                    out[4 * k] += 1;
                    int q = sp % ks[k];
                    if (owner[k][q] >= 0 && owner[k][q] < sp) out[4 * k + 1] += 1;
                    owner[k][q] = sp;
                }
                stk_node[sp] = farn;
                stk_t[sp] = t;
                stk_tmax[sp] = tmax;
                sp++;
                tmax = t;
                node = nearn;
            }
        }
    }
    return 0;
}
