/* cert_bound.c -- empirical check of the certified culling margin (test code;
 * DESIGN.md section 4 "Certified culling", rt_kernels.hip bsp_box_miss).
 *
 * The claim: when intersect_triangle (w7e3.wgsl:286-332, f32, no contraction,
 * correctly rounded division) accepts a ray (o, w) at distance t, the point
 * Q = o + t*w (exact) lies within m (L-inf) of the triangle's bounding box,
 * where m is bsp_box_miss's certified margin for a subtree holding that
 * triangle:
 *   m = D1 * (36u * w1 / max(F, 2 Dlb - 20u w1) + 2u) + max(|o|inf, scene) * 2^-19
 * D1 = sum_a max(|bmin_a - o_a|, |bmax_a - o_a|), w1 = |w|_1, F = 1e-10 / E2,
 * E2 = max(|e0|inf, |e1|inf)^2, 2 Dlb = |w . c| - |w| . r, the lower bound of
 * |w . n*| / E2 over the normal box stored as f16 centre c and radius r.  This harness draws adversarial rays -- at
 * the 1e-10 denominator floor, at grazing angles, from far away -- against
 * random triangles, runs the f32 test, and for every accept measures the
 * distance of Q from the box in units of m (it must stay below 1), with Q
 * evaluated in long double.
 * Build: gcc -O2 -ffp-contract=off -o cert_bound cert_bound.c -lm
 * usage: cert_bound <trials> <seed> [camera 0/1]   prints: accepts max_ratio floor_accepts
 * With camera 1 the margin also takes the camera bound (rt_kernels.hip bsp_box_miss)
 * with each ray's origin as the eye -- every trial is then a camera ray. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int g_cam = 0;
static long g_cam_binds = 0;   /* accepts whose margin the camera bound set */   /* argv[3] = 1: the camera bound too, with every ray's origin as the eye */

typedef struct { float x, y, z; } v3;
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 cross(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static float cmp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* intersect_triangle_indexed, w7e3.wgsl:286-332 (records: e0 = v1 - v0, e1 = v2 - v0, n = cross) */
static int tri_test(v3 v0, v3 v1, v3 v2, v3 o, v3 w, float tmin, float tmax, float* dist, float* den_out)
{
    v3 e0 = sub(v1, v0), e1 = sub(v2, v0), ov = sub(v0, o);
    v3 n = cross(e0, e1), nom = cross(ov, w);
    float den = dot(w, n);
    *den_out = den;
    if (fabsf(den) < 1e-10f) return 0;
    float b = dot(nom, e1) / den, g = -dot(nom, e0) / den, d = dot(ov, n) / den;
    if (b < 0.0f || g < 0.0f || b + g > 1.0f || d > tmax || d < tmin) return 0;
    *dist = d;
    return 1;
}

static uint64_t st = 0x9E3779B97F4A7C15ull;
static double U(void)
{
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return (double)(st >> 11) * 0x1p-53;
}
static double N01(void) { return sqrt(-2.0 * log(U() + 1e-300)) * cos(6.283185307179586 * U()); }

/* round to the f16 grid toward -inf (dir < 0) or +inf (dir > 0), |x| <= 2 */
static float h_round(double x, int dir)
{
    double ax = fabs(x);
    double ulp = ax >= 0x1p-14 ? ldexp(1.0, (int)floor(log2(ax)) - 10) : 0x1p-24;
    double q = x / ulp;
    q = dir < 0 ? floor(q) : ceil(q);
    return (float)(q * ulp);
}

/* bsp_box_miss's certified margin (f32, the kernel's operation order) for the
 * one-triangle subtree {v0, v1, v2} */
static float cert_margin(v3 v0, v3 v1, v3 v2, v3 o, v3 w, float scene, float bmin[3], float bmax[3])
{
    v3 vs[3] = {v0, v1, v2};
    for (int a = 0; a < 3; a++) {
        bmin[a] = fminf(fminf(cmp(vs[0], a), cmp(vs[1], a)), cmp(vs[2], a));
        bmax[a] = fmaxf(fmaxf(cmp(vs[0], a), cmp(vs[1], a)), cmp(vs[2], a));
    }
    /* the repack's certification data (rt_bsp_build.hip k_leaf_boxes / k_bsp_repack) */
    v3 e0 = sub(v1, v0), e1 = sub(v2, v0);
    double n[3] = {(double)e0.y * e1.z - (double)e0.z * e1.y, (double)e0.z * e1.x - (double)e0.x * e1.z,
                   (double)e0.x * e1.y - (double)e0.y * e1.x};
    double E = fmax(fmax(fmax(fabs(e0.x), fabs(e0.y)), fabs(e0.z)), fmax(fmax(fabs(e1.x), fabs(e1.y)), fabs(e1.z)));
    double E2 = E * E;
    float F = INFINITY, cc[3] = {0, 0, 0}, rr[3] = {0, 0, 0};
    if (E2 > 0) {
        F = (float)(1e-10 / E2 * (1.0 - 0x1p-30));   /* rounded down (the kernel: __double2float_rd) */
        F = nextafterf(F, 0.0f);
        for (int k = 0; k < 3; k++) {
            double a = n[k] * (1.0 / E2);
            double lo = a - fabs(a) * 0x1p-40, hi = a + fabs(a) * 0x1p-40;
            double mid = 0.5 * (lo + hi);
            /* nearest f16 to the centre, then the radius rounded up */
            float cd = h_round(mid, -1), cu = h_round(mid, +1);
            cc[k] = (mid - cd <= cu - mid) ? cd : cu;
            rr[k] = h_round(fmax(hi - cc[k], cc[k] - lo) * (1.0 + 0x1p-40), +1);
        }
    }
    float oo[3] = {o.x, o.y, o.z};
    float D1 = 0.0f;
    for (int a = 0; a < 3; a++) {
        float dl = bmin[a] - oo[a], dh = bmax[a] - oo[a];
        D1 += fmaxf(fabsf(dl), fabsf(dh));
    }
    float w1 = fabsf(w.x) + fabsf(w.y) + fabsf(w.z);
    float wc = fmaf(w.z, cc[2], fmaf(w.y, cc[1], w.x * cc[0]));
    float wr = fmaf(fabsf(w.z), rr[2], fmaf(fabsf(w.y), rr[1], fabsf(w.x) * rr[0]));
    float dlb2 = fabsf(wc) - wr;
    float den = fmaxf(F, dlb2 - (20.0f * 0x1p-24f) * w1);
    if (g_cam) {
        /* the camera bound, with the ray's origin as the eye: H = |(v0 - o) . n*| / E2
         * rounded down (rt_bsp_build.hip tri_hcam), bf16-truncated as the treelet stores it */
        double dd[3] = {(double)v0.x - o.x, (double)v0.y - o.y, (double)v0.z - o.z};
        double dot = dd[0] * n[0] + dd[1] * n[1] + dd[2] * n[2];
        double err = 0x1p-45 * (fabs(dd[0] * n[0]) + fabs(dd[1] * n[1]) + fabs(dd[2] * n[2]));
        double eta = fabs(dot) - err;
        float H = E2 > 0 ? (eta > 0 ? (float)(eta / E2 * (1.0 - 0x1p-19)) : 0.0f) : INFINITY;
        H = nextafterf(H, 0.0f);
        /* the treelet's camera term G (rt_bsp_build.hip k_treelet_hcam): from H (f32),
         * the box's L1 / L-inf distances to the eye (f64, rounded up), rounded down,
         * an f16 rounded down as the treelet stores it */
        double D1e = 0.0, Dinfe = 0.0;
        for (int a = 0; a < 3; a++) {
            double d = fmax(fabs((double)bmin[a] - oo[a]), fabs((double)bmax[a] - oo[a]));
            D1e += d;
            Dinfe = fmax(Dinfe, d);
        }
        D1e *= 1.0 + 0x1p-40;
        Dinfe *= 1.0 + 0x1p-40;
        float G = 0.0f;
        if (H == INFINITY) G = INFINITY;
        else if (Dinfe > 0.0 && H - 128.0 * 0x1p-24 * D1e > 0.0) {
            G = (float)((H - 128.0 * 0x1p-24 * D1e) / Dinfe * (1.0 - 0x1p-20));
            G = nextafterf(G, 0.0f);
        }
        G = isinf(G) ? G : (float)h_round(G, -1);   /* f16, rounded down */
        float winf = fmaxf(fmaxf(fabsf(w.x), fabsf(w.y)), fabsf(w.z));
        float dcam = G * winf;
        if (dcam > den) g_cam_binds++;
        den = fmaxf(den, dcam);
    }
    float mo = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    /* v_rcp_f32 is within 1 ulp: emulate the worse side */
    float rc = nextafterf(1.0f / den, 0.0f);
    return fmaf(D1, fmaf((36.0f * 0x1p-24f) * w1, rc, 2.0f * 0x1p-24f), fmaxf(mo * 0x1p-19f, scene * 0x1p-19f));
}

int main(int argc, char** argv)
{
    long trials = argc > 1 ? atol(argv[1]) : 1000000;
    st ^= (uint64_t)(argc > 2 ? atol(argv[2]) : 1) * 0x2545F4914F6CDD1Dull;
    g_cam = argc > 3 ? atoi(argv[3]) : 0;
    long acc = 0, floor_acc = 0;
    double worst = 0.0;
    for (long it = 0; it < trials; it++) {
        /* a triangle: size 10^[-4, 0.5], centre within the scene, random shape (slivers too) */
        double scale = pow(10.0, -4.0 + 4.5 * U()), cen[3];
        double scene = pow(10.0, -1.0 + 3.0 * U());
        for (int a = 0; a < 3; a++) cen[a] = (2 * U() - 1) * scene;
        v3 vs[3];
        for (int k = 0; k < 3; k++)
            vs[k] = V((float)(cen[0] + scale * N01()), (float)(cen[1] + scale * N01()), (float)(cen[2] + scale * N01()));
        if (U() < 0.1) vs[2] = V((float)(vs[0].x + 1e-3 * (vs[1].x - vs[0].x)), vs[1].y, vs[1].z);   /* slivers */
        v3 e0 = sub(vs[1], vs[0]), e1 = sub(vs[2], vs[0]);
        double n[3] = {(double)e0.y * e1.z - (double)e0.z * e1.y, (double)e0.z * e1.x - (double)e0.x * e1.z,
                       (double)e0.x * e1.y - (double)e0.y * e1.x};
        double ln = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (!(ln > 0)) continue;
        /* a target point near the triangle (inside or up to 3 sizes off), a direction
         * at an elevation from its plane chosen so |denom| lands near the 1e-10 floor
         * (half of the trials) or anywhere down to 1e-9 rad */
        double bu = U(), bv = U();
        if (bu + bv > 1) { bu = 1 - bu; bv = 1 - bv; }
        double off = U() < 0.5 ? 0.0 : 3.0 * U();
        double p[3];
        for (int a = 0; a < 3; a++)
            p[a] = cmp(vs[0], a) + bu * cmp(e0, a) + bv * cmp(e1, a) + off * scale * N01();
        double t1[3] = {N01(), N01(), N01()};
        double nn[3] = {n[0] / ln, n[1] / ln, n[2] / ln};
        double dt = t1[0] * nn[0] + t1[1] * nn[1] + t1[2] * nn[2];
        for (int a = 0; a < 3; a++) t1[a] -= dt * nn[a];
        double lt = sqrt(t1[0] * t1[0] + t1[1] * t1[1] + t1[2] * t1[2]);
        double wlen = pow(10.0, -1.0 + 2.0 * U());
        double se = U() < 0.5 ? (1e-10 * (1.0 + 3.0 * U())) / (ln * wlen) : pow(10.0, -9.0 + 8.0 * U());
        if (se > 1) se = 1;
        double ce = sqrt(1 - se * se), sg = U() < 0.5 ? -1 : 1;
        double w[3];
        for (int a = 0; a < 3; a++) w[a] = wlen * (ce * t1[a] / lt + sg * se * nn[a]);
        double dist = pow(10.0, -2.0 + 3.0 * U()) * scene;
        v3 o = V((float)(p[0] - dist * w[0] / wlen), (float)(p[1] - dist * w[1] / wlen), (float)(p[2] - dist * w[2] / wlen));
        v3 wf = V((float)w[0], (float)w[1], (float)w[2]);
        float t, den;
        if (!tri_test(vs[0], vs[1], vs[2], o, wf, 1e-4f, 5000.0f, &t, &den)) continue;
        acc++;
        if (fabsf(den) < 1e-9f) floor_acc++;
        float bmin[3], bmax[3];
        float m = cert_margin(vs[0], vs[1], vs[2], o, wf, (float)(scene + 4 * scale), bmin, bmax);
        long double q[3] = {(long double)o.x + (long double)t * wf.x, (long double)o.y + (long double)t * wf.y,
                            (long double)o.z + (long double)t * wf.z};
        long double dd = 0;
        for (int a = 0; a < 3; a++) {
            long double lo = bmin[a] - q[a], hi = q[a] - bmax[a];
            long double g = lo > hi ? lo : hi;
            if (g > dd) dd = g;
        }
        double ratio = (double)(dd / m);
        if (ratio > worst) worst = ratio;
    }
    printf("%ld %.6g %ld %ld\n", acc, worst, floor_acc, g_cam_binds);
    return 0;
}
