/*
 * rt_detmath.h -- the f32 transcendental functions this implementation pins.
 *
 * WGSL leaves the precision of sin/cos/acos implementation-defined (the
 * reference's values come from naga 0.13 -> SPIR-V -> the Vulkan driver and
 * are "parity unpinned").  One ulp of difference in
 * setup_indirect (res/shaders/w7e3.wgsl:472-489) changes a path's next
 * direction, so the HIP kernel and the CPU oracle must evaluate the SAME
 * f32 operation sequence.  This header is that specification: Cody-Waite
 * range reduction + minimax polynomials (Cephes single-precision
 * coefficients), every operation an IEEE-754 binary32 add/mul/div/sqrt with
 * round-to-nearest-even.  It must be compiled WITHOUT fp contraction
 * (-ffp-contract=off) and without fast-math, with correctly rounded f32
 * division/sqrt (clang HIP: -fhip-fp32-correctly-rounded-divide-sqrt).
 *
 * Included by the product kernels (C++/HIP) and by the C oracle.
 */
#ifndef RT02562_DETMATH_H
#define RT02562_DETMATH_H

#if defined(__HIPCC__) || defined(__HIP__)
#define RT_HD __host__ __device__ static inline
#else
#define RT_HD static inline
#endif

#define RT_DET_PIF    3.14159265358979323846f   /* == f32 PI of the shaders */
#define RT_DET_PIO2F  1.57079632679489661923f

RT_HD float rt_det_sqrtf(float x) { return __builtin_sqrtf(x); }

/* Correctly rounded x / d from r = RN(1/d) (Markstein's theorem: with y within
 * 1/2 ulp of 1/d and q within 1 ulp of x/d, RN(q + (x - d*q)*y) == RN(x/d); the
 * first correction brings RN(x*r), up to 2 ulp off, within 1 ulp).  Exact when
 * d is a finite normal number, r == RN(1/d) and 2^-100 <= |x| <= 2^100 with
 * |x/d| < 2^127 (no overflow, and every residual representable); callers use
 * x / d outside that range.  tests/test_fastdiv.py checks it bitwise against
 * IEEE division on ~10^8 operand pairs. */
RT_HD float rt_div_by_recip(float x, float d, float r)
{
    float q = x * r;
    float e = __builtin_fmaf(-d, q, x);
    q = __builtin_fmaf(e, r, q);
    e = __builtin_fmaf(-d, q, x);
    return __builtin_fmaf(e, r, q);
}
RT_HD int rt_div_by_recip_ok(float x) { float a = __builtin_fabsf(x); return a >= 0x1p-100f && a <= 0x1p100f; }

/* WGSL min/max/saturate/sign on f32 are implementation-defined for NaN and
 * for the sign of zero; these are the pinned choices (ternaries, so the host
 * libm and the GPU min/max instructions cannot disagree on +-0). */
RT_HD float rt_minf(float a, float b) { return (b < a) ? b : a; }
RT_HD float rt_maxf(float a, float b) { return (a < b) ? b : a; }
RT_HD float rt_satf(float x) { return x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f; }
RT_HD float rt_max0f(float x) { return x > 0.0f ? x : 0.0f; }
RT_HD float rt_signf(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
RT_HD float rt_absf(float x) { return __builtin_fabsf(x); }

/* Reduced-argument kernels on |x| <= pi/4 (z = x*x). */
RT_HD float rt_det__sin_poly(float x, float z)
{
    return ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
}
RT_HD float rt_det__cos_poly(float z)
{
    return ((2.443315711809948E-5f * z - 1.388731625493765E-3f) * z + 4.166664568298827E-2f) * z * z
           - 0.5f * z + 1.0f;
}

/* Cody-Waite reduction by pi/4 (three-part split of pi/4). Valid for |x| < 8192. */
RT_HD float rt_det__reduce(float ax, int* octant)
{
    int j = (int)(1.27323954473516f * ax);
    float y = (float)j;
    if (j & 1) {
        j += 1;
        y += 1.0f;
    }
    *octant = j & 7;
    return ((ax - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
}

RT_HD float rt_det_sinf(float x)
{
    int neg = 0;
    float ax = x;
    if (x < 0.0f) {
        neg = 1;
        ax = -x;
    }
    if (!(ax < 8192.0f)) return x - x;   /* NaN for inf/NaN/huge (never reached by the shaders) */
    int j;
    float r = rt_det__reduce(ax, &j);
    if (j > 3) {
        neg = !neg;
        j -= 4;
    }
    float z = r * r;
    float y = (j == 1 || j == 2) ? rt_det__cos_poly(z) : rt_det__sin_poly(r, z);
    return neg ? -y : y;
}

RT_HD float rt_det_cosf(float x)
{
    float ax = x < 0.0f ? -x : x;
    if (!(ax < 8192.0f)) return x - x;
    int j;
    float r = rt_det__reduce(ax, &j);
    int neg = 0;
    if (j > 3) {
        j -= 4;
        neg = 1;
    }
    if (j > 1) neg = !neg;
    float z = r * r;
    float y = (j == 1 || j == 2) ? rt_det__sin_poly(r, z) : rt_det__cos_poly(z);
    return neg ? -y : y;
}

/* asin on |x| <= 0.5 */
RT_HD float rt_det__asin_small(float x)
{
    float a = x < 0.0f ? -x : x;
    if (a < 1.0e-4f) return x;
    float z = x * x;
    return ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z
            + 1.6666752422E-1f) * z * x + x;
}

RT_HD float rt_det_acosf(float x)
{
    if (x > 0.5f) {
        float s = rt_det_sqrtf(0.5f * (1.0f - x));   /* NaN for x > 1 */
        return 2.0f * rt_det__asin_small(s);
    }
    if (x < -0.5f) {
        float s = rt_det_sqrtf(0.5f * (1.0f + x));
        return RT_DET_PIF - 2.0f * rt_det__asin_small(s);
    }
    return RT_DET_PIO2F - rt_det__asin_small(x);  /* NaN propagates */
}

/* exp: Cephes expf (range reduction by ln 2 in two parts, degree-5
 * polynomial), scaled by ldexp (exact).  Used by W9E1's transparent shader
 * (w9e1.wgsl:525, T_r = exp(-rho_t * s)). */
RT_HD float rt_det_expf(float x)
{
    if (x != x) return x;
    if (x > 88.72283905206835f) return __builtin_inff();
    if (x < -103.972077083991796f) return 0.0f;
    const float fx = __builtin_floorf(x * 1.44269504088896341f + 0.5f);
    x = x - fx * 0.693359375f;
    x = x - fx * -2.12194440e-4f;
    const float z = x * x;
    const float y = ((((( 1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x
                       + 4.1665795894E-2f) * x + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    const int n = (int)fx;
    /* 2^n in two exact steps (n in [-150, 128]) */
    const int n1 = n / 2, n2 = n - n1;
    return __builtin_ldexpf(__builtin_ldexpf(y, n1), n2);
}

/* exp2: Cephes exp2f (round-to-nearest integer split, degree-6 polynomial on
 * [-0.5, 0.5]), scaled by ldexp (exact).  Exact powers of two for integer x.
 * Used as WGSL pow(2.0, e) by W9E2's RGBE environment decode
 * (w9e2.wgsl:240-245). */
RT_HD float rt_det_exp2f(float x)
{
    if (x != x) return x;
    if (x > 128.0f) return __builtin_inff();
    if (x < -151.0f) return 0.0f;
    const float i0 = __builtin_floorf(x + 0.5f);
    const float f = x - i0;
    float px = f * (((((1.535336188319500e-4f * f + 1.339887440266574e-3f) * f + 9.618437357674640e-3f) * f
                      + 5.550332471162809e-2f) * f + 2.402264791363012e-1f) * f + 6.931472028550421e-1f);
    px = 1.0f + px;
    const int n = (int)i0;
    const int n1 = n / 2, n2 = n - n1;
    return __builtin_ldexpf(__builtin_ldexpf(px, n1), n2);
}

/* log2: Cephes log2f (frexp split about sqrt(1/2), degree-9 polynomial,
 * log2(e) applied in two parts); log2(0) = -inf, negative or NaN -> NaN. */
RT_HD float rt_det_log2f(float xx)
{
    if (xx != xx || xx < 0.0f) return __builtin_nanf("");
    if (xx == 0.0f) return -__builtin_inff();
    if (xx == __builtin_inff()) return xx;
    int e;
    float x = __builtin_frexpf(xx, &e);
    if (x < 0.707106781186547524f) {
        e -= 1;
        x = x + x - 1.0f;
    } else {
        x = x - 1.0f;
    }
    const float z = x * x;
    float y = ((((((((7.0376836292e-2f * x - 1.1514610310e-1f) * x + 1.1676998740e-1f) * x - 1.2420140846e-1f) * x
                   + 1.4249322787e-1f) * x - 1.6668057665e-1f) * x + 2.0000714765e-1f) * x - 2.4999993993e-1f) * x
              + 3.3333331174e-1f) * x * z;
    y = y + -0.5f * z;
    float r = y * 0.44269504088896340736f;
    r = r + x * 0.44269504088896340736f;
    r = r + y;
    r = r + x;
    return r + (float)e;
}

/* WGSL pow(x, y) = exp2(y * log2(x)) for x >= 0 (the phong lobe, w6e3.wgsl:418) */
RT_HD float rt_det_powf(float x, float y)
{
    if (x == 0.0f) return y > 0.0f ? 0.0f : (y == 0.0f ? 1.0f : __builtin_inff());
    return rt_det_exp2f(y * rt_det_log2f(x));
}

/* atan on |x| <= tan(pi/8) after the Cephes atanf reduction */
RT_HD float rt_det_atanf(float x)
{
    int neg = 0;
    if (x < 0.0f) {
        neg = 1;
        x = -x;
    }
    float y0 = 0.0f;
    if (x > 2.414213562373095f) {            /* tan(3pi/8) */
        y0 = RT_DET_PIO2F;
        x = -1.0f / x;
    } else if (x > 0.4142135623730950f) {    /* tan(pi/8) */
        y0 = 0.78539816339744830962f;
        x = (x - 1.0f) / (x + 1.0f);
    }
    float z = x * x;
    float y = (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x
              + x;
    y = y0 + y;
    return neg ? -y : y;   /* NaN propagates */
}

/* WGSL atan2(y, x); pinned choices where IEEE atan2 distinguishes signed
 * zeros: atan2(+-0, x < 0) = +pi, atan2(+-0, +-0) = 0. */
RT_HD float rt_det_atan2f(float y, float x)
{
    if (x == 0.0f) {
        if (y > 0.0f) return RT_DET_PIO2F;
        if (y < 0.0f) return -RT_DET_PIO2F;
        return y == y ? 0.0f : y;
    }
    float z = rt_det_atanf(y / x);
    if (x < 0.0f) z = (y < 0.0f) ? z - RT_DET_PIF : z + RT_DET_PIF;
    return z;
}

/* environment_map (res/shaders/w9e1.wgsl:232-239) on an RGBA8 (Rgba8Unorm)
 * equirectangular texture of w x h texels, row 0 at v = 0: the direction's
 * (u, 1 - v) sampled with the hdri0 sampler's magnification filter --
 * bilinear, ClampToEdge (src/bindings/texture.rs:134-141).  Pinned choices:
 * textureSample's LOD comes from fragment-quad derivatives inside the
 * bounce loop's non-uniform control flow (implementation-defined), so the
 * magnification (Linear) filter is used for every lookup; texel weights and
 * the unorm conversion c/255 are f32, evaluated as written here. */
RT_HD float rt_det__unorm8(unsigned int c) { return (float)c / 255.0f; }
RT_HD void rt_det_env_sample(const unsigned int* tex, unsigned int w, unsigned int h, float dx, float dy, float dz,
                             float* rgb)
{
    const float u = 0.5f * (1.0f + (1.0f / RT_DET_PIF) * rt_det_atan2f(dx, -dz));
    const float v = 1.0f / RT_DET_PIF * rt_det_acosf(-dy);
    const float s = u, t = 1.0f - v;
    float x = s * (float)w - 0.5f, y = t * (float)h - 0.5f;
    x = x == x ? x : 0.0f;   /* NaN direction: texel 0 (pinned) */
    y = y == y ? y : 0.0f;
    const float fx = __builtin_floorf(x), fy = __builtin_floorf(y);
    const float a = x - fx, b = y - fy;
    int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const int wm = (int)w - 1, hm = (int)h - 1;
    x0 = x0 < 0 ? 0 : (x0 > wm ? wm : x0);
    x1 = x1 < 0 ? 0 : (x1 > wm ? wm : x1);
    y0 = y0 < 0 ? 0 : (y0 > hm ? hm : y0);
    y1 = y1 < 0 ? 0 : (y1 > hm ? hm : y1);
    const unsigned int t00 = tex[(unsigned int)y0 * w + (unsigned int)x0], t10 = tex[(unsigned int)y0 * w + (unsigned int)x1];
    const unsigned int t01 = tex[(unsigned int)y1 * w + (unsigned int)x0], t11 = tex[(unsigned int)y1 * w + (unsigned int)x1];
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    for (int c = 0; c < 3; c++) {
        const unsigned int sh = 8u * (unsigned int)c;
        rgb[c] = rt_det__unorm8((t00 >> sh) & 255u) * w00 + rt_det__unorm8((t10 >> sh) & 255u) * w10 +
                 rt_det__unorm8((t01 >> sh) & 255u) * w01 + rt_det__unorm8((t11 >> sh) & 255u) * w11;
    }
}

/* environment_map of w9e2.wgsl:234-246: the same lookup on an RGBE-encoded
 * texture (luxo_pxr_campus.hdr.png): all four channels filtered, then
 * rgb * pow(2, a*255 - 128) on the filtered alpha, as the shader decodes after
 * textureSample. */
RT_HD void rt_det_env_sample_rgbe(const unsigned int* tex, unsigned int w, unsigned int h, float dx, float dy,
                                  float dz, float* rgb)
{
    const float u = 0.5f * (1.0f + (1.0f / RT_DET_PIF) * rt_det_atan2f(dx, -dz));
    const float v = 1.0f / RT_DET_PIF * rt_det_acosf(-dy);
    const float s = u, t = 1.0f - v;
    float x = s * (float)w - 0.5f, y = t * (float)h - 0.5f;
    x = x == x ? x : 0.0f;
    y = y == y ? y : 0.0f;
    const float fx = __builtin_floorf(x), fy = __builtin_floorf(y);
    const float a = x - fx, b = y - fy;
    int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const int wm = (int)w - 1, hm = (int)h - 1;
    x0 = x0 < 0 ? 0 : (x0 > wm ? wm : x0);
    x1 = x1 < 0 ? 0 : (x1 > wm ? wm : x1);
    y0 = y0 < 0 ? 0 : (y0 > hm ? hm : y0);
    y1 = y1 < 0 ? 0 : (y1 > hm ? hm : y1);
    const unsigned int t00 = tex[(unsigned int)y0 * w + (unsigned int)x0], t10 = tex[(unsigned int)y0 * w + (unsigned int)x1];
    const unsigned int t01 = tex[(unsigned int)y1 * w + (unsigned int)x0], t11 = tex[(unsigned int)y1 * w + (unsigned int)x1];
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    float c4[4];
    for (int c = 0; c < 4; c++) {
        const unsigned int sh = 8u * (unsigned int)c;
        c4[c] = rt_det__unorm8((t00 >> sh) & 255u) * w00 + rt_det__unorm8((t10 >> sh) & 255u) * w10 +
                rt_det__unorm8((t01 >> sh) & 255u) * w01 + rt_det__unorm8((t11 >> sh) & 255u) * w11;
    }
    const float e = rt_det_exp2f(c4[3] * 255.0f - 128.0f);
    for (int c = 0; c < 3; c++) rgb[c] = c4[c] * e;
}

#endif /* RT02562_DETMATH_H */
