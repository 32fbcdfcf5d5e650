/* Bitwise check of rt_div_by_recip (include/rt_detmath.h) against IEEE
 * binary32 division, over the operand range the BSP walk feeds it:
 * x = plane - origin (0, or 2^-100 <= |x| <= 2^100), d = a direction component
 * (1e-8 <= |d| <= 1, or the 1e-8 clamp).  usage: fastdiv_check <n> <seed>
 * prints the number of mismatches and the first few. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "../../include/rt_detmath.h"

static uint64_t s_state;
static uint32_t rnd32(void)
{
    s_state = s_state * 6364136223846793005ull + 1442695040888963407ull;
    uint32_t x = (uint32_t)(((s_state >> 18) ^ s_state) >> 27), r = (uint32_t)(s_state >> 59);
    return (x >> r) | (x << ((-r) & 31));
}
static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* mantissa patterns: uniform, near all-ones, near zero, sparse */
static uint32_t mant(void)
{
    uint32_t k = rnd32() & 7u, m = rnd32() & 0x7FFFFFu;
    if (k == 0) return 0x7FFFFFu ^ (m & 0xFFu);
    if (k == 1) return m & 0xFFu;
    if (k == 2) return 1u << (rnd32() % 23u);
    return m;
}

int main(int argc, char** argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ull;
    s_state = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    uint64_t bad = 0, tested = 0, zsign = 0;
    for (uint64_t i = 0; i < n; i++) {
        /* d: |d| in [1e-8, 1] (exponent -27..0), or exactly the clamp value */
        float d;
        if ((rnd32() & 63u) == 0) d = 1.0e-8f;
        else {
            int e = -27 + (int)(rnd32() % 28u);
            d = bits(((uint32_t)(e + 127) << 23) | mant());
            if (d < 1.0e-8f) d = 1.0e-8f;
        }
        if (rnd32() & 1u) d = -d;
        /* x = +-0 (a plane through the ray origin's coordinate), which the walk's
         * unchecked divisions (rt_kernels.hip bsp_decide without chk) also take: the
         * result must be a zero; its sign is x / d's for x = +0 and may differ for
         * x = -0 (counted apart), which the walk does not see -- it only compares t */
        for (int zs = 0; zs < 2; zs++) {
            const float z = zs ? -0.0f : 0.0f;
            const float gz = rt_div_by_recip(z, d, 1.0f / d), wz = z / d;
            tested++;
            if (gz != wz || (!zs && ubits(gz) != ubits(wz))) {
                if (bad < 5) printf("mismatch x=%a d=%a got=%a want=%a\n", z, d, gz, wz);
                bad++;
            } else if (ubits(gz) != ubits(wz)) {
                zsign++;
            }
        }
        /* x: exponent -100..100, biased toward scene scales */
        int ex = (rnd32() & 3u) ? -30 + (int)(rnd32() % 45u) : -100 + (int)(rnd32() % 201u);
        float x = bits(((uint32_t)(ex + 127) << 23) | mant());
        if (rnd32() & 1u) x = -x;
        if (!rt_div_by_recip_ok(x)) continue;
        const float r = 1.0f / d;
        const float want = x / d;
        if (!(fabsf(want) < 0x1p127f)) continue;
        const float got = rt_div_by_recip(x, d, r);
        tested++;
        if (ubits(got) != ubits(want)) {
            if (bad < 5) printf("mismatch x=%a d=%a got=%a want=%a\n", x, d, got, want);
            bad++;
        }
    }
    printf("tested %llu mismatches %llu (x = -0: %llu zeros of the other sign)\n", (unsigned long long)tested,
           (unsigned long long)bad, (unsigned long long)zsign);
    return bad != 0;
}
