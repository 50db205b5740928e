/* sincos_check.c — rt_sincosf (isaklm-raytracer_amd/csrc/rt_libm.h) against
 * rt_sinf / rt_cosf, bit for bit: every float in [-8, 8] (the shading angles
 * xi * TAU lie in [0, 2 pi]) and every 4096th float up to |x| = 1e6.
 * usage: sincos_check [stride]  (every stride-th float of [-8, 8]); exit 0 = identical. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_libm.h"

int main(int argc, char **argv)
{
    const long long stride = argc > 1 ? atoll(argv[1]) : 1;
    long long bad = 0, n = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(dynamic, 1 << 20)
    for (long long u = 0; u < (1LL << 32); ++u) {
        float x;
        const uint32_t b = (uint32_t)u;
        memcpy(&x, &b, 4);
        if (!(x == x)) continue;
        const float ax = x < 0 ? -x : x;
        if (ax > 1e6f || (ax > 8.0f ? (u & 4095) != 0 : u % stride != 0)) continue;
        float s, c;
        rt_sincosf(x, &s, &c);
        const float s0 = rt_sinf(x), c0 = rt_cosf(x);
        ++n;
        if (memcmp(&s, &s0, 4) != 0 || memcmp(&c, &c0, 4) != 0) ++bad;
    }
    printf("checked %lld mismatches %lld\n", n, bad);
    return bad != 0;
}
