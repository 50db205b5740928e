// div_structured.cpp — structured check of rt_div_by (csrc/rt_vecmath.h)
// against IEEE '/', the division the reference performs for the KD split
// distance (rt/trace_ray.cuh:193-210, intersect_plane).
//
// Random pairs rarely hit the cases where a reciprocal-based division can go
// wrong, so this enumerates them:
//   * every one of the 2^23 divisor significands (all-ones included),
//   * numerator significands chosen per divisor: 1.0, all-ones, the divisor's
//     own significand and its neighbours (quotient at / around a binade
//     edge), twice the divisor's significand and its neighbours when that is
//     in range (quotient just below 2), near-midpoint quotients (numerator =
//     RN(d * (q + ulp/2)) for pseudo-random q), and pseudo-random ones,
//   * exponent pairs inside the guards, including the guard boundaries
//     2^-60 and 2^40 on both operands, and every sign combination.
// Prints "tested <n> mismatches <m>" and the first mismatches.
// Build: g++ -O2 -std=c++17 -fopenmp -ffp-contract=off -I include -I isaklm-raytracer_amd/csrc
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <initializer_list>

#include "rt_vecmath.h"

static float from_bits(uint32_t b)
{
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}
static uint32_t to_bits(float f)
{
    uint32_t b;
    std::memcpy(&b, &f, 4);
    return b;
}
// a float with significand bits m (23 bits, implicit 1) and unbiased exponent e
static float make(uint32_t m, int e) { return from_bits((uint32_t)(e + 127) << 23 | (m & 0x7fffffu)); }
static uint32_t mix(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}

int main(int argc, char **argv)
{
    const uint32_t step = argc > 1 ? (uint32_t)atoi(argv[1]) : 1; // 1 = every divisor significand
    // (numerator exponent, divisor exponent): quotients from 2^-100 to 2^100 and the guard edges
    static const int EXP[][2] = {{0, 0},     {0, 1},     {1, 0},     {-1, 0},    {7, -5},   {-9, 12},
                                 {39, -60},  {-60, 39},  {39, 39},   {-60, -60}, {-60, 0},  {39, 0},
                                 {0, -60},   {0, 39},    {-59, -60}, {38, 39}};
    const int nexp = sizeof EXP / sizeof EXP[0];
    unsigned long long tested = 0, bad = 0;
    unsigned long long first[8][2] = {};
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : tested, bad)
    for (long long md = 0; md < (1ll << 23); md += step) {
        uint32_t mn[40];
        int k = 0;
        mn[k++] = 0;
        mn[k++] = 0x7fffff;
        for (int j = -3; j <= 3; ++j) {
            const long long v = md + j;
            if (v >= 0 && v <= 0x7fffff) mn[k++] = (uint32_t)v;
        }
        // numerator = 2 * divisor significand (quotient just below / at 2): as a
        // significand with the exponent one up it is the same bits; cover its
        // neighbours in the lower binade instead
        for (int j = 1; j <= 3; ++j) {
            const long long v = 2 * (md + (1ll << 23)) - j - (1ll << 23);
            if (v >= 0 && v <= 0x7fffff) mn[k++] = (uint32_t)v;
        }
        for (int j = 0; j < 8; ++j) mn[k++] = mix((uint64_t)md * 64 + j) & 0x7fffff;
        const int nrand = k;
        for (int ei = 0; ei < nexp; ++ei) {
            const float dpos = make((uint32_t)md, EXP[ei][1]);
            // near-midpoint quotients: q = (1 + (2r+1) 2^-24) for pseudo-random r, n = RN(d q)
            float extra[6];
            int ne = 0;
            for (int j = 0; j < 6; ++j) {
                const uint32_t r = mix((uint64_t)md * 977 + ei * 31 + j) & 0x7fffff;
                const double q = (1.0 + (2.0 * r + 1.0) * 0x1p-24) * std::ldexp(1.0, EXP[ei][0] - EXP[ei][1]);
                const float n = (float)((double)dpos * q);
                if (std::fabs(n) >= 0x1p-60f && std::fabs(n) <= 0x1p40f) extra[ne++] = n;
            }
            for (int s = 0; s < 4; ++s) {
                const float d = (s & 1) ? -dpos : dpos;
                const float y = rt_recip_guard(d);
                for (int i = 0; i < nrand + ne; ++i) {
                    float n = i < nrand ? make(mn[i], EXP[ei][0]) : extra[i - nrand];
                    if (s & 2) n = -n;
                    const float got = rt_div_by(n, d, y);
                    const float want = n / d;
                    ++tested;
                    if (to_bits(got) != to_bits(want)) {
                        ++bad;
#pragma omp critical
                        {
                            for (auto &f : first)
                                if (f[0] == 0 && f[1] == 0) {
                                    f[0] = to_bits(n);
                                    f[1] = to_bits(d);
                                    break;
                                }
                        }
                    }
                }
            }
        }
    }
    // the guard boundaries themselves, exhaustively over the numerator significand
    for (int dexp : {-60, 39, 40}) {
        for (uint32_t m = 0; m <= 0x7fffff; ++m) {
            for (int nexp2 : {-60, 39}) {
                const float d = dexp == 40 ? 0x1p40f : make(0x7fffff - (m & 0xff), dexp);
                const float n = make(m, nexp2);
                const float got = rt_div_by(n, d, rt_recip_guard(d));
                ++tested;
                if (to_bits(got) != to_bits(n / d)) ++bad;
            }
        }
    }
    printf("tested %llu mismatches %llu\n", tested, bad);
    for (auto &f : first)
        if (f[0] | f[1]) printf("n=%a d=%a\n", from_bits((uint32_t)f[0]), from_bits((uint32_t)f[1]));
    return bad != 0;
}
