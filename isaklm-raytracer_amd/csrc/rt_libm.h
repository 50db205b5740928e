/*
 * rt_libm.h — the transcendental functions of the path-tracing hot path,
 * evaluated identically on the host CPU and on gfx950.
 *
 * Why this file exists
 * --------------------
 * The reference calls sinf/cosf (rt/path_tracing.cuh:49-50,113-114,332-333),
 * cos/sin on floats (rt/math_library.cuh:388-404 via rotation_matrix), tanf
 * (rt/path_tracing.cuh:381) and powf (rt/math_library.cuh:43, tonemap only),
 * all from CUDA 11.7 libdevice (<= 2 ulp, not correctly rounded, unavailable
 * here).  Monte-Carlo paths branch on every float, so
 * the CPU oracle and the GPU kernel must agree bit for bit on these
 * functions.  Both therefore use the code below: the argument is widened to
 * double, reduced with a Cody–Waite split of pi/2 and evaluated with the
 * (public-domain) fdlibm minimax kernels, then rounded once to float.  Only
 * IEEE-exact double operations (+ - * / floor frexp ldexp) are used, and every
 * translation unit that includes this header is compiled with
 * -ffp-contract=off, so the result is the same bits on x86-64 (SSE2) and on
 * CDNA4 (v_*_f64).  The double result carries ~1e-16 relative error, so the
 * float result is the correctly rounded one except in vanishingly rare
 * hard-to-round cases (tests/test_libm.py measures this against glibc).
 *
 * This header is C99/C++/HIP: RT_LIBM_FN adds __host__ __device__ under hipcc.
 */
#ifndef RT_LIBM_H
#define RT_LIBM_H

#include <math.h>

#if defined(__HIPCC__)
#define RT_LIBM_FN __host__ __device__ static inline
#else
#define RT_LIBM_FN static inline
#endif

/* pi/2 split into three parts; the first two have 33 significant bits so
 * k * part is exact for |k| < 2^20 (fdlibm pio2_1, pio2_2, pio2_3). */
#define RT_PIO2_1 1.57079632673412561417e+00
#define RT_PIO2_2 6.07710050630396597660e-11
#define RT_PIO2_3 2.02226624871116645580e-21
#define RT_INVPIO2 6.36619772367581382433e-01

RT_LIBM_FN double rt_ksin(double r)
{
    /* fdlibm __kernel_sin, |r| <= ~pi/4 */
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = r * r;
    double v = z * r;
    double p = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return r + v * (S1 + z * p);
}

RT_LIBM_FN double rt_kcos(double r)
{
    /* fdlibm __kernel_cos, |r| <= ~pi/4 */
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = r * r;
    double p = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    return 1.0 - (0.5 * z - z * p);
}

/* x = k*pi/2 + r, |r| <~ pi/4.  Valid for |x| < 2^19 * pi/2 (all call sites
 * pass angles of a few radians). */
RT_LIBM_FN double rt_reduce_pio2(double x, int *quadrant)
{
    double k = floor(x * RT_INVPIO2 + 0.5);
    *quadrant = (int)k;
    return ((x - k * RT_PIO2_1) - k * RT_PIO2_2) - k * RT_PIO2_3;
}

RT_LIBM_FN double rt_sin_d(double x)
{
    if (x == 0.0) return x; /* keeps the sign of zero */
    int q;
    double r = rt_reduce_pio2(x, &q);
    switch (q & 3) {
    case 0: return rt_ksin(r);
    case 1: return rt_kcos(r);
    case 2: return -rt_ksin(r);
    default: return -rt_kcos(r);
    }
}

RT_LIBM_FN double rt_cos_d(double x)
{
    int q;
    double r = rt_reduce_pio2(x, &q);
    switch (q & 3) {
    case 0: return rt_kcos(r);
    case 1: return -rt_ksin(r);
    case 2: return -rt_kcos(r);
    default: return rt_ksin(r);
    }
}

RT_LIBM_FN float rt_sinf(float x) { return (float)rt_sin_d((double)x); }
RT_LIBM_FN float rt_cosf(float x) { return (float)rt_cos_d((double)x); }

/* rt_sinf(x) and rt_cosf(x) from one reduction (the same r and quadrant, the
 * same kernels, the same signs: bit for bit the two calls' results).  The
 * shading code wants both of one angle; on the GPU a wave whose lanes fall
 * in different quadrants runs both kernels for each call anyway. */
RT_LIBM_FN void rt_sincosf(float xf, float *sf, float *cf)
{
    const double x = (double)xf;
    int q;
    const double r = rt_reduce_pio2(x, &q);
    const double s = rt_ksin(r), c = rt_kcos(r);
    double sv, cv;
    switch (q & 3) {
    case 0: sv = s; cv = c; break;
    case 1: sv = c; cv = -s; break;
    case 2: sv = -s; cv = -c; break;
    default: sv = -c; cv = s; break;
    }
    *sf = x == 0.0 ? xf : (float)sv; /* (rt_sin_d keeps the sign of zero) */
    *cf = (float)cv;
}

RT_LIBM_FN float rt_tanf(float xf)
{
    if (xf == 0.0f) return xf;
    int q;
    double r = rt_reduce_pio2((double)xf, &q);
    double s = rt_ksin(r), c = rt_kcos(r);
    return (float)((q & 1) ? -c / s : s / c);
}

/* natural log of a positive finite double: x = m * 2^e, m in [sqrt(1/2), sqrt(2)) */
RT_LIBM_FN double rt_log_d(double x)
{
    int e;
    double m = frexp(x, &e); /* m in [0.5, 1) */
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e = e - 1;
    }
    double f = (m - 1.0) / (m + 1.0);
    double f2 = f * f;
    /* 2 atanh(f) = 2 (f + f^3/3 + f^5/5 + ...), |f| < 0.1716 */
    double s = 1.0 / 21.0;
    s = 1.0 / 19.0 + f2 * s;
    s = 1.0 / 17.0 + f2 * s;
    s = 1.0 / 15.0 + f2 * s;
    s = 1.0 / 13.0 + f2 * s;
    s = 1.0 / 11.0 + f2 * s;
    s = 1.0 / 9.0 + f2 * s;
    s = 1.0 / 7.0 + f2 * s;
    s = 1.0 / 5.0 + f2 * s;
    s = 1.0 / 3.0 + f2 * s;
    s = 1.0 + f2 * s;
    const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    return ((double)e * LN2_HI + 2.0 * f * s) + (double)e * LN2_LO;
}

RT_LIBM_FN double rt_exp_d(double x)
{
    const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double INV_LN2 = 1.44269504088896338700e+00;
    double k = floor(x * INV_LN2 + 0.5);
    double r = (x - k * LN2_HI) - k * LN2_LO; /* |r| <= ~0.347 */
    double t = 1.0 / 6227020800.0;            /* 1/13! */
    t = 1.0 / 479001600.0 + r * t;
    t = 1.0 / 39916800.0 + r * t;
    t = 1.0 / 3628800.0 + r * t;
    t = 1.0 / 362880.0 + r * t;
    t = 1.0 / 40320.0 + r * t;
    t = 1.0 / 5040.0 + r * t;
    t = 1.0 / 720.0 + r * t;
    t = 1.0 / 120.0 + r * t;
    t = 1.0 / 24.0 + r * t;
    t = 1.0 / 6.0 + r * t;
    t = 0.5 + r * t;
    t = 1.0 + r * t;
    t = 1.0 + r * t;
    return ldexp(t, (int)k);
}

/* powf for the tonemap's gamma curve (rt/math_library.cuh:43): x > 0.0031308 there. */
RT_LIBM_FN float rt_powf(float x, float y)
{
    if (!(x > 0.0f)) {
        if (x == 0.0f) return (y > 0.0f) ? 0.0f : (float)INFINITY;
        return (float)NAN;
    }
    if (x == (float)INFINITY) return (y > 0.0f) ? (float)INFINITY : 0.0f;
    return (float)rt_exp_d((double)y * rt_log_d((double)x));
}


/* sqrtf(2.0f) * erfinvf(1.0f - tolerance), the adaptive test's z constant
 * (rt/path_tracing.cuh:370).  Host-only (a frame constant).  For the
 * reference's MAX_TOLERANCE = 0.05f the correctly rounded erfinvf(0.95f) =
 * 1.3859037160873413f is used; other tolerances invert erf by Newton steps
 * in double. */
static inline float rt_adaptive_z(float tolerance)
{
    float p = 1.0f - tolerance;
    float e;
    if (p == 0.95f) {
        e = 1.3859037160873413f;
    } else {
        double y = (double)p, x = 0.0;
        for (int it = 0; it < 100; ++it) {
            double fx = erf(x) - y;
            double d = 1.1283791670955126 * exp(-x * x);
            double nx = x - fx / d;
            if (nx == x) break;
            x = nx;
        }
        e = (float)x;
    }
    return sqrtf(2.0f) * e;
}

#endif /* RT_LIBM_H */
