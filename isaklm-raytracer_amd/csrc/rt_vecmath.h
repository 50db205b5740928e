// rt_vecmath.h — the reference's vector/matrix arithmetic on its own types
// (rt/math_library.cuh), for host C++ and gfx950 device code alike.
//
// Every operator keeps the reference's operand order and rounding points:
// a dot product is ((x*x' + y*y') + z*z'), a matrix-vector product is
// ((i*v.x + j*v.y) + k*v.z), normalize multiplies by 1/sqrt.  All code that
// includes this header is compiled with -ffp-contract=off, so a
// value computed on the host and on the GPU is the same bits.
#pragma once

#include "../../include/isaklm_rt.h"
#include "rt_libm.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

#define RT_PI 3.1415926536f        /* rt/math_library.cuh:9 */
#define RT_TAU (RT_PI * 2)         /* rt/math_library.cuh:10 */
#define RT_HALF_PI (RT_PI / 2)     /* rt/math_library.cuh:11 */
#define RT_KD_TREE_DEPTH 19        /* rt/macros.h:11 */
#define RT_MAX_COLOR_CHANNEL 255   /* rt/macros.h:9 */

struct RtM3 { Vec3D i, j, k; };    // Matrix3X3 (rt/math_library.cuh:319-335), column vectors

RT_HD Vec3D rt_v3(float x, float y, float z) { Vec3D r; r.x = x; r.y = y; r.z = z; return r; }
RT_HD Vec2D rt_v2(float x, float y) { Vec2D r; r.x = x; r.y = y; return r; }
RT_HD float rt_square(float x) { return x * x; }                                   // :17-20
RT_HD float rt_clamp(float x, float lo, float hi) { return fmaxf(lo, fminf(hi, x)); } // :22-25
RT_HD float rt_mod(float x, float m) { return x - m * floorf(x / m); }            // :32-35

// Correctly rounded n / d for a fixed d from its reciprocal (Markstein):
// with y = RN(1/d), q0 = RN(n*y) is within 1 ulp of n/d, the residual
// e = n - d*q0 is exact in one fma, and RN(q0 + e*y) = RN(n/d) — the same
// bits as the IEEE division the reference performs, in 3 VALU ops instead of
// the ~10 of a full division.  Valid without over/underflow, which the range
// guards (|n|, |d| in [2^-60, 2^40]) ensure; outside them (axis-parallel rays,
// origins on a split plane) the plain division runs.  Used for the KD split
// distance t = (split - o) / d, whose d is one of the ray's 3 components.
// tests/test_host.py::test_division_matches_ieee checks it against '/'.
// The barycentric range test of intersect_triangle (rt/trace_ray.cuh:97-110):
// every coordinate in [0, 1].  On the device as IEEE minimum / maximum
// (v_minimum3_f32 / v_maximum3_f32): they propagate a NaN, which then fails
// its compare as a NaN coordinate fails the six; -0 passes both ways.
RT_HD bool rt_bary_inside(float cx, float cy, float cz)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const float lo = __builtin_elementwise_minimum(__builtin_elementwise_minimum(cx, cy), cz);
    const float hi = __builtin_elementwise_maximum(__builtin_elementwise_maximum(cx, cy), cz);
    return lo >= 0.0f && hi <= 1.0f;
#else
    return cx >= 0.0f && cx <= 1.0f && cy >= 0.0f && cy <= 1.0f && cz >= 0.0f && cz <= 1.0f;
#endif
}

RT_HD float rt_recip_guard(float d)
{
    const float a = fabsf(d);
    return (a >= 0x1p-60f && a <= 0x1p40f) ? 1.0f / d : 0.0f; // 0: use the plain division
}
RT_HD float rt_div_by(float n, float d, float y)
{
    const float a = fabsf(n);
    if (y != 0.0f && a >= 0x1p-60f && a <= 0x1p40f) {
        const float q0 = n * y;
        const float e = fmaf(-d, q0, n);
        return fmaf(e, y, q0);
    }
    return n / d;
}

RT_HD Vec2D operator+(Vec2D a, Vec2D b) { return rt_v2(a.x + b.x, a.y + b.y); }   // :68-71
RT_HD Vec2D operator*(Vec2D v, float s) { return rt_v2(v.x * s, v.y * s); }       // :78-81
RT_HD Vec3D operator+(Vec3D a, Vec3D b) { return rt_v3(a.x + b.x, a.y + b.y, a.z + b.z); } // :117-120
RT_HD Vec3D operator-(Vec3D a, Vec3D b) { return rt_v3(a.x - b.x, a.y - b.y, a.z - b.z); } // :122-125
RT_HD Vec3D operator-(Vec3D a) { return rt_v3(-a.x, -a.y, -a.z); }                       // :127-130
RT_HD Vec3D operator*(Vec3D v, float s) { return rt_v3(v.x * s, v.y * s, v.z * s); }     // :132-135
RT_HD Vec3D operator*(float s, Vec3D v) { return rt_v3(v.x * s, v.y * s, v.z * s); }     // :137-140
RT_HD Vec3D operator*(Vec3D a, Vec3D b) { return rt_v3(a.x * b.x, a.y * b.y, a.z * b.z); } // :142-145
RT_HD float rt_dot(Vec3D a, Vec3D b) { return a.x * b.x + a.y * b.y + a.z * b.z; }         // :212-215
RT_HD Vec3D rt_cross(Vec3D a, Vec3D b)                                                      // :217-220
{
    return rt_v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
RT_HD float rt_magnitude(Vec3D v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }     // :222-225
RT_HD float rt_magnitude_squared(Vec3D v) { return v.x * v.x + v.y * v.y + v.z * v.z; }    // :227-230
RT_HD Vec3D rt_normalize(Vec3D v)                                                           // :232-237
{
    float r = 1.0f / sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return rt_v3(v.x * r, v.y * r, v.z * r);
}
RT_HD float rt_luminance(Vec3D c) { return rt_dot(c, rt_v3(0.2126f, 0.7152f, 0.0722f)); }  // :263-266

RT_HD Vec3D operator*(RtM3 m, Vec3D v) { return v.x * m.i + v.y * m.j + v.z * m.k; }       // :347-350
RT_HD RtM3 operator*(RtM3 m2, RtM3 m1) { RtM3 r = {m2 * m1.i, m2 * m1.j, m2 * m1.k}; return r; } // :352-355
RT_HD RtM3 operator*(RtM3 m, float s) { RtM3 r = {s * m.i, s * m.j, s * m.k}; return r; }  // :337-340

// rotation_matrix(yaw, pitch, roll = 0) (:384-408) with the shared trig (rt_libm.h)
RT_HD RtM3 rt_rotation_matrix(float yaw, float pitch)
{
    const float roll = 0.0f;
    RtM3 y = {rt_v3(rt_cosf(yaw), 0.0f, -rt_sinf(yaw)), rt_v3(0.0f, 1.0f, 0.0f), rt_v3(rt_sinf(yaw), 0.0f, rt_cosf(yaw))};
    RtM3 x = {rt_v3(1.0f, 0.0f, 0.0f), rt_v3(0.0f, rt_cosf(pitch), rt_sinf(pitch)),
              rt_v3(0.0f, -rt_sinf(pitch), rt_cosf(pitch))};
    RtM3 z = {rt_v3(rt_cosf(roll), rt_sinf(roll), 0.0f), rt_v3(-rt_sinf(roll), rt_cosf(roll), 0.0f),
              rt_v3(0.0f, 0.0f, 1.0f)};
    return z * y * x;
}

// ---- tonemap (rt/math_library.cuh:37-52, 422-460) ----
RT_HD float rt_gamma_correction(float x)                                                    // :37-47
{
    float output = (float)(12.92 * (double)x);
    if ((double)x > 0.0031308) output = (float)(1.055 * (double)rt_powf(x, (float)(1.0 / 2.4)) - 0.055);
    return output;
}
RT_HD float rt_aces_curve(float x)                                                          // :49-52
{
    return (x * (x + 0.0245786f) - 0.000090537f) / (x * (0.983729f * x + 0.4329510f) + 0.238081f);
}
RT_HD Vec3D rt_correct_color(Vec3D c)                                                       // :422-460
{
    const RtM3 in = {rt_v3(0.59719f, 0.07600f, 0.02840f), rt_v3(0.35458f, 0.90834f, 0.13383f),
                     rt_v3(0.04823f, 0.01566f, 0.83777f)};
    const RtM3 out = {rt_v3(1.60475f, -0.10208f, -0.00327f), rt_v3(-0.53108f, 1.10813f, -0.07276f),
                      rt_v3(-0.07367f, -0.00605f, 1.07602f)};
    c.x = fmaxf(c.x, 0.0f);
    c.y = fmaxf(c.y, 0.0f);
    c.z = fmaxf(c.z, 0.0f);
    c = in * c;
    c = rt_v3(rt_aces_curve(c.x), rt_aces_curve(c.y), rt_aces_curve(c.z));
    c = out * c;
    c = rt_v3(rt_gamma_correction(c.x), rt_gamma_correction(c.y), rt_gamma_correction(c.z));
    c.x = rt_clamp(c.x, 0.0f, 1.0f);
    c.y = rt_clamp(c.y, 0.0f, 1.0f);
    c.z = rt_clamp(c.z, 0.0f, 1.0f);
    return c;
}
