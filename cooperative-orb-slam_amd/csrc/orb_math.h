/*
 * orb_math.h -- bit-exact scalar math shared by the gfx950 kernels.
 *
 * Every float operation the reference performs on the hot path is reproduced with
 * explicitly rounded intrinsics (no FMA contraction; the library is also built with
 * -ffp-contract=off), so device results equal the host oracle bit for bit.
 *
 *  - glibc_cosf/glibc_sinf: the float cos/sin that computeOrbDescriptor calls
 *    (ORBextractor.cc:113, `cos(angle)` on a float = glibc cosf). Restated from glibc 2.35's
 *    sincosf algorithm (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c): double evaluation,
 *    constants read from libm's __sincosf_table. Verified equal to the host libm (both the
 *    FMA and the SSE2 ifunc variants) for every float in [0, 2*pi] (tools/check_trig.c).
 *  - fast_atan2: cv::fastAtan2 (OpenCV 3.x scalar form), called by IC_Angle
 *    (ORBextractor.cc:103).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbamd {

__device__ __forceinline__ int cv_round(float v) { return __float2int_rn(v); }

__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float r2d = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d,
                p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
    const float eps = (float)2.220446049250313080847e-16; /* (float)DBL_EPSILON */
    float ax = fabsf(x), ay = fabsf(y), a, c, c2, poly;
    if (ax >= ay) {
        c = __fdiv_rn(ay, __fadd_rn(ax, eps));
    } else {
        c = __fdiv_rn(ax, __fadd_rn(ay, eps));
    }
    c2 = __fmul_rn(c, c);
    poly = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
    a = (ax >= ay) ? poly : __fsub_rn(90.f, poly);
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

/* glibc 2.35 __sincosf_table (values read from libm.so.6 .rodata). Table 1 is table 0 with the
 * cosine coefficients negated and identical sine coefficients, and sign[n&3] = -1 for n&3 in
 * {1,2}; all constants are immediates (no memory loads on the hot path). */
#define SC_HPI_INV 0x1.45f306dc9c883p+23
#define SC_HPI 0x1.921fb54442d18p+0
#define SC_C0 1.0
#define SC_C1 -0x1.ffffffd0c621cp-2
#define SC_S1 -0x1.555545995a603p-3
#define SC_C2 0x1.55553e1068f19p-5
#define SC_S2 0x1.1107605230bc4p-7
#define SC_C3 -0x1.6c087e89a359dp-10
#define SC_S3 -0x1.994eb3774cf24p-13
#define SC_C4 0x1.99343027bf8c3p-16

__device__ __forceinline__ float sinf_poly(double xs, double x2) {
    double x3 = __dmul_rn(x2, xs);
    double a = __fma_rn(x2, SC_S3, SC_S2);
    double x5 = __dmul_rn(x3, x2);
    double s = __fma_rn(x3, SC_S1, xs);
    return __double2float_rn(__fma_rn(a, x5, s));
}
/* neg = 1 selects table 1 (cosine coefficients negated) */
__device__ __forceinline__ float cosf_poly(double x2, bool neg) {
    const double c0 = neg ? -SC_C0 : SC_C0, c1 = neg ? -SC_C1 : SC_C1, c2 = neg ? -SC_C2 : SC_C2;
    const double c3 = neg ? -SC_C3 : SC_C3, c4 = neg ? -SC_C4 : SC_C4;
    double x4 = __dmul_rn(x2, x2);
    double t1 = __fma_rn(x2, c1, c0);
    double t2 = __fma_rn(x2, c4, c3);
    double x6 = __dmul_rn(x2, x4);
    double c = __fma_rn(x4, c2, t1);
    return __double2float_rn(__fma_rn(t2, x6, c));
}
__device__ __forceinline__ unsigned top12(float y) { return (__float_as_uint(y) >> 20) & 0x7ff; }
/* valid for |y| < 120 (all ORB angles are in [0, 2*pi]) */
__device__ __forceinline__ void glibc_sincosf(float y, float* s_out, float* c_out) {
    double x = (double)y;
    if (top12(y) <= 0x3f3) {
        double x2 = __dmul_rn(x, x);
        if (top12(y) <= 0x397) {
            *s_out = y;
            *c_out = 1.0f;
            return;
        }
        *s_out = sinf_poly(x, x2);
        *c_out = cosf_poly(x2, false);
        return;
    }
    double r = __dmul_rn(x, SC_HPI_INV);
    int n = ((int)r + 0x800000) >> 24;
    double xr = __fma_rn(-(double)n, SC_HPI, x);
    const bool neg = (n & 2) != 0;
    double x2 = __dmul_rn(xr, xr);
    const int q = n & 3;
    double xs = (q == 1 || q == 2) ? -xr : xr;  // xr * sign[n&3], exact
    if (n & 1) {
        *s_out = cosf_poly(x2, neg);
        *c_out = sinf_poly(xs, x2);
    } else {
        *s_out = sinf_poly(xs, x2);
        *c_out = cosf_poly(x2, neg);
    }
}

}  // namespace orbamd
