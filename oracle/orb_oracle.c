/*
 * orb_oracle.c -- plain-C restatement of the reference ORB front-end and matcher.
 *
 * TEST INFRASTRUCTURE (see orb_oracle.h): the parity checker and the timed CPU baseline
 * ("port"). Never linked into the product. Written to follow the reference's control flow
 * literally (linked list + pointer-order sort in DistributeOctTree, per-cell cv::FAST with
 * threshold fallback, ...) so that the GPU's re-formulations are checked against an
 * independent statement. PARITY UNPINNED at the OpenCV boundary (see header).
 *
 * Citations are to files under /root/reference/ORB_SLAM2/src (identical to ORB_SLAM2.1).
 * Build: -O3 -ffp-contract=off (no FMA contraction: the pinned float semantics).
 */
#define _POSIX_C_SOURCE 199309L /* clock_gettime for the stage timers */
#include "orb_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <time.h>
#include <string.h>

#include "orb_pattern_data.h"

#define PATCH_SIZE 31     /* ORBextractor.cc:72 */
#define HALF_PATCH_SIZE 15 /* ORBextractor.cc:73 */
#define EDGE_THRESHOLD 19 /* ORBextractor.cc:74 */
#define MAXL 32

/* ---------------------------------------------------------------- OpenCV helpers --- */
/* cvRound(float/double): SSE2 cvtss2si / cvtsd2si = round half to even (default MXCSR). */
static int cv_round_f(float v) { return (int)lrintf(v); }
static int cv_round_d(double v) { return (int)lrint(v); }
static int cv_floor_f(float v) { int i = (int)v; return i - (i > v); }
static int cv_ceil_f(float v) { int i = (int)v; return i + (i < v); }
static short sat_short_f(float v) {
    int i = cv_round_f(v);
    return (short)(i < -32768 ? -32768 : i > 32767 ? 32767 : i);
}
static uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* cv::fastAtan2 (OpenCV 3.x mathfuncs, scalar form). Called from
 * IC_Angle, ORBextractor.cc:103. */
float oc_fast_atan2(float y, float x) {
    const float r2d = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d,
                p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) on 8UC1 (OpenCV 3.3 resizeGeneric_ with
 * HResizeLinear<uchar,int,short,2048> + VResizeLinear<...,FixedPtCast<int,uchar,22>,
 * VResizeLinearVec_32s8u>). Called at ORBextractor.cc:1120. */
void oc_resize_linear(const uint8_t* src, int sw, int sh, size_t sstep, uint8_t* dst, int dw,
                      int dh, size_t dstep) {
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int* xofs = (int*)malloc(sizeof(int) * dw);
    short* ialpha = (short*)malloc(sizeof(short) * 2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor_f(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        ialpha[2 * dx] = sat_short_f((1.f - fx) * 2048);
        ialpha[2 * dx + 1] = sat_short_f(fx * 2048);
    }
    /* SSE2 VResizeLinearVec_32s8u covers x in [0, simd_end): 16-wide while x <= w-16,
     * then 4-wide while x < w-4; the rest is the scalar FixedPtCast path. */
    int simd_end = 0;
    while (simd_end <= dw - 16) simd_end += 16;
    while (simd_end < dw - 4) simd_end += 4;
    int* h0 = (int*)malloc(sizeof(int) * dw);
    int* h1 = (int*)malloc(sizeof(int) * dw);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor_f(fy);
        fy -= sy;
        int b0 = sat_short_f((1.f - fy) * 2048), b1 = sat_short_f(fy * 2048);
        int r0 = sy < 0 ? 0 : (sy < sh ? sy : sh - 1);
        int r1 = sy + 1 < 0 ? 0 : (sy + 1 < sh ? sy + 1 : sh - 1);
        const uint8_t* S0 = src + (size_t)r0 * sstep;
        const uint8_t* S1 = src + (size_t)r1 * sstep;
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) {
                int a0 = ialpha[2 * dx], a1 = ialpha[2 * dx + 1];
                h0[dx] = S0[sx] * a0 + S0[sx + 1] * a1;
                h1[dx] = S1[sx] * a0 + S1[sx + 1] * a1;
            } else {
                h0[dx] = S0[sx] * 2048;
                h1[dx] = S1[sx] * 2048;
            }
        }
        uint8_t* D = dst + (size_t)dy * dstep;
        for (int x = 0; x < dw; x++) {
            int v;
            if (x < simd_end) {
                int t0 = ((h0[x] >> 4) * b0) >> 16; /* _mm_mulhi_epi16 */
                int t1 = ((h1[x] >> 4) * b1) >> 16;
                v = (t0 + t1 + 2) >> 2;
            } else {
                v = (h0[x] * b0 + h1[x] * b1 + (1 << 21)) >> 22;
            }
            D[x] = sat_u8(v);
        }
    }
    free(xofs); free(ialpha); free(h0); free(h1);
}

/* cv::getGaussianKernel(7, 2, CV_32F) scaled by 256 and rounded as
 * createSeparableLinearFilter does for 8U smooth symmetric kernels.
 * Writes the 7 taps, returns their sum (257). */
int oc_gauss_kernel_q8(int32_t* k7) {
    float cf[7];
    double sum = 0, sigmaX = 2.0, scale2X = -0.5 / (sigmaX * sigmaX);
    for (int i = 0; i < 7; i++) {
        double x = i - (7 - 1) * 0.5;
        double t = exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    int s = 0;
    for (int i = 0; i < 7; i++) {
        cf[i] = (float)(cf[i] * sum);
        k7[i] = cv_round_f(cf[i] * 256.f);
        s += k7[i];
    }
    return s;
}

static int reflect101(int p, int n) {
    while (p < 0 || p >= n) {
        if (n == 1) return 0;
        p = p < 0 ? -p : 2 * n - 2 - p;
    }
    return p;
}

/* cv::GaussianBlur(m, m, Size(7,7), 2, 2, BORDER_REFLECT_101) on a contiguous 8UC1 clone
 * (ORBextractor.cc:1085-1086): RowFilter<uchar,int> integer row pass, then
 * SymmColumnFilter<FixedPtCastEx<int,uchar>(16)> with SSE2 SymmColumnVec_32s8u on
 * x < 4*floor(w/4) (float sum, exact, _mm_cvtps_epi32 = round half even) and the scalar
 * (s + 2^15) >> 16 tail. */
void oc_gauss7(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst, size_t dstep) {
    int32_t k[7];
    oc_gauss_kernel_q8(k);
    int* rows = (int*)malloc(sizeof(int) * (size_t)w * h);
    /* the same sums as written per pixel with reflect101 on every tap, arranged so the compiler can
     * vectorise them: reflected taps only for the 3 border columns on each side, contiguous inner loops */
    const int xi0 = w < 3 ? w : 3, xi1 = w - 3 > xi0 ? w - 3 : xi0;  /* interior columns [xi0, xi1) */
    for (int y = 0; y < h; y++) {
        const uint8_t* S = src + (size_t)y * sstep;
        int* R = rows + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            if (x == xi0) x = xi1;  /* skip the interior (below) */
            if (x >= w) break;
            int sum = 0;
            for (int i = -3; i <= 3; i++) sum += k[i + 3] * S[reflect101(x + i, w)];
            R[x] = sum;
        }
        for (int x = xi0; x < xi1; x++)
            R[x] = k[0] * S[x - 3] + k[1] * S[x - 2] + k[2] * S[x - 1] + k[3] * S[x] + k[4] * S[x + 1] +
                   k[5] * S[x + 2] + k[6] * S[x + 3];
    }
    const int vec_end = w & ~3;
    for (int y = 0; y < h; y++) {
        uint8_t* D = dst + (size_t)y * dstep;
        const int* r0 = rows + (size_t)y * w;
        const int* rp[3];
        const int* rm[3];
        for (int i = 1; i <= 3; i++) {
            rp[i - 1] = rows + (size_t)reflect101(y + i, h) * w;
            rm[i - 1] = rows + (size_t)reflect101(y - i, h) * w;
        }
        for (int x = 0; x < w; x++) {
            const int sum = k[3] * r0[x] + k[4] * (rp[0][x] + rm[0][x]) + k[5] * (rp[1][x] + rm[1][x]) +
                            k[6] * (rp[2][x] + rm[2][x]);
            /* x < vec_end: the SSE2 path's float sum scaled by 2^-16 and rounded half to even
             * (_mm_cvtps_epi32), exact for sum < 2^24 and saturating above, = the integer round half even
             * below; the scalar tail (sum + 2^15) >> 16. sum >= 0 (non-negative taps and pixels). */
            const int v = x < vec_end ? (sum + 0x7FFF + ((sum >> 16) & 1)) >> 16 : (sum + (1 << 15)) >> 16;
            D[x] = (uint8_t)(v > 255 ? 255 : v);
        }
    }
    free(rows);
}

/* ------------------------------------------------------------------ cv::FAST ------ */
/* OpenCV 3.x cornerScore<16> (scalar form; the SSE2 form computes the same value). */
static int corner_score16(const uint8_t* ptr, const int pixel[], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[25];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
        if (d[k + 3] < a) a = d[k + 3];
        if (a <= a0) continue;
        for (int q = 4; q <= 8; q++) if (d[k + q] < a) a = d[k + q];
        int m = a < d[k] ? a : d[k];
        if (m > a0) a0 = m;
        m = a < d[k + 9] ? a : d[k + 9];
        if (m > a0) a0 = m;
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
        for (int q = 3; q <= 5; q++) if (d[k + q] > b) b = d[k + q];
        if (b >= b0) continue;
        for (int q = 6; q <= 8; q++) if (d[k + q] > b) b = d[k + q];
        int m = b > d[k] ? b : d[k];
        if (m < b0) b0 = m;
        m = b > d[k + 9] ? b : d[k + 9];
        if (m < b0) b0 = m;
    }
    return -b0 - 1;
}

/* 1: FAST decides 16 pixels of a row at a time with SSE2, as OpenCV's FAST_t<16> vector form does (the
 * CPU baseline then times the form the reference runs through OpenCV; unlike OpenCV, a row's tail is one
 * more, overlapping, vector step instead of scalar pixels); 0: the scalar form for every pixel. Both give
 * the same keypoints and scores (tests/test_oracle_primitives.py compares them). */
static int g_fast_simd = 1;
void oc_set_fast_simd(int on) { g_fast_simd = on; }

#if defined(__SSE2__)
#include <emmintrin.h>
/* OpenCV FAST_t<16> vector step over the 16 pixels at ptr: a pixel is a corner when some 9 contiguous
 * circle pixels (of the 25-long wrapped circle, as the scalar count > K) are all brighter than v+t or all
 * darker than v-t, with v+t / v-t saturated to [0,255] (an x beyond them never exists, as in the scalar
 * int comparison). Bytes are compared signed after ^0x80. The cardinal pre-test (two consecutive
 * cardinal points both brighter / both darker) is necessary for a 9-arc. Returns the 16-bit corner mask. */
static unsigned fast_sse2_16(const uint8_t* ptr, const int pixel[25], int threshold) {
    const __m128i delta = _mm_set1_epi8((char)0x80), t = _mm_set1_epi8((char)threshold);
    const __m128i vv = _mm_loadu_si128((const __m128i*)ptr);
    const __m128i vlo = _mm_xor_si128(_mm_subs_epu8(vv, t), delta);
    const __m128i vhi = _mm_xor_si128(_mm_adds_epu8(vv, t), delta);
#define LDX(k) _mm_xor_si128(_mm_loadu_si128((const __m128i*)(ptr + pixel[k])), delta)
    const __m128i x0 = LDX(0), x1 = LDX(4), x2 = LDX(8), x3 = LDX(12);
    const __m128i b0 = _mm_cmpgt_epi8(x0, vhi), b1 = _mm_cmpgt_epi8(x1, vhi), b2 = _mm_cmpgt_epi8(x2, vhi),
                  b3 = _mm_cmpgt_epi8(x3, vhi);
    const __m128i d0 = _mm_cmpgt_epi8(vlo, x0), d1 = _mm_cmpgt_epi8(vlo, x1), d2 = _mm_cmpgt_epi8(vlo, x2),
                  d3 = _mm_cmpgt_epi8(vlo, x3);
    __m128i m = _mm_or_si128(_mm_and_si128(b0, b1), _mm_and_si128(b1, b2));
    m = _mm_or_si128(m, _mm_or_si128(_mm_and_si128(b2, b3), _mm_and_si128(b3, b0)));
    m = _mm_or_si128(m, _mm_or_si128(_mm_and_si128(d0, d1), _mm_and_si128(d1, d2)));
    m = _mm_or_si128(m, _mm_or_si128(_mm_and_si128(d2, d3), _mm_and_si128(d3, d0)));
    if (_mm_movemask_epi8(m) == 0) return 0;
    __m128i c0 = _mm_setzero_si128(), c1 = c0, max0 = c0, max1 = c0;
    for (int k = 0; k < 25; k++) { /* run lengths: c = (c + 1) & hit, per byte */
        const __m128i x = LDX(k);
        const __m128i h0 = _mm_cmpgt_epi8(x, vhi), h1 = _mm_cmpgt_epi8(vlo, x);
        c0 = _mm_and_si128(_mm_sub_epi8(c0, h0), h0);
        c1 = _mm_and_si128(_mm_sub_epi8(c1, h1), h1);
        max0 = _mm_max_epu8(max0, c0);
        max1 = _mm_max_epu8(max1, c1);
    }
#undef LDX
    max0 = _mm_max_epu8(max0, max1);
    return (unsigned)_mm_movemask_epi8(_mm_cmpgt_epi8(max0, _mm_set1_epi8(8)));
}

/* cornerScore<16>, OpenCV's SSE2 form: for the 16 arcs of 9 (8 at a time, as int16 lanes), the dark
 * bound max_k min(d[k..k+8]) and the bright bound min_k max(d[k..k+8]); score = max(dark, -bright) - 1.
 * For a corner it equals corner_score16 (whose threshold floor is below both). */
static int corner_score16_sse2(const uint8_t* ptr, const int pixel[25]) {
    short d[32];
    const int v = ptr[0];
    for (int k = 0; k < 25; k++) d[k] = (short)(v - ptr[pixel[k]]);
    __m128i q0 = _mm_set1_epi16(-1000), q1 = _mm_set1_epi16(1000);
    for (int k = 0; k < 16; k += 8) {
        __m128i a = _mm_loadu_si128((const __m128i*)(d + k + 1)), b = a;
        for (int q = 2; q <= 8; q++) {
            const __m128i x = _mm_loadu_si128((const __m128i*)(d + k + q));
            a = _mm_min_epi16(a, x);
            b = _mm_max_epi16(b, x);
        }
        const __m128i e0 = _mm_loadu_si128((const __m128i*)(d + k)), e9 = _mm_loadu_si128((const __m128i*)(d + k + 9));
        q0 = _mm_max_epi16(q0, _mm_max_epi16(_mm_min_epi16(a, e0), _mm_min_epi16(a, e9)));
        q1 = _mm_min_epi16(q1, _mm_min_epi16(_mm_max_epi16(b, e0), _mm_max_epi16(b, e9)));
    }
    q0 = _mm_max_epi16(q0, _mm_sub_epi16(_mm_setzero_si128(), q1));
    q0 = _mm_max_epi16(q0, _mm_unpackhi_epi64(q0, q0));
    q0 = _mm_max_epi16(q0, _mm_srli_si128(q0, 4));
    q0 = _mm_max_epi16(q0, _mm_srli_si128(q0, 2));
    return (short)_mm_cvtsi128_si32(q0) - 1;
}
#endif

/* cv::FAST(img, keypoints, threshold, nonmaxSuppression=true), TYPE_9_16: OpenCV 3.x
 * FAST_t<16>. Called per cell at ORBextractor.cc:809-816. */
int oc_fast(const uint8_t* img, int cols, int rows, size_t step, int threshold, float* xyr,
            int cap) {
    static const int off16[16][2] = {{0, 3}, {1, 3},  {2, 2},  {3, 1},  {3, 0},   {3, -1},
                                     {2, -2}, {1, -3}, {0, -3}, {-1, -3}, {-2, -2}, {-3, -1},
                                     {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    const int K = 8, N = 25;
    int pixel[25], i, j, k, nkp = 0;
    for (k = 0; k < 16; k++) pixel[k] = off16[k][0] + off16[k][1] * (int)step;
    for (; k < 25; k++) pixel[k] = pixel[k - 16];
    threshold = threshold < 0 ? 0 : threshold > 255 ? 255 : threshold;
    uint8_t tab[512];
    for (i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols < 7 || rows < 7) return 0;
    /* row buffers on the stack for a cell-sized ROI, as cv::FAST's AutoBuffer keeps them (no heap
     * allocation per ORBextractor cell) */
    uint8_t sbuf[3 * 128];
    int scp[3 * 129];
    const int small = cols <= 128;
    uint8_t* bufmem = small ? sbuf : (uint8_t*)malloc((size_t)cols * 3);
    int* cpmem = small ? scp : (int*)malloc(sizeof(int) * (size_t)(cols + 1) * 3);
    memset(bufmem, 0, (size_t)cols * 3);
    uint8_t* buf[3] = {bufmem, bufmem + cols, bufmem + 2 * cols};
    int* cpbuf[3] = {cpmem + 1, cpmem + 1 + (cols + 1), cpmem + 1 + 2 * (cols + 1)};
    for (i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            j = 3;
#if defined(__SSE2__)
            if (g_fast_simd && cols - 3 - 16 >= 3) {
                for (; j < cols - 3; j += 16, ptr += 16) {
                    unsigned skip = 0;  /* the row's tail: one step ending at cols-4, its first columns done */
                    if (j + 16 > cols - 3) {
                        skip = (unsigned)(j - (cols - 3 - 16));
                        ptr -= skip;
                        j -= (int)skip;
                    }
                    for (unsigned m = fast_sse2_16(ptr, pixel, threshold) >> skip << skip; m; m &= m - 1) {
                        const int b = __builtin_ctz(m);
                        cornerpos[ncorners++] = j + b;
                        curr[j + b] = (uint8_t)corner_score16_sse2(ptr + b, pixel);
                    }
                }
            }
#endif
            for (; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* t = tab - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (k = 0; k < ncorners; k++) {
            j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                score > curr[j] && score > curr[j + 1]) {
                if (nkp < cap) {
                    xyr[3 * nkp] = (float)j;
                    xyr[3 * nkp + 1] = (float)(i - 1);
                    xyr[3 * nkp + 2] = (float)score;
                }
                nkp++;
            }
        }
    }
    if (!small) {
        free(bufmem);
        free(cpmem);
    }
    return nkp;
}

/* ------------------------------------------------------------ DistributeOctTree --- */
typedef struct { float x, y, r; } okey;
typedef struct ocnode {
    int ulx, uly, urx, ury, blx, bly, brx, bry; /* UL, UR, BL, BR (ORBextractor.h:40) */
    int* keys; /* indices into the level's candidate array (vKeys) */
    int nk, cap;
    int bNoMore;
    long seq; /* creation order: stands in for the heap address the reference sorts on */
    struct ocnode *prev, *next;
} ocnode;

typedef struct {
    ocnode *head, *tail;
    int size;
    long next_seq;
} olist;

static void node_add(ocnode* n, int k) {
    if (n->nk == n->cap) {
        n->cap = n->cap ? n->cap * 2 : 4;
        n->keys = (int*)realloc(n->keys, sizeof(int) * n->cap);
    }
    n->keys[n->nk++] = k;
}
/* list node creation: std::list::push_front/push_back copy-constructs the temporary into a
 * fresh allocation; under a bump allocator its address grows with creation order. */
static ocnode* olist_push(olist* L, const ocnode* tmp, int front) {
    ocnode* n = (ocnode*)malloc(sizeof(ocnode));
    *n = *tmp;
    n->seq = L->next_seq++;
    if (front) {
        n->prev = NULL; n->next = L->head;
        if (L->head) L->head->prev = n; else L->tail = n;
        L->head = n;
    } else {
        n->next = NULL; n->prev = L->tail;
        if (L->tail) L->tail->next = n; else L->head = n;
        L->tail = n;
    }
    L->size++;
    return n;
}
static ocnode* olist_erase(olist* L, ocnode* n) {
    ocnode* nx = n->next;
    if (n->prev) n->prev->next = n->next; else L->head = n->next;
    if (n->next) n->next->prev = n->prev; else L->tail = n->prev;
    free(n->keys);
    free(n);
    L->size--;
    return nx;
}

/* ExtractorNode::DivideNode (ORBextractor.cc:481-537) */
static void divide_node(const ocnode* p, const okey* K, ocnode c[4]) {
    const int halfX = (int)ceilf((float)(p->urx - p->ulx) / 2);
    const int halfY = (int)ceilf((float)(p->bry - p->uly) / 2);
    memset(c, 0, sizeof(ocnode) * 4);
    c[0].ulx = p->ulx; c[0].uly = p->uly;
    c[0].urx = p->ulx + halfX; c[0].ury = p->uly;
    c[0].blx = p->ulx; c[0].bly = p->uly + halfY;
    c[0].brx = p->ulx + halfX; c[0].bry = p->uly + halfY;
    c[1].ulx = c[0].urx; c[1].uly = c[0].ury;
    c[1].urx = p->urx; c[1].ury = p->ury;
    c[1].blx = c[0].brx; c[1].bly = c[0].bry;
    c[1].brx = p->urx; c[1].bry = p->uly + halfY;
    c[2].ulx = c[0].blx; c[2].uly = c[0].bly;
    c[2].urx = c[0].brx; c[2].ury = c[0].bry;
    c[2].blx = p->blx; c[2].bly = p->bly;
    c[2].brx = c[0].brx; c[2].bry = p->bly;
    c[3].ulx = c[2].urx; c[3].uly = c[2].ury;
    c[3].urx = c[1].brx; c[3].ury = c[1].bry;
    c[3].blx = c[2].brx; c[3].bly = c[2].bry;
    c[3].brx = p->brx; c[3].bry = p->bry;
    for (int i = 0; i < p->nk; i++) {
        const okey* kp = &K[p->keys[i]];
        if (kp->x < c[0].urx) {
            if (kp->y < c[0].bry) node_add(&c[0], p->keys[i]);
            else node_add(&c[2], p->keys[i]);
        } else if (kp->y < c[0].bry)
            node_add(&c[1], p->keys[i]);
        else
            node_add(&c[3], p->keys[i]);
    }
    for (int q = 0; q < 4; q++) if (c[q].nk == 1) c[q].bNoMore = 1;
}

typedef struct { int size; ocnode* node; } sizeptr;
static int sizeptr_cmp(const void* a, const void* b) {
    const sizeptr* x = (const sizeptr*)a;
    const sizeptr* y = (const sizeptr*)b;
    if (x->size != y->size) return x->size < y->size ? -1 : 1;
    return x->node->seq < y->node->seq ? -1 : (x->node->seq > y->node->seq ? 1 : 0);
}
typedef struct { sizeptr* v; int n, cap; } spvec;
static void spvec_push(spvec* s, int size, ocnode* n) {
    if (s->n == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 64;
        s->v = (sizeptr*)realloc(s->v, sizeof(sizeptr) * s->cap);
    }
    s->v[s->n].size = size;
    s->v[s->n].node = n;
    s->n++;
}

/* push the non-empty children in the order n1,n2,n3,n4 (ORBextractor.cc:621-660) */
static int push_children(olist* L, ocnode c[4], spvec* rec) {
    int nexp = 0;
    for (int q = 0; q < 4; q++) {
        if (c[q].nk > 0) {
            ocnode* n = olist_push(L, &c[q], 1);
            if (c[q].nk > 1) {
                nexp++;
                spvec_push(rec, n->nk, n);
            }
        } else {
            free(c[q].keys);
        }
    }
    return nexp;
}

/* ORBextractor::DistributeOctTree (ORBextractor.cc:539-763). The phase-2 sort's tie-break
 * on ExtractorNode* (ORBextractor.cc:681-684) is pinned to creation order. Output: level
 * keypoints (relative coords) written to out (xyr triplets); returns the count. */
static int distribute_octtree(const okey* K, int nkeys, int minX, int maxX, int minY, int maxY,
                              int N, okey* out) {
    const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    olist L = {NULL, NULL, 0, 0};
    ocnode** ini = (ocnode**)malloc(sizeof(ocnode*) * (nIni > 0 ? nIni : 1));
    for (int i = 0; i < nIni; i++) {
        ocnode ni;
        memset(&ni, 0, sizeof(ni));
        ni.ulx = (int)(hX * (float)i); ni.uly = 0;
        ni.urx = (int)(hX * (float)(i + 1)); ni.ury = 0;
        ni.blx = ni.ulx; ni.bly = maxY - minY;
        ni.brx = ni.urx; ni.bry = maxY - minY;
        ini[i] = olist_push(&L, &ni, 0);
    }
    for (int i = 0; i < nkeys; i++) {
        size_t r = (size_t)(K[i].x / hX);
        if (r >= (size_t)nIni) abort(); /* out of range in the reference too (UB) */
        node_add(ini[r], i);
    }
    free(ini);
    ocnode* lit = L.head;
    while (lit) {
        if (lit->nk == 1) {
            lit->bNoMore = 1;
            lit = lit->next;
        } else if (lit->nk == 0)
            lit = olist_erase(&L, lit);
        else
            lit = lit->next;
    }
    int bFinish = 0;
    spvec rec = {NULL, 0, 0}, prevrec = {NULL, 0, 0};
    while (!bFinish) {
        int prevSize = L.size;
        lit = L.head;
        int nToExpand = 0;
        rec.n = 0;
        while (lit) {
            if (lit->bNoMore) {
                lit = lit->next;
                continue;
            }
            ocnode c[4];
            divide_node(lit, K, c);
            nToExpand += push_children(&L, c, &rec);
            lit = olist_erase(&L, lit);
        }
        if (L.size >= N || L.size == prevSize) {
            bFinish = 1;
        } else if (L.size + nToExpand * 3 > N) {
            while (!bFinish) {
                prevSize = L.size;
                spvec t = prevrec; prevrec = rec; rec = t; /* vPrev = v; v.clear() */
                rec.n = 0;
                qsort(prevrec.v, prevrec.n, sizeof(sizeptr), sizeptr_cmp);
                for (int j = prevrec.n - 1; j >= 0; j--) {
                    ocnode c[4];
                    divide_node(prevrec.v[j].node, K, c);
                    push_children(&L, c, &rec);
                    olist_erase(&L, prevrec.v[j].node);
                    if (L.size >= N) break;
                }
                if (L.size >= N || L.size == prevSize) bFinish = 1;
            }
        }
    }
    int nout = 0;
    for (lit = L.head; lit; lit = lit->next) {
        int best = lit->keys[0];
        float maxResponse = K[best].r;
        for (int k = 1; k < lit->nk; k++) {
            if (K[lit->keys[k]].r > maxResponse) {
                best = lit->keys[k];
                maxResponse = K[best].r;
            }
        }
        out[nout++] = K[best];
    }
    while (L.head) olist_erase(&L, L.head);
    free(rec.v);
    free(prevrec.v);
    return nout;
}

/* ---------------------------------------------------------- orientation, rBRIEF --- */
/* IC_Angle (ORBextractor.cc:77-104) */
static float ic_angle(const uint8_t* img, size_t step, float px, float py, const int* umax) {
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = img + (size_t)cv_round_f(py) * step + cv_round_f(px);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    int st = (int)step;
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * st], val_minus = center[u - v * st];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return oc_fast_atan2((float)m_01, (float)m_10);
}

/* computeOrbDescriptor (ORBextractor.cc:107-147) */
static void orb_descriptor(float px, float py, float angle_deg, const uint8_t* img, size_t step,
                           uint8_t* desc) {
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float angle = angle_deg * factorPI;
    float a = cosf(angle), b = sinf(angle);
    const uint8_t* center = img + (size_t)cv_round_f(py) * step + cv_round_f(px);
    const int st = (int)step;
    const signed char* pat = (const signed char*)orb_oracle_pattern_u8;
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int j = 0; j < 8; j++) {
            const signed char* p = pat + 4 * (8 * i + j);
            float x0 = (float)p[0], y0 = (float)p[1], x1 = (float)p[2], y1 = (float)p[3];
            int t0 = center[cv_round_f(x0 * b + y0 * a) * st + cv_round_f(x0 * a - y0 * b)];
            int t1 = center[cv_round_f(x1 * b + y1 * a) * st + cv_round_f(x1 * a - y1 * b)];
            val |= (t0 < t1) << j;
        }
        desc[i] = (uint8_t)val;
    }
}

/* ----------------------------------------------------------------- extractor ------ */
struct oc_extractor {
    int nfeatures;
    double scaleFactor; /* double member: ORBextractor.h:100 */
    int nlevels, iniThFAST, minThFAST;
    float scale[MAXL], inv_scale[MAXL], sigma2[MAXL], inv_sigma2[MAXL];
    int nfeat[MAXL];
    int umax[HALF_PATCH_SIZE + 1];
    int lw[MAXL], lh[MAXL];
    uint8_t* pyr[MAXL];
    uint8_t* blur[MAXL];
    okey* cand[MAXL];
    int ncand[MAXL], capcand[MAXL];
    okey* oct[MAXL];
    int noct[MAXL];
    /* per-stage wall time (bench.py's CPU breakdown): pyramid, FAST, octree, orientation, blur, descriptor */
    double stage_s[6];
    int stage_frames;
};

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ORBextractor::ORBextractor (ORBextractor.cc:410-470) */
oc_extractor* oc_create(const orbx_params* p) {
    if (!p || p->nlevels < 1 || p->nlevels > MAXL || p->nfeatures < 0) return NULL;
    oc_extractor* e = (oc_extractor*)calloc(1, sizeof(oc_extractor));
    e->nfeatures = p->nfeatures;
    e->scaleFactor = p->scale_factor;
    e->nlevels = p->nlevels;
    e->iniThFAST = p->ini_th_fast;
    e->minThFAST = p->min_th_fast;
    e->scale[0] = 1.0f;
    e->sigma2[0] = 1.0f;
    for (int i = 1; i < e->nlevels; i++) {
        e->scale[i] = (float)(e->scale[i - 1] * e->scaleFactor);
        e->sigma2[i] = e->scale[i] * e->scale[i];
    }
    for (int i = 0; i < e->nlevels; i++) {
        e->inv_scale[i] = 1.0f / e->scale[i];
        e->inv_sigma2[i] = 1.0f / e->sigma2[i];
    }
    float factor = (float)(1.0f / e->scaleFactor);
    float nDesired = e->nfeatures * (1 - factor) /
                     (1 - (float)pow((double)factor, (double)e->nlevels));
    int sumFeatures = 0;
    for (int level = 0; level < e->nlevels - 1; level++) {
        e->nfeat[level] = cv_round_f(nDesired);
        sumFeatures += e->nfeat[level];
        nDesired *= factor;
    }
    int last = e->nfeatures - sumFeatures;
    e->nfeat[e->nlevels - 1] = last > 0 ? last : 0;
    int v, v0, vmax = cv_floor_f(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    int vmin = cv_ceil_f(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) e->umax[v] = cv_round_d(sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (e->umax[v0] == e->umax[v0 + 1]) ++v0;
        e->umax[v] = v0;
        ++v0;
    }
    return e;
}

static void free_frame(oc_extractor* e) {
    for (int l = 0; l < MAXL; l++) {
        free(e->pyr[l]); e->pyr[l] = NULL;
        free(e->blur[l]); e->blur[l] = NULL;
        free(e->cand[l]); e->cand[l] = NULL;
        free(e->oct[l]); e->oct[l] = NULL;
        e->ncand[l] = e->capcand[l] = e->noct[l] = 0;
    }
}

void oc_destroy(oc_extractor* e) {
    if (!e) return;
    free_frame(e);
    free(e);
}

static void add_cand(oc_extractor* e, int l, float x, float y, float r) {
    if (e->ncand[l] == e->capcand[l]) {
        e->capcand[l] = e->capcand[l] ? e->capcand[l] * 2 : 1024;
        e->cand[l] = (okey*)realloc(e->cand[l], sizeof(okey) * e->capcand[l]);
    }
    okey k = {x, y, r};
    e->cand[l][e->ncand[l]++] = k;
}

/* ORBextractor::ComputeKeyPointsOctTree (ORBextractor.cc:765-853), minus orientation */
static void compute_keypoints_octtree(oc_extractor* e) {
    const float W = 30;
    float* cell = NULL;
    int cellcap = 0;
    for (int level = 0; level < e->nlevels; ++level) {
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = e->lw[level] - EDGE_THRESHOLD + 3;
        const int maxBorderY = e->lh[level] - EDGE_THRESHOLD + 3;
        const float width = (float)(maxBorderX - minBorderX);
        const float height = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width / W), nRows = (int)(height / W);
        const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
        const uint8_t* img = e->pyr[level];
        const size_t step = (size_t)e->lw[level];
        const double t_fast = now_s();
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                const int y0 = (int)iniY, y1 = (int)maxY, x0 = (int)iniX, x1 = (int)maxX;
                const uint8_t* roi = img + (size_t)y0 * step + x0;
                int need = (x1 - x0) * (y1 - y0);
                if (need * 3 > cellcap) {
                    cellcap = need * 3;
                    cell = (float*)realloc(cell, sizeof(float) * cellcap);
                }
                int n = oc_fast(roi, x1 - x0, y1 - y0, step, e->iniThFAST, cell, cellcap / 3);
                if (n == 0) n = oc_fast(roi, x1 - x0, y1 - y0, step, e->minThFAST, cell, cellcap / 3);
                for (int k = 0; k < n; k++)
                    add_cand(e, level, cell[3 * k] + j * wCell, cell[3 * k + 1] + i * hCell,
                             cell[3 * k + 2]);
            }
        }
        const double t_oct = now_s();
        e->stage_s[1] += t_oct - t_fast;
        e->oct[level] = (okey*)malloc(sizeof(okey) * (size_t)(e->ncand[level] + 1));
        e->noct[level] = e->ncand[level] == 0
                             ? 0
                             : distribute_octtree(e->cand[level], e->ncand[level], minBorderX,
                                                  maxBorderX, minBorderY, maxBorderY,
                                                  e->nfeat[level], e->oct[level]);
        for (int k = 0; k < e->noct[level]; k++) {
            e->oct[level][k].x += minBorderX;
            e->oct[level][k].y += minBorderY;
        }
        e->stage_s[2] += now_s() - t_oct;
    }
    free(cell);
}

/* ORBextractor::operator() (ORBextractor.cc:1043-1105) */
int oc_extract(oc_extractor* e, const uint8_t* img, int w, int h, size_t pitch, orbx_kp* kps,
               uint8_t* desc, int cap, int* n) {
    *n = 0;
    if (w <= 0 || h <= 0 || !img) return 0;
    free_frame(e);
    double t0 = now_s();
    /* ComputePyramid (ORBextractor.cc:1107-1132); padded borders are never read. */
    for (int level = 0; level < e->nlevels; ++level) {
        float scale = e->inv_scale[level];
        int sw = cv_round_f((float)w * scale), sh = cv_round_f((float)h * scale);
        e->lw[level] = sw;
        e->lh[level] = sh;
        e->pyr[level] = (uint8_t*)malloc((size_t)sw * sh);
        if (level == 0) {
            for (int y = 0; y < h; y++) memcpy(e->pyr[0] + (size_t)y * w, img + (size_t)y * pitch, w);
        } else {
            oc_resize_linear(e->pyr[level - 1], e->lw[level - 1], e->lh[level - 1],
                             (size_t)e->lw[level - 1], e->pyr[level], sw, sh, (size_t)sw);
        }
    }
    e->stage_s[0] += now_s() - t0;
    compute_keypoints_octtree(e);
    int total = 0;
    for (int level = 0; level < e->nlevels; ++level) total += e->noct[level];
    if (total > cap) return ORBX_ECAPACITY;
    int offset = 0;
    for (int level = 0; level < e->nlevels; ++level) {
        const int nl = e->noct[level];
        if (nl == 0) continue;
        const int lw = e->lw[level], lh = e->lh[level];
        /* computeOrientation (ORBextractor.cc:851-852) runs before the per-level blur + describe
         * loop in the reference; the two per-keypoint loops are independent, so timing them
         * separately does not change any output */
        t0 = now_s();
        for (int k = 0; k < nl; k++) {
            const okey* kp = &e->oct[level][k];
            kps[offset + k].angle = ic_angle(e->pyr[level], (size_t)lw, kp->x, kp->y, e->umax);
        }
        double t1 = now_s();
        e->stage_s[3] += t1 - t0;
        e->blur[level] = (uint8_t*)malloc((size_t)lw * lh);
        oc_gauss7(e->pyr[level], lw, lh, (size_t)lw, e->blur[level], (size_t)lw);
        t0 = now_s();
        e->stage_s[4] += t0 - t1;
        const float scaledPatchSize = (float)(int)(PATCH_SIZE * e->scale[level]);
        for (int k = 0; k < nl; k++) {
            const okey* kp = &e->oct[level][k];
            const float ang = kps[offset + k].angle;
            orb_descriptor(kp->x, kp->y, ang, e->blur[level], (size_t)lw, desc + 32 * (offset + k));
            orbx_kp* o = &kps[offset + k];
            o->x = kp->x;
            o->y = kp->y;
            if (level != 0) {
                o->x = kp->x * e->scale[level];
                o->y = kp->y * e->scale[level];
            }
            o->size = scaledPatchSize;
            o->angle = ang;
            o->response = kp->r;
            o->octave = level;
        }
        e->stage_s[5] += now_s() - t0;
        offset += nl;
    }
    e->stage_frames++;
    *n = total;
    return 0;
}

void oc_stage_times(const oc_extractor* e, double* sec6, int* nframes) {
    for (int i = 0; i < 6; i++) sec6[i] = e->stage_s[i];
    *nframes = e->stage_frames;
}

int oc_level_size(const oc_extractor* e, int level, int* w, int* h) {
    if (level < 0 || level >= e->nlevels) return ORBX_EARG;
    *w = e->lw[level];
    *h = e->lh[level];
    return 0;
}
const uint8_t* oc_pyramid(const oc_extractor* e, int level) { return e->pyr[level]; }
const uint8_t* oc_blurred(const oc_extractor* e, int level) { return e->blur[level]; }
int oc_level_candidates(const oc_extractor* e, int level, float* xyr, int cap) {
    int n = e->ncand[level];
    for (int k = 0; k < n && k < cap; k++) {
        xyr[3 * k] = e->cand[level][k].x;
        xyr[3 * k + 1] = e->cand[level][k].y;
        xyr[3 * k + 2] = e->cand[level][k].r;
    }
    return n;
}
int oc_level_octree(const oc_extractor* e, int level, float* xyr, int cap) {
    int n = e->noct[level];
    for (int k = 0; k < n && k < cap; k++) {
        xyr[3 * k] = e->oct[level][k].x;
        xyr[3 * k + 1] = e->oct[level][k].y;
        xyr[3 * k + 2] = e->oct[level][k].r;
    }
    return n;
}
void oc_get_tables(const oc_extractor* e, float* scale, float* inv_scale, float* sigma2,
                   float* inv_sigma2, int32_t* nfeat, int32_t* umax16) {
    for (int l = 0; l < e->nlevels; l++) {
        if (scale) scale[l] = e->scale[l];
        if (inv_scale) inv_scale[l] = e->inv_scale[l];
        if (sigma2) sigma2[l] = e->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = e->inv_sigma2[l];
        if (nfeat) nfeat[l] = e->nfeat[l];
    }
    if (umax16) for (int v = 0; v <= HALF_PATCH_SIZE; v++) umax16[v] = e->umax[v];
}

/* host libm sinf/cosf over an array (what computeOrbDescriptor calls, ORBextractor.cc:113) */
void oc_sincosf_batch(const float* in, float* s, float* c, int n) {
    for (int i = 0; i < n; i++) {
        s[i] = sinf(in[i]);
        c[i] = cosf(in[i]);
    }
}

/* ------------------------------------------------------------------- matcher ------ */
/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:1647-1663) */
int oc_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        int32_t pa, pb;
        memcpy(&pa, a + 4 * i, 4);
        memcpy(&pb, b + 4 * i, 4);
        unsigned int v = (unsigned int)(pa ^ pb);
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

#define TH_HIGH 100   /* ORBmatcher.cc:37 */
#define TH_LOW 50     /* ORBmatcher.cc:38 */
#define HISTO_LENGTH 30 /* ORBmatcher.cc:39 */

typedef struct { int* v; int n, cap; } ivec;
static void ivec_push(ivec* s, int x) {
    if (s->n == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 64;
        s->v = (int*)realloc(s->v, sizeof(int) * s->cap);
    }
    s->v[s->n++] = x;
}

/* ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:1601-1642) */
static void three_maxima(const ivec* histo, int L, int* ind1, int* ind2, int* ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = histo[i].n;
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            *ind3 = *ind2; *ind2 = i;
        } else if (s > max3) {
            max3 = s;
            *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        *ind2 = -1; *ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        *ind3 = -1;
    }
}

static int rot_bin(float a1, float a2) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

/* ORBmatcher::CheckDistEpipolarLine (ORBmatcher.cc:140-157) */
static int check_dist_epipolar(float x1, float y1, float x2, float y2, const float* F,
                               float sigma2) {
    const float a = x1 * F[0] + y1 * F[3] + F[6];
    const float b = x1 * F[1] + y1 * F[4] + F[7];
    const float c = x1 * F[2] + y1 * F[5] + F[8];
    const float num = a * x2 + b * y2 + c;
    const float den = a * a + b * b;
    if (den == 0) return 0;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * sigma2;
}

static int lower_bound_u32(const uint32_t* a, int n, int from, uint32_t key) {
    int lo = from, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

static int has_mp(const orbm_kf_view* v, int i) { return v->has_mp ? v->has_mp[i] != 0 : 0; }
static int mp_bad(const orbm_kf_view* v, int i) { return v->mp_bad ? v->mp_bad[i] != 0 : 0; }

/* ORBmatcher::SearchForTriangulation (ORBmatcher.cc:657-823) */
int oc_search_for_triangulation(const orbm_kf_view* kf1, const orbm_kf_view* kf2,
                                const float F12[9], float ex, float ey, int bOnlyStereo,
                                int checkOri, int32_t* match12) {
    int nmatches = 0;
    ivec rotHist[HISTO_LENGTH];
    memset(rotHist, 0, sizeof(rotHist));
    for (int i = 0; i < kf1->n; i++) match12[i] = -1;
    int f1 = 0, f2 = 0;
    while (f1 < kf1->n_nodes && f2 < kf2->n_nodes) {
        if (kf1->node_id[f1] == kf2->node_id[f2]) {
            for (int i1 = kf1->node_off[f1]; i1 < kf1->node_off[f1 + 1]; i1++) {
                const int idx1 = kf1->node_feat[i1];
                if (has_mp(kf1, idx1)) continue;
                const int bStereo1 = kf1->uright ? kf1->uright[idx1] >= 0 : 0;
                if (bOnlyStereo && !bStereo1) continue;
                const uint8_t* d1 = kf1->desc + 32 * (size_t)idx1;
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int i2 = kf2->node_off[f2]; i2 < kf2->node_off[f2 + 1]; i2++) {
                    const int idx2 = kf2->node_feat[i2];
                    if (has_mp(kf2, idx2)) continue; /* vbMatched2 is never set (:677) */
                    const int bStereo2 = kf2->uright ? kf2->uright[idx2] >= 0 : 0;
                    if (bOnlyStereo && !bStereo2) continue;
                    const int dist = oc_descriptor_distance(d1, kf2->desc + 32 * (size_t)idx2);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const int oct2 = kf2->octave[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ex - kf2->x[idx2];
                        const float distey = ey - kf2->y[idx2];
                        if (distex * distex + distey * distey < 100 * kf2->scale_factors[oct2])
                            continue;
                    }
                    if (check_dist_epipolar(kf1->x[idx1], kf1->y[idx1], kf2->x[idx2],
                                            kf2->y[idx2], F12, kf2->level_sigma2[oct2])) {
                        bestIdx2 = idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    match12[idx1] = bestIdx2;
                    nmatches++;
                    if (checkOri)
                        ivec_push(&rotHist[rot_bin(kf1->angle[idx1], kf2->angle[bestIdx2])], idx1);
                }
            }
            f1++;
            f2++;
        } else if (kf1->node_id[f1] < kf2->node_id[f2]) {
            f1 = lower_bound_u32(kf1->node_id, kf1->n_nodes, f1, kf2->node_id[f2]);
        } else {
            f2 = lower_bound_u32(kf2->node_id, kf2->n_nodes, f2, kf1->node_id[f1]);
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j = 0; j < rotHist[i].n; j++) {
                match12[rotHist[i].v[j]] = -1;
                nmatches--;
            }
        }
    }
    for (int i = 0; i < HISTO_LENGTH; i++) free(rotHist[i].v);
    return nmatches;
}

/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (ORBmatcher.cc:159-288) */
int oc_search_by_bow_kf_f(const orbm_kf_view* kf, const orbm_kf_view* f, float nnratio,
                          int checkOri, int32_t* match_f) {
    int nmatches = 0;
    ivec rotHist[HISTO_LENGTH];
    memset(rotHist, 0, sizeof(rotHist));
    for (int i = 0; i < f->n; i++) match_f[i] = -1;
    int a = 0, b = 0;
    while (a < kf->n_nodes && b < f->n_nodes) {
        if (kf->node_id[a] == f->node_id[b]) {
            for (int iKF = kf->node_off[a]; iKF < kf->node_off[a + 1]; iKF++) {
                const int realIdxKF = kf->node_feat[iKF];
                if (!has_mp(kf, realIdxKF)) continue;
                if (mp_bad(kf, realIdxKF)) continue;
                const uint8_t* dKF = kf->desc + 32 * (size_t)realIdxKF;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (int iF = f->node_off[b]; iF < f->node_off[b + 1]; iF++) {
                    const int realIdxF = f->node_feat[iF];
                    if (match_f[realIdxF] >= 0) continue;
                    const int dist = oc_descriptor_distance(dKF, f->desc + 32 * (size_t)realIdxF);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdxF = realIdxF;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 <= TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        match_f[bestIdxF] = realIdxKF;
                        if (checkOri)
                            ivec_push(&rotHist[rot_bin(kf->angle[realIdxKF], f->angle[bestIdxF])],
                                      bestIdxF);
                        nmatches++;
                    }
                }
            }
            a++;
            b++;
        } else if (kf->node_id[a] < f->node_id[b]) {
            a = lower_bound_u32(kf->node_id, kf->n_nodes, a, f->node_id[b]);
        } else {
            b = lower_bound_u32(f->node_id, f->n_nodes, b, kf->node_id[a]);
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j = 0; j < rotHist[i].n; j++) {
                match_f[rotHist[i].v[j]] = -1;
                nmatches--;
            }
        }
    }
    for (int i = 0; i < HISTO_LENGTH; i++) free(rotHist[i].v);
    return nmatches;
}

/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, ...) (ORBmatcher.cc:522-655) */
int oc_search_by_bow_kf_kf(const orbm_kf_view* kf1, const orbm_kf_view* kf2, float nnratio,
                           int checkOri, int32_t* match12) {
    int nmatches = 0;
    ivec rotHist[HISTO_LENGTH];
    memset(rotHist, 0, sizeof(rotHist));
    for (int i = 0; i < kf1->n; i++) match12[i] = -1;
    uint8_t* matched2 = (uint8_t*)calloc(kf2->n > 0 ? kf2->n : 1, 1);
    int f1 = 0, f2 = 0;
    while (f1 < kf1->n_nodes && f2 < kf2->n_nodes) {
        if (kf1->node_id[f1] == kf2->node_id[f2]) {
            for (int i1 = kf1->node_off[f1]; i1 < kf1->node_off[f1 + 1]; i1++) {
                const int idx1 = kf1->node_feat[i1];
                if (!has_mp(kf1, idx1)) continue;
                if (mp_bad(kf1, idx1)) continue;
                const uint8_t* d1 = kf1->desc + 32 * (size_t)idx1;
                int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
                for (int i2 = kf2->node_off[f2]; i2 < kf2->node_off[f2 + 1]; i2++) {
                    const int idx2 = kf2->node_feat[i2];
                    if (matched2[idx2] || !has_mp(kf2, idx2)) continue;
                    if (mp_bad(kf2, idx2)) continue;
                    int dist = oc_descriptor_distance(d1, kf2->desc + 32 * (size_t)idx2);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdx2 = idx2;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 < TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        match12[idx1] = bestIdx2;
                        matched2[bestIdx2] = 1;
                        if (checkOri)
                            ivec_push(&rotHist[rot_bin(kf1->angle[idx1], kf2->angle[bestIdx2])], idx1);
                        nmatches++;
                    }
                }
            }
            f1++;
            f2++;
        } else if (kf1->node_id[f1] < kf2->node_id[f2]) {
            f1 = lower_bound_u32(kf1->node_id, kf1->n_nodes, f1, kf2->node_id[f2]);
        } else {
            f2 = lower_bound_u32(kf2->node_id, kf2->n_nodes, f2, kf1->node_id[f1]);
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j = 0; j < rotHist[i].n; j++) {
                match12[rotHist[i].v[j]] = -1;
                nmatches--;
            }
        }
    }
    for (int i = 0; i < HISTO_LENGTH; i++) free(rotHist[i].v);
    free(matched2);
    return nmatches;
}
