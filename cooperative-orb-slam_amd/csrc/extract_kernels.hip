/*
 * extract_kernels.hip -- gfx950 kernels for ORBextractor::operator() (ORBextractor.cc:1043-1105).
 *
 * One launch per stage over a whole batch of frames (grid.y / grid.z = frame):
 *   k_pyramid_frames ComputePyramid, one workgroup per frame (or row band)  (ORBextractor.cc:1107-1132)
 *                    (k_resize_tiled / k_resize_level: per-level forms for geometries it does not fit)
 *   k_fast_cells2    per-cell cv::FAST + 3x3 NMS + threshold fallback (ORBextractor.cc:789-829)
 *   k_octree         DistributeOctTree, one workgroup per (frame,level) (ORBextractor.cc:539-763)
 *   k_describe_blur  GaussianBlur 7x7 sigma 2 REFLECT_101 of each keypoint's window + IC_Angle + rBRIEF +
 *                    output assembly, 16 lanes per keypoint (ORBextractor.cc:77-147, 851-852, 1075-1104)
 *   k_blur_strips +  the same as two stages (whole-level blur, then describe) for frames whose level-0 rows
 *   k_describe       are not 4-aligned
 * capi.cpp runs them in order on the caller's stream (the separate blur on a side stream beside FAST and the
 * octree; DESIGN.md "Schedule").
 * All of it is integer/byte work bounded by HBM/LDS and VALU issue; no MFMA.
 * Exact-semantics notes live in DESIGN.md "Pinned semantics".
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbslam_amd.h"
#include "orb_device.h"
#include "orb_wave.h"
#include "orb_math.h"
#include "orb_pattern.h"


namespace orbamd {

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_prefix(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0));
}

__device__ __forceinline__ int iclamp(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

typedef short short2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef unsigned int uint2v __attribute__((ext_vector_type(2)));
static inline int iclamp_host(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* n consecutive little-endian dwords starting at an arbitrary byte address, from n+1 aligned
 * dword loads + v_alignbyte (rows of the input frame need not be 4-byte aligned). Reads only
 * dwords that overlap the span, so it never touches memory past the span's last byte's dword. */
/* dword of bytes [c, c+4) of a row whose valid bytes are [0, w): two aligned dword loads,
 * addresses clamped into the row's valid dwords (always issued, never out of bounds); bytes
 * outside [0, w) come back as garbage and must be overwritten by the caller. */
__device__ __forceinline__ uint32_t load_row_u32_clamped(const uint8_t* row, int c, int w) {
    // offsets stay relative to `row` (pointer arithmetic keeps the global address space, so
    // these become global_load_dword, not flat loads)
    const int mr = (int)((uintptr_t)row & 3);
    const int lo = -mr, hi = ((mr + w - 1) & ~3) - mr;
    int o0 = ((mr + c) & ~3) - mr;
    o0 = o0 < lo ? lo : (o0 > hi ? hi : o0);
    const int o1 = o0 + 4 > hi ? hi : o0 + 4;
    const uint32_t w0 = *(const uint32_t*)(row + o0), w1 = *(const uint32_t*)(row + o1);
    return __builtin_amdgcn_alignbyte(w1, w0, (unsigned)((mr + c) & 3));
}

template <int N>
__device__ __forceinline__ void load_u32_unaligned(const uint8_t* p, uint32_t out[N]) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
    const unsigned sh = (unsigned)(a & 3);
    uint32_t w[N + 1];
#pragma unroll
    for (int i = 0; i < N; i++) w[i] = q[i];
    w[N] = sh ? q[N] : 0u;  // an aligned span never touches the dword after it
#pragma unroll
    for (int i = 0; i < N; i++) out[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}

/* ----------------------------------------------------------------------------------- */
/* Pyramid: cv::resize(INTER_LINEAR) 8U fixed point, one output pixel per lane.        */
/* xofs/alpha/yofs/beta are the host-built tables of resizeGeneric_.       */
/* ----------------------------------------------------------------------------------- */
__device__ __forceinline__ int resize_px(const uint8_t* S0, const uint8_t* S1, int x, int xmax, int simd_end,
                                         const int* __restrict__ xofs, const short2* __restrict__ alpha, short2 b) {
    const int sx = xofs[x];
    int h0, h1;
    if (x < xmax) {
        const short2 a = alpha[x];
        h0 = S0[sx] * a.x + S0[sx + 1] * a.y;
        h1 = S1[sx] * a.x + S1[sx + 1] * a.y;
    } else {
        h0 = S0[sx] * 2048;
        h1 = S1[sx] * 2048;
    }
    int v;
    if (x < simd_end)  // SSE2 VResizeLinearVec_32s8u: mulhi_epi16 on (h >> 4)
        v = (((__mul24(h0 >> 4, (int)b.x)) >> 16) + ((__mul24(h1 >> 4, (int)b.y)) >> 16) + 2) >> 2;
    else  // scalar FixedPtCast<int, uchar, 22>
        v = (__mul24(h0, (int)b.x) + __mul24(h1, (int)b.y) + (1 << 21)) >> 22;
    return iclamp(v, 0, 255);
}

/* 4 adjacent output pixels per lane, one dword store (rows are 64-B aligned). */
__global__ __launch_bounds__(256) void k_resize_level(
    const uint8_t* __restrict__ src, long long src_fstride, int src_pitch, int sw, int sh,
    uint8_t* __restrict__ dst, long long dst_fstride, int dst_pitch, int dw, int dh,
    const int* __restrict__ xofs, const short2* __restrict__ alpha, const int* __restrict__ yofs,
    const short2* __restrict__ beta, int xmax, int simd_end) {
    const int x0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x0 >= dw || y >= dh) return;
    const uint8_t* S = src + (long long)blockIdx.z * src_fstride;
    const int sy = yofs[y];
    const int r0 = iclamp(sy, 0, sh - 1), r1 = iclamp(sy + 1, 0, sh - 1);
    const uint8_t* S0 = S + (long long)r0 * src_pitch;
    const uint8_t* S1 = S + (long long)r1 * src_pitch;
    const short2 b = beta[y];
    uint8_t* D = dst + (long long)blockIdx.z * dst_fstride + (long long)y * dst_pitch;
    if (x0 + 4 <= dw) {
        uint32_t packed = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) packed |= (uint32_t)resize_px(S0, S1, x0 + i, xmax, simd_end, xofs, alpha, b) << (8 * i);
        *(uint32_t*)(D + x0) = packed;
    } else {
        for (int x = x0; x < dw; x++) D[x] = (uint8_t)resize_px(S0, S1, x, xmax, simd_end, xofs, alpha, b);
    }
}

/* Tiled form: a 64 x kRsTH output tile per workgroup; its source window (<= kRsW x kRsH
 * bytes, checked on the host by resize_tile_fits) is staged in LDS with aligned dword loads,
 * then each thread produces kRsTH/4 rows of one column from LDS. Every table load (window
 * bounds, xofs/alpha of the thread's column, yofs/beta of its rows) is issued before the
 * staging loads, so a tile costs two memory round trips (tables, source). */
constexpr int kRsTW = kRsTileW, kRsTH = kRsTileH, kRsW = 144, kRsH = 48, kRsRows = kRsTH / 4;

__device__ __forceinline__ void resize_tile(const uint8_t* __restrict__ S, int src_pitch, int sw, int sh,
                                            uint8_t* __restrict__ D, int dst_pitch, int dw, int dh,
                                            const int* __restrict__ xofs, const short2* __restrict__ alpha,
                                            const int* __restrict__ yofs, const short2* __restrict__ beta, int xmax,
                                            int simd_end, int bx, int by, uint8_t (*tile)[kRsW]) {
    const int c0 = bx * kRsTW, r0 = by * kRsTH;
    const int c1 = min(c0 + kRsTW, dw), r1 = min(r0 + kRsTH, dh);
    const int tid = threadIdx.x;
    // this thread's column and rows (indices clamped so every load is unconditional)
    const int c = c0 + (tid & 63);
    const int cc = min(c, dw - 1);
    const int yr0 = r0 + (tid >> 6) * kRsRows;
    const int sx = xofs[cc];
    const short2 al = alpha[cc];
    int syv[kRsRows];
    short2 bv[kRsRows];
#pragma unroll
    for (int k = 0; k < kRsRows; k++) {
        const int y = min(yr0 + k, dh - 1);
        syv[k] = yofs[y];
        bv[k] = beta[y];
    }
    // source window (uniform): columns [sx_lo, sx_hi], rows [yb, ye]
    const int sx_lo = xofs[c0];
    const int sx_hi = min(sw - 1, xofs[c1 - 1] + 1);
    const int yb = iclamp(yofs[r0], 0, sh - 1), ye = iclamp(yofs[r1 - 1] + 1, 0, sh - 1);
    const int nrows = ye - yb + 1;
    {
        constexpr int kPer = (kRsH * (kRsW / 4) + 255) / 256;
        uint32_t v[kPer];
        int slot[kPer];
        // unconditional loads (row and dword clamped into the source window), stores masked
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int i = tid + k * 256;
            const int r = i / (kRsW / 4), d = i - r * (kRsW / 4);
            const int rr = min(r, nrows - 1);
            const uint8_t* rp = S + (long long)(yb + rr) * src_pitch + sx_lo;
            const int mis = (int)((uintptr_t)rp & 3);
            const int span = mis + (sx_hi - sx_lo + 1);
            const int dmax = (span - 1) >> 2;
            v[k] = *(const uint32_t*)(rp - mis + 4 * (d < dmax ? d : dmax));
            slot[k] = (r < nrows && d <= dmax) ? r * kRsW + 4 * d : -1;
        }
#pragma unroll
        for (int k = 0; k < kPer; k++)
            if (slot[k] >= 0) *(uint32_t*)(&tile[0][0] + slot[k]) = v[k];
    }
    __syncthreads();
    if (c >= c1) return;  // (no barrier follows inside the tile)
    // LDS column of source x in row r: (x - sx_lo) + mis(r), mis = misalignment of that row's start
    const int a0 = c < xmax ? al.x : 2048, a1 = c < xmax ? al.y : 0;
    const int sxn = c < xmax ? sx + 1 : sx;
    const int mis0 = (int)((uintptr_t)(S + sx_lo) & 3);
#pragma unroll
    for (int k = 0; k < kRsRows; k++) {
        const int y = yr0 + k;
        if (y >= r1) break;
        const int sy = syv[k];
        const int q0 = iclamp(sy, 0, sh - 1) - yb, q1 = iclamp(sy + 1, 0, sh - 1) - yb;
        const int m0 = (mis0 + (yb + q0) * src_pitch) & 3;
        const int m1 = (mis0 + (yb + q1) * src_pitch) & 3;
        const int h0 = tile[q0][sx - sx_lo + m0] * a0 + tile[q0][sxn - sx_lo + m0] * a1;
        const int h1 = tile[q1][sx - sx_lo + m1] * a0 + tile[q1][sxn - sx_lo + m1] * a1;
        const short2 b = bv[k];
        int v;
        if (c < simd_end)
            v = (((__mul24(h0 >> 4, (int)b.x)) >> 16) + ((__mul24(h1 >> 4, (int)b.y)) >> 16) + 2) >> 2;
        else
            v = (__mul24(h0, (int)b.x) + __mul24(h1, (int)b.y) + (1 << 21)) >> 22;
        D[(long long)y * dst_pitch + c] = (uint8_t)iclamp(v, 0, 255);
    }
}


__global__ __launch_bounds__(256) void k_resize_tiled(
    const uint8_t* __restrict__ src, long long src_fstride, int src_pitch, int sw, int sh,
    uint8_t* __restrict__ dst, long long dst_fstride, int dst_pitch, int dw, int dh,
    const int* __restrict__ xofs, const short2* __restrict__ alpha, const int* __restrict__ yofs,
    const short2* __restrict__ beta, int xmax, int simd_end) {
    __shared__ __align__(16) uint8_t tile[kRsH][kRsW];
    resize_tile(src + (long long)blockIdx.z * src_fstride, src_pitch, sw, sh, dst + (long long)blockIdx.z * dst_fstride,
                dst_pitch, dw, dh, xofs, alpha, yofs, beta, xmax, simd_end, blockIdx.x, blockIdx.y, tile);
}

/* ----------------------------------------------------------------------------------- */
/* GaussianBlur 7x7, sigma 2, REFLECT_101, 8U fixed point (kernel 18,34,49,55,...; sum  */
/* 257). Row strips of all levels of all frames in one grid.                            */
/* ----------------------------------------------------------------------------------- */
__device__ __forceinline__ int reflect101(int p, int n) {
    p = p < 0 ? -p : p;
    p = p >= n ? 2 * n - 2 - p : p;
    return p;
}

constexpr int kBlurSeg = 264; // bytes of one staged row segment: strip (256) + 4 left + 4 right

/* One wave per (frame, level, 256-column strip, 64-row chunk); each lane owns 4 adjacent output
 * columns x0 = sx + 4*lane.
 *  - Source row segment [sx-4, sx+260) is fetched once per wave with coalesced dword loads
 *    (addresses clamped into the row), staged in LDS, and the REFLECT_101 halo bytes are
 *    patched there by three lanes. Rows are prefetched 7 rows ahead into a register ring.
 *  - Horizontal: the lane's 12 bytes are three LDS dwords; output i's taps are two byte
 *    windows (alignbyte) dotted with the packed kernel by v_dot4_u32_u8.
 *  - Vertical: the 7 row sums of the window live in registers as float pairs; the loop is
 *    unrolled by 7 so the window rotates by renaming. All values are integers < 2^24 and the
 *    weights are k/2^16, so every packed fma is exact: sf = s / 2^16 exactly.
 *  - Rounding: OpenCV's SSE2 column path (x < w&~3) rounds s/2^16 half to even = rint(sf),
 *    v_cvt_pk_u8_f32 (round-to-nearest-even, saturating); the scalar tail rounds half up,
 *    floor(sf + 0.5) (DESIGN.md "Pinned semantics"; checked by tools/check_cvtpk.hip). */
__device__ __forceinline__ float2v blur_vsum(const float2v r0, const float2v r1, const float2v r2, const float2v r3,
                                            const float2v r4, const float2v r5, const float2v r6) {
    // symmetric taps paired first (sums of two row sums < 2^17, exact), so the dependent chain is 4 packed ops deep
    // instead of 7; every partial sum is an exact multiple of 2^-16 below 256 whenever the result is (products of a
    // < 2^17 integer and k / 2^16 are exact), so the order does not change the value; a result >= 256 saturates to
    // 255 whichever way it rounds
    const float k18 = 18.f / 65536.f, k34 = 34.f / 65536.f, k49 = 49.f / 65536.f, k55 = 55.f / 65536.f;
    const float2v s06 = r0 + r6, s15 = r1 + r5, s24 = r2 + r4;
    float2v v = r3 * (float2v){k55, k55};
    v = __builtin_elementwise_fma(s24, (float2v){k49, k49}, v);
    v = __builtin_elementwise_fma(s15, (float2v){k34, k34}, v);
    v = __builtin_elementwise_fma(s06, (float2v){k18, k18}, v);
    return v;
}

/* one blur job: rows [chunk*kRows, +kRows) x columns [strip*256, +256) of a level (img / pitch,
 * output out with the level's pitch), by one wave; rows = that wave's 7 x kBlurSeg LDS staging slots */
template <bool kAligned, int kRows>
__device__ __forceinline__ void blur_job(const uint8_t* __restrict__ img, int pitch, const LevelDesc& lv,
                                         uint8_t* __restrict__ out, int strip, int chunk, uint8_t (*rows)[kBlurSeg],
                                         int lane) {
    const int w = lv.w, h = lv.h;
    const int sx = strip * 256;
    const int x0 = sx + lane * 4;
    const int ya = chunk * kRows, yb = min(h, ya + kRows);
    const bool lane_on = x0 < w;
    const bool tail = x0 + 3 >= lv.blur_vec_end;  // some of this lane's columns take the scalar path
    const int seg0 = sx - 4;                      // segment byte 0 = column seg0
    const int need_hi = min(sx + 256, w) + 3;     // columns [sx-3, need_hi) are read
    // kAligned: every row of every level starts 4-aligned (pyramid levels always do; the
    // caller's frames are checked at launch), so segment dwords are plain clamped loads
    const int lastd = (w - 1) & ~3;
    const int dA = iclamp(seg0 + 4 * lane, 0, lastd);
    const int dB = lane < 2 ? iclamp(seg0 + 4 * (lane + 64), 0, lastd) : dA;
    // dwords `lane` and `lane+64` (lanes 0..1) of source row yy's segment
    auto fetch = [&](int yy, uint32_t& v0, uint32_t& v1) {
        const uint8_t* row = img + (long long)reflect101(yy, h) * pitch;
        if (kAligned) {
            v0 = *(const uint32_t*)(row + dA);
            v1 = *(const uint32_t*)(row + dB);
        } else {
            v0 = load_row_u32_clamped(row, seg0 + 4 * lane, w);
            v1 = load_row_u32_clamped(row, seg0 + 4 * (lane + 64), w);
        }
    };
    // stage one row into LDS slot k, patch its halo, return the lane's 4 row sums (as floats)
    auto rowsum = [&](int k, uint32_t v0, uint32_t v1, float2v& lo, float2v& hi) {
        ((uint32_t*)rows[k])[lane] = v0;
        if (lane < 2) ((uint32_t*)rows[k])[lane + 64] = v1;
        wave_sync();
        // REFLECT_101 halo over the garbage bytes: column -1-q <- 1+q, column w+q <- w-2-q
        if (lane < 3) {
            const int q = lane;
            if (sx == 0) rows[k][(-1 - q) - seg0] = rows[k][(1 + q) - seg0];
            const int xr = w + q;
            if (xr >= sx && xr < need_hi) rows[k][xr - seg0] = rows[k][(w - 2 - q) - seg0];
        }
        wave_sync();
        const uint32_t* d = (const uint32_t*)rows[k] + lane;
        const uint32_t w0 = d[0], w1 = d[1], w2 = d[2];  // columns x0-4 .. x0+7
        const uint32_t K1 = 18u | 34u << 8 | 49u << 16 | 55u << 24, K2 = 49u | 34u << 8 | 18u << 16;
        const uint32_t r0 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 1), K1,
                                                   __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 1), K2, 0u, false), false);
        const uint32_t r1 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 2), K1,
                                                   __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 2), K2, 0u, false), false);
        const uint32_t r2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 3), K1,
                                                   __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 3), K2, 0u, false), false);
        const uint32_t r3 = __builtin_amdgcn_udot4(w1, K1, __builtin_amdgcn_udot4(w2, K2, 0u, false), false);
        lo = (float2v){(float)r0, (float)r1};
        hi = (float2v){(float)r2, (float)r3};
    };
    auto emit = [&](int yo, float2v a, float2v b) {
        if (!lane_on || yo >= yb) return;
        float o[4] = {a.x, a.y, b.x, b.y};
        if (tail) {
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (x0 + i >= lv.blur_vec_end) o[i] = floorf(o[i] + 0.5f);
        }
        uint32_t packed = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) packed = __builtin_amdgcn_cvt_pk_u8_f32(o[i], (unsigned)i, packed);
        uint8_t* p = out + (long long)yo * lv.pitch + x0;
        if (x0 + 4 <= w) {
            *(uint32_t*)p = packed;
        } else {
            for (int i = 0; i < 4 && x0 + i < w; i++) p[i] = (uint8_t)(packed >> (8 * i));
        }
    };
    // window: rows y-3 .. y+3 of output row y live in slots (y - ya) .. (y - ya + 6) mod 7
    float2v WL[7], WH[7];
    uint32_t D0[7], D1[7];  // prefetched source rows: row ya+3+m in D[m mod 7]
#pragma unroll
    for (int m = 0; m < 6; m++) fetch(ya - 3 + m, D0[m], D1[m]);
#pragma unroll
    for (int m = 0; m < 6; m++) rowsum(m, D0[m], D1[m], WL[m], WH[m]);
#pragma unroll
    for (int m = 0; m < 7; m++) fetch(ya + 3 + m, D0[m], D1[m]);
    // straight-line body: every step fetches (rows past the chunk are reflected, valid rows)
    // and computes; only the stores are masked, so the prefetch waits stay counted (vmcnt(N))
    for (int yi = ya; yi < yb; yi += 7) {
#pragma unroll
        for (int s = 0; s < 7; s++) {
            const int y = yi + s;
            const int ns = (s + 6) % 7;  // slot of the new row y+3
            rowsum(ns, D0[s], D1[s], WL[ns], WH[ns]);
            fetch(y + 10, D0[s], D1[s]);
            const float2v a = blur_vsum(WL[s], WL[(s + 1) % 7], WL[(s + 2) % 7], WL[(s + 3) % 7], WL[(s + 4) % 7],
                                       WL[(s + 5) % 7], WL[ns]);
            const float2v b = blur_vsum(WH[s], WH[(s + 1) % 7], WH[(s + 2) % 7], WH[(s + 3) % 7], WH[(s + 4) % 7],
                                       WH[(s + 5) % 7], WH[ns]);
            emit(y, a, b);
        }
    }
}

/* Whole-pyramid form: one 512-thread workgroup per frame builds levels 1..L-1 in order
 * (level l+1 is read back from L2 right after this CU wrote level l; a workgroup barrier
 * separates the levels). A batch of >= 256 frames fills every CU with equal work, and the
 * seven dependent per-level launches (each too small to hide its own latency) become one.
 *
 * Per level each thread owns one 4-column output group (column table in registers) and walks
 * rows. For a group the host precomputed (PyrColGroup): the 8-byte source window start W
 * (relative to the row; all 4 outputs' taps lie in [W, W+8)), per output a v_perm selector
 * that extracts the tap pair as two u16 lanes, and the tap weights as a short2 (alpha, with
 * (2048, 0) past xmax). Horizontal = one v_dot2 per output and source row; vertical = the
 * SSE2 VResizeLinearVec_32s8u formula, scalar FixedPtCast for x >= simd_end (as k_resize_*).
 * Rows' (r0, r1, beta) come from an LDS copy of the level's row table. */
struct PyrColGroup {
    int sel[4];
    int alpha[4];  // short2 bit patterns
    int W;
    int pad[3];
};
static_assert(sizeof(PyrColGroup) == 48, "PyrColGroup layout");

template <int U, int NT>
__global__ __launch_bounds__(NT) void k_pyramid_frames(const uint8_t* __restrict__ frames, long long fstride,
                                                         int pitch0, uint8_t* __restrict__ pyr, ExtractParams ep,
                                                         const LevelDesc* __restrict__ levels,
                                                         const int* __restrict__ ptab,
                                                         const int2* __restrict__ bands) {
    // the current level's row table; sized at launch for the tallest level >= 1 (rows x 16 B: 6.4 KB at
    // 640x480) instead of kPyrMaxRows, so the LDS the long-lived pyramid workgroup holds stays free for the
    // other graphs' FAST / describe workgroups beside it
    extern __shared__ int4 s_rt[];
    // whole frames: block = frame; row bands (small batches): block (band, frame), rows [x, y) of each level
    // from the host's cone table (every row a band's next level reads was made by this workgroup, so the
    // read-back after the level barrier is of its own writes)
    const int f = bands ? blockIdx.y : blockIdx.x, band = bands ? blockIdx.x : 0, tid = threadIdx.x;
    uint8_t* P = pyr + (long long)f * ep.pyr_frame_bytes;
    for (int l = 1; l < ep.L; l++) {
        const LevelDesc sv = levels[l - 1];
        const LevelDesc lv = levels[l];
        const uint8_t* src = l == 1 ? frames + (long long)f * fstride : P + sv.pyr_off;
        const int sp = l == 1 ? pitch0 : sv.pitch;
        uint8_t* dst = P + lv.pyr_off;
        int lo = 0, hi = lv.h;
        if (bands) {
            const int2 r = bands[band * kMaxLevels + l];
            lo = r.x;
            hi = r.y;
        }
        const int4* rt = (const int4*)(ptab + lv.rt_off) + lo;
        for (int i = tid; i < hi - lo; i += NT) s_rt[i] = rt[i];
        const int gw = (lv.w + 3) >> 2;
        const int R = NT / gw;  // rows per pass
        const int ry = tid / gw, xg = tid - ry * gw;
        const PyrColGroup cg = ((const PyrColGroup*)(ptab + lv.cg_off))[min(xg, gw - 1)];
        const int A = cg.W & ~3, k = cg.W & 3;
        const int edge4 = A + 8 > cg.pad[0] ? 4 : 0;  // pad[0]: the row's last dword (host: align4(sw) - 4)
        const int x0 = 4 * xg;
        const bool tail = x0 + 3 >= lv.simd_end;
        __syncthreads();
        // one pass = U output rows of this thread's column group: the 2 x 3 source dwords of each (rows clamped,
        // so every load is valid and unconditional), then the taps
        if (ry < R) {
            for (int y0 = lo + ry; y0 < hi; y0 += U * R) {
                uint32_t w[U][2][3];
                int4 rr[U];
#pragma unroll
                for (int u = 0; u < U; u++) rr[u] = s_rt[min(y0 + u * R, hi - 1) - lo];
#pragma unroll
                for (int u = 0; u < U; u++) {
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const int r = q ? rr[u].y : rr[u].x;
                        // (a 24-bit multiply here frees 11 VGPRs, and the 6th wave per SIMD it allows costs the step
                        // 0.9 %: profiles/r06l_ab_pyramid_mul24.log)
                        const unsigned rs = (unsigned)(r * sp);
                        // the window's 3 dwords by one 12-byte load; the row's last group (whose third dword would
                        // start past the row's last dword) loads 4 bytes earlier and takes the clamped dword twice.
                        // The dwordx2 + dword pair requested the window's lines twice: pyramid alone 0.181 -> 0.168
                        // ms per 256 frames, 80 instead of 85 VGPRs, the step +0.8 % (profiles/r06zc_ab_pyr_x3.log)
                        typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));
                        const u32x3a4 L3 = *(const u32x3a4*)(src + (rs + (unsigned)(A - edge4)));
                        w[u][q][0] = edge4 ? L3.y : L3.x;
                        w[u][q][1] = edge4 ? L3.z : L3.y;
                        w[u][q][2] = L3.z;
                    }
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int y = y0 + u * R;
                    if (y >= hi) break;
                    const short2 b = __builtin_bit_cast(short2, rr[u].z);
                    int h[2][4];
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const uint32_t lw = __builtin_amdgcn_alignbyte(w[u][q][1], w[u][q][0], k);
                        const uint32_t hw = __builtin_amdgcn_alignbyte(w[u][q][2], w[u][q][1], k);
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const uint32_t pr = __builtin_amdgcn_perm(hw, lw, cg.sel[i]);
                            // VOP3P v_dot2_i32_i16 with an inline-zero accumulator (the builtin becomes a v_mov + v_dot2c)
                            asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(h[q][i]) : "v"(pr), "v"(cg.alpha[i]));
                        }
                    }
                    uint32_t packed = 0;
                    // (b * (h >> 4)) >> 16 as the high word of a 24 x 24-bit product: (h & ~15) * (b << 12) >> 32, one
                    // full-rate v_mul_hi_u32_u24 and an and for the shift-multiply-shift (h < 2^20, b <= 2049 < 2^12).
                    // No clamp: the weights of a row (a0 + a1) and of a column pair (b0 + b1) are >= 0 and sum to at
                    // most 2049, so every result lies in [0, 255] (the SSE2 path's saturation never engages)
                    const uint64_t B0 = (uint64_t)(((uint32_t)b.x & 0xFFFu) << 12), B1 = (uint64_t)(((uint32_t)b.y & 0xFFFu) << 12);
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const uint64_t t0 = (uint64_t)((uint32_t)h[0][i] & 0xFFFF0u) * B0;
                        const uint64_t t1 = (uint64_t)((uint32_t)h[1][i] & 0xFFFF0u) * B1;
                        uint32_t v = ((uint32_t)(t0 >> 32) + (uint32_t)(t1 >> 32) + 2u) >> 2;
                        if (tail && x0 + i >= lv.simd_end)
                            v = (uint32_t)(__mul24(h[0][i], (int)b.x) + __mul24(h[1][i], (int)b.y) + (1 << 21)) >> 22;
                        packed |= v << (8 * i);
                    }
                    if (xg < gw) *(uint32_t*)(dst + (unsigned)(y * lv.pitch + x0)) = packed;
                }
            }
        }
        __syncthreads();
    }
}

/* ----------------------------------------------------------------------------------- */
/* FAST-9/16 "strength": S = max over the 16 cyclic 9-arcs of min(v-ring) or min(ring-v). */
/* A pixel is a cv::FAST corner at threshold t iff S > t, and then cornerScore<16> = S-1  */
/* (threshold-independent), so one S map serves both thresholds of the cell fallback.    */
/* ----------------------------------------------------------------------------------- */
/* FAST strength S as packed f16 (integers in [-255, 255] are exact in f16, and min/max are exact):
 * X_k = (v - r_k, r_k - v) from the byte r_k as f16(1024 + r_k) = bits 0x6400 | r_k (one v_perm) and one
 * v_pk_fma_f16; every 9-arc minimum is min3(min3 of 3 consecutive) and the arc maximum a max3 tree, on
 * gfx950's v_pk_minimum3_f16 / v_pk_maximum3_f16: about half the min/max instructions of a packed-i16 form. */
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int fast_strength_h2(const uint8_t* roi, int o, int P) {
    int ow = o - 3 * P - 3;  // 7x7 window origin: every ring offset is a non-negative immediate
    asm volatile("" : "+v"(ow));
    const uint8_t* w = roi + ow;
    const int v = w[3 * P + 3];
    const uint32_t vb = __builtin_amdgcn_perm(0x64646464u, (uint32_t)v, 0x04000400u);  // (1024+v, 1024+v)
    const half2v vp = __builtin_bit_cast(half2v, vb ^ 0x80000000u);                  // (1024+v, -(1024+v))
    const half2v sg = {(_Float16)-1.0f, (_Float16)1.0f};
    const int off[16] = {6 * P + 3, 6 * P + 4, 5 * P + 5, 4 * P + 6, 3 * P + 6, 2 * P + 6, P + 5, 4,
                         3, 2, P + 1, 2 * P, 3 * P, 4 * P, 5 * P + 1, 6 * P + 2};
    half2v x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t rb = __builtin_amdgcn_perm(0x64646464u, (uint32_t)w[off[k]], 0x04000400u);
        x[k] = __builtin_elementwise_fma(__builtin_bit_cast(half2v, rb), sg, vp);
    }
    half2v m3[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        m3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(x[k], x[(k + 1) & 15]), x[(k + 2) & 15]);
    half2v m9[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        m9[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]);
    half2v a = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m9[0], m9[1]), m9[2]);
#pragma unroll
    for (int k = 3; k < 15; k += 2) a = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, m9[k]), m9[k + 1]);
    a = __builtin_elementwise_maximum(a, m9[15]);
    const int S = max((int)(float)a.x, (int)(float)a.y);
    return S < 0 ? 0 : S;
}

/* NMS survivor test of cv::FAST (FAST_t, nonmax_suppression) at threshold t, on the
 * cell's S buffer (zero outside the detection band [3, rows-3) x [3, cols-3)).
 * cv::FAST keeps a corner (S > t, score S-1) iff its score is strictly greater than the score of
 * every neighbouring corner. A neighbour with S_n >= S_c > t is a corner, and one with
 * S_n < S_c never suppresses, so the test is S_c > t && S_c > 1 && max8(S_n) < S_c. */
/* (the centre's S c is passed in: the caller holds it in a register or has read s[0]) */
__device__ __forceinline__ bool fast_survivor_c(const uint8_t* s, int P, int t, int c) {
    const int n0 = s[-P - 1], n1 = s[-P], n2 = s[-P + 1], n3 = s[-1], n4 = s[1], n5 = s[P - 1], n6 = s[P],
              n7 = s[P + 1];
    const int mx = max(max(max(n0, n1), max(n2, n3)), max(max(n4, n5), max(n6, n7)));
    return c > t && c > 1 && mx < c;
}

/* LDS bytes per wave of k_fast_cells2: ROI + S map (RP x RH each) + candidate list (u16 per
 * band pixel; a band is at most (RP-6) x (RH-6)) + 64 per-lane dummy slots of the compaction */
#ifndef ORBX_FAST_WAVES
#define ORBX_FAST_WAVES 4
#endif
constexpr int kFastWaves = ORBX_FAST_WAVES;  // cells (one per wave) per k_fast_cells2 workgroup
__host__ __device__ inline int fast_wave_lds(int RP, int RH) {
    return 2 * RP * RH + ((2 * ((RP - 6) * (RH - 6) + 64) + 15) & ~15);
}

template <int kMaxPass, int kRP>
__device__ __forceinline__ void fast_cells_body(
    const uint8_t* __restrict__ frames, long long fstride, int pitch0, const uint8_t* __restrict__ pyr,
    const ExtractParams& ep, const LevelDesc* __restrict__ levels, const CellDesc* __restrict__ cells,
    uint32_t* __restrict__ cellkey, int* __restrict__ cellcnt, int RP_, int RH, int cell_lo, int cell_hi, int bx,
    int f, uint8_t* lds, int wpb) {
    // compile-time ROI pitch for the common geometries: every LDS offset of the ring/NMS reads becomes an
    // instruction immediate
    const int RP = kRP ? kRP : RP_;
    // wave index through readfirstlane: the cell descriptor, loop bounds and addressing are wave-uniform
    // (scalar loads / SALU) instead of per-lane VALU
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int ci = cell_lo + bx * wpb + wave;  // wpb: cells (waves) per workgroup
    if (ci >= cell_hi) return;  // wave-uniform; no block barriers in this kernel
    const int roi_bytes = RP * RH;
    uint8_t* roi = lds + wave * fast_wave_lds(RP, RH);
    uint8_t* str = roi + roi_bytes;
    uint16_t* clist = (uint16_t*)(str + roi_bytes);  // <= (RP-6)(RH-6) entries (band pixels)
    const CellDesc c = cells[ci];
    const LevelDesc lv = levels[c.level];
    const uint8_t* img = c.level == 0 ? frames + (long long)f * fstride
                                      : pyr + (long long)f * ep.pyr_frame_bytes + lv.pyr_off;
    const int pitch = c.level == 0 ? pitch0 : lv.pitch;
    {
        // D dwords per ROI row, 64/D rows per pass; all passes' loads issued before the LDS writes
        const int D = c.D;
        const int rpp = c.rpp;
        // 24-bit index products (full-rate v_mul_u32_u24 / v_mad_u32_u24; v_mul_lo_u32 is quarter rate)
        const int lr = __mul24(lane, c.magD) >> 16, ld = lane - __mul24(lr, D);
        const bool on = lane < rpp * D;
        uint32_t v[kMaxPass];  // kMaxPass >= ceil(h / rpp) for every cell (host-chosen)
        const int ldc = on ? ld : 0;
        const bool rows_aligned = (((uintptr_t)img | (uintptr_t)pitch) & 3) == 0;  // wave-uniform
        if (rows_aligned) {
            // every row starts 4-aligned: one column schedule for all rows (two clamped dwords + alignbyte)
            const int k = c.x0 & 3;
            const int lastd = (lv.w - 1) & ~3;
            const int o0 = min((c.x0 & ~3) + 4 * ldc, lastd), o1 = min(o0 + 4, lastd);
            const uint8_t* base = img + (long long)c.y0 * pitch;
#pragma unroll
            for (int kk = 0; kk < kMaxPass; kk++) {
                const unsigned ro = (unsigned)__mul24(min(kk * rpp + lr, c.h - 1), pitch);
                // both dwords by one 8-byte load (an active lane's o0 + 4 is always inside the row: cells end 13
                // columns before the level's edge, so the clamp to lastd never binds for them). Two dword loads
                // request every line of the ROI twice, and the staging is bound by those requests: 398.0k -> 403.2k
                // frames/s, FAST alone 0.220 -> 0.215 ms per 256 frames (profiles/r06zb_ab_fast_x2.log; staging alone with
                // half the requests 0.46 -> 0.31 ms per 1024 frames, r06z_fast_half_loads.txt)
                typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
                const u32x2a4 w = *(const u32x2a4*)(base + (ro + o0));
                v[kk] = __builtin_amdgcn_alignbyte(w.y, w.x, k);
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < kMaxPass; kk++) {
                const int r = min(kk * rpp + lr, c.h - 1);  // clamped: loads always valid, issued back to back
                v[kk] = load_row_u32_clamped(img + (long long)(c.y0 + r) * pitch, c.x0 + 4 * ldc, lv.w);
            }
        }
#pragma unroll
        for (int kk = 0; kk < kMaxPass; kk++) {
            const int r = kk * rpp + lr;
            if (on && r < c.h) {
                ((uint32_t*)(roi + __mul24(r, RP)))[ld] = v[kk];
                ((uint32_t*)(str + __mul24(r, RP)))[ld] = 0u;
            }
        }
    }
    wave_sync();
    const int bw = c.w - 6, bh = c.h - 6;
    int total = 0;
    if (bw > 0 && bh > 0) {
        // One pass per threshold: iniThFAST first; only a cell with no corner there is scanned again at
        // minThFAST (ORBextractor.cc:811-826). Each pass pretests, computes S and stores it in the S map
        // only at its own threshold t: the NMS at t is exact with the S of the pretest(t) candidates alone
        // (a neighbour can suppress a corner with S_c > t only if S_n >= S_c > t, and then it passed the
        // pretest at t), so the common first pass computes S for the ~9% of band pixels passing the
        // pretest at 20 instead of the ~15% passing it at 7. The fallback pass sees a superset of the
        // first pass's candidates and stores the same S for them (S does not depend on t).
        const int G = c.G;  // dword groups covering columns [0, bw+3): (bw + 6) / 4
        const int rpc = c.rpc;
        const int lr = __mul24(lane, c.magG) >> 16, j = lane - __mul24(lr, G);
        const bool lane_ok = lane < rpc * G;
        // band-column mask at the candidate bits: pixel i of this lane's dword -> bit 8 i + 7
        auto colok = [&](int i) { return 4 * j + i >= 3 && 4 * j + i < 3 + bw; };
        const uint32_t colm = (colok(0) ? 0x80u : 0u) | (colok(1) ? 0x8000u : 0u) | (colok(2) ? 0x800000u : 0u) |
                              (colok(3) ? 0x80000000u : 0u);
        uint32_t* out = cellkey + (long long)f * ep.keys_per_frame + c.slot;
        for (int t = ep.ini_th;; t = ep.min_th) {
            int ncand = 0;
            {
                // SWAR pretest: each lane tests the 4 pixels of one aligned ROI dword (band columns
                // [3, 3+bw)) as 4 bytes with v_lerp_u8 (per byte (a + b + r) >> 1, exact in 9 bits):
                // m = lerp(c, 255 - v, r) = floor((c - v + 255 + r) / 2), and m >= M <=> bit 7 of lerp(m, 255 - M, 1).
                // With r of the right parity, c - v > t <=> m_b >= (t + 256 + r_b) / 2 (r_b = t & 1) and
                // c - v < -t <=> NOT m_d >= (255 - t + r_d) / 2 (r_d = 1 - r_b); for t = 255 the bright bound is
                // clamped to 255 (looser: the pretest stays a necessary condition). Exhaustive check over
                // (c, v, t): tests/test_oracle_primitives.py::test_fast_pretest_lerp_exact.
                uint32_t* rec = (uint32_t*)str;  // <= bh x G records, zeroed again by the expansion
                int nrec = 0;
                const uint32_t RB = (t & 1) ? 0x01010101u : 0u, RD = RB ^ 0x01010101u;
                const uint32_t CB = (uint32_t)(255 - min((t + 256 + (t & 1)) >> 1, 255)) * 0x01010101u;
                const uint32_t CD = (uint32_t)(255 - ((256 - t - (t & 1)) >> 1)) * 0x01010101u;
                // candidate bits of the row pass starting at band row r0 (bit 8 i + 7: pixel i of this lane's dword)
                auto pretest = [&](int r0) -> uint32_t {
                    const int rr = 3 + r0 + lr;
                    const int rrc = min(rr, bh + 2);
                    const uint8_t* q = roi + __mul24(rrc, RP) + 4 * j;
                    const uint32_t xv = *(const uint32_t*)q;
                    const uint32_t xn = *(const uint32_t*)(q + 4);
                    const uint32_t xp = *(const uint32_t*)(q - 4);
                    const uint32_t xd = *(const uint32_t*)(q + 3 * RP);  // ring 0 (row + 3)
                    const uint32_t xu = *(const uint32_t*)(q - 3 * RP);  // ring 8 (row - 3)
                    const uint32_t xr = __builtin_amdgcn_alignbyte(xn, xv, 3);  // ring 4 (col + 3)
                    const uint32_t xl = __builtin_amdgcn_alignbyte(xv, xp, 1);  // ring 12 (col - 3)
                    const uint32_t nv = ~xv;  // 255 - v per byte
                    auto bright = [&](uint32_t cb) {
                        return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(cb, nv, RB), CB, 0x01010101u);
                    };
                    auto notdark = [&](uint32_t cb) {
                        return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(cb, nv, RD), CD, 0x01010101u);
                    };
                    const uint32_t b0 = bright(xd), b4 = bright(xr), b8 = bright(xu), b12 = bright(xl);
                    const uint32_t n0 = notdark(xd), n4 = notdark(xr), n8 = notdark(xu), n12 = notdark(xl);
                    // candidate iff two cyclically adjacent cardinals are both brighter ((b0|b8)&(b4|b12)) or
                    // both darker (NOT((n0&n8)|(n4&n12)))
                    const uint32_t cand = ((b0 | b8) & (b4 | b12)) | ~((n0 & n8) | (n4 & n12));
                    // mask, not a branch: the loads of both row passes stay unconditional and in flight together
                    const uint32_t live = 0u - (uint32_t)(lane_ok && rr < 3 + bh);
                    return cand & colm & live;
                };
                // sparse ordered record of this dword (lanes with a candidate, ~1 in 5): row-major = lane order
                // within a row pass; record = candidate bits | group j | ROI row << 8 (j, rr < 128 fit the 7 free
                // bits of bytes 0 / 1)
                auto record = [&](uint32_t k, int r0) {
                    const unsigned long long Bk = __ballot(k != 0u);
                    if (k != 0u) {
                        const int at = nrec + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(Bk >> 32),
                                                                              __builtin_amdgcn_mbcnt_lo((unsigned)Bk, 0));
                        rec[at] = k | (uint32_t)j | ((uint32_t)(3 + r0 + lr) << 8);
                    }
                    nrec += __popcll(Bk);
                };
                for (int r0 = 0; r0 < bh; r0 += rpc) record(pretest(r0), r0);
                wave_sync();
                // expand the records into the candidate list (order kept: records in order, pixels of a
                // record ascending); the record area is zeroed behind, so str is the S map again (zero
                // except S values of an earlier pass, which this pass rewrites unchanged)
                for (int c0 = 0; c0 < nrec; c0 += 64) {
                    const int i = c0 + lane;
                    uint32_t r = 0u;
                    if (i < nrec) {
                        r = rec[i];
                        rec[i] = 0u;
                    }
                    const uint32_t km = r & 0x80808080u;
                    const int cntl = __popc(km);
                    int pos = ncand;
#pragma unroll
                    for (int bit = 0; bit < 3; bit++) {  // cntl <= 4
                        const unsigned long long B = __ballot((cntl >> bit) & 1);
                        pos += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(B >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)B, 0))
                               << bit;
                        ncand += __popcll(B) << bit;
                    }
                    const int e = (int)(((r >> 8) & 127u) << 8) | (int)(4u * (r & 127u));
                    if (km & 0x80u) clist[pos++] = (uint16_t)e;
                    if (km & 0x8000u) clist[pos++] = (uint16_t)(e + 1);
                    if (km & 0x800000u) clist[pos++] = (uint16_t)(e + 2);
                    if (km & 0x80000000u) clist[pos++] = (uint16_t)(e + 3);
                }
            }
            wave_sync();
            // the first 64 candidates (all of them in most cells) keep their list entry and strength in
            // registers for the NMS pass: one dependent LDS read fewer
            const int e0 = lane < ncand ? (int)clist[lane] : 0;
            int s0 = 0;
            for (int i0 = 0; i0 < ncand; i0 += 64) {
                const int i = i0 + lane;
                if (i < ncand) {
                    const int e = i0 == 0 ? e0 : (int)clist[i];
                    const int o = __mul24(e >> 8, RP) + (e & 0xFF);
                    const int S = fast_strength_h2(roi, o, RP);
                    if (S > t) str[o] = (uint8_t)S;
                    if (i0 == 0) s0 = S > t ? S : 0;
                }
            }
            wave_sync();
            // NMS + row-major emission at t
            for (int i0 = 0; i0 < ncand; i0 += 64) {
                const int i = i0 + lane;
                bool keep = false;
                int e = 0;
                int cS = 0;
                if (i < ncand) {
                    const uint8_t* sp;
                    if (i0 == 0) {
                        e = e0;
                        sp = str + __mul24(e >> 8, RP) + (e & 0xFF);
                        cS = s0;
                    } else {
                        e = clist[i];
                        sp = str + __mul24(e >> 8, RP) + (e & 0xFF);
                        cS = sp[0];
                    }
                    keep = fast_survivor_c(sp, RP, t, cS);
                }
                const unsigned long long m = __ballot(keep);
                if (keep) {
                    const int pos = total + lane_prefix(m);
                    const int sc = cS - 1;
                    const uint32_t xr = (uint32_t)((e & 0xFF) + c.xoff), yr = (uint32_t)((e >> 8) + c.yoff);
                    if (pos < c.cap) out[pos] = xr | (yr << 12) | ((uint32_t)sc << 24);
                }
                total += __popcll(m);
            }
            if (total != 0 || t == ep.min_th) break;  // wave-uniform
            wave_sync();  // the fallback pass rewrites the record area / candidate list
        }
        if (total > c.cap) total = c.cap;
    }
    if (lane == 0) cellcnt[(long long)f * ep.ncells + ci] = total;
}

template <int kMaxPass, int kRP>
__global__ __launch_bounds__(64 * kFastWaves) void k_fast_cells2(
    const uint8_t* __restrict__ frames, long long fstride, int pitch0, const uint8_t* __restrict__ pyr,
    ExtractParams ep, const LevelDesc* __restrict__ levels, const CellDesc* __restrict__ cells,
    uint32_t* __restrict__ cellkey, int* __restrict__ cellcnt, int RP_, int RH, int cell_lo, int cell_hi) {
    extern __shared__ __align__(16) uint8_t lds[];
    fast_cells_body<kMaxPass, kRP>(frames, fstride, pitch0, pyr, ep, levels, cells, cellkey, cellcnt, RP_, RH, cell_lo,
                                   cell_hi, blockIdx.x, blockIdx.y, lds, kFastWaves);
}

/* ----------------------------------------------------------------------------------- */
/* DistributeOctTree, one 256-thread workgroup per (frame, level).                       */
/*                                                                                       */
/* Re-formulation (proved equivalent in DESIGN.md): keys never move; each key carries   */
/* the index of its live node. The std::list order is kept as the node table's order:   */
/* children of a round are pushed to the front (reverse creation order) ahead of the    */
/* surviving nodes. Phase 1 divides every node with >1 key in list order; phase 2        */
/* divides them by (size desc, creation desc) and stops at the first division that      */
/* reaches N (ORBextractor.cc:676-737; pointer tie-break pinned to creation order).      */
/* ----------------------------------------------------------------------------------- */
template <int NW>
__device__ int block_scan_excl(int v, int* total, int* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int inc = wave_scan_incl_i32(v);
    if (lane == 63) red[w] = inc;
    __syncthreads();
    int woff = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const int s = red[i];
        woff += (i < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return woff + inc - v;
}

/* how many of the first m LDS keys are above `key` (rank counting): 8 independent broadcast reads in flight per
 * step -- one dependent read per key waited out the LDS latency m times */
__device__ __forceinline__ int count_above(const unsigned long long* a, int m, unsigned long long key) {
    int c = 0, t = 0;
    for (; t + 8 <= m; t += 8) {
        unsigned long long v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = a[t + k];
#pragma unroll
        for (int k = 0; k < 8; k++) c += v[k] > key ? 1 : 0;
    }
    for (; t < m; t++) c += a[t] > key ? 1 : 0;
    return c;
}

template <int NW>
__device__ __forceinline__ int block_sum(int v, int* red) {
    int tot;
    block_scan_excl<NW>(v, &tot, red);
    return tot;
}

/* LDS layout (bytes), NC = node capacity (pow2-rounded for the sort):
 *   nodes A/B : 2 x NC x {u16 x0,y0,x1,y1; int nk; uint seq} = 32 NC
 *   cnt4      : NC x 4 int                                 = 16 NC
 *   cpos      : NC x 4 u16                                 =  8 NC
 *   spos, dflag, dbase : 3 x NC int                        = 12 NC
 *   sortkey   : NC x u64                                   =  8 NC
 *   keys      : KL x (4 + 2 + 1) (if n <= KL, else global scratch)
 */
/* node rectangles as u16 (level coordinates < 4096, the 12-bit key fields): 76 B of LDS per node
 * instead of 92, so a 256-node table plus 1888 keys fits 32 KB and five workgroups share a CU with
 * the other graphs' kernels */
struct NodeT {
    uint16_t* x0; uint16_t* y0; uint16_t* x1; uint16_t* y1; int* nk; uint32_t* seq;
};

#ifdef ORBX_OCT_TRACE
__device__ unsigned long long g_oct_trace[kMaxLevels][40];
#define OCT_T(k) do { if (threadIdx.x == 0 && blockIdx.y == 0) g_oct_trace[l][(k)] = wall_clock64(); } while (0)
#else
#define OCT_T(k) do { } while (0)
#endif
template <int NT>
__global__ __launch_bounds__(NT) void k_octree(ExtractParams ep, const LevelDesc* __restrict__ levels,
                                                const CellDesc* __restrict__ cells,
                                                const uint32_t* __restrict__ cellkey,
                                                const int* __restrict__ cellcnt, uint32_t* __restrict__ lvkey,
                                                int* __restrict__ lvcnt, uint8_t* __restrict__ gscratch,
                                                long long gscratch_frame_bytes, int NC, int KL, int level0,
                                                int* __restrict__ err, HostCopy hc) {
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int red[16];
    __shared__ int sh_size, sh_jstar, sh_tc, sh_nexp, sh_ndiv;
    const int tid = threadIdx.x;
    if ((int)blockIdx.x >= (int)gridDim.x - hc.nblocks) {
        // the host path's mvImagePyramid (orbx_set_host_pyramid): this frame's levels 1..L-1 into mapped pinned host
        // memory, beside the octree's few barrier-chained workgroups; visible to the host before the call's done
        // word (k_call_done, a later launch on the same queue)
        const long long stride = (long long)hc.nblocks * NT;
        uint4* dst = hc.dst_ref ? *(uint4* const volatile*)hc.dst_ref : hc.dst;
        for (long long i = (long long)(blockIdx.x - (gridDim.x - hc.nblocks)) * NT + tid; i < hc.n16; i += stride)
            dst[i] = hc.src[i];
        __threadfence_system();
        return;
    }
    const int l = level0 + blockIdx.x, f = blockIdx.y;
    OCT_T(0);
    const LevelDesc lv = levels[l];
    // --- carve LDS
    uint8_t* p = lds;
    NodeT A, Bt;
    A.x0 = (uint16_t*)p; p += 2 * NC; A.y0 = (uint16_t*)p; p += 2 * NC; A.x1 = (uint16_t*)p; p += 2 * NC;
    A.y1 = (uint16_t*)p; p += 2 * NC; A.nk = (int*)p; p += 4 * NC; A.seq = (uint32_t*)p; p += 4 * NC;
    Bt.x0 = (uint16_t*)p; p += 2 * NC; Bt.y0 = (uint16_t*)p; p += 2 * NC; Bt.x1 = (uint16_t*)p; p += 2 * NC;
    Bt.y1 = (uint16_t*)p; p += 2 * NC; Bt.nk = (int*)p; p += 4 * NC; Bt.seq = (uint32_t*)p; p += 4 * NC;
    int* cnt4 = (int*)p; p += 16 * NC;
    int* spos = (int*)p; p += 4 * NC;
    int* dflag = (int*)p; p += 4 * NC;
    int* dbase = (int*)p; p += 4 * NC;
    unsigned long long* skey = (unsigned long long*)p; p += 8 * NC;
    uint16_t* cpos = (uint16_t*)p; p += 8 * NC;
    uint8_t* kbase = p;

    // --- 1. gather this level's candidates (cell order = ORBextractor.cc:789-829 order)
    const int* ccnt = cellcnt + (long long)f * ep.ncells + lv.cell_begin;
    const uint32_t* ckey = cellkey + (long long)f * ep.keys_per_frame;
    int carry = 0;
    // the level's key count; for the flat gather below also each cell's key offset and slot, in LDS (cnt4's space,
    // unused until the roots): the counts and slots come in one round of loads, with one scan
    const bool flat = 2 * lv.ncells + 2 <= 4 * NC;
    int* coff = cnt4;                   // [ncells + 1]
    int* cslot = cnt4 + lv.ncells + 1;  // [ncells]
    __syncthreads();
    int n = 0;
    for (int c0 = 0; c0 < lv.ncells; c0 += NT) {
        const int c = c0 + tid;
        const int v = c < lv.ncells ? ccnt[c] : 0;
        const int sl = flat && c < lv.ncells ? cells[lv.cell_begin + c].slot : 0;
        int tot;
        const int off = block_scan_excl<NT / 64>(v, &tot, red) + carry;
        if (flat && c < lv.ncells) {
            coff[c] = off;
            cslot[c] = sl;
        }
        carry += tot;
    }
    n = carry;
    if (flat && tid == 0) coff[lv.ncells] = n;
    OCT_T(1);
    // The rest runs with the keys either in LDS (n <= KL) or in global scratch; the two
    // instantiations keep every key access a plain ds_* or global_* instruction (a pointer
    // that may be either would make all of them flat accesses).
    struct KeysLds { uint32_t* key; uint16_t* label; uint8_t* quad; };
    struct KeysGlobal { uint32_t* key; uint16_t* label; uint8_t* quad; };
    auto tail = [&](auto K) {
        carry = 0;
        if (flat) {
            // flat gather: thread t copies keys t, t+NT, ... finding each key's cell by a fixed-trip binary search
            // over the cell offsets (in LDS since the count pass), four keys in flight per thread. (A thread per
            // cell copying its keys one by one waited on one global load per key of the level's fullest cell: the
            // level-0 workgroup's long pole.)
            __syncthreads();
            int top = 1;
            while (top < lv.ncells) top <<= 1;
            constexpr int kG = 4;
            for (int i0 = tid; i0 < n; i0 += NT * kG) {
                int pos[kG];
#pragma unroll
                for (int g = 0; g < kG; g++) pos[g] = 0;
                for (int step = top >> 1; step > 0; step >>= 1) {  // largest c with coff[c] <= i
#pragma unroll
                    for (int g = 0; g < kG; g++) {
                        const int i = min(i0 + NT * g, n - 1);
                        const int q = pos[g] + step;
                        if (q < lv.ncells && coff[q] <= i) pos[g] = q;
                    }
                }
                uint32_t kv[kG];
#pragma unroll
                for (int g = 0; g < kG; g++) {
                    const int i = min(i0 + NT * g, n - 1);
                    kv[g] = ckey[cslot[pos[g]] + (i - coff[pos[g]])];
                }
#pragma unroll
                for (int g = 0; g < kG; g++)
                    if (i0 + NT * g < n) K.key[i0 + NT * g] = kv[g];
            }
        } else {
            for (int c0 = 0; c0 < lv.ncells; c0 += NT) {
                const int c = c0 + tid;
                const int v = c < lv.ncells ? ccnt[c] : 0;
                int tot;
                const int off = block_scan_excl<NT / 64>(v, &tot, red) + carry;
                if (c < lv.ncells) {
                    const uint32_t* src = ckey + cells[lv.cell_begin + c].slot;
                    for (int k = 0; k < v; k++) K.key[off + k] = src[k];
                }
                carry += tot;
            }
        }
        __syncthreads();
        uint32_t* outk = lvkey + (long long)f * ep.kp_per_frame + lv.kp_off;
        if (n == 0) {
            if (tid == 0) lvcnt[f * ep.L + l] = 0;
            return;
        }
        OCT_T(2);
        // --- 2. roots (ORBextractor.cc:542-585)
        const int nIni = lv.nIni;
        for (int s = tid; s < nIni; s += NT) cnt4[s] = 0;
        __syncthreads();
        if (nIni <= 8) {  // a handful of roots (1 at 4:3, 3 at C4's 3.3:1): one LDS atomic per wave and root
            for (int i0 = 0; i0 < n; i0 += NT) {
                const int i = i0 + tid;
                int r = -1;
                if (i < n) {
                    const float x = (float)(K.key[i] & 0xFFF);
                    r = (int)__fdiv_rn(x, lv.hX);
                    if (r >= nIni) { atomicOr(err, 1); r = nIni - 1; }
                    K.label[i] = (uint16_t)r;
                }
                for (int q = 0; q < nIni; q++) {
                    const unsigned long long m = __ballot(r == q);
                    if ((tid & 63) == 0 && m) atomicAdd(&cnt4[q], (int)__popcll(m));
                }
            }
        } else {
            for (int i = tid; i < n; i += NT) {
                const float x = (float)(K.key[i] & 0xFFF);
                int r = (int)__fdiv_rn(x, lv.hX);
                if (r >= nIni) { atomicOr(err, 1); r = nIni - 1; }
                K.label[i] = (uint16_t)r;
                atomicAdd(&cnt4[r], 1);
            }
        }
        __syncthreads();
        int size = 0;
        {
            int carry2 = 0;
            for (int r0 = 0; r0 < nIni; r0 += NT) {
                const int r = r0 + tid;
                const int nonempty = (r < nIni && cnt4[r] > 0) ? 1 : 0;
                int tot;
                const int pos = block_scan_excl<NT / 64>(nonempty, &tot, red) + carry2;
                if (nonempty) {
                    spos[r] = pos;
                    A.x0[pos] = (int)__fmul_rn(lv.hX, (float)r);
                    A.x1[pos] = (int)__fmul_rn(lv.hX, (float)(r + 1));
                    A.y0[pos] = 0;
                    A.y1[pos] = lv.maxY - lv.minY;
                    A.nk[pos] = cnt4[r];
                    A.seq[pos] = (uint32_t)r;
                }
                carry2 += tot;
            }
            size = carry2;
        }
        __syncthreads();
        for (int i = tid; i < n; i += NT) K.label[i] = (uint16_t)spos[K.label[i]];
        if (size > NC) {  // capacity overflow: flag it and leave this level empty (never a stale count)
            if (tid == 0) { atomicOr(err, 2); lvcnt[f * ep.L + l] = 0; }
            return;
        }
        __syncthreads();
        uint32_t next_seq = (uint32_t)nIni;
        int phase = 1;
        const int N = lv.N;
        OCT_T(3);
        // --- 3. division rounds (ORBextractor.cc:594-739)
        bool cnt_clean = false;  // cnt4[0, 4 size) already zero (cleared by the previous fast round)
        bool counted = false;    // this round's quadrant counts are in cntc already (the previous round's relabel)
        int* cntc = cnt4;        // this round's counts (cnt4, or dflag..skey when a relabel pass counted there)
        int iters = 0;
        for (int iter = 0; iter < 100000; iter++) {
            if (iter < 30) OCT_T(4 + iter);
            iters = iter + 1;
            const int prevSize = size;
            if (!cnt_clean && !counted) {
                for (int s = tid; s < size; s += NT) {
                    cnt4[4 * s] = 0; cnt4[4 * s + 1] = 0; cnt4[4 * s + 2] = 0; cnt4[4 * s + 3] = 0;
                }
                __syncthreads();
            }
            cnt_clean = false;
            // node-per-thread rounds: slot s = tid (size <= NT), and the packed scan's survivor field holds 9 bits
            constexpr int kFast1 = NT < 512 ? NT : 511;
            if (phase == 1 && size <= kFast1) {
                // Phase-1 round with every node in one thread (slot s = tid): every node with > 1 key divides,
                // in list order, so one packed scan gives the children's creation indices, the survivors'
                // positions and the number of children with > 1 key at once (4 barriers per round instead of
                // ~20 for the general path below, which phase 2 and tables of > 256 nodes take). When the next
                // round is one of these too, this round's relabel pass also counts the keys' quadrants in the new
                // table (into the other counts buffer), so that round has no count pass of its own.
                if (!counted) {
                    for (int i = tid; i < n; i += NT) {
                        const int s = K.label[i];
                        if (A.nk[s] >= 2) {
                            const uint32_t kk = K.key[i];
                            const int x = (int)(kk & 0xFFF), y = (int)((kk >> 12) & 0xFFF);
                            const int hx = (A.x1[s] - A.x0[s] + 1) >> 1, hy = (A.y1[s] - A.y0[s] + 1) >> 1;
                            const int q = (x >= A.x0[s] + hx ? 1 : 0) + (y >= A.y0[s] + hy ? 2 : 0);
                            K.quad[i] = (uint8_t)q;
                            atomicAdd(&cntc[4 * s + q], 1);
                        }
                    }
                    __syncthreads();
                }
                const int s = tid;
                const bool live = s < size;
                const bool isD = live && A.nk[s] >= 2;
                int c4[4] = {0, 0, 0, 0};
                if (isD) {
#pragma unroll
                    for (int q = 0; q < 4; q++) c4[q] = cntc[4 * s + q];
                }
                const int nc = (c4[0] > 0) + (c4[1] > 0) + (c4[2] > 0) + (c4[3] > 0);
                const int ne = (c4[0] > 1) + (c4[1] > 1) + (c4[2] > 1) + (c4[3] > 1);
                const int sv = (live && !isD) ? 1 : 0;
                // fields: children (<= 1024, bits 0-10), survivors (<= 256, bits 11-19), children with
                // > 1 key (<= 1024, bits 20-30)
                int tot;
                const int ex = block_scan_excl<NT / 64>(nc | (sv << 11) | (ne << 20), &tot, red);
                const int TC = tot & 0x7FF, nsurv = (tot >> 11) & 0x1FF, nToExpand = tot >> 20;
                const int newSize = TC + nsurv;
                if (newSize > NC) {
                    if (tid == 0) { atomicOr(err, 4); lvcnt[f * ep.L + l] = 0; }
                    return;
                }
                if (isD) {
                    const int x0 = A.x0[s], y0 = A.y0[s], x1 = A.x1[s], y1 = A.y1[s];
                    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;
                    int ci = ex & 0x7FF;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (c4[q] > 0) {
                            const int np = TC - 1 - ci;  // children pushed to the front, reverse creation order
                            Bt.x0[np] = (q & 1) ? x0 + hx : x0;
                            Bt.x1[np] = (q & 1) ? x1 : x0 + hx;
                            Bt.y0[np] = (q & 2) ? y0 + hy : y0;
                            Bt.y1[np] = (q & 2) ? y1 : y0 + hy;
                            Bt.nk[np] = c4[q];
                            Bt.seq[np] = next_seq + (uint32_t)ci;
                            cpos[4 * s + q] = (uint16_t)np;
                            ci++;
                        }
                    }
                    spos[s] = -1;
                } else if (live) {
                    const int np = TC + ((ex >> 11) & 0x1FF);
                    Bt.x0[np] = A.x0[s]; Bt.y0[np] = A.y0[s]; Bt.x1[np] = A.x1[s]; Bt.y1[np] = A.y1[s];
                    Bt.nk[np] = A.nk[s]; Bt.seq[np] = A.seq[s];
                    spos[s] = np;
                }
                // the next round is a phase-1 round of this form: count its quadrants in the relabel pass below, into
                // the buffer this round did not use (cnt4, or the phase-2 arrays dflag..skey, idle in phase 1)
                const bool fuse = !(newSize >= N || newSize == prevSize) && !(newSize + nToExpand * 3 > N) &&
                                  newSize <= kFast1;
                int* cntn = cntc == cnt4 ? dflag : cnt4;
                if (fuse)
                    for (int i = tid; i < 4 * newSize; i += NT) cntn[i] = 0;
                __syncthreads();
                for (int i = tid; i < n; i += NT) {
                    const int s2 = K.label[i];
                    const int np0 = spos[s2];
                    const int np = np0 >= 0 ? np0 : cpos[4 * s2 + K.quad[i]];
                    K.label[i] = (uint16_t)np;
                    if (fuse && Bt.nk[np] >= 2) {
                        const uint32_t kk = K.key[i];
                        const int x = (int)(kk & 0xFFF), y = (int)((kk >> 12) & 0xFFF);
                        const int hx = (Bt.x1[np] - Bt.x0[np] + 1) >> 1, hy = (Bt.y1[np] - Bt.y0[np] + 1) >> 1;
                        const int q = (x >= Bt.x0[np] + hx ? 1 : 0) + (y >= Bt.y0[np] + hy ? 2 : 0);
                        K.quad[i] = (uint8_t)q;
                        atomicAdd(&cntn[4 * np + q], 1);
                    }
                }
                if (!fuse)
                    for (int i = tid; i < 4 * newSize; i += NT) cnt4[i] = 0;  // for the next round's count pass
                __syncthreads();
                cnt_clean = !fuse;
                counted = fuse;
                cntc = fuse ? cntn : cnt4;
                { NodeT t = A; A = Bt; Bt = t; }
                next_seq += (uint32_t)TC;
                size = newSize;
                if (size >= N || size == prevSize) break;
                if (size + nToExpand * 3 > N) phase = 2;
                continue;
            }
            if (phase == 2 && size <= NT) {
                // Phase-2 round with every node in one thread (slot s = tid): the divisible nodes' processing order
                // is their rank by (size, creation) descending (rank counting over the LDS keys), one scan in that
                // order finds the first division reaching N and the children's creation indices, one packed scan in
                // list order gives the survivors' positions and the children with > 1 key: 11 barriers per round
                // instead of the general path's ~20 (the same table, the same order).
                for (int i = tid; i < n; i += NT) {
                    const int s = K.label[i];
                    if (A.nk[s] >= 2) {
                        const uint32_t kk = K.key[i];
                        const int x = (int)(kk & 0xFFF), y = (int)((kk >> 12) & 0xFFF);
                        const int hx = (A.x1[s] - A.x0[s] + 1) >> 1, hy = (A.y1[s] - A.y0[s] + 1) >> 1;
                        const int q = (x >= A.x0[s] + hx ? 1 : 0) + (y >= A.y0[s] + hy ? 2 : 0);
                        K.quad[i] = (uint8_t)q;
                        atomicAdd(&cnt4[4 * s + q], 1);
                    }
                }
                __syncthreads();
                const int s = tid;
                const bool live = s < size;
                const bool isD = live && A.nk[s] >= 2;
                int nc = 0, ne = 0;
                if (isD) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int cq = cnt4[4 * s + q];
                        nc += cq > 0;
                        ne += cq > 1;
                    }
                }
                const unsigned long long key = isD ? ((unsigned long long)(uint32_t)A.nk[s] << 32) | A.seq[s] : 0ull;
                if (live) skey[s] = key;  // 0 for a node that does not divide: below every divisible key
                if (tid == 0) sh_tc = -1;
                int nD;
                block_scan_excl<NT / 64>(isD ? 1 : 0, &nD, red);  // (its barriers publish skey / sh_tc)
                if (nD == 0) break;  // cannot happen while size changes, kept for safety
                int rank = 0;
                if (isD)
                    rank = count_above(skey, size, key);
                if (isD) {
                    dflag[rank] = s;
                    dbase[rank] = nc;
                }
                if (tid == 0) sh_jstar = nD - 1;
                __syncthreads();
                // processing position r = tid: children before it and the first division that reaches N
                const int r = tid;
                const int ncr = r < nD ? dbase[r] : 0;
                int TCall;
                const int exr = block_scan_excl<NT / 64>(ncr, &TCall, red);
                if (r < nD) {
                    const int before = prevSize + exr - r, after = before + ncr - 1;
                    if (after >= N && before < N) {  // first crossing (unique)
                        sh_jstar = r;
                        sh_tc = exr + ncr;
                    }
                }
                __syncthreads();
                const int jstar = sh_jstar;
                const int TC = sh_tc >= 0 ? sh_tc : TCall;
                // survivors in list order + children with > 1 key of the divided nodes, one packed scan
                const bool divided = isD && rank <= jstar;
                const bool sv = live && !divided;
                int tot;
                const int ex = block_scan_excl<NT / 64>((sv ? 1 : 0) | ((divided ? ne : 0) << 16), &tot, red);
                const int nsurv = tot & 0xFFFF, nToExpand = tot >> 16;
                const int newSize = TC + nsurv;
                if (newSize > NC) {
                    if (tid == 0) { atomicOr(err, 4); lvcnt[f * ep.L + l] = 0; }
                    return;
                }
                if (sv) {
                    const int np = TC + (ex & 0xFFFF);
                    Bt.x0[np] = A.x0[s]; Bt.y0[np] = A.y0[s]; Bt.x1[np] = A.x1[s]; Bt.y1[np] = A.y1[s];
                    Bt.nk[np] = A.nk[s]; Bt.seq[np] = A.seq[s];
                    spos[s] = np;
                } else if (divided) {
                    spos[s] = -1;
                }
                if (r <= jstar) {  // the node at processing position r divides: its children pushed to the front
                    const int d = dflag[r];
                    const int x0 = A.x0[d], y0 = A.y0[d], x1 = A.x1[d], y1 = A.y1[d];
                    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;
                    int ci = exr;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int cn = cnt4[4 * d + q];
                        if (cn > 0) {
                            const int np = TC - 1 - ci;
                            Bt.x0[np] = (q & 1) ? x0 + hx : x0;
                            Bt.x1[np] = (q & 1) ? x1 : x0 + hx;
                            Bt.y0[np] = (q & 2) ? y0 + hy : y0;
                            Bt.y1[np] = (q & 2) ? y1 : y0 + hy;
                            Bt.nk[np] = cn;
                            Bt.seq[np] = next_seq + (uint32_t)ci;
                            cpos[4 * d + q] = (uint16_t)np;
                            ci++;
                        }
                    }
                }
                __syncthreads();
                for (int i = tid; i < n; i += NT) {
                    const int s2 = K.label[i];
                    const int np = spos[s2];
                    K.label[i] = (uint16_t)(np >= 0 ? np : cpos[4 * s2 + K.quad[i]]);
                }
                for (int i = tid; i < 4 * newSize; i += NT) cnt4[i] = 0;  // for the next round's count pass
                __syncthreads();
                cnt_clean = true;
                { NodeT t = A; A = Bt; Bt = t; }
                next_seq += (uint32_t)TC;
                size = newSize;
                (void)nToExpand;
                if (size >= N || size == prevSize) break;
                continue;
            }
            for (int i = tid; i < n; i += NT) {
                const int s = K.label[i];
                if (A.nk[s] >= 2) {
                    const uint32_t kk = K.key[i];
                    const int x = (int)(kk & 0xFFF), y = (int)((kk >> 12) & 0xFFF);
                    const int hx = (A.x1[s] - A.x0[s] + 1) >> 1, hy = (A.y1[s] - A.y0[s] + 1) >> 1;
                    const int q = (x >= A.x0[s] + hx ? 1 : 0) + (y >= A.y0[s] + hy ? 2 : 0);
                    K.quad[i] = (uint8_t)q;
                    atomicAdd(&cnt4[4 * s + q], 1);
                }
            }
            __syncthreads();
            // D = nodes with >1 key; processing order: list order (phase 1) or sorted (phase 2)
            int nD;
            {
                int carry3 = 0;
                for (int s0 = 0; s0 < size; s0 += NT) {
                    const int s = s0 + tid;
                    const int isD = (s < size && A.nk[s] >= 2) ? 1 : 0;
                    int tot;
                    const int pos = block_scan_excl<NT / 64>(isD, &tot, red) + carry3;
                    if (isD) {
                        dflag[pos] = s;  // D array (slot ids) in list order
                        skey[pos] = ((unsigned long long)(uint32_t)A.nk[s] << 32) | A.seq[s];
                    }
                    carry3 += tot;
                }
                nD = carry3;
            }
            __syncthreads();
            if (nD == 0) break;  // cannot happen while size changes, kept for safety
            if (phase == 2) {
                // processing order = descending (size, creation) key; keys are unique (seq), so a node's
                // rank is the number of larger keys: nD broadcast LDS reads per node and two barriers
                // instead of a bitonic network's log2(P)(log2(P)+1)/2 barriers
                for (int j = tid; j < nD; j += NT) {
                    const unsigned long long key = skey[j];
                    const int rank = count_above(skey, nD, key);
                    dbase[rank] = dflag[j];
                }
                __syncthreads();
                for (int j = tid; j < nD; j += NT) dflag[j] = dbase[j];
                __syncthreads();
            }
            // children counts per processing position; prefix -> creation indices
            int TC = 0, jstar = nD - 1;
            {
                int carry4 = 0;
                if (tid == 0) sh_jstar = nD - 1;
                __syncthreads();
                for (int j0 = 0; j0 < nD; j0 += NT) {
                    const int j = j0 + tid;
                    int nc = 0;
                    if (j < nD) {
                        const int s = dflag[j];
                        nc = (cnt4[4 * s] > 0) + (cnt4[4 * s + 1] > 0) + (cnt4[4 * s + 2] > 0) + (cnt4[4 * s + 3] > 0);
                    }
                    int tot;
                    const int excl = block_scan_excl<NT / 64>(nc, &tot, red) + carry4;
                    const int excl2 = excl - j;  // sum of (children - 1) before position j (active j only)
                    if (j < nD) {
                        dbase[j] = excl;
                        if (phase == 2) {
                            const int after = prevSize + excl2 + (nc - 1);
                            const int before = prevSize + excl2;
                            if (after >= N && before < N) sh_jstar = j;  // first crossing (unique)
                        }
                    }
                    carry4 += tot;
                }
                __syncthreads();
                jstar = sh_jstar;
                TC = (jstar == nD - 1) ? carry4 : dbase[jstar + 1];
            }
            const int ndiv = jstar + 1;
            // survivors = live slots not divided, in list order
            for (int s = tid; s < size; s += NT) spos[s] = 0;
            __syncthreads();
            for (int j = tid; j < ndiv; j += NT) spos[dflag[j]] = -1;  // mark divided
            __syncthreads();
            int nsurv;
            {
                int carry5 = 0;
                for (int s0 = 0; s0 < size; s0 += NT) {
                    const int s = s0 + tid;
                    const int sv = (s < size && spos[s] == 0) ? 1 : 0;
                    int tot;
                    const int pos = block_scan_excl<NT / 64>(sv, &tot, red) + carry5;
                    __syncthreads();
                    if (s < size) spos[s] = sv ? (TC + pos) : -1;
                    carry5 += tot;
                }
                nsurv = carry5;
            }
            __syncthreads();
            const int newSize = TC + nsurv;
            if (newSize > NC) {
                if (tid == 0) { atomicOr(err, 4); lvcnt[f * ep.L + l] = 0; }
                return;
            }
            // write new table: survivors copy, children created
            for (int s = tid; s < size; s += NT) {
                const int np = spos[s];
                if (np >= 0) {
                    Bt.x0[np] = A.x0[s]; Bt.y0[np] = A.y0[s]; Bt.x1[np] = A.x1[s]; Bt.y1[np] = A.y1[s];
                    Bt.nk[np] = A.nk[s]; Bt.seq[np] = A.seq[s];
                }
            }
            int nexp_local = 0;
            for (int j = tid; j < ndiv; j += NT) {
                const int s = dflag[j];
                const int x0 = A.x0[s], y0 = A.y0[s], x1 = A.x1[s], y1 = A.y1[s];
                const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;
                int ci = dbase[j];
    #pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int cn = cnt4[4 * s + q];
                    if (cn > 0) {
                        const int np = TC - 1 - ci;
                        const int cx0 = (q & 1) ? x0 + hx : x0, cx1 = (q & 1) ? x1 : x0 + hx;
                        const int cy0 = (q & 2) ? y0 + hy : y0, cy1 = (q & 2) ? y1 : y0 + hy;
                        Bt.x0[np] = cx0; Bt.y0[np] = cy0; Bt.x1[np] = cx1; Bt.y1[np] = cy1;
                        Bt.nk[np] = cn; Bt.seq[np] = next_seq + (uint32_t)ci;
                        cpos[4 * s + q] = (uint16_t)np;
                        nexp_local += cn > 1;
                        ci++;
                    }
                }
            }
            const int nToExpand = block_sum<NT / 64>(nexp_local, red);
            // relabel keys
            for (int i = tid; i < n; i += NT) {
                const int s = K.label[i];
                const int np = spos[s];
                K.label[i] = (uint16_t)(np >= 0 ? np : cpos[4 * s + K.quad[i]]);
            }
            __syncthreads();
            // swap tables
            { NodeT t = A; A = Bt; Bt = t; }
            next_seq += (uint32_t)TC;
            size = newSize;
            if (size >= N || size == prevSize) break;
            if (phase == 1 && size + nToExpand * 3 > N) phase = 2;
        }
        OCT_T(34);
#ifdef ORBX_OCT_TRACE
        if (threadIdx.x == 0 && blockIdx.y == 0) g_oct_trace[l][36] = (unsigned long long)iters | ((unsigned long long)n << 16) | ((unsigned long long)phase << 40) | ((unsigned long long)size << 48);
#endif
        (void)iters;
        // --- 4. keep the best key of each node (first max response, ORBextractor.cc:741-760)
        uint32_t* best = (uint32_t*)cnt4;
        for (int s = tid; s < size; s += NT) best[s] = 0u;
        __syncthreads();
        for (int i = tid; i < n; i += NT) {
            const uint32_t kk = K.key[i];
            atomicMax(&best[K.label[i]], (kk & 0xFF000000u) | (0xFFFFFFu - (uint32_t)i));
        }
        __syncthreads();
        if (size > lv.kp_cap) { if (tid == 0) atomicOr(err, 8); size = lv.kp_cap; }
        for (int s = tid; s < size; s += NT) {
            const int i = (int)(0xFFFFFFu - (best[s] & 0xFFFFFFu));
            const uint32_t kk = K.key[i];
            const uint32_t x = (kk & 0xFFF) + (uint32_t)lv.minX, y = ((kk >> 12) & 0xFFF) + (uint32_t)lv.minY;
            outk[s] = x | (y << 12) | (kk & 0xFF000000u);
        }
        if (tid == 0) lvcnt[f * ep.L + l] = size;
        OCT_T(35);
    };
    if (n <= KL) {
        tail(KeysLds{(uint32_t*)kbase, (uint16_t*)(kbase + 4 * KL), kbase + 6 * KL});
    } else {
        uint8_t* g = gscratch + (long long)f * gscratch_frame_bytes + (long long)lv.key_begin * 8;
        tail(KeysGlobal{(uint32_t*)g, (uint16_t*)(g + 4ll * lv.key_cap), g + 6ll * lv.key_cap});
    }
}

template <bool kAligned, int kRows>
__device__ __forceinline__ void blur_strips_body(const uint8_t* __restrict__ frames, long long fstride, int pitch0,
                                                 const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                                 const ExtractParams& ep, const LevelDesc* __restrict__ levels,
                                                 int job0, int job1, const int* __restrict__ lvcnt, int bx, int f,
                                                 uint8_t (*s_rows)[7][kBlurSeg]) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    int j = job0 + bx * 4 + wave;
    if (j >= job1) return;
    const int l = level_of(ep.bjob_begin, ep.L, j);
    j -= ep.bjob_begin[l];
    // the reference blurs only levels with keypoints (:1081); lvcnt == nullptr blurs every level
    // (the result of an unused level is never read), so the blur can run before the octree
    if (lvcnt && lvcnt[f * ep.L + l] == 0) return;
    const LevelDesc lv = levels[l];
    const int nstrips = (lv.w + 255) / 256;
    const uint8_t* img = l == 0 ? frames + (long long)f * fstride : pyr + (long long)f * ep.pyr_frame_bytes + lv.pyr_off;
    const int pitch = l == 0 ? pitch0 : lv.pitch;
    uint8_t* out = blur + (long long)f * ep.blur_frame_bytes + lv.blur_off;
    blur_job<kAligned, kRows>(img, pitch, lv, out, j % nstrips, j / nstrips, s_rows[wave], lane);
}

template <bool kAligned, int kRows>
__global__ __launch_bounds__(256) void k_blur_strips(const uint8_t* __restrict__ frames, long long fstride, int pitch0,
                                                     const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                                     ExtractParams ep, const LevelDesc* __restrict__ levels,
                                                     int job0, int job1, const int* __restrict__ lvcnt) {
    __shared__ __align__(16) uint8_t s_rows[4][7][kBlurSeg];
    blur_strips_body<kAligned, kRows>(frames, fstride, pitch0, pyr, blur, ep, levels, job0, job1, lvcnt, blockIdx.x,
                                      blockIdx.y, s_rows);
}

/* FAST and the blur in one launch (small batches: both need only the pyramid, and one frame's FAST cells and
 * blur chunks each fill a few dozen CUs): blocks [0, nfast) take FAST cells as k_fast_cells2, the rest take
 * blur jobs (kBlurRowsSmall-row chunks, job table in eb) as k_blur_strips; every wave works alone */
template <int kMaxPass, int kRP, bool kAligned>
__global__ __launch_bounds__(256) void k_fast_blur(
    const uint8_t* __restrict__ frames, long long fstride, int pitch0, const uint8_t* __restrict__ pyr,
    ExtractParams ep, const LevelDesc* __restrict__ levels, const CellDesc* __restrict__ cells,
    uint32_t* __restrict__ cellkey, int* __restrict__ cellcnt, int RP_, int RH, int cell_lo, int cell_hi, int nfast,
    uint8_t* __restrict__ blur, ExtractParams eb, int njobs) {
    extern __shared__ __align__(16) uint8_t lds[];
    if ((int)blockIdx.x < nfast)
        fast_cells_body<kMaxPass, kRP>(frames, fstride, pitch0, pyr, ep, levels, cells, cellkey, cellcnt, RP_, RH,
                                       cell_lo, cell_hi, blockIdx.x, blockIdx.y, lds, 4);
    else
        blur_strips_body<kAligned, kBlurRowsSmall>(frames, fstride, pitch0, pyr, blur, eb, levels, 0, njobs, nullptr,
                                                   blockIdx.x - nfast, blockIdx.y, (uint8_t(*)[7][kBlurSeg])lds);
}

/* rBRIEF test pairs as floats, one 16-byte load per test; stored (x0, x1, y0, y1) so the two points'
 * x and y coordinates are float pairs for the packed-f32 rotation */
struct PatPt {
    float x0, x1, y0, y1;
};
struct PatTable {
    PatPt t[256];
};
constexpr float pat_s8(unsigned char c) { return (float)(c < 128 ? (int)c : (int)c - 256); }
constexpr PatTable make_pattern_table() {
    PatTable p{};
    for (int t = 0; t < 256; t++) {
        p.t[t].x0 = pat_s8(orbx_pattern_soa_u8[t]);
        p.t[t].y0 = pat_s8(orbx_pattern_soa_u8[256 + t]);
        p.t[t].x1 = pat_s8(orbx_pattern_soa_u8[512 + t]);
        p.t[t].y1 = pat_s8(orbx_pattern_soa_u8[768 + t]);
    }
    return p;
}
__device__ constexpr PatTable kPatternF = make_pattern_table();
/* the same pairs transposed (pair p at (p % 16) * 16 + p / 16): the 16 lanes of a keypoint read 256
 * contiguous bytes per step */
constexpr PatTable make_pattern_table_t() {
    PatTable p{};
    const PatTable a = make_pattern_table();
    for (int t = 0; t < 256; t++) p.t[(t & 15) * 16 + (t >> 4)] = a.t[t];
    return p;
}
__device__ constexpr PatTable kPatternT = make_pattern_table_t();

/* ----------------------------------------------------------------------------------- */
/* IC_Angle + rBRIEF + output: 16 lanes per keypoint, 4 keypoints per wave.               */
/*                                                                                       */
/*  - IC_Angle (ORBextractor.cc:77-104): lane (column group g4 = ln&7, row parity ln>>3)  */
/*    takes rows ri = (ln>>3) + 2p, p = 0..15 (v = ri - 15 in -15..16, 16 masked); its 4  */
/*    pixels are one dword (8-byte aligned load + alignbyte); the circular mask and the   */
/*    column weights u+15 are packed bytes of a host table (LDS copy), so per row two     */
/*    v_dot4 give sum (u+15)*I and sum I: m10 = sum (u+15)I - 15 sum I, m01 = sum v*I.     */
/*  - fastAtan2 + glibc sincosf once per 16 lanes (orb_math.h).                           */
/*  - rBRIEF (ORBextractor.cc:107-147): test t = 16k + ln, k = 0..15, pattern from LDS;   */
/*    bit t%8 of byte t/8 = ballot bit (16 sub + ln) of round k.                          */
/* ----------------------------------------------------------------------------------- */
constexpr int kDescPatchR = 18;                   // |round(rotated pattern coordinate)| <= 13*sqrt(2)
constexpr int kDescPatchRows = 2 * kDescPatchR + 1;  // 37
constexpr int kDescPatchPitch = 40;                 // 10 dwords: 37 columns + up to 3 bytes misalignment
constexpr int kDescWaves = 4;                      // waves (x 4 keypoints) per k_describe workgroup
constexpr int kDescKps = 4 * kDescWaves;            // keypoints per workgroup

/* kEvenPitch: every row pitch is even (levels >= 1 always are; level 0 when the caller's pitch is), so the IC rows a
 * lane reads (2 rows apart) share one misalignment and their addresses are one running 32-bit offset */
template <bool kEvenPitch>
__global__ __launch_bounds__(64 * kDescWaves) void k_describe(const uint8_t* __restrict__ frames, long long fstride, int pitch0,
                                                  const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur,
                                                  ExtractParams ep, const LevelDesc* __restrict__ levels,
                                                  const uint32_t* __restrict__ lvkey, const int* __restrict__ lvcnt,
                                                  orbx_kp* __restrict__ out_kps, uint8_t* __restrict__ out_desc,
                                                  int* __restrict__ out_counts, int kp_stride,
                                                  const int* __restrict__ ptab) {
    __shared__ PatPt s_pat[256];
    __shared__ int2 s_ic[256];
    __shared__ __align__(8) uint8_t s_patch[kDescKps][kDescPatchRows * kDescPatchPitch];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int sub = lane >> 4, ln = lane & 15;
    // XCD-aware block mapping (1-D grid of G groups x F frames): workgroups are dispatched to the 8
    // XCDs round-robin, so with F % 8 == 0 block b runs on XCD b % 8 and serves frame
    // (b % 8) + 8 * ((b / 8) / G): every workgroup of a frame shares one XCD's L2, where the
    // overlapping 37x37 patches and IC rows of neighbouring keypoints hit
    const int G = (ep.kp_per_frame + kDescKps - 1) / kDescKps;
    int f, blk;
    {
        const int b = blockIdx.x;
        if ((gridDim.x / G) % 8 == 0) {
            const int k = b >> 3;
            f = (b & 7) + 8 * (k / G);
            blk = k % G;
        } else {
            f = b / G;
            blk = b % G;
        }
    }
    // everything that depends only on the slot is issued before the table barrier
    constexpr int NT = 64 * kDescWaves;
    constexpr int kTab = (256 + NT - 1) / NT;  // table entries per thread (workgroups of more than 256 threads: 1)
    PatPt my_pat[kTab];
    int2 my_ic[kTab];
#pragma unroll
    for (int q = 0; q < kTab; q++) {
        const int t = min(tid + q * NT, 255);
        // the transposed table, read and stored linearly (slot t): the 8 lanes of a ds_write_b128 group
        // write 128 consecutive bytes (a transposing store, slot (t % 16) * 16 + t / 16, put the group's
        // eight 16-byte words 256 bytes apart: one bank, an 8-way conflict)
        my_pat[q] = kPatternT.t[t];
        my_ic[q] = ((const int2*)(ptab + ep.ic_off))[t];
    }
    const int g = (blk * kDescWaves + wave) * 4 + sub;  // octree output slot of this lane group
    const int gc = min(g, ep.kp_per_frame - 1);
    const uint32_t kk_raw = lvkey[(long long)f * ep.kp_per_frame + gc];
    // per-level counts of this frame (lvcnt is padded by kMaxLevels ints; entries >= L masked)
    const int* cnt = lvcnt + f * ep.L;
    int cl[kMaxLevels];
#pragma unroll
    for (int q = 0; q < kMaxLevels; q++) cl[q] = q < ep.L ? cnt[q] : 0;
#pragma unroll
    for (int q = 0; q < kTab; q++) {
        const int t = tid + q * NT;
        if (t >= 256) break;
        s_pat[t] = my_pat[q];  // pair p at (p % 16) * 16 + p / 16 (kPatternT's order)
        s_ic[t] = my_ic[q];
    }
    if (blk == 0 && tid == 0) {
        int tot = 0;
#pragma unroll
        for (int q = 0; q < kMaxLevels; q++) tot += cl[q];
        out_counts[f] = tot;
        if (ep.host_out) __threadfence_system();
    }
    __syncthreads();
    if (__ballot(g < ep.kp_per_frame) == 0) return;  // wave-uniform
    // level, index in the level and output row of the keypoint: one select chain over the frame's L levels
    int l = 0, koff = 0, mycnt = cl[0], below = 0;
#pragma unroll
    for (int q = 1; q < kMaxLevels; q++) {
        if (q >= ep.L) break;  // wave-uniform
        const bool ge = gc >= ep.kp_off[q];
        l += ge ? 1 : 0;
        koff = ge ? ep.kp_off[q] : koff;
        below += ge ? cl[q - 1] : 0;
        mycnt = ge ? cl[q] : mycnt;
    }
    const int k = gc - koff;
    const int outidx = k + below;
    const bool valid = g < ep.kp_per_frame && k < mycnt;
    if (__ballot(valid) == 0) return;  // wave-uniform
    const LevelDesc lv = levels[l];
    const uint32_t kk = valid ? kk_raw : 0u;
    // invalid groups run on a safe dummy position (results discarded)
    const int x = valid ? (int)(kk & 0xFFF) : 32, y = valid ? (int)((kk >> 12) & 0xFFF) : 32;
    const int resp = (int)(kk >> 24);
    const uint8_t* img = l == 0 ? frames + (long long)f * fstride : pyr + (long long)f * ep.pyr_frame_bytes + lv.pyr_off;
    const int pitch = l == 0 ? pitch0 : lv.pitch;
    const uint8_t* bl = blur + (long long)f * ep.blur_frame_bytes + lv.blur_off;
    // one memory round trip: the IC_Angle rows of the level image and the blurred 37x37 patch
    // around the keypoint (staged in LDS for the 512 rBRIEF samples)
    const int g4 = ln & 7, r = ln >> 3;
    const int off0 = (y + r - 15) * pitch + x - 15 + 4 * g4;  // >= 0: keypoints lie in [19, dim - 19)
    const uint32_t mis = ((uint32_t)(uintptr_t)img + (uint32_t)off0) & 3u;
    const uint32_t dmis = kEvenPitch ? 0u : (uint32_t)(2 * pitch) & 3u;  // misalignment step between a lane's rows
    uint2 wv[16];
#pragma unroll
    for (int p = 0; p < 16; p++) {
        const uint32_t al = (mis + (uint32_t)p * dmis) & 3u;
        wv[p] = *(const uint2*)(img + ((uint32_t)off0 + (uint32_t)(2 * p * pitch) - al));
    }
    // patch: 37 rows x 5 aligned 8-byte words (row start rounded down to 4; patch column 0 =
    // image column x-18-pmis[row])
    const int bp = lv.pitch;  // blurred rows are 64-aligned: one misalignment for every row
    const int pmis = (int)((uint32_t)(x - kDescPatchR) & 3u);
    const int pbase = (y - kDescPatchR) * bp + x - kDescPatchR - pmis;
    // patch by LDS-DMA (global_load_lds_dword, no VGPR staging): per keypoint of the wave 37 rows x
    // 10 dwords = 370 dwords, linear in LDS (pitch 40), as 6 wave-instructions of lanes
    // d = 64q + lane < 370; the keypoint's patch origin and level pitch are wave-uniform (readlane)
    uint8_t* patch = s_patch[wave * 4 + sub];
    {
        const uint64_t pg = (uint64_t)(uintptr_t)(bl + pbase);
        int rq[6], cq[6];
#pragma unroll
        for (int q = 0; q < 6; q++) {
            const int d = 64 * q + lane;
            rq[q] = d / 10;
            cq[q] = 4 * (d - 10 * rq[q]);
        }
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pg, 16 * s);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pg >> 32), 16 * s);
            const uint8_t* sb = (const uint8_t*)(uintptr_t)(((uint64_t)hi << 32) | lo);
            const int sbp = __builtin_amdgcn_readlane(bp, 16 * s);
            uint8_t* dst = s_patch[wave * 4 + s];
#pragma unroll
            for (int q = 0; q < 6; q++) {
                if (64 * q + lane < kDescPatchRows * kDescPatchPitch / 4)
                    __builtin_amdgcn_global_load_lds(
                        (__attribute__((address_space(1))) void*)(sb + (unsigned)(rq[q] * sbp + cq[q])),
                        (__attribute__((address_space(3))) void*)(dst + 256 * q), 4, 0, 0);
            }
        }
    }
    int m10, m01;
    {
        // per row ri = r + 2p: A' += sum (u+15) I, S += sum I, M' += 2p * sum I (24-bit multiply by a
        // constant); then m10 = A' - 15 S and m01 = M' + (r - 15) S
        uint32_t Ap = 0, S = 0, Mp = 0;
#pragma unroll
        for (int p = 0; p < 16; p++) {
            const int ri = r + 2 * p;
            const uint32_t al = (mis + (uint32_t)p * dmis) & 3u;
            const uint32_t I4 = __builtin_amdgcn_alignbyte(wv[p].y, wv[p].x, al);
            const int2 msk = s_ic[ri * 8 + g4];
            const uint32_t sI = __builtin_amdgcn_udot4(I4, (uint32_t)msk.y, 0u, false);
            Ap = __builtin_amdgcn_udot4(I4, (uint32_t)msk.x, Ap, false);
            S += sI;
            Mp += __umul24(sI, 2u * (uint32_t)p);
        }
        // 24-bit products (S < 2^24): full-rate v_mad_i32_i24, not a 64-bit / quarter-rate multiply
        m10 = row16_sum_i32((int)Ap - __mul24(15, (int)S));
        m01 = row16_sum_i32((int)Mp + __mul24(r - 15, (int)S));
    }
    const float angle = fast_atan2((float)m01, (float)m10);
    // computeOrbDescriptor (ORBextractor.cc:107-147)
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float theta = __fmul_rn(angle, factorPI);
    float sa, ca;
    glibc_sincosf(theta, &sa, &ca);
    const float a = ca, b = sa;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA patch writes have landed
    wave_sync();  // patch stores of the other lanes of this group
    const uint8_t* pc0 = patch + kDescPatchR * kDescPatchPitch + kDescPatchR + pmis;  // keypoint
    uint32_t myword = 0;  // descriptor bytes 2ln, 2ln+1 of this lane's keypoint = pairs 16ln .. 16ln+15
    {
        // Both points of a pair at once in packed f32 (v_pk_mul_f32 / v_pk_add_f32: per component the
        // same IEEE products and sums as the reference's x*b + y*a, no contraction). cvRound (RNE) by
        // adding 1.5*2^23: the sum's bits are 0x4B400000 + round(v) for |v| < 2^22, so the rounded
        // row/column feed v_mad_u32_u24 (low 24 bits 0x400000 + r) and the constant bias
        // K = 0x400000 * pitch + 0x4B400000 is removed once per address.
#pragma clang fp contract(off)
        const float2v A2 = {a, a}, B2 = {b, b};
        const float2v MAG = {12582912.f, 12582912.f};
        constexpr uint32_t K = 0x400000u * (uint32_t)kDescPatchPitch + 0x4B400000u;
#pragma unroll
        for (int j = 15; j >= 0; j--) {  // bit j is shifted up j times: v_cmp + v_addc per test
            // global table: pairs fetched 4 steps at a time (a scheduling fence per group keeps the compiler
            // from hoisting all 16 loads, i.e. 64 live VGPRs)
            const PatPt pp = s_pat[16 * j + ln];  // pair 16ln + j (transposed)
            const float2v X = {pp.x0, pp.x1}, Y = {pp.y0, pp.y1};
            float2v R = (X * B2 + Y * A2) + MAG;  // rows    round(x*b + y*a) of points 0, 1
            float2v C = (X * A2 - Y * B2) + MAG;  // columns round(x*a - y*b)
            // opaque to the optimizer: keeps the pairs packed (v_pk_*_f32) and the bit patterns unfolded
            asm("" : "+v"(R), "+v"(C));
            // (bit_cast of the whole pair: clang folds a bit_cast of a single vector element to undef here)
            const uint2v RB = __builtin_bit_cast(uint2v, R), CB = __builtin_bit_cast(uint2v, C);
            const uint32_t rb0 = RB.x, rb1 = RB.y, cb0 = CB.x, cb1 = CB.y;
            const uint32_t o0 = (rb0 & 0xFFFFFFu) * (uint32_t)kDescPatchPitch + cb0 - K;
            const uint32_t o1 = (rb1 & 0xFFFFFFu) * (uint32_t)kDescPatchPitch + cb1 - K;
            const int t0 = pc0[(int)o0];
            const int t1 = pc0[(int)o1];
            myword = myword + myword + (uint32_t)(t0 < t1);
        }
    }
    if (valid) {
        const long long o = (long long)f * kp_stride + outidx;
        ((uint16_t*)(out_desc + o * 32))[ln] = (uint16_t)myword;
        if (ln == 0) {
            orbx_kp kp;
            const float fx = (float)x, fy = (float)y;
            kp.x = l ? __fmul_rn(fx, lv.scale) : fx;
            kp.y = l ? __fmul_rn(fy, lv.scale) : fy;
            kp.size = lv.patch_size;
            kp.angle = angle;
            kp.response = (float)resp;
            kp.octave = l;
            out_kps[o] = kp;
        }
    }
    // the host path's results land in mapped host memory: visible to the CPU before the call's done word
    // (k_call_done, a later launch) is
    if (ep.host_out) __threadfence_system();
}

/* ----------------------------------------------------------------------------------- */
/* GaussianBlur + IC_Angle + rBRIEF in one kernel: no blurred pyramid in HBM.            */
/*                                                                                       */
/*  Per keypoint (x, y) the unblurred neighbourhood rows y-21..y+21 x 12 dwords from      */
/*  column cx0 = (x-22) & ~3 is staged in LDS by LDS-DMA (pitch 48; rows REFLECT_101 by   */
/*  address, columns clamped into the row and the two halo columns on either side        */
/*  patched as REFLECT_101 for keypoints near an edge). IC_Angle (ORBextractor.cc:77-104) */
/*  reads its 31x31 window there. After a workgroup barrier waves 0-2 blur the 16 patches  */
/*  in place (ORBextractor.cc:1085-1086), 6 patches per wave at 10 lanes each: lane = 4    */
/*  output columns (dword g = 1..10), a 7-row register window of float row sums walking    */
/*  the 43 rows; output row r (image row y-18+r) overwrites source row r, which no later   */
/*  row sum reads (a patch's lanes are lanes of one wave: they issue in lockstep and its   */
/*  LDS operations complete in order); wave 3 computes the 16 angles meanwhile. Row sums:  */
/*  ten v_dot4 per 4 outputs on the three aligned dwords around them (no alignbyte); the   */
/*  vertical sums, the rounding (SSE2 column path RNE, scalar tail half-up) are those of   */
/*  k_blur_strips, so every blurred byte rBRIEF samples equals the whole-level blur's.     */
/*  rBRIEF (ORBextractor.cc:107-147) then samples rows 0..36 as k_describe does.          */
/*  Requires 4-aligned level-0 rows (the DMA moves dwords); launch_describe falls back to */
/*  k_blur_strips + k_describe otherwise.                                                  */
/* ----------------------------------------------------------------------------------- */
constexpr int kFusedRows = 43;   // source rows y-21 .. y+21
constexpr int kFusedPitch = 48;  // 12 dwords: columns cx0 .. cx0+47 cover x-21 .. x+21 for any (x-22) & 3
constexpr int kFusedDwords = kFusedRows * kFusedPitch / 4;  // 516 per keypoint
#ifndef ORBX_FUSED_STRIDE
#define ORBX_FUSED_STRIDE 2088  // 522 dwords = 10 banks mod 64: the blur's 60 lanes of a wave hit 60 distinct banks
#endif
constexpr int kFusedStride = ORBX_FUSED_STRIDE;  // bytes between the keypoints' patches in LDS

// waves (x 4 keypoints) per k_describe_blur workgroup (2 waves: -0.2 %, 1 wave: -5 %, profiles/r05_ab_mf4_fw2.log,
// r05_ab_graphs_batch2.log)
#ifndef ORBX_FUSED_WAVES
#define ORBX_FUSED_WAVES 4
#endif
constexpr int kFusedWaves = ORBX_FUSED_WAVES;
constexpr int kFusedKps = 4 * kFusedWaves;

/* One lane's share of the in-place patch blur of k_describe_blur: output dword gd (patch columns 4gd..4gd+3,
 * image column col0 of the first) of rows 0..36 from source rows 0..42, walking down with a 7-row register
 * window. In place: output row r overwrites source row r after every lane of the wave read it (row sum r was
 * taken at step r-6), so all lanes of one patch must be lanes of one wave. */
__device__ __forceinline__ void blur_patch_column(uint8_t* patch, int gd, int col0, int vec_end) {
    {
        const uint32_t* src = (const uint32_t*)patch + (gd - 1);
        uint32_t* dsw = (uint32_t*)patch + gd;
        const bool tail = col0 + 3 >= vec_end;
        // taps 18 34 49 55 49 34 18 against bytes of dwords g-1 (a), g (b), g+1 (c): output j sums bytes j+1 .. j+7
        constexpr uint32_t A0 = 18u << 8 | 34u << 16 | 49u << 24, B0 = 55u | 49u << 8 | 34u << 16 | 18u << 24;
        constexpr uint32_t A1 = 18u << 16 | 34u << 24, B1 = 49u | 55u << 8 | 49u << 16 | 34u << 24, C1 = 18u;
        constexpr uint32_t A2 = 18u << 24, B2 = 34u | 49u << 8 | 55u << 16 | 49u << 24, C2 = 34u | 18u << 8;
        constexpr uint32_t B3 = 18u | 34u << 8 | 49u << 16 | 55u << 24, C3 = 49u | 34u << 8 | 18u << 16;
        auto rowsum = [&](int i, float2v& lo, float2v& hi) {
            const uint32_t a = src[i * (kFusedPitch / 4)], b = src[i * (kFusedPitch / 4) + 1],
                           c = src[i * (kFusedPitch / 4) + 2];
            // each dot chain starts at the bit pattern of 2^23, so a row sum s (< 2^16) lands as the float
            // 2^23 + s; one packed subtract of 2^23 per pair converts two sums exactly (for 4 cvt_f32_u32)
            constexpr uint32_t Z = 0x4B000000u;
            const uint32_t o0 = __builtin_amdgcn_udot4(a, A0, __builtin_amdgcn_udot4(b, B0, Z, false), false);
            const uint32_t o1 = __builtin_amdgcn_udot4(
                a, A1, __builtin_amdgcn_udot4(b, B1, __builtin_amdgcn_udot4(c, C1, Z, false), false), false);
            const uint32_t o2 = __builtin_amdgcn_udot4(
                a, A2, __builtin_amdgcn_udot4(b, B2, __builtin_amdgcn_udot4(c, C2, Z, false), false), false);
            const uint32_t o3 = __builtin_amdgcn_udot4(b, B3, __builtin_amdgcn_udot4(c, C3, Z, false), false);
            const float2v M23 = {8388608.f, 8388608.f};
            lo = __builtin_bit_cast(float2v, (uint2v){o0, o1}) - M23;
            hi = __builtin_bit_cast(float2v, (uint2v){o2, o3}) - M23;
        };
        float2v WL[7], WH[7];
#pragma unroll
        for (int m = 0; m < 6; m++) rowsum(m, WL[m], WH[m]);
        for (int r0 = 0; r0 < kDescPatchRows; r0 += 7) {
#pragma unroll
            for (int s = 0; s < 7; s++) {
                const int r = r0 + s;
                if (r < kDescPatchRows) {
                    const int ns = (s + 6) % 7;
                    rowsum(r + 6, WL[ns], WH[ns]);
                    const float2v av = blur_vsum(WL[s], WL[(s + 1) % 7], WL[(s + 2) % 7], WL[(s + 3) % 7],
                                                 WL[(s + 4) % 7], WL[(s + 5) % 7], WL[ns]);
                    const float2v bv = blur_vsum(WH[s], WH[(s + 1) % 7], WH[(s + 2) % 7], WH[(s + 3) % 7],
                                                 WH[(s + 4) % 7], WH[(s + 5) % 7], WH[ns]);
                    float o[4] = {av.x, av.y, bv.x, bv.y};
                    if (tail) {
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            if (col0 + i >= vec_end) o[i] = floorf(o[i] + 0.5f);
                    }
                    uint32_t packed = 0;
#pragma unroll
                    for (int i = 0; i < 4; i++) packed = __builtin_amdgcn_cvt_pk_u8_f32(o[i], (unsigned)i, packed);
                    dsw[r * (kFusedPitch / 4)] = packed;
                }
            }
        }
    }
}

__global__ __launch_bounds__(64 * kFusedWaves) void k_describe_blur(
    const uint8_t* __restrict__ frames, long long fstride, int pitch0, const uint8_t* __restrict__ pyr,
    ExtractParams ep, const LevelDesc* __restrict__ levels, const uint32_t* __restrict__ lvkey,
    const int* __restrict__ lvcnt, orbx_kp* __restrict__ out_kps, uint8_t* __restrict__ out_desc,
    int* __restrict__ out_counts, int kp_stride, const int* __restrict__ ptab) {
    __shared__ PatPt s_pat[256];
    __shared__ int2 s_ic[256];
    __shared__ __align__(16) uint8_t s_patch[kFusedKps][kFusedStride];
    __shared__ int s_bcx[kFusedKps], s_bve[kFusedKps];  // per patch: cx0, blur_vec_end (-1: no keypoint)
    __shared__ float4 s_trig[kFusedKps];  // per patch: (m10, m01) after IC_Angle, then (angle, cos, sin)
    // wave index through readfirstlane: the LDS-DMA destinations (m0) are scalar
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int sub = lane >> 4, ln = lane & 15;
    // XCD-aware block mapping as k_describe: every workgroup of a frame on one XCD
    const int G = (ep.kp_per_frame + kFusedKps - 1) / kFusedKps;
    int f, blk;
    {
        const int b = blockIdx.x;
        if ((gridDim.x / G) % 8 == 0) {
            const int k = b >> 3;
            f = (b & 7) + 8 * (k / G);
            blk = k % G;
        } else {
            f = b / G;
            blk = b % G;
        }
    }
    constexpr int NT = 64 * kFusedWaves;
    constexpr int kTab = (256 + NT - 1) / NT;
    PatPt my_pat[kTab];
    int2 my_ic[kTab];
#pragma unroll
    for (int q = 0; q < kTab; q++) {
        const int t = min(tid + q * NT, 255);
        my_pat[q] = kPatternT.t[t];
        my_ic[q] = ((const int2*)(ptab + ep.ic_off))[t];
    }
    const int g = (blk * kFusedWaves + wave) * 4 + sub;
    const int gc = min(g, ep.kp_per_frame - 1);
    const uint32_t kk_raw = lvkey[(long long)f * ep.kp_per_frame + gc];
    const int* cnt = lvcnt + f * ep.L;
    int cl[kMaxLevels];
#pragma unroll
    for (int q = 0; q < kMaxLevels; q++) cl[q] = q < ep.L ? cnt[q] : 0;
#pragma unroll
    for (int q = 0; q < kTab; q++) {
        const int t = tid + q * NT;
        if (t >= 256) break;
        s_pat[t] = my_pat[q];
        s_ic[t] = my_ic[q];
    }
    if (blk == 0 && tid == 0) {
        int tot = 0;
#pragma unroll
        for (int q = 0; q < kMaxLevels; q++) tot += cl[q];
        out_counts[f] = tot;
        if (ep.host_out) __threadfence_system();
    }
    __syncthreads();
    // the keypoint's level, its index in the level and its output row (level_of, then the counts of the levels
    // below): one select chain over the frame's L levels (a uniform trip count), not three over kMaxLevels
    int l = 0, koff = 0, mycnt = cl[0], below = 0;
#pragma unroll
    for (int q = 1; q < kMaxLevels; q++) {
        if (q >= ep.L) break;  // wave-uniform
        const bool ge = gc >= ep.kp_off[q];
        l += ge ? 1 : 0;
        koff = ge ? ep.kp_off[q] : koff;
        below += ge ? cl[q - 1] : 0;
        mycnt = ge ? cl[q] : mycnt;
    }
    const int k = gc - koff;
    const int outidx = k + below;
    const bool valid = g < ep.kp_per_frame && k < mycnt;
    const bool wave_on = __ballot(valid) != 0;  // wave-uniform
    const LevelDesc lv = levels[l];
    const uint32_t kk = valid ? kk_raw : 0u;
    const int x = valid ? (int)(kk & 0xFFF) : 32, y = valid ? (int)((kk >> 12) & 0xFFF) : 32;
    const int resp = (int)(kk >> 24);
    const uint8_t* img = l == 0 ? frames + (long long)f * fstride : pyr + (long long)f * ep.pyr_frame_bytes + lv.pyr_off;
    const int pitch = l == 0 ? pitch0 : lv.pitch;
    const int cx0 = (x - 22) & ~3;  // image column of patch column 0
    const int pm = (x - 22) & 3;    // x = cx0 + 22 + pm
    const int lastd = (lv.w - 1) & ~3;
    // a patch that reaches past an image edge (REFLECT_101 rows or halo columns) or whose last dword lies past the
    // row's last valid dword takes the clamped / reflected staging
    const int edge = (y < 21 || y + 21 >= lv.h || x < 22 || x + 21 >= lv.w || cx0 + 44 > lastd) ? 1 : 0;
    uint8_t* patch = s_patch[wave * 4 + sub];
    if (wave_on) {  // a wave without keypoints stages nothing (it still reaches the barriers)
        // dword d = 64 q + lane of a window is row rq = d / 12, byte 4 (d - 12 rq): at row pitch sp its source
        // offset is rq (sp - 48) + 4 d, kept per q for the pitch of the last staged keypoint (the 4 keypoints of a
        // wave are mostly of one level, so it is computed once per wave and a load is saddr + that voffset)
        int rq[9], offq[9];
        int cur_sp = -1;
#pragma unroll
        for (int q = 0; q < 9; q++) {
            const int d = 64 * q + lane;
            rq[q] = d / 12;
            offq[q] = 0;
        }
        const uint64_t ib = (uint64_t)(uintptr_t)img;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ib, 16 * s);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ib >> 32), 16 * s);
            const uint8_t* sb = (const uint8_t*)(uintptr_t)(((uint64_t)hi << 32) | lo);
            const int sp = __builtin_amdgcn_readlane(pitch, 16 * s);
            const int sy = __builtin_amdgcn_readlane(y, 16 * s);
            const int scx = __builtin_amdgcn_readlane(cx0, 16 * s);
            uint8_t* dst = s_patch[wave * 4 + s];
            if (__builtin_amdgcn_readlane(edge, 16 * s) == 0) {
                if (sp != cur_sp) {  // wave-uniform
                    cur_sp = sp;
#pragma unroll
                    for (int q = 0; q < 9; q++) offq[q] = __mul24(rq[q], sp - 48) + 4 * (64 * q + lane);
                }
                const uint8_t* b0 = sb + (long long)(sy - 21) * sp + scx;
#pragma unroll
                for (int q = 0; q < 9; q++) {
                    if (64 * q + lane < kFusedDwords)
                        __builtin_amdgcn_global_load_lds(
                            (__attribute__((address_space(1))) void*)(b0 + (unsigned)offq[q]),
                            (__attribute__((address_space(3))) void*)(dst + 256 * q), 4, 0, 0);
                }
            } else {
                const int sh = __builtin_amdgcn_readlane(lv.h, 16 * s);
                const int sld = __builtin_amdgcn_readlane(lastd, 16 * s);
#pragma unroll
                for (int q = 0; q < 9; q++) {
                    if (64 * q + lane < kFusedDwords) {
                        const int rr = reflect101(sy - 21 + rq[q], sh);
                        const int cc = iclamp(scx + 4 * (64 * q + lane) - 48 * rq[q], 0, sld);
                        __builtin_amdgcn_global_load_lds(
                            (__attribute__((address_space(1))) void*)(sb + (unsigned)(__mul24(rr, sp) + cc)),
                            (__attribute__((address_space(3))) void*)(dst + 256 * q), 4, 0, 0);
                    }
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA writes have landed
    wave_sync();
    // REFLECT_101 halo columns of edge patches: image columns -1, -2 <- 1, 2 and w, w+1 <- w-2, w-3
#pragma unroll
    for (int s = 0; s < 4; s++) {
        if (__builtin_amdgcn_readlane(edge, 16 * s) == 0) continue;
        const int scx = __builtin_amdgcn_readlane(cx0, 16 * s);
        const int sw = __builtin_amdgcn_readlane(lv.w, 16 * s);
        if (lane < kFusedRows) {
            uint8_t* row = s_patch[wave * 4 + s] + lane * kFusedPitch;
#pragma unroll
            for (int q = 1; q <= 2; q++) {
                const int lc = -q - scx;
                if (lc >= 0) row[lc] = row[q - scx];
            }
#pragma unroll
            for (int q = 0; q <= 1; q++) {
                const int lc = sw + q - scx;
                if (lc < kFusedPitch) row[lc] = row[sw - 2 - q - scx];
            }
        }
    }
    wave_sync();
    int m10, m01;
    {
        // IC_Angle window: image rows y-15+ri = patch row ri+6, columns x-15+4g4.. = patch column 7+pm+4g4
        const int g4 = ln & 7, r = ln >> 3;
        const int c0 = 7 + pm + 4 * g4;
        const uint32_t al = (uint32_t)c0 & 3u;
        const uint32_t* pw = (const uint32_t*)patch + (c0 >> 2);
        uint32_t Ap = 0, S = 0, Mp = 0;
#pragma unroll
        for (int p = 0; p < 16; p++) {
            const int ri = r + 2 * p;
            const uint32_t w0 = pw[(ri + 6) * (kFusedPitch / 4)], w1 = pw[(ri + 6) * (kFusedPitch / 4) + 1];
            const uint32_t I4 = __builtin_amdgcn_alignbyte(w1, w0, al);
            const int2 msk = s_ic[ri * 8 + g4];
            const uint32_t sI = __builtin_amdgcn_udot4(I4, (uint32_t)msk.y, 0u, false);
            Ap = __builtin_amdgcn_udot4(I4, (uint32_t)msk.x, Ap, false);
            S += sI;
            Mp += __umul24(sI, 2u * (uint32_t)p);
        }
        // 24-bit products (S < 2^24): full-rate v_mad_i32_i24, not a 64-bit / quarter-rate multiply
        m10 = row16_sum_i32((int)Ap - __mul24(15, (int)S));
        m01 = row16_sum_i32((int)Mp + __mul24(r - 15, (int)S));
    }
    float angle, a, b;
    // blur across the workgroup: wave w blurs patches 6w .. 6w+5 with 10 lanes each (60 of 64 lanes busy,
    // 3 waves for 16 patches instead of 4 at 10 of 16), after every wave's IC_Angle read its raw rows. The
    // last wave, which has no blur share, computes the 16 keypoints' angle / cos / sin once each meanwhile
    // (instead of on all 16 lanes of every keypoint in every wave)
    static_assert((kFusedWaves - 1) * 6 >= kFusedKps, "the last wave has no blur share");
    if (ln == 0) {
        s_bcx[wave * 4 + sub] = cx0;  // negative near the left edge
        s_bve[wave * 4 + sub] = valid ? lv.blur_vec_end : -1;
        s_trig[wave * 4 + sub] = make_float4((float)m10, (float)m01, 0.f, 0.f);
    }
    __syncthreads();
    if (wave == kFusedWaves - 1) {
        if (lane < kFusedKps) {
            const float4 m = s_trig[lane];
            const float ang = fast_atan2(m.y, m.x);
            float sa, ca;
            glibc_sincosf(__fmul_rn(ang, (float)(3.14159265358979323846 / 180.f)), &sa, &ca);
            s_trig[lane] = make_float4(ang, ca, sa, 0.f);
        }
    } else {
        const int kq = wave * 6 + lane / 10, gd = lane - 10 * (lane / 10) + 1;
        if (lane < 60 && kq < kFusedKps) {
            const int bve = s_bve[kq];
            if (bve >= 0) blur_patch_column(s_patch[kq], gd, s_bcx[kq] + 4 * gd, bve);
        }
    }
    __syncthreads();
    if (!wave_on) return;  // wave-uniform, past the last barrier
    {
        const float4 t = s_trig[wave * 4 + sub];
        angle = t.x;
        a = t.y;
        b = t.z;
    }
    // blurred row r = image row y-18+r; image column x+dx = patch column 22+pm+dx
    const uint8_t* pc0 = patch + kDescPatchR * kFusedPitch + 22 + pm;
    uint32_t myword = 0;
    {
#pragma clang fp contract(off)
        const float2v A2v = {a, a}, B2v = {b, b};
        const float2v MAG = {12582912.f, 12582912.f};
        constexpr uint32_t K = 0x400000u * (uint32_t)kFusedPitch + 0x4B400000u;
#pragma unroll
        for (int j = 15; j >= 0; j--) {  // bit j is shifted up j times: v_cmp + v_addc per test
            const PatPt pp = s_pat[16 * j + ln];
            const float2v X = {pp.x0, pp.x1}, Y = {pp.y0, pp.y1};
            float2v R = (X * B2v + Y * A2v) + MAG;
            float2v C = (X * A2v - Y * B2v) + MAG;
            asm("" : "+v"(R), "+v"(C));
            const uint2v RB = __builtin_bit_cast(uint2v, R), CB = __builtin_bit_cast(uint2v, C);
            const uint32_t o0 = (RB.x & 0xFFFFFFu) * (uint32_t)kFusedPitch + CB.x - K;
            const uint32_t o1 = (RB.y & 0xFFFFFFu) * (uint32_t)kFusedPitch + CB.y - K;
            const int t0 = pc0[(int)o0];
            const int t1 = pc0[(int)o1];
            myword = myword + myword + (uint32_t)(t0 < t1);
        }
    }
    if (valid) {
        const long long o = (long long)f * kp_stride + outidx;
        ((uint16_t*)(out_desc + o * 32))[ln] = (uint16_t)myword;
        if (ln == 0) {
            orbx_kp kp;
            const float fx = (float)x, fy = (float)y;
            kp.x = l ? __fmul_rn(fx, lv.scale) : fx;
            kp.y = l ? __fmul_rn(fy, lv.scale) : fy;
            kp.size = lv.patch_size;
            kp.angle = angle;
            kp.response = (float)resp;
            kp.octave = l;
            out_kps[o] = kp;
        }
    }
    if (ep.host_out) __threadfence_system();
}

/* self-test hook: the device restatement of glibc sinf/cosf on an array (tests only) */
__global__ void k_sincos_selftest(const float* __restrict__ in, float* __restrict__ s, float* __restrict__ c, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) glibc_sincosf(in[i], s + i, c + i);
}

}  // namespace orbamd

/* ----------------------------------------------------------------------------------- */
/* host-side launchers (called from capi.cpp)                                           */
/* ----------------------------------------------------------------------------------- */
#include "launch.h"

namespace orbamd {

hipError_t launch_resize(const uint8_t* src, long long src_fstride, int src_pitch, int sw, int sh, uint8_t* dst,
                         long long dst_fstride, int dst_pitch, int dw, int dh, const int* coef, int xmax,
                         int simd_end, int nframes, hipStream_t st) {
    const int* xofs = coef;
    const short2* alpha = (const short2*)(coef + dw);
    const int* yofs = coef + 2 * dw;
    const short2* beta = (const short2*)(coef + 2 * dw + dh);
    dim3 grid((dw + 255) / 256, (dh + 3) / 4, nframes);
    hipLaunchKernelGGL(k_resize_level, grid, dim3(256), 0, st, src, src_fstride, src_pitch, sw, sh, dst,
                       dst_fstride, dst_pitch, dw, dh, xofs, alpha, yofs, beta, xmax, simd_end);
    return hipGetLastError();
}

hipError_t launch_pyramid_frames(const uint8_t* frames, long long fstride, int pitch0, uint8_t* pyr,
                                 const ExtractParams& ep, const LevelDesc* levels, const int* ptab, int max_rows,
                                 int max_groups, int nframes, hipStream_t st, const int2* bands, int nbands) {
    if (max_rows < 1 || max_rows > kPyrMaxRows) return hipErrorInvalidValue;
    const size_t lds = (size_t)max_rows * sizeof(int4);
    if (bands) {  // row bands: 1024 threads, so a band's rows of a level are one or two passes
        if (nbands < 1) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_pyramid_frames<kPyrUMax, kPyrThreadsMax>), dim3(nbands, nframes), dim3(kPyrThreadsMax),
                           lds, st, frames, fstride, pitch0, pyr, ep, levels, ptab, bands);
        return hipGetLastError();
    }
    // 512-thread workgroups pack beside the other graphs' kernels while every level
    // keeps >= 2 rows per pass; a level 1 wider than 4 x 256 columns (C4's 1034) would leave half the
    // threads idle, so such geometries take 1024 threads
    if (max_groups <= kPyrThreads / 2)
        hipLaunchKernelGGL((k_pyramid_frames<kPyrU, kPyrThreads>), dim3(nframes), dim3(kPyrThreads), lds, st, frames,
                           fstride, pitch0, pyr, ep, levels, ptab, (const int2*)nullptr);
    else
        hipLaunchKernelGGL((k_pyramid_frames<kPyrUMax, kPyrThreadsMax>), dim3(nframes), dim3(kPyrThreadsMax), lds, st,
                           frames, fstride, pitch0, pyr, ep, levels, ptab, (const int2*)nullptr);
    return hipGetLastError();
}

hipError_t launch_resize_tiled(const uint8_t* src, long long src_fstride, int src_pitch, int sw, int sh, uint8_t* dst,
                               long long dst_fstride, int dst_pitch, int dw, int dh, const int* coef, int xmax,
                               int simd_end, int nframes, hipStream_t st) {
    const int* xofs = coef;
    const short2* alpha = (const short2*)(coef + dw);
    const int* yofs = coef + 2 * dw;
    const short2* beta = (const short2*)(coef + 2 * dw + dh);
    dim3 grid((dw + kRsTW - 1) / kRsTW, (dh + kRsTH - 1) / kRsTH, nframes);
    hipLaunchKernelGGL(k_resize_tiled, grid, dim3(256), 0, st, src, src_fstride, src_pitch, sw, sh, dst, dst_fstride,
                       dst_pitch, dw, dh, xofs, alpha, yofs, beta, xmax, simd_end);
    return hipGetLastError();
}

int resize_tile_fits(const int* xofs, const int* yofs, int sw, int sh, int dw, int dh) {
    for (int c0 = 0; c0 < dw; c0 += kRsTW) {
        const int c1 = c0 + kRsTW < dw ? c0 + kRsTW : dw;
        const int hi = xofs[c1 - 1] + 1 < sw - 1 ? xofs[c1 - 1] + 1 : sw - 1;
        if (hi - xofs[c0] + 1 + 3 + 4 > kRsW) return 0;
    }
    for (int r0 = 0; r0 < dh; r0 += kRsTH) {
        const int r1 = r0 + kRsTH < dh ? r0 + kRsTH : dh;
        const int lo = iclamp_host(yofs[r0], 0, sh - 1), hi = iclamp_host(yofs[r1 - 1] + 1, 0, sh - 1);
        if (hi - lo + 1 > kRsH) return 0;
    }
    return 1;
}

hipError_t launch_fast_cells2(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                              const ExtractParams& ep, const LevelDesc* levels, const CellDesc* cells,
                              uint32_t* cellkey, int* cellcnt, int RP, int RH, int max_pass, int cell_lo,
                              int cell_hi, int nframes, hipStream_t st) {
    if (cell_hi <= cell_lo) return hipSuccess;
    dim3 grid((cell_hi - cell_lo + kFastWaves - 1) / kFastWaves, nframes);
    const size_t lds = kFastWaves * (size_t)fast_wave_lds(RP, RH);
#define ORBX_FAST(MP, RPC)                                                                                        \
    hipLaunchKernelGGL((k_fast_cells2<MP, RPC>), grid, dim3(64 * kFastWaves), lds, st, frames, fstride, pitch0, pyr, ep, levels, \
                       cells, cellkey, cellcnt, RP, RH, cell_lo, cell_hi)
    if (max_pass <= 8 && RP == 40)
        ORBX_FAST(8, 40);
    else if (max_pass <= 8 && RP == 44)
        ORBX_FAST(8, 44);
    else if (max_pass <= 8 && RP == 48)
        ORBX_FAST(8, 48);
    else if (max_pass <= 8)
        ORBX_FAST(8, 0);
    else if (max_pass <= 12)
        ORBX_FAST(12, 0);
    else
        ORBX_FAST(24, 0);
#undef ORBX_FAST
    return hipGetLastError();
}

hipError_t launch_fast_blur(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                            const ExtractParams& ep, const LevelDesc* levels, const CellDesc* cells, uint32_t* cellkey,
                            int* cellcnt, int RP, int RH, int max_pass, uint8_t* blur, const ExtractParams& eb,
                            int njobs, int nframes, hipStream_t st) {
    const int nfast = (ep.ncells + 3) / 4;
    dim3 grid(nfast + (njobs + 3) / 4, nframes);
    const size_t lds = std::max((size_t)4 * fast_wave_lds(RP, RH), sizeof(uint8_t) * 4 * 7 * kBlurSeg);
    const bool aligned = (((uintptr_t)frames | (uintptr_t)fstride | (uintptr_t)pitch0) & 3) == 0;
#define ORBX_FAST(MP, RPC)                                                                                          \
    do {                                                                                                            \
        if (aligned)                                                                                                \
            hipLaunchKernelGGL((k_fast_blur<MP, RPC, true>), grid, dim3(256), lds, st, frames, fstride, pitch0, pyr,  \
                               ep, levels, cells, cellkey, cellcnt, RP, RH, 0, ep.ncells, nfast, blur, eb, njobs);   \
        else                                                                                                        \
            hipLaunchKernelGGL((k_fast_blur<MP, RPC, false>), grid, dim3(256), lds, st, frames, fstride, pitch0, pyr, \
                               ep, levels, cells, cellkey, cellcnt, RP, RH, 0, ep.ncells, nfast, blur, eb, njobs);   \
    } while (0)
    if (max_pass <= 8 && RP == 40)
        ORBX_FAST(8, 40);
    else if (max_pass <= 8 && RP == 44)
        ORBX_FAST(8, 44);
    else if (max_pass <= 8 && RP == 48)
        ORBX_FAST(8, 48);
    else if (max_pass <= 8)
        ORBX_FAST(8, 0);
    else if (max_pass <= 12)
        ORBX_FAST(12, 0);
    else
        ORBX_FAST(24, 0);
#undef ORBX_FAST
    return hipGetLastError();
}

hipError_t launch_sincos_selftest(const float* in, float* so, float* co, int n, hipStream_t st) {
    hipLaunchKernelGGL(k_sincos_selftest, dim3((n + 255) / 256), dim3(256), 0, st, in, so, co, n);
    return hipGetLastError();
}

hipError_t octree_setup(int lds_bytes) {
    hipError_t e = hipFuncSetAttribute((const void*)k_octree<256>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)k_octree<512>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute((const void*)k_octree<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

hipError_t launch_octree(const ExtractParams& ep, const LevelDesc* levels, const CellDesc* cells,
                         const uint32_t* cellkey, const int* cellcnt, uint32_t* lvkey, int* lvcnt,
                         uint8_t* gscratch, long long gscratch_frame_bytes, int NC, int KL, int lds_bytes,
                         int* err, int nframes, hipStream_t st, int level0, int nlevels, const HostCopy* copy) {
    if (nlevels < 0) nlevels = ep.L - level0;
    if (level0 < 0 || nlevels < 1 || level0 + nlevels > ep.L) return hipErrorInvalidValue;
    HostCopy hc{nullptr, nullptr, 0, 0};
    if (copy) {
        // one frame only: the copy blocks sit at the end of grid.x, and grid.y would repeat them per frame
        if (nframes != 1 || copy->nblocks < 1 || copy->n16 < 0) return hipErrorInvalidValue;
        hc = *copy;
    }
    dim3 grid(nlevels + hc.nblocks, nframes);
    // a small batch (one frame per Tracking call) has a workgroup per level and nothing beside it: 16 waves walk
    // each round's keys in a quarter of the iterations; batches pack four 256-thread workgroups per CU instead
    if (nframes < kPyrFramesMinBatch)
        hipLaunchKernelGGL(k_octree<1024>, grid, dim3(1024), lds_bytes, st, ep, levels, cells, cellkey, cellcnt, lvkey,
                           lvcnt, gscratch, gscratch_frame_bytes, NC, KL, level0, err, hc);
    else if (NC > 256)  // levels of up to 512 live nodes (C4's 2000 features): every round node-per-thread
        hipLaunchKernelGGL(k_octree<512>, grid, dim3(512), lds_bytes, st, ep, levels, cells, cellkey, cellcnt, lvkey,
                           lvcnt, gscratch, gscratch_frame_bytes, NC, KL, level0, err, hc);
    else
        hipLaunchKernelGGL(k_octree<256>, grid, dim3(256), lds_bytes, st, ep, levels, cells, cellkey, cellcnt, lvkey,
                           lvcnt, gscratch, gscratch_frame_bytes, NC, KL, level0, err, hc);
    return hipGetLastError();
}

hipError_t launch_blur_strips(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr, uint8_t* blur,
                              const ExtractParams& ep, const LevelDesc* levels, int job0, int job1, const int* lvcnt,
                              int nframes, hipStream_t st, int rows) {
    if (job1 <= job0) return hipSuccess;
    if (rows != kBlurRows && rows != kBlurRowsSmall) return hipErrorInvalidValue;
    dim3 grid((job1 - job0 + 3) / 4, nframes);
    const bool aligned = (((uintptr_t)frames | (uintptr_t)fstride | (uintptr_t)pitch0) & 3) == 0;
    // ep.bjob_begin must be the job table of `rows`-row chunks (Geometry::bjob_begin / bjob_small)
    if (rows == kBlurRows) {
        if (aligned)
            hipLaunchKernelGGL((k_blur_strips<true, kBlurRows>), grid, dim3(256), 0, st, frames, fstride, pitch0, pyr,
                               blur, ep, levels, job0, job1, lvcnt);
        else
            hipLaunchKernelGGL((k_blur_strips<false, kBlurRows>), grid, dim3(256), 0, st, frames, fstride, pitch0, pyr,
                               blur, ep, levels, job0, job1, lvcnt);
    } else {
        if (aligned)
            hipLaunchKernelGGL((k_blur_strips<true, kBlurRowsSmall>), grid, dim3(256), 0, st, frames, fstride, pitch0,
                               pyr, blur, ep, levels, job0, job1, lvcnt);
        else
            hipLaunchKernelGGL((k_blur_strips<false, kBlurRowsSmall>), grid, dim3(256), 0, st, frames, fstride, pitch0,
                               pyr, blur, ep, levels, job0, job1, lvcnt);
    }
    return hipGetLastError();
}

hipError_t launch_describe(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                           const uint8_t* blur, const ExtractParams& ep, const LevelDesc* levels,
                           const uint32_t* lvkey, const int* lvcnt, orbx_kp* out_kps, uint8_t* out_desc,
                           int* out_counts, int kp_stride, const int* ptab, int nframes, hipStream_t st) {
    dim3 grid(((ep.kp_per_frame + kDescKps - 1) / kDescKps) * nframes);
    if ((pitch0 & 1) == 0)
        hipLaunchKernelGGL(k_describe<true>, grid, dim3(64 * kDescWaves), 0, st, frames, fstride, pitch0, pyr, blur, ep,
                           levels, lvkey, lvcnt, out_kps, out_desc, out_counts, kp_stride, ptab);
    else
        hipLaunchKernelGGL(k_describe<false>, grid, dim3(64 * kDescWaves), 0, st, frames, fstride, pitch0, pyr, blur, ep,
                           levels, lvkey, lvcnt, out_kps, out_desc, out_counts, kp_stride, ptab);
    return hipGetLastError();
}

bool describe_blur_ok(const uint8_t* frames, long long fstride, int pitch0) {
    return ((((uintptr_t)frames | (uintptr_t)fstride | (uintptr_t)pitch0) & 3) == 0);
}

hipError_t launch_describe_blur(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                                const ExtractParams& ep, const LevelDesc* levels, const uint32_t* lvkey,
                                const int* lvcnt, orbx_kp* out_kps, uint8_t* out_desc, int* out_counts, int kp_stride,
                                const int* ptab, int nframes, hipStream_t st) {
    if (!describe_blur_ok(frames, fstride, pitch0)) return hipErrorInvalidValue;
    dim3 grid(((ep.kp_per_frame + kFusedKps - 1) / kFusedKps) * nframes);
    hipLaunchKernelGGL(k_describe_blur, grid, dim3(64 * kFusedWaves), 0, st, frames, fstride, pitch0, pyr, ep, levels,
                       lvkey, lvcnt, out_kps, out_desc, out_counts, kp_stride, ptab);
    return hipGetLastError();
}

}  // namespace orbamd

#ifdef ORBX_OCT_TRACE
extern "C" int orbx_debug_octree_trace(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbamd::g_oct_trace), sizeof(orbamd::g_oct_trace)) == hipSuccess ? 0 : -1;
}
#endif
