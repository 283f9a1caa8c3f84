/*
 * frame_kernels.hip -- gfx950 kernels for the Frame-level consumers of the extractor output
 * (SURVEY.md 8(f)).
 *
 *   k_stereo   Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641), one workgroup
 *              per stereo pair of a batch: right keypoints bucketed by their row band in LDS
 *              (counting sort replaces vRowIndices, Frame.cc:477-498), one wave per left
 *              keypoint for the band/octave/disparity-filtered Hamming search (the minimum of
 *              (dist, iR) is the reference's first-strict-minimum, so bucket order is free),
 *              the 11x11 SAD over 11 shifts on the device-resident pyramids staged per wave in
 *              LDS (integers: exact, as cv::norm's double sum of integer-valued floats is),
 *              the parabola fit in IEEE float (no contraction), then the per-frame median
 *              rejection (Frame.cc:636-650) as an LDS radix select.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbslam_amd.h"
#include "orb_frame.h"

namespace orbamd {

constexpr int kStereoThreads = 1024;
constexpr int kStereoWaves = kStereoThreads / 64;
constexpr int kStereoWaveBytes = 124 + 232 + 4 * 56 + 4 * 12;  // IL 11x11, IR 11x21, SAD parts, totals

/* dynamic LDS layout of k_stereo for kp capacity `cap` and `nrows` level-0 rows */
struct StereoLds {
    int rx, rband, roct, sorted, row, sad, wave, hist, misc, total;
    __host__ __device__ StereoLds(int cap, int nrows) {
        const int c4 = (cap + 3) & ~3;
        rx = 0;
        rband = rx + 4 * c4;
        roct = rband + 4 * c4;
        sorted = roct + c4;
        row = sorted + 2 * c4;
        sad = row + 4 * ((nrows + 2 + 3) & ~3);
        wave = sad + 4 * c4;
        hist = wave + kStereoWaves * kStereoWaveBytes;
        misc = hist + 4 * 512;
        total = misc + 4 * 8;
    }
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

__device__ __forceinline__ const uint8_t* level_base(const PyrSide& s, const StereoArgs& a, int f, int l,
                                                     int* pitch) {
    if (l == 0) {
        *pitch = s.l0_pitch;
        return s.l0 + (long long)f * s.l0_fstride;
    }
    *pitch = a.lpitch[l];
    return s.pyr + (long long)f * s.pyr_fstride + a.pyr_off[l];
}

__global__ __launch_bounds__(kStereoThreads) void k_stereo(StereoArgs a, const int32_t* __restrict__ fl_idx,
                                                           const int32_t* __restrict__ fr_idx,
                                                           const orbx_kp* __restrict__ kpsL,
                                                           const uint8_t* __restrict__ descL,
                                                           const int32_t* __restrict__ cntL,
                                                           const orbx_kp* __restrict__ kpsR,
                                                           const uint8_t* __restrict__ descR,
                                                           const int32_t* __restrict__ cntR, int stride,
                                                           float* __restrict__ uright, float* __restrict__ depth,
                                                           int32_t* __restrict__ nstereo, int* __restrict__ err) {
    extern __shared__ __align__(16) uint8_t lds[];
    const StereoLds o(stride, a.nrows);
    float* s_rx = (float*)(lds + o.rx);
    int* s_rband = (int*)(lds + o.rband);
    int8_t* s_roct = (int8_t*)(lds + o.roct);
    uint16_t* s_sorted = (uint16_t*)(lds + o.sorted);
    int* s_row = (int*)(lds + o.row);
    int* s_sad = (int*)(lds + o.sad);
    int* s_hist = (int*)(lds + o.hist);
    int* s_misc = (int*)(lds + o.misc);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int p = blockIdx.x;
    const int fl = fl_idx[p], fr = fr_idx[p];
    if (fl < 0 || fl >= a.left.nframes || fr < 0 || fr >= a.right.nframes) {
        if (tid == 0) atomicOr(err, 4);
        return;
    }
    const int nL = cntL[fl], nR = cntR[fr];
    if (nL < 0 || nL > stride || nR < 0 || nR > stride) {
        if (tid == 0) atomicOr(err, 4);
        return;
    }
    const orbx_kp* kL = kpsL + (long long)fl * stride;
    const orbx_kp* kR = kpsR + (long long)fr * stride;
    const uint8_t* dL = descL + (long long)fl * stride * 32;
    const uint8_t* dR = descR + (long long)fr * stride * 32;
    float* ur = uright + (long long)p * stride;
    float* dp = depth + (long long)p * stride;
    const int nrows = a.nrows;

    // mvuRight = mvDepth = -1 (Frame.cc:472-473); row-bucket counts
    for (int i = tid; i < nL; i += kStereoThreads) {
        ur[i] = -1.0f;
        dp[i] = -1.0f;
        s_sad[i] = -1;
    }
    for (int i = tid; i <= nrows + 1; i += kStereoThreads) s_row[i] = 0;
    for (int i = tid; i < 512; i += kStereoThreads) s_hist[i] = 0;
    if (tid < 8) s_misc[tid] = 0;
    __syncthreads();
    // row band of each right keypoint (Frame.cc:487-498): rows minr..maxr
    for (int iR = tid; iR < nR; iR += kStereoThreads) {
        const orbx_kp k = kR[iR];
        const float r = __fmul_rn(2.0f, a.scale[k.octave]);
        const int maxr = (int)ceilf(__fadd_rn(k.y, r));
        const int minr = (int)floorf(__fsub_rn(k.y, r));
        s_rx[iR] = k.x;
        s_rband[iR] = (minr & 0xffff) | (maxr << 16);
        s_roct[iR] = (int8_t)k.octave;
        const int b = min(max(minr, 0), nrows - 1);
        atomicAdd(&s_row[b + 1], 1);
    }
    __syncthreads();
    // exclusive scan of the bucket counts (s_row[b+1] = count of bucket b) by wave 0
    if (wv == 0) {
        const int C = (nrows + 63) / 64;
        const int b0 = min(lane * C, nrows), b1 = min(b0 + C, nrows);
        int sum = 0;
        for (int b = b0; b < b1; b++) sum += s_row[b + 1];
        int incl = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        int run = incl - sum;
        for (int b = b0; b < b1; b++) {
            const int c = s_row[b + 1];
            s_row[b + 1] = run;
            run += c;
        }
    }
    __syncthreads();
    // scatter: afterwards bucket b = s_sorted[s_row[b] .. s_row[b+1])
    for (int iR = tid; iR < nR; iR += kStereoThreads) {
        const int minr = (int)(int16_t)(s_rband[iR] & 0xffff);
        const int b = min(max(minr, 0), nrows - 1);
        const int pos = atomicAdd(&s_row[b + 1], 1);
        s_sorted[pos] = (uint16_t)iR;
    }
    __syncthreads();

    uint8_t* s_il = lds + o.wave + wv * kStereoWaveBytes;
    uint8_t* s_ir = s_il + 124;
    int* s_part = (int*)(s_ir + 232);
    int* s_tot = s_part + 56;
    for (int iL = wv; iL < nL; iL += kStereoWaves) {
        const orbx_kp kpL = kL[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const int v = (int)vL;  // vRowIndices[vL] (Frame.cc:514)
        if (!(vL >= 0.f) || v >= nrows) continue;
        const float minU = __fsub_rn(uL, a.maxD);
        const float maxU = __fsub_rn(uL, 0.0f);
        if (maxU < 0) continue;
        const uint4* qd = (const uint4*)(dL + (long long)iL * 32);
        const uint4 q0 = qd[0], q1 = qd[1];
        const int cb = s_row[max(v - a.rspan, 0)], ce = s_row[v + 1];
        uint32_t best = 0xffffffffu;
        for (int c0 = cb; c0 < ce; c0 += 64) {  // Frame.cc:531-550
            const int c = c0 + lane;
            if (c < ce) {
                const int iR = s_sorted[c];
                const int band = s_rband[iR];
                const int minr = (int)(int16_t)(band & 0xffff), maxr = band >> 16;
                const int oct = s_roct[iR];
                const float uR = s_rx[iR];
                if (minr <= v && v <= maxr && oct >= levelL - 1 && oct <= levelL + 1 && uR >= minU && uR <= maxU) {
                    const uint4* cd = (const uint4*)(dR + (long long)iR * 32);
                    const uint4 c0v = cd[0], c1v = cd[1];
                    const int dist = __popc(q0.x ^ c0v.x) + __popc(q0.y ^ c0v.y) + __popc(q0.z ^ c0v.z) +
                                     __popc(q0.w ^ c0v.w) + __popc(q1.x ^ c1v.x) + __popc(q1.y ^ c1v.y) +
                                     __popc(q1.z ^ c1v.z) + __popc(q1.w ^ c1v.w);
                    if (dist < 100) best = min(best, ((uint32_t)dist << 16) | (uint32_t)iR);  // TH_HIGH
                }
            }
        }
        best = wave_min_u32(best);
        if (best == 0xffffffffu || (int)(best >> 16) >= 75) continue;  // thOrbDist (Frame.cc:475, 553)
        const int bestIdxR = (int)(best & 0xffff);
        // sub-pixel match by correlation (Frame.cc:555-621)
        const float uR0 = s_rx[bestIdxR];
        const float sf = a.inv_scale[levelL];
        const float suL = roundf(__fmul_rn(uL, sf));
        const float svL = roundf(__fmul_rn(vL, sf));
        const float suR0 = roundf(__fmul_rn(uR0, sf));
        const float iniu = __fsub_rn(__fadd_rn(suR0, 5.0f), 5.0f);
        const float endu = __fadd_rn(__fadd_rn(__fadd_rn(suR0, 5.0f), 5.0f), 1.0f);
        const int lw = a.lw[levelL], lh = a.lh[levelL];
        if (iniu < 0 || endu >= (float)lw) continue;
        const int r0 = (int)__fsub_rn(svL, 5.0f), c0l = (int)__fsub_rn(suL, 5.0f), c0r = (int)__fsub_rn(suR0, 10.0f);
        if (r0 < 0 || r0 + 11 > lh || c0l < 0 || c0l + 11 > lw || c0r < 0 || c0r + 21 > lw) {
            if (lane == 0) atomicOr(err, 2);  // the reference's cv::Mat::colRange/rowRange would assert
            continue;
        }
        int pitchL, pitchR;
        const uint8_t* PL = level_base(a.left, a, fl, levelL, &pitchL) + (long long)r0 * pitchL + c0l;
        const uint8_t* PR = level_base(a.right, a, fr, levelL, &pitchR) + (long long)r0 * pitchR + c0r;
        for (int k = lane; k < 121; k += 64) s_il[k] = PL[(k / 11) * pitchL + k % 11];
        for (int k = lane; k < 231; k += 64) s_ir[k] = PR[(k / 21) * pitchR + k % 21];
        wave_lds_sync();
        int part = 0;
        if (lane < 55) {
            const int s = lane % 11, g = lane / 11;
            const int cL = s_il[5 * 11 + 5], cR = s_ir[5 * 21 + s + 5];
            for (int r = g; r < 11; r += 5)
#pragma unroll
                for (int c = 0; c < 11; c++)
                    part += abs((s_il[r * 11 + c] - cL) - (s_ir[r * 21 + s + c] - cR));
            s_part[lane] = part;
        }
        wave_lds_sync();
        if (lane < 11)
            s_tot[lane] = s_part[lane] + s_part[lane + 11] + s_part[lane + 22] + s_part[lane + 33] + s_part[lane + 44];
        wave_lds_sync();
        int bestS = 0x7fffffff, bi = 0;
        for (int s = 0; s < 11; s++) {
            const int d = s_tot[s];
            if (d < bestS) {
                bestS = d;
                bi = s;
            }
        }
        const float d1 = (float)s_tot[max(bi - 1, 0)], d2 = (float)s_tot[bi], d3 = (float)s_tot[min(bi + 1, 10)];
        wave_lds_sync();  // s_tot/s_il/s_ir are rewritten by this wave's next keypoint
        if (bi == 0 || bi == 10) continue;
        const float deltaR = __fdiv_rn(__fsub_rn(d1, d3), __fmul_rn(2.0f, __fsub_rn(__fadd_rn(d1, d3), __fmul_rn(2.0f, d2))));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = __fmul_rn(a.scale[levelL], __fadd_rn(__fadd_rn(suR0, (float)(bi - 5)), deltaR));
        float disparity = __fsub_rn(uL, bestuR);
        if (disparity >= 0.0f && disparity < a.maxD) {  // Frame.cc:623-633
            if (disparity <= 0) {
                disparity = 0.01f;
                bestuR = (float)((double)uL - 0.01);
            }
            if (lane == 0) {
                dp[iL] = __fdiv_rn(a.bf, disparity);
                ur[iL] = bestuR;
                s_sad[iL] = bestS;
            }
        }
    }
    __syncthreads();
    // median rejection (Frame.cc:636-650): k-th smallest SAD, k = n/2, by a two-digit radix select
    int nloc = 0;
    for (int i = tid; i < nL; i += kStereoThreads) {
        const int d = s_sad[i];
        if (d >= 0) {
            nloc++;
            atomicAdd(&s_hist[d >> 8], 1);
        }
    }
    if (nloc) atomicAdd(&s_misc[0], nloc);
    __syncthreads();
    const int n = s_misc[0];
    if (n == 0) {
        if (tid == 0) nstereo[p] = 0;
        return;
    }
    if (tid == 0) {
        int k = n / 2, hb = 0;
        while (k >= s_hist[hb]) k -= s_hist[hb++];
        s_misc[1] = hb;
        s_misc[2] = k;
    }
    __syncthreads();
    const int hb = s_misc[1];
    for (int i = tid; i < nL; i += kStereoThreads) {
        const int d = s_sad[i];
        if (d >= 0 && (d >> 8) == hb) atomicAdd(&s_hist[256 + (d & 255)], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int k = s_misc[2], lb = 0;
        while (k >= s_hist[256 + lb]) k -= s_hist[256 + lb++];
        s_misc[3] = (hb << 8) | lb;
    }
    __syncthreads();
    const float median = (float)s_misc[3];
    const float thDist = __fmul_rn(a.thc, median);
    int kept = 0;
    for (int i = tid; i < nL; i += kStereoThreads) {
        const int d = s_sad[i];
        if (d < 0) continue;
        if ((float)d < thDist) {
            kept++;
        } else {
            ur[i] = -1.0f;
            dp[i] = -1.0f;
        }
    }
    if (kept) atomicAdd(&s_misc[4], kept);
    __syncthreads();
    if (tid == 0) nstereo[p] = s_misc[4];
}

int stereo_lds_bytes(int cap, int nrows) { return StereoLds(cap, nrows).total; }

hipError_t stereo_setup(int lds_bytes) {
    return hipFuncSetAttribute((const void*)k_stereo, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

hipError_t launch_stereo(const StereoArgs& a, int npairs, const int32_t* fl, const int32_t* fr, const orbx_kp* kpsL,
                         const uint8_t* descL, const int32_t* cntL, const orbx_kp* kpsR, const uint8_t* descR,
                         const int32_t* cntR, int stride, float* uright, float* depth, int32_t* nstereo, int* err,
                         hipStream_t st) {
    const int lds = stereo_lds_bytes(stride, a.nrows);
    hipLaunchKernelGGL(k_stereo, dim3(npairs), dim3(kStereoThreads), lds, st, a, fl, fr, kpsL, descL, cntL, kpsR,
                       descR, cntR, stride, uright, depth, nstereo, err);
    return hipGetLastError();
}

}  // namespace orbamd
