/*
 * frame_kernels.hip -- gfx950 kernels for the Frame-level consumers of the extractor output
 * (SURVEY.md 8(f)).
 *
 *   k_stereo   Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641), 4 workgroups of
 *              256 threads per stereo pair of a batch: right keypoints bucketed by their row band in
 *              LDS (counting sort replaces vRowIndices, Frame.cc:477-498), 16 lanes per left
 *              keypoint for the band/octave/disparity-filtered Hamming search (the minimum of
 *              (dist, iR) is the reference's first-strict-minimum, so bucket order is free),
 *              the 11x11 SAD over 11 shifts (a lane per shift) on the device-resident pyramids
 *              staged per keypoint in LDS (integers: exact, as cv::norm's double sum of
 *              integer-valued floats is), the parabola fit in IEEE float (no contraction);
 *   k_stereo_median
 *              then the per-frame median rejection (Frame.cc:636-650) as an LDS radix select.
 *   k_grid     Frame::AssignFeaturesToGrid (Frame.cc:235-250, PosInGrid 391-401): CSR cell lists
 *              (counting sort in LDS; order inside a cell is free, see k_proj_scan).
 *   k_proj_scan / k_proj_resolve
 *              SearchByProjection x4 (ORBmatcher.cc:45-129, 290-403, 1328-1470, 1472-1599) with
 *              GetFeaturesInArea (Frame.cc:332-389, KeyFrame.cc:569-608). The scan gives every
 *              MapPoint query 16 lanes over the window's grid cells and keeps the best and
 *              second-best candidate as 64-bit keys (dist, window cell order, feature index):
 *              the reference's scan order is (cell, position in cell), position in a cell is
 *              ascending feature index, so the minimum key is its first strict minimum and the
 *              next key its `bestDist2` element. Matching assigns F.mvpMapPoints in MapPoint
 *              order and later MapPoints skip occupied features; a claim can only change a
 *              later result if it takes that query's best or second element, so the resolve
 *              wave commits 64 queries at a time up to the first such conflict, re-scans that
 *              one query against the live occupancy bitmap, and continues. Then the rotation
 *              histogram + ComputeThreeMaxima (ORBmatcher.cc:1437-1467, 1601-1642).
 *   k_init_resolve
 *              SearchForInitialization (ORBmatcher.cc:405-520) on the same grid + scan: in-order
 *              resolution against vMatchedDistance (accepts may take a feature from an earlier query).
 *   k_distinctive
 *              MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307) for a batch of
 *              MapPoints: one wave per MapPoint, row i of the Hamming distance matrix in LDS,
 *              its median (sorted element floor(0.5*(N-1))) by a 9-bit ballot radix select,
 *              first strict minimum of the medians.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbslam_amd.h"
#include "orb_frame.h"
#include "orb_wave.h"

namespace orbamd {

/* k_stereo: kStereoSplit workgroups of kStereoThreads per stereo pair, each over every kStereoSplit-th block of 16 left
 * keypoints; 16 lanes per left keypoint, so a wave carries 4 keypoints through the band search and the SAD at once
 * (round 5's form: one wave per keypoint and one 1024-thread workgroup per pair, a long dependent chain per keypoint
 * and a workgroup that needs a whole CU's wave slots beside the other graphs' kernels). Every workgroup buckets the
 * pair's right keypoints by row band itself (nR records, cheap beside the search); the median rejection, which needs
 * every keypoint of the pair, is k_stereo_median's. */
constexpr int kStereoThreads = 256;
constexpr int kStereoWaves = kStereoThreads / 64;
constexpr int kStereoGroups = kStereoThreads / 16;  // left keypoints in flight per workgroup
constexpr int kStereoSplit = 4;                     // workgroups per pair
/* the correlation windows of one keypoint in LDS, as whole dwords from the dword that holds their first column: the
 * 11x11 IL window as 11 rows x 4 dwords (columns (c0l & ~3) .. +15), the 11x21 IR strip as 11 rows x 6 dwords
 * ((c0r & ~3) .. +23). An LDS-DMA round q of a wave writes its 64 lanes' dwords to 64 consecutive LDS dwords, so
 * group g (lanes 16 g .. 16 g + 15) owns the 16-dword block q of every round: 7 blocks of 16 dwords, and each row is
 * kept whole inside one block so the SAD reads it at constant offsets: block q < 5 = IL row q | IR row 2q | IR row 2q+1
 * (4 + 6 + 6 dwords), block 5 = IL rows 5..8, block 6 = IL rows 9, 10 | IR row 10 */
constexpr int kStereoStageQ = 7;
constexpr int kStereoWaveStage = kStereoStageQ * 64 * 4 + 16;  // bytes per wave (+16: the IR over-read of group 3)
__host__ __device__ constexpr int il_dw(int r) {  // block-local dword index of IL row r (block q * 64 + offset)
    return r < 5 ? 64 * r : r < 9 ? 64 * 5 + 4 * (r - 5) : 64 * 6 + 4 * (r - 9);
}
__host__ __device__ constexpr int ir_dw(int r) {
    return r < 10 ? 64 * (r >> 1) + ((r & 1) ? 10 : 4) : 64 * 6 + 8;
}

/* dynamic LDS layout of k_stereo for kp capacity `cap` and `nrows` level-0 rows */
struct StereoLds {
    int rec, idx, row, stage, total;
    __host__ __device__ StereoLds(int cap, int nrows) {
        const int c4 = (cap + 3) & ~3;
        rec = 0;                                  // per right keypoint in bucket order: {uR, minr | maxr << 12 | oct << 24}
        idx = rec + 8 * c4;                       // its index iR (u16)
        row = idx + ((2 * c4 + 15) & ~15);        // bucket offsets (nrows + 2)
        stage = row + ((4 * (nrows + 2) + 15) & ~15);
        total = stage + kStereoWaves * kStereoWaveStage;
    }
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* minimum over each row of 16 lanes (DPP quad butterfly + row rotations), every lane of the row holds it */
__device__ __forceinline__ uint32_t row16_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
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

typedef short short2v __attribute__((ext_vector_type(2)));

/* sum over 4 pixel pairs of |a - b + d| (bytes of a and b; d in each 16-bit half of d2), as two u16 partial sums:
 * bytes 0, 2 and 1, 3 of each word spread into 16-bit lanes by v_perm; keep3 drops byte 3 (the 12th column) */
__device__ __forceinline__ short2v sad4(uint32_t a, uint32_t b, short2v d2, short2v acc, bool keep3) {
    const uint32_t alo = __builtin_amdgcn_perm(0u, a, 0x0c020c00u), ahi = __builtin_amdgcn_perm(0u, a, 0x0c030c01u);
    const uint32_t blo = __builtin_amdgcn_perm(0u, b, 0x0c020c00u), bhi = __builtin_amdgcn_perm(0u, b, 0x0c030c01u);
    short2v xlo = __builtin_bit_cast(short2v, alo) - __builtin_bit_cast(short2v, blo) + d2;
    short2v xhi = __builtin_bit_cast(short2v, ahi) - __builtin_bit_cast(short2v, bhi) + d2;
    if (!keep3) xhi = (short2v){xhi.x, 0};
    return acc + __builtin_elementwise_max(xlo, -xlo) + __builtin_elementwise_max(xhi, -xhi);
}

template <bool kDwordRows>
__global__ __launch_bounds__(kStereoThreads) void k_stereo(StereoArgs a, const int32_t* __restrict__ fl_idx,
                                                           const int32_t* __restrict__ fr_idx,
                                                           const orbx_kp* __restrict__ kpsL,
                                                           const uint8_t* __restrict__ descL,
                                                           const int32_t* __restrict__ cntL,
                                                           const orbx_kp* __restrict__ kpsR,
                                                           const uint8_t* __restrict__ descR,
                                                           const int32_t* __restrict__ cntR, int stride,
                                                           float* __restrict__ uright, float* __restrict__ depth,
                                                           int32_t* __restrict__ sad, int* __restrict__ err) {
    extern __shared__ __align__(16) uint8_t lds[];
    const StereoLds o(stride, a.nrows);
    uint2* s_rec = (uint2*)(lds + o.rec);
    uint16_t* s_idx = (uint16_t*)(lds + o.idx);
    int* s_row = (int*)(lds + o.row);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = tid >> 4, li = tid & 15;
    const int p = blockIdx.x / kStereoSplit, part = blockIdx.x % kStereoSplit;
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
    int32_t* sd = sad + (long long)p * stride;
    const int nrows = a.nrows;

    // vRowIndices (Frame.cc:477-498) as buckets by the first row of each right keypoint's band: counts, scan, scatter
    for (int i = tid; i <= nrows + 1; i += kStereoThreads) s_row[i] = 0;
    __syncthreads();
    for (int iR = tid; iR < nR; iR += kStereoThreads) {
        const orbx_kp k = kR[iR];
        const float r = __fmul_rn(2.0f, a.scale[k.octave]);
        const int minr = (int)floorf(__fsub_rn(k.y, r));
        atomicAdd(&s_row[min(max(minr, 0), nrows - 1) + 1], 1);
    }
    __syncthreads();
    if (wv == 0) {  // exclusive scan of the bucket counts (s_row[b+1] = count of bucket b)
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
    for (int iR = tid; iR < nR; iR += kStereoThreads) {
        const orbx_kp k = kR[iR];
        const float r = __fmul_rn(2.0f, a.scale[k.octave]);
        const int maxr = (int)ceilf(__fadd_rn(k.y, r));
        const int minr = (int)floorf(__fsub_rn(k.y, r));
        // a band test minr <= v <= maxr for 0 <= v < nrows (< 4096) is unchanged by clamping both ends to [0, nrows]
        const uint32_t band = (uint32_t)min(max(minr, 0), nrows) | ((uint32_t)min(max(maxr, 0), nrows) << 12) |
                              ((uint32_t)k.octave << 24);
        const int pos = atomicAdd(&s_row[min(max(minr, 0), nrows - 1) + 1], 1);
        s_rec[pos] = make_uint2(__float_as_uint(k.x), band);
        s_idx[pos] = (uint16_t)iR;
    }
    __syncthreads();

    uint8_t* stage = lds + o.stage + wv * kStereoWaveStage;
    const uint32_t* sg = (const uint32_t*)stage + 16 * (g & 3);  // this group's blocks: sg[64 q + 0..15]
    const int gbase = lane & ~15;
    const int nblk = (nL + kStereoGroups - 1) / kStereoGroups;
    for (int blk = part; blk < nblk; blk += kStereoSplit) {  // wave-uniform trip count
        const int iL = blk * kStereoGroups + g;
        const bool on = iL < nL;
        orbx_kp kpL;
        kpL.x = kpL.y = 0.f;
        kpL.octave = 0;
        if (on) kpL = kL[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const int v = (int)vL;  // vRowIndices[vL] (Frame.cc:514)
        const float minU = __fsub_rn(uL, a.maxD);
        const float maxU = __fsub_rn(uL, 0.0f);
        const bool search = on && vL >= 0.f && v < nrows && !(maxU < 0);
        uint32_t best = 0xffffffffu;
        float bestU = 0.f;  // uR of this lane's best candidate (the winner's is shuffled to the group below)
        if (search) {  // Frame.cc:531-550: the first strict minimum over the band = the minimum of (dist, iR)
            const uint4* qd = (const uint4*)(dL + (long long)iL * 32);
            const uint4 q0 = qd[0], q1 = qd[1];
            const int cb = s_row[max(v - a.rspan, 0)], ce = s_row[v + 1];
            // 4 candidates per lane per round: their records, then all 8 descriptor loads in flight together (a
            // candidate that fails the tests, or past the bucket range, loads row 0 and is ignored), one memory round
            // trip per 64 candidates instead of one per 16
            for (int c0 = cb; c0 < ce; c0 += 64) {
                uint2 rc[4];
                int ir[4];
                bool ok[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int c = c0 + 16 * k + li;
                    const bool in = c < ce;
                    rc[k] = s_rec[in ? c : cb];
                    ir[k] = s_idx[in ? c : cb];
                    const int minr = (int)(rc[k].y & 0xfffu), maxr = (int)((rc[k].y >> 12) & 0xfffu),
                              oct = (int)(rc[k].y >> 24);
                    const float uR = __uint_as_float(rc[k].x);
                    ok[k] = in && minr <= v && v <= maxr && oct >= levelL - 1 && oct <= levelL + 1 && uR >= minU &&
                            uR <= maxU;
                }
                uint4 cv0[4], cv1[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint4* cd = (const uint4*)(dR + (long long)(ok[k] ? ir[k] : 0) * 32);
                    cv0[k] = cd[0];
                    cv1[k] = cd[1];
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int dist = __popc(q0.x ^ cv0[k].x) + __popc(q0.y ^ cv0[k].y) + __popc(q0.z ^ cv0[k].z) +
                                     __popc(q0.w ^ cv0[k].w) + __popc(q1.x ^ cv1[k].x) + __popc(q1.y ^ cv1[k].y) +
                                     __popc(q1.z ^ cv1[k].z) + __popc(q1.w ^ cv1[k].w);
                    const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)ir[k];
                    if (ok[k] && dist < 100 && key < best) {  // TH_HIGH
                        best = key;
                        bestU = __uint_as_float(rc[k].x);
                    }
                }
            }
        }
        const uint32_t mine = best;
        best = row16_min_u32(best);
        // sub-pixel match by correlation (Frame.cc:555-621) for best distance < thOrbDist (Frame.cc:475, 553)
        bool corr = search && best != 0xffffffffu && (int)(best >> 16) < 75;
        // the winner's uR from the lane that holds it (keys are unique: iR is in the key)
        const unsigned long long wm = __ballot(mine == best && best != 0xffffffffu) & (0xFFFFull << gbase);
        const int wl = wm ? (int)__builtin_ctzll(wm) : lane;
        const float wU = __shfl(bestU, wl);  // every lane takes part (the winner lane is active here)
        const float uR0 = corr ? wU : 0.f;
        const float sf = a.inv_scale[levelL];
        const float suL = roundf(__fmul_rn(uL, sf));
        const float svL = roundf(__fmul_rn(vL, sf));
        const float suR0 = roundf(__fmul_rn(uR0, sf));
        const float iniu = __fsub_rn(__fadd_rn(suR0, 5.0f), 5.0f);
        const float endu = __fadd_rn(__fadd_rn(__fadd_rn(suR0, 5.0f), 5.0f), 1.0f);
        const int lw = a.lw[levelL], lh = a.lh[levelL];
        corr = corr && !(iniu < 0 || endu >= (float)lw);
        const int r0 = (int)__fsub_rn(svL, 5.0f), c0l = (int)__fsub_rn(suL, 5.0f), c0r = (int)__fsub_rn(suR0, 10.0f);
        if (corr && (r0 < 0 || r0 + 11 > lh || c0l < 0 || c0l + 11 > lw || c0r < 0 || c0r + 21 > lw)) {
            if (li == 0) atomicOr(err, 2);  // the reference's cv::Mat::colRange/rowRange would assert
            corr = false;
        }
        int pitchL = 0, pitchR = 0;
        const uint8_t* PL = level_base(a.left, a, fl, levelL, &pitchL) + (long long)r0 * pitchL;
        const uint8_t* PR = level_base(a.right, a, fr, levelL, &pitchR) + (long long)r0 * pitchR;
        if (kDwordRows) {
            // every row 4-aligned: 7 LDS-DMA rounds per wave, lane j of a group carrying the dword of its block slot
            // (round q, j); a dword past the level's last one is clamped to it (its bytes lie past column lw - 1: never
            // read)
            const int lastd = (lw - 1) & ~3;
            const bool any = __ballot(corr) != 0;  // wave-uniform: a wave with no window to stage issues nothing
            // lanes without a window load a valid dummy (their keypoint array); r0 / c0 of such a lane are arbitrary
            const uint8_t* dummy = (const uint8_t*)kL;
#pragma unroll
            for (int q = 0; q < kStereoStageQ; q++) {
                bool il;
                int rr, dd;
                if (q < 5) {
                    il = li < 4;
                    rr = il ? q : 2 * q + (li >= 10 ? 1 : 0);
                    dd = il ? li : (li >= 10 ? li - 10 : li - 4);
                } else if (q == 5) {
                    il = true;
                    rr = 5 + (li >> 2);
                    dd = li & 3;
                } else {
                    il = li < 8;
                    rr = il ? 9 + (li >> 2) : 10;
                    dd = il ? (li & 3) : min(li - 8, 5);
                }
                const int col = min(((il ? c0l : c0r) & ~3) + 4 * dd, lastd);
                const uint8_t* src = (il ? PL + rr * pitchL : PR + rr * pitchR) + col;
                if (any)
                    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(corr ? src : dummy),
                                                     (__attribute__((address_space(3))) void*)(stage + 256 * q), 4, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (corr) {  // unaligned rows (a packed odd-width level 0): the same layout a byte at a time
            for (int k = li; k < 11 * 16 + 11 * 24; k += 16) {
                const bool il = k < 11 * 16;
                const int kk = il ? k : k - 11 * 16;
                const int rr = il ? kk >> 4 : kk / 24, bb = il ? kk & 15 : kk - 24 * rr;
                const int col = min(((il ? c0l : c0r) & ~3) + bb, lw - 1);
                ((uint8_t*)sg)[4 * (il ? il_dw(rr) : ir_dw(rr)) + bb] = il ? PL[rr * pitchL + col] : PR[rr * pitchR + col];
            }
        }
        wave_lds_sync();
        // lane li < 11: the L1 distance at shift incR = li - 5 (cv::norm(IL, IR, NORM_L1) of the centre-subtracted
        // windows: |IL - IR + (cR - cL)| summed, integers, exact); every row read at constant offsets
        int tot = 0x7fffffff;
        if (corr && li < 11) {
            const int shl = c0l & 3, orr = (c0r & 3) + li;
            const uint8_t* sb = (const uint8_t*)sg;
            const int cL = sb[4 * il_dw(5) + shl + 5];
            const int cR = sb[4 * ir_dw(5) + orr + 5];
            const short2v d2 = (short2v){(short)(cR - cL), (short)(cR - cL)};
            short2v acc = (short2v){0, 0};
            const int shr = orr & 3;
            const uint32_t* irb = sg + (orr >> 2);  // this lane's IR rows start (orr >> 2) dwords in
#pragma unroll
            for (int r = 0; r < 11; r++) {
                const uint4 lw4 = *(const uint4*)(sg + il_dw(r));
                const uint32_t* rw = irb + ir_dw(r);
                const uint32_t w0 = rw[0], w1 = rw[1], w2 = rw[2], w3 = rw[3];
                const uint32_t l0 = __builtin_amdgcn_alignbyte(lw4.y, lw4.x, shl), l1 = __builtin_amdgcn_alignbyte(lw4.z, lw4.y, shl),
                               l2 = __builtin_amdgcn_alignbyte(lw4.w, lw4.z, shl);
                const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, shr), x1 = __builtin_amdgcn_alignbyte(w2, w1, shr),
                               x2 = __builtin_amdgcn_alignbyte(w3, w2, shr);
                acc = sad4(l0, x0, d2, acc, true);
                acc = sad4(l1, x1, d2, acc, true);
                acc = sad4(l2, x2, d2, acc, false);
            }
            tot = (int)(uint16_t)acc.x + (int)(uint16_t)acc.y;
        }
        // first strict minimum over the 11 shifts (Frame.cc:594-602) and its neighbours for the parabola
        const uint32_t key = row16_min_u32(tot == 0x7fffffff ? 0xffffffffu : ((uint32_t)tot << 4) | (uint32_t)li);
        const int bi = (int)(key & 15u), bestS = (int)(key >> 4);
        const float d1 = (float)__shfl(tot, gbase + max(bi - 1, 0)), d2f = (float)bestS,
                    d3 = (float)__shfl(tot, gbase + min(bi + 1, 10));
        wave_lds_sync();  // this group's window is rewritten by its next keypoint
        if (!on || li != 0) continue;
        float u_out = -1.0f, d_out = -1.0f;
        int s_out = -1;
        if (corr && bi != 0 && bi != 10) {
            const float deltaR =
                __fdiv_rn(__fsub_rn(d1, d3), __fmul_rn(2.0f, __fsub_rn(__fadd_rn(d1, d3), __fmul_rn(2.0f, d2f))));
            if (!(deltaR < -1 || deltaR > 1)) {
                float bestuR = __fmul_rn(a.scale[levelL], __fadd_rn(__fadd_rn(suR0, (float)(bi - 5)), deltaR));
                float disparity = __fsub_rn(uL, bestuR);
                if (disparity >= 0.0f && disparity < a.maxD) {  // Frame.cc:623-633
                    if (disparity <= 0) {
                        disparity = 0.01f;
                        bestuR = (float)((double)uL - 0.01);
                    }
                    d_out = __fdiv_rn(a.bf, disparity);
                    u_out = bestuR;
                    s_out = bestS;
                }
            }
        }
        ur[iL] = u_out;  // mvuRight = mvDepth = -1 unless matched (Frame.cc:472-473)
        dp[iL] = d_out;
        sd[iL] = s_out;
    }
}

/* the median rejection of a pair's stereo matches (Frame.cc:636-650), one workgroup per pair after k_stereo: the
 * n/2-th smallest SAD (sort(vDistIdx), vDistIdx[n/2]) by a two-digit radix select in LDS, thDist = 1.5f*1.4f*median,
 * every match at or above it reset to -1; d_nstereo = the matches kept */
__global__ __launch_bounds__(256) void k_stereo_median(const int32_t* __restrict__ fl_idx, const int32_t* __restrict__ fr_idx,
                                                      const int32_t* __restrict__ cntL, const int32_t* __restrict__ cntR,
                                                      int left_nframes, int right_nframes, int stride, float thc,
                                                      float* __restrict__ uright, float* __restrict__ depth,
                                                      const int32_t* __restrict__ sad, int32_t* __restrict__ nstereo) {
    __shared__ int s_hist[512];
    __shared__ int s_misc[8];
    const int tid = threadIdx.x, p = blockIdx.x;
    const int fl = fl_idx[p], fr = fr_idx[p];
    if (fl < 0 || fl >= left_nframes || fr < 0 || fr >= right_nframes) return;  // k_stereo raised the error flag
    const int nL = cntL[fl], nR = cntR[fr];
    if (nL < 0 || nL > stride || nR < 0 || nR > stride) return;
    float* ur = uright + (long long)p * stride;
    float* dp = depth + (long long)p * stride;
    const int32_t* sd = sad + (long long)p * stride;
    for (int i = tid; i < 512; i += 256) s_hist[i] = 0;
    if (tid < 8) s_misc[tid] = 0;
    __syncthreads();
    int nloc = 0;
    for (int i = tid; i < nL; i += 256) {
        const int d = sd[i];
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
    for (int i = tid; i < nL; i += 256) {
        const int d = sd[i];
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
    const float thDist = __fmul_rn(thc, median);
    int kept = 0;
    for (int i = tid; i < nL; i += 256) {
        const int d = sd[i];
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

/* ============================ SearchByProjection ============================ */

constexpr unsigned long long kNoKey = ~0ull;
/* a projection-scan candidate key: dist << 40 | cell order << 20 | feature idx << 4 | octave. Keys order by
 * (dist, cell order, idx) as the reference's scan does (the octave is a function of idx); the octave rides
 * along so the resolve's ratio test reads no feature array (no dependent global load per round). */
__device__ __forceinline__ int key_idx(unsigned long long k) { return (int)((k >> 4) & 0xffffu); }
__device__ __forceinline__ int key_oct(unsigned long long k) { return (int)(k & 15u); }

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
    const int lo = __shfl_xor((int)(uint32_t)v, o), hi = __shfl_xor((int)(uint32_t)(v >> 32), o);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ void keep2(unsigned long long k, unsigned long long& b, unsigned long long& s) {
    if (k < b) {
        s = b;
        b = k;
    } else if (k < s) {
        s = k;
    }
}

/* block-wide exclusive scan of one int per thread (1024 threads); returns the exclusive prefix,
 * *total = sum. s_tmp: 16 ints of LDS. */
__device__ int block_scan_1024(int v, int* s_tmp, int* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) s_tmp[wv] = incl;
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 16; w++) {
        const int t = s_tmp[w];
        off += w < wv ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}

/* Frame::AssignFeaturesToGrid (Frame.cc:235-250): cell = posX*48 + posY with PosInGrid's
 * round((x - mnMinX) * mfGridElementWidthInv) (Frame.cc:391-401) */
__device__ __forceinline__ int grid_cell(const ProjCall& c, int i) {
    const int posX = (int)roundf(__fmul_rn(__fsub_rn(c.x[i], c.min_x), c.gw_inv));
    const int posY = (int)roundf(__fmul_rn(__fsub_rn(c.y[i], c.min_y), c.gh_inv));
    if (posX < 0 || posX >= kGridCols || posY < 0 || posY >= kGridRows) return -1;
    return posX * kGridRows + posY;
}

__global__ __launch_bounds__(1024) void k_grid(const ProjCall* __restrict__ calls) {
    constexpr int NC = kGridCols * kGridRows;  // 3072 = 3 per thread
    __shared__ int s_cnt[NC];
    __shared__ int s_tmp[16];
    const ProjCall& c = calls[blockIdx.x];
    const int tid = threadIdx.x;
    for (int i = tid; i < NC; i += 1024) s_cnt[i] = 0;
    __syncthreads();
    for (int i = tid; i < c.n; i += 1024) {
        const int cell = grid_cell(c, i);
        if (cell >= 0) atomicAdd(&s_cnt[cell], 1);
    }
    __syncthreads();
    const int a0 = s_cnt[3 * tid], a1 = s_cnt[3 * tid + 1], a2 = s_cnt[3 * tid + 2];
    int total;
    const int off = block_scan_1024(a0 + a1 + a2, s_tmp, &total);
    s_cnt[3 * tid] = off;
    s_cnt[3 * tid + 1] = off + a0;
    s_cnt[3 * tid + 2] = off + a0 + a1;
    c.grid_start[3 * tid] = off;
    c.grid_start[3 * tid + 1] = off + a0;
    c.grid_start[3 * tid + 2] = off + a0 + a1;
    if (tid == 0) c.grid_start[NC] = total;
    __syncthreads();
    for (int i = tid; i < c.n; i += 1024) {
        const int cell = grid_cell(c, i);
        if (cell >= 0) c.grid_idx[atomicAdd(&s_cnt[cell], 1)] = (uint16_t)i;
    }
}

/* GetFeaturesInArea (Frame.cc:332-389) + the per-candidate tests of the variants, G lanes of one
 * query (gl = lane in group). Returns (all lanes) the group's K smallest candidate keys, sorted,
 * and the number of candidates (keys with dist < 256). */
template <int K>
__device__ __forceinline__ void topk_insert(unsigned long long k, unsigned long long (&a)[K]) {
#pragma unroll
    for (int t = 0; t < K; t++) {
        const unsigned long long lo = min(k, a[t]), hi = max(k, a[t]);
        a[t] = lo;
        k = hi;
    }
}

struct AnyDist {
    __device__ bool operator()(int, int) const { return true; }
};

/* elig(idx, dist): a candidate-specific filter after the distance (SearchForInitialization's
 * vMatchedDistance[i2] > dist test, ORBmatcher.cc:444-445) */
template <int G, int K, class Occ, class Elig = AnyDist>
__device__ __forceinline__ int proj_scan(const ProjCall& c, const ProjQuery& q, const uint4 qd0, const uint4 qd1, int gl,
                                         Occ occupied, unsigned long long (&top)[K], Elig elig = Elig()) {
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = kNoKey;
    int ncand = 0;
    const float r = q.radius;
    const int nMinCellX = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(q.u, c.min_x), r), c.gw_inv)));
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(q.u, c.min_x), r), c.gw_inv)));
    const int nMinCellY = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(q.v, c.min_y), r), c.gh_inv)));
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(q.v, c.min_y), r), c.gh_inv)));
    if (nMinCellX < kGridCols && nMaxCellX >= 0 && nMinCellY < kGridRows && nMaxCellY >= 0) {
        const int ny = nMaxCellY - nMinCellY + 1;
        const int ncell = (nMaxCellX - nMinCellX + 1) * ny;
        for (int k = gl; k < ncell; k += G) {
            const int dx = k / ny;
            const int cell = (nMinCellX + dx) * kGridRows + nMinCellY + (k - dx * ny);
            const int j1 = c.grid_start[cell + 1];
            for (int j = c.grid_start[cell]; j < j1; j++) {
                const int idx = c.grid_idx[j];
                const int oct = c.octave[idx];
                if (oct < q.min_level) continue;
                if (q.max_level >= 0 && oct > q.max_level) continue;
                if (!(fabsf(__fsub_rn(c.x[idx], q.u)) < r && fabsf(__fsub_rn(c.y[idx], q.v)) < r)) continue;
                if (occupied(idx)) continue;
                if ((q.flags & kProjStereo) && c.uright) {
                    const float urf = c.uright[idx];
                    if (urf > 0 && fabsf(__fsub_rn(q.ur, urf)) > q.er_th) continue;
                }
                if (q.flags & kProjChi2) {  // ORBmatcher.cc:904-929 (float residual, double threshold)
                    const float ex = __fsub_rn(q.u, c.x[idx]), ey = __fsub_rn(q.v, c.y[idx]);
                    float e2 = __fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey));
                    const float urf = c.uright ? c.uright[idx] : -1.0f;
                    if (urf >= 0) {
                        const float er = __fsub_rn(q.ur, urf);
                        e2 = __fadd_rn(e2, __fmul_rn(er, er));
                    }
                    if ((double)__fmul_rn(e2, c.inv_sigma2[oct]) > (urf >= 0 ? 7.8 : 5.99)) continue;
                }
                const uint4* fd = (const uint4*)(c.desc + (long long)idx * 32);
                const uint4 f0 = fd[0], f1 = fd[1];
                const int dist = __popc(qd0.x ^ f0.x) + __popc(qd0.y ^ f0.y) + __popc(qd0.z ^ f0.z) +
                                 __popc(qd0.w ^ f0.w) + __popc(qd1.x ^ f1.x) + __popc(qd1.y ^ f1.y) +
                                 __popc(qd1.z ^ f1.z) + __popc(qd1.w ^ f1.w);
                if (dist < 256 && elig(idx, dist)) {  // bestDist starts at 256 (ORBmatcher.cc:78, 349, 1397, 1550)
                    topk_insert<K>(((unsigned long long)dist << 40) | ((unsigned long long)k << 20) |
                                       ((unsigned long long)idx << 4) | (unsigned)oct, top);
                    ncand++;
                }
            }
        }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
        unsigned long long other[K];
#pragma unroll
        for (int t = 0; t < K; t++) other[t] = shfl_xor_u64(top[t], o);
#pragma unroll
        for (int t = 0; t < K; t++) topk_insert<K>(other[t], top);
        ncand += __shfl_xor(ncand, o);
    }
    return ncand;
}

constexpr int kProjTopK = 4;  // candidate keys kept per query by the scan (more keys = fewer whole-wave rescans)
static_assert(kProjTopK >= 2 && kProjTopK <= 16, "the scan writes one key per lane of a 16-lane query group");
int proj_topk() { return kProjTopK; }

/* one result of a per-call host API launch: a single 64-bit store of (value, call seq) to pinned host memory;
 * the host takes an entry once it carries its call's seq, whatever order the stores land in */
__device__ __forceinline__ void host_put(unsigned long long* p, int v, int seq) {
    __hip_atomic_store(p, (unsigned long long)(uint32_t)v | (unsigned long long)(uint32_t)seq << 32, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

/* the call's match[0 .. n) and nmatches to host_out (the last step of a resolve wave) */
__device__ __forceinline__ void host_put_matches(const ProjCall& c, int32_t* match, int n, int nm, int lane) {
    // this wave's own match[] atomics / stores complete before its loads (they were never loaded into L1, so
    // the loads read them from L2); 8 independent loads per lane in flight before their stores
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    constexpr int U = 8;
    unsigned long long* const out = c.host_out;
    const int seq = c.seq;
    if (n > 0)
        for (int i0 = 0; i0 < n; i0 += 64 * U) {
            int v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = match[min(i0 + 64 * u + lane, n - 1)];  // unconditional: no waits
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int i = i0 + 64 * u + lane;
                if (i < n) host_put(out + i, v[u], seq);
            }
        }
    if (lane == 0) host_put(out + n, nm, seq);
}

__global__ __launch_bounds__(256) void k_proj_scan(const ProjCall* __restrict__ calls) {
    const ProjCall& c = calls[blockIdx.y];
    const int qi = blockIdx.x * 16 + (threadIdx.x >> 4), gl = threadIdx.x & 15;
    if (blockIdx.x * 16 >= c.nq) return;  // block-uniform
    const bool in = qi < c.nq;
    ProjQuery q;
    uint4 qd0 = make_uint4(0, 0, 0, 0), qd1 = qd0;
    if (in) {
        q = c.q[qi];
        const uint4* qd = (const uint4*)(c.qdesc + (long long)qi * 32);
        qd0 = qd[0];
        qd1 = qd[1];
    } else {
        q.u = q.v = -1e30f;  // empty window
        q.radius = 0.f;
        q.flags = 0;
        q.min_level = 0;
        q.max_level = -1;
    }
    const uint8_t* occ0 = c.occ0;
    unsigned long long top[kProjTopK];
    const int ncand = proj_scan<16, kProjTopK>(c, q, qd0, qd1, gl, [occ0](int i) { return occ0 && occ0[i]; }, top);
    if (in && gl < kProjTopK) {
        unsigned long long v = top[0];
#pragma unroll
        for (int t = 1; t < kProjTopK; t++)
            if (gl == t) v = top[t];
        c.scan[(long long)kProjTopK * qi + gl] = v;
        if (gl == 0) c.scan_cnt[qi] = ncand;
        // Fuse: nothing claims, so the query's answer is its best key (occupied features are already
        // excluded by the scan), accepted when bestDist <= the threshold -- what k_proj_resolve would write
        if (c.direct && gl == 0) {
            const bool acc = top[0] != kNoKey && (int)(top[0] >> 40) <= c.accept_th;
            const int r = acc ? key_idx(top[0]) : -1;
            if (c.host_out) {
                host_put(c.host_out + qi, r, c.seq);
            } else {
                c.res[2 * qi] = r;
                c.res[2 * qi + 1] = 0;
            }
        }
    }
}

/* accept rule of the variant: bestDist <= threshold, and for SearchByProjection(F, vpMapPoints)
 * the ratio test when best and second lie on one level (ORBmatcher.cc:116-125) */
__device__ __forceinline__ bool proj_accept(const ProjCall& c, unsigned long long b, unsigned long long s) {
    if (b == kNoKey) return false;
    const int dist = (int)(b >> 40);
    if (dist > c.accept_th) return false;
    if (c.ratio) {
        const int level = key_oct(b);
        const int level2 = s != kNoKey ? key_oct(s) : -1;
        const int dist2 = s != kNoKey ? (int)(s >> 40) : 256;
        if (level == level2 && (float)dist > __fmul_rn(c.nnratio, (float)dist2)) return false;
    }
    return true;
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {  // ORBmatcher.cc:1423-1430
    float rot = __fsub_rn(a1, a2);
    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
    int bin = (int)roundf(__fmul_rn(rot, 1.0f / 30));
    if (bin == 30) bin = 0;
    return min(max(bin, 0), 29);
}

constexpr int kProjMaxFeatures = 65536;
constexpr int kClaimTab = 2048;  // claim table of one resolve round (power of 2)

/* rotation bins of every accepted query (res[2q] >= 0: bin of q.angle - angle[res[2q]]) into res[2q+1] and the
 * histogram; kQU queries per lane with their loads in flight together (a per-query loop would pay two
 * dependent global loads per query) */
constexpr int kQU = 4;
__device__ __forceinline__ void rot_bins(const ProjCall& c, int lane, int* hist) {
    const int nq = c.nq;
    for (int q0 = 0; q0 < nq; q0 += 64 * kQU) {
        int f[kQU];
        float qa[kQU], fa[kQU];
#pragma unroll
        for (int u = 0; u < kQU; u++) {
            const int qc = min(q0 + 64 * u + lane, nq - 1);
            f[u] = c.res[2 * qc];
            qa[u] = c.q[qc].angle;
        }
#pragma unroll
        for (int u = 0; u < kQU; u++) fa[u] = c.angle[max(f[u], 0)];
#pragma unroll
        for (int u = 0; u < kQU; u++) {
            const int q = q0 + 64 * u + lane;
            if (q < nq && f[u] >= 0) {
                const int bin = rot_bin(qa[u], fa[u]);
                c.res[2 * q + 1] = bin;
                atomicAdd(&hist[bin], 1);
            }
        }
    }
}

/* One wave per call. Chunks of 64 queries (lane j = query base+j) are evaluated in registers: each
 * lane's best / second are the first two entries of its top-K list not occupied in the live bitmap
 * (claims only remove candidates, so the remaining order is unchanged). Lanes commit in order up to
 * the first lane whose best (or, with the ratio test, second) element is claimed by an earlier
 * uncommitted lane of the chunk; that lane is re-filtered in the next round against the bitmap that
 * now holds those claims. A lane whose filtered list ran out while the list was truncated (more than
 * K candidates) is re-scanned by the whole wave against the bitmap. */
__global__ __launch_bounds__(64) void k_proj_resolve(const ProjCall* __restrict__ calls) {
    __shared__ uint32_t s_occ[kProjMaxFeatures / 32];
    __shared__ int s_claim[kClaimTab];
    __shared__ int s_hist[32];
    const ProjCall& c = calls[blockIdx.x];
    const int lane = threadIdx.x;
    // the occupancy bitmap by ballots over coalesced byte loads, 4 loads per lane in flight (a per-lane loop
    // over 32 bytes costs one dependent load each)
    {
        const int n = c.n;
        const uint8_t* occ0 = c.occ0;
        for (int b0 = 0; b0 < n; b0 += 256) {
            int v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = occ0 ? occ0[min(b0 + 64 * u + lane, max(n - 1, 0))] : 0;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int f = b0 + 64 * u + lane;
                const unsigned long long m = __ballot(f < n && v[u] != 0);
                if (lane < 2 && f - lane < n) s_occ[(b0 + 64 * u) / 32 + lane] = (uint32_t)(m >> (32 * lane));
            }
        }
    }
    for (int i = lane; i < c.n; i += 64) c.match[i] = -1;
    if (lane < 32) s_hist[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // one wave: order its own global accesses (no L2 write-back)
    wave_lds_sync();
    auto occ_get = [](int i) { return (s_occ[i >> 5] >> (i & 31)) & 1u; };
    const int need = c.ratio ? 2 : 1;  // list entries that decide the result
    for (int i = lane; i < kClaimTab; i += 64) s_claim[i] = 64;
    wave_lds_sync();
    int nacc = 0;
    // chunk registers; the next chunk's loads are issued before the current chunk's rounds
    unsigned long long top[kProjTopK], ntop[kProjTopK];
    int ncand = 0, flags = 0, src = 0, nncand = 0, nflags = 0, nsrc = 0;
    auto load_chunk = [&](int b0, unsigned long long (&t)[kProjTopK], int& cnt, int& fl, int& sr) {
        const int qi = b0 + lane;
#pragma unroll
        for (int k = 0; k < kProjTopK; k++) t[k] = kNoKey;
        cnt = 0;
        fl = 0;
        sr = 0;
        if (qi < c.nq) {
#pragma unroll
            for (int k = 0; k < kProjTopK; k++) t[k] = c.scan[(long long)kProjTopK * qi + k];
            cnt = c.scan_cnt[qi];
            const ProjQuery& q = c.q[qi];
            fl = q.flags;
            sr = q.src;
        }
    };
    load_chunk(0, ntop, nncand, nflags, nsrc);
    for (int base = 0; base < c.nq; base += 64) {
        const int qi = base + lane;
        const bool in = qi < c.nq;
#pragma unroll
        for (int t = 0; t < kProjTopK; t++) top[t] = ntop[t];
        ncand = nncand;
        flags = nflags;
        src = nsrc;
        if (base + 64 < c.nq) load_chunk(base + 64, ntop, nncand, nflags, nsrc);
        int done = 0;  // lanes < done are committed
        while (done < 64 && base + done < c.nq) {
            const bool act = in && lane >= done;
            unsigned long long b = kNoKey, s = kNoKey;
            int found = 0;
#pragma unroll
            for (int t = 0; t < kProjTopK; t++) {
                const unsigned long long k = top[t];
                if (k == kNoKey || occ_get(key_idx(k))) continue;
                if (found == 0) b = k; else if (found == 1) s = k;
                found++;
            }
            const bool rescan = act && found < need && ncand > kProjTopK;
            const int bi = b != kNoKey ? key_idx(b) : -1;
            const int si = s != kNoKey ? key_idx(s) : -1;
            const bool acc = act && !rescan && proj_accept(c, b, s);
            const int my_claim = acc && (flags & kProjClaims) ? bi : -1;
            // conflicts with earlier uncommitted claims of this round: claim table (lane ids, hashed by feature;
            // a collision only delays a lane to the next round)
            if (my_claim >= 0) atomicMin(&s_claim[my_claim & (kClaimTab - 1)], lane);
            wave_lds_sync();
            bool dirty = rescan;
            if (act && bi >= 0 && s_claim[bi & (kClaimTab - 1)] < lane) dirty = true;
            if (act && need == 2 && si >= 0 && s_claim[si & (kClaimTab - 1)] < lane) dirty = true;
            const unsigned long long dm = __ballot(act && dirty);
            const int d = dm ? __ffsll((long long)dm) - 1 : 64;
            wave_lds_sync();
            if (my_claim >= 0) s_claim[my_claim & (kClaimTab - 1)] = 64;
            if (act && lane < d) {
                if (acc) {
                    atomicMax(&c.match[bi], src);
                    if (my_claim >= 0) atomicOr(&s_occ[bi >> 5], 1u << (bi & 31));
                    c.res[2 * qi] = bi;  // the rotation bin is taken after the chunks (no load in a round)
                    nacc++;
                } else {
                    c.res[2 * qi] = -1;
                }
            }
            wave_lds_sync();
            if (d < 64 && __shfl((int)rescan, d)) {  // whole-wave re-scan of query base+d
                const int qd = base + d;
                const ProjQuery q = c.q[qd];
                const uint4* qp = (const uint4*)(c.qdesc + (long long)qd * 32);
                unsigned long long t2[2];
                proj_scan<64, 2>(c, q, qp[0], qp[1], lane, occ_get, t2);
                const bool acc2 = proj_accept(c, t2[0], t2[1]);
                if (lane == 0) {
                    if (acc2) {
                        const int bi2 = key_idx(t2[0]);
                        atomicMax(&c.match[bi2], q.src);
                        if (q.flags & kProjClaims) atomicOr(&s_occ[bi2 >> 5], 1u << (bi2 & 31));
                        c.res[2 * qd] = bi2;
                        nacc++;
                    } else {
                        c.res[2 * qd] = -1;
                    }
                }
                wave_lds_sync();
                done = d + 1;
            } else {
                done = d;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // one wave: order its own global accesses (no L2 write-back)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nacc += __shfl_xor(nacc, o);
    if (c.check_ori) {  // rotation consistency (ORBmatcher.cc:1437-1467)
        rot_bins(c, lane, s_hist);
        wave_lds_sync();
        int ind1 = -1, ind2 = -1, ind3 = -1, max1 = 0, max2 = 0, max3 = 0;  // ComputeThreeMaxima (:1601-1642)
        for (int i = 0; i < 30; i++) {
            const int sz = s_hist[i];
            if (sz > max1) {
                max3 = max2; max2 = max1; max1 = sz;
                ind3 = ind2; ind2 = ind1; ind1 = i;
            } else if (sz > max2) {
                max3 = max2; max2 = sz;
                ind3 = ind2; ind2 = i;
            } else if (sz > max3) {
                max3 = sz; ind3 = i;
            }
        }
        if (max2 < __fmul_rn(0.1f, (float)max1)) {
            ind2 = -1; ind3 = -1;
        } else if (max3 < __fmul_rn(0.1f, (float)max1)) {
            ind3 = -1;
        }
        int removed = 0;
        for (int q0 = 0; q0 < c.nq; q0 += 64 * kQU) {  // kQU queries per lane, their loads in flight together
            int f[kQU], b[kQU];
#pragma unroll
            for (int u = 0; u < kQU; u++) {
                const int qc = min(q0 + 64 * u + lane, c.nq - 1);
                f[u] = c.res[2 * qc];
                b[u] = c.res[2 * qc + 1];
            }
#pragma unroll
            for (int u = 0; u < kQU; u++)
                if (q0 + 64 * u + lane < c.nq && f[u] >= 0 && b[u] != ind1 && b[u] != ind2 && b[u] != ind3) {
                    c.match[f[u]] = -2;
                    removed++;
                }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) removed += __shfl_xor(removed, o);
        nacc -= removed;
    }
    if (lane == 0) *c.nmatches = nacc;
    if (c.host_out) host_put_matches(c, c.match, c.n, nacc, lane);
}

/* ============================ SearchForInitialization ============================ */

/* ORBmatcher::SearchForInitialization (ORBmatcher.cc:405-520) after k_grid + k_proj_scan over F2 with one
 * query per level-0 keypoint of F1 (window vbPrevMatched[i1] +- windowSize, levels 0..0, q.src = i1).
 * The reference visits i1 in order; a candidate i2 is usable iff dist < vMatchedDistance[i2] (the best
 * distance it was matched with so far, :444-445), and an accept steals i2 from its previous i1 (:463-467).
 * vMatchedDistance only decreases, so a query's ineligible list entries stay ineligible: its decision
 * (best = first usable entry of its top-K list, best2 = the next one) can only change if an earlier query
 * takes its best or second entry. One wave, chunks of 64 queries: lanes commit in order up to the first
 * lane whose best / second entry an earlier uncommitted lane of the chunk takes (LDS claim table), that
 * lane is re-evaluated next round; a lane whose usable entries ran out in a truncated list is re-scanned
 * by the whole wave against the live vMatchedDistance. Then the rotation histogram over every accept
 * (stolen matches stay in their bins, :482) + ComputeThreeMaxima (:489-512). Writes vnMatches12 to
 * c.match[0 .. c.n_out) and nmatches. */
constexpr int kInitMaxN = 8192;

__global__ __launch_bounds__(64) void k_init_resolve(const ProjCall* __restrict__ calls) {
    __shared__ uint16_t s_md[kInitMaxN];   // vMatchedDistance (0xffff = INT_MAX)
    __shared__ int16_t s_v21[kInitMaxN];   // vnMatches21
    __shared__ int16_t s_v12[kInitMaxN];   // vnMatches12
    __shared__ int s_claim[kClaimTab];
    __shared__ int s_hist[32];
    const ProjCall& c = calls[blockIdx.x];
    const int lane = threadIdx.x;
    for (int i = lane; i < c.n; i += 64) {
        s_md[i] = 0xffff;
        s_v21[i] = -1;
    }
    for (int i = lane; i < c.n_out; i += 64) s_v12[i] = -1;
    for (int i = lane; i < kClaimTab; i += 64) s_claim[i] = 64;
    if (lane < 32) s_hist[lane] = 0;
    wave_lds_sync();
    auto usable = [](int idx, int dist) { return dist < (int)s_md[idx]; };
    // accept rule (:459-461): bestDist <= TH_LOW and bestDist < (float)bestDist2 * mfNNratio, bestDist2 =
    // INT_MAX when there is no second usable candidate
    auto accept = [&](unsigned long long b, unsigned long long s2) {
        if (b == kNoKey) return false;
        const int d1 = (int)(b >> 40);
        const float d2 = s2 != kNoKey ? (float)(int)(s2 >> 40) : 2147483647.0f;
        return d1 <= 50 && (float)d1 < __fmul_rn(d2, c.nnratio);
    };
    auto commit = [&](int qi, int i1, unsigned long long b) {
        const int i2 = key_idx(b);
        const int prev = s_v21[i2];
        if (prev >= 0) s_v12[prev] = -1;
        s_v12[i1] = (int16_t)i2;
        s_v21[i2] = (int16_t)i1;
        s_md[i2] = (uint16_t)(b >> 40);
        c.res[2 * qi] = i2;  // its rotation bin is taken after the chunks
    };
    for (int base = 0; base < c.nq; base += 64) {
        const int qi = base + lane;
        const bool in = qi < c.nq;
        unsigned long long top[kProjTopK];
        int ncand = 0, src = 0;
#pragma unroll
        for (int k = 0; k < kProjTopK; k++) top[k] = in ? c.scan[(long long)kProjTopK * qi + k] : kNoKey;
        if (in) {
            ncand = c.scan_cnt[qi];
            src = c.q[qi].src;
        }
        int done = 0;
        while (done < 64 && base + done < c.nq) {
            const bool act = in && lane >= done;
            unsigned long long b = kNoKey, s2 = kNoKey;
            int found = 0;
#pragma unroll
            for (int t = 0; t < kProjTopK; t++) {
                const unsigned long long k = top[t];
                if (k == kNoKey || !usable(key_idx(k), (int)(k >> 40))) continue;
                if (found == 0) b = k; else if (found == 1) s2 = k;
                found++;
            }
            const bool rescan = act && found < 2 && ncand > kProjTopK;
            const bool acc = act && !rescan && accept(b, s2);
            const int bi = b != kNoKey ? key_idx(b) : -1;
            const int si = s2 != kNoKey ? key_idx(s2) : -1;
            if (acc) atomicMin(&s_claim[bi & (kClaimTab - 1)], lane);
            wave_lds_sync();
            bool dirty = rescan;
            if (act && bi >= 0 && s_claim[bi & (kClaimTab - 1)] < lane) dirty = true;
            if (act && si >= 0 && s_claim[si & (kClaimTab - 1)] < lane) dirty = true;
            const unsigned long long dm = __ballot(act && dirty);
            const int d = dm ? __ffsll((long long)dm) - 1 : 64;
            wave_lds_sync();
            if (acc) s_claim[bi & (kClaimTab - 1)] = 64;
            if (act && lane < d) {
                if (acc) commit(qi, src, b);
                else c.res[2 * qi] = -1;
            }
            wave_lds_sync();
            if (d < 64 && __shfl((int)rescan, d)) {  // whole-wave re-scan of query base+d
                const int qd = base + d;
                const ProjQuery q = c.q[qd];
                const uint4* qp = (const uint4*)(c.qdesc + (long long)qd * 32);
                unsigned long long t2[2];
                proj_scan<64, 2>(c, q, qp[0], qp[1], lane, [](int) { return false; }, t2, usable);
                if (lane == 0) {
                    if (accept(t2[0], t2[1])) commit(qd, q.src, t2[0]);
                    else c.res[2 * qd] = -1;
                }
                wave_lds_sync();
                done = d + 1;
            } else {
                done = d;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // one wave: order its own global accesses (no L2 write-back)
    if (c.check_ori) {  // every accept is in its bin, stolen ones too (:482); ComputeThreeMaxima (:1601-1642)
        rot_bins(c, lane, s_hist);
        wave_lds_sync();
        int ind1 = -1, ind2 = -1, ind3 = -1, max1 = 0, max2 = 0, max3 = 0;
        for (int i = 0; i < 30; i++) {
            const int sz = s_hist[i];
            if (sz > max1) {
                max3 = max2; max2 = max1; max1 = sz;
                ind3 = ind2; ind2 = ind1; ind1 = i;
            } else if (sz > max2) {
                max3 = max2; max2 = sz;
                ind3 = ind2; ind2 = i;
            } else if (sz > max3) {
                max3 = sz; ind3 = i;
            }
        }
        if (max2 < __fmul_rn(0.1f, (float)max1)) {
            ind2 = -1; ind3 = -1;
        } else if (max3 < __fmul_rn(0.1f, (float)max1)) {
            ind3 = -1;
        }
        for (int q0 = 0; q0 < c.nq; q0 += 64 * kQU) {  // :497-510 (a stolen i1 is already -1)
            int f[kQU], b[kQU], src[kQU];
#pragma unroll
            for (int u = 0; u < kQU; u++) {
                const int qc = min(q0 + 64 * u + lane, c.nq - 1);
                f[u] = c.res[2 * qc];
                b[u] = c.res[2 * qc + 1];
                src[u] = c.q[qc].src;
            }
#pragma unroll
            for (int u = 0; u < kQU; u++)
                if (q0 + 64 * u + lane < c.nq && f[u] >= 0 && b[u] != ind1 && b[u] != ind2 && b[u] != ind3)
                    s_v12[src[u]] = -1;
        }
        wave_lds_sync();
    }
    int nm = 0;
    for (int i = lane; i < c.n_out; i += 64) {
        const int m = s_v12[i];
        if (c.host_out) host_put(c.host_out + i, m, c.seq);
        else c.match[i] = m;
        nm += m >= 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nm += __shfl_xor(nm, o);
    if (lane == 0) {
        if (c.host_out) host_put(c.host_out + c.n_out, nm, c.seq);
        else *c.nmatches = nm;
    }
}

int init_max_features() { return kInitMaxN; }

hipError_t launch_projection(const ProjCall* d_calls, int ncalls, int max_nq, hipStream_t st, bool resolve,
                             bool init, bool grid) {
    if (grid) hipLaunchKernelGGL(k_grid, dim3(ncalls), dim3(1024), 0, st, d_calls);
    if (max_nq > 0) hipLaunchKernelGGL(k_proj_scan, dim3((max_nq + 15) / 16, ncalls), dim3(256), 0, st, d_calls);
    if (init) hipLaunchKernelGGL(k_init_resolve, dim3(ncalls), dim3(64), 0, st, d_calls);
    else if (resolve) hipLaunchKernelGGL(k_proj_resolve, dim3(ncalls), dim3(64), 0, st, d_calls);
    return hipGetLastError();
}

/* ============================ ComputeDistinctiveDescriptors ============================ */

constexpr int kDistinctMaxObs = 1024;
constexpr int kDistinctWaves = 4;

__device__ __forceinline__ int desc_dist(const uint4 q0, const uint4 q1, const uint8_t* dj) {
    const uint4 c0 = ((const uint4*)dj)[0], c1 = ((const uint4*)dj)[1];
    return __popc(q0.x ^ c0.x) + __popc(q0.y ^ c0.y) + __popc(q0.z ^ c0.z) + __popc(q0.w ^ c0.w) +
           __popc(q1.x ^ c1.x) + __popc(q1.y ^ c1.y) + __popc(q1.z ^ c1.z) + __popc(q1.w ^ c1.w);
}

__global__ __launch_bounds__(64 * kDistinctWaves) void k_distinctive(int npoints, const int32_t* __restrict__ off,
                                                                      const uint8_t* __restrict__ desc,
                                                                      int32_t* __restrict__ best_idx,
                                                                      uint8_t* __restrict__ out_desc) {
    __shared__ uint16_t s_d[kDistinctWaves][kDistinctMaxObs];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int p = blockIdx.x * kDistinctWaves + wv;
    if (p >= npoints) return;
    const int b = off[p], N = off[p + 1] - b;
    if (N <= 0) {  // no observations / all observing KeyFrames bad: mDescriptor unchanged
        if (lane == 0) best_idx[p] = -1;
        return;
    }
    const bool in_lds = N <= kDistinctMaxObs;  // longer rows are recomputed per radix pass
    uint16_t* d = s_d[wv];
    const uint8_t* rows = desc + (long long)b * 32;
    const int k = (int)(0.5 * (N - 1));  // vDists[0.5*(N-1)] (MapPoint.cc:290)
    int bestMedian = 0x7fffffff, bestIdx = 0;
    for (int i = 0; i < N; i++) {
        const uint4 q0 = ((const uint4*)(rows + (long long)i * 32))[0], q1 = ((const uint4*)(rows + (long long)i * 32))[1];
        if (in_lds) {
            for (int j = lane; j < N; j += 64) d[j] = (uint16_t)desc_dist(q0, q1, rows + (long long)j * 32);
            wave_lds_sync();
        }
        // k-th smallest of row i (Distances[i][i] = 0 is part of the row): 9-bit radix select
        int prefix = 0, rank = k;
        for (int bit = 8; bit >= 0; bit--) {
            int cnt0 = 0;
            for (int j0 = 0; j0 < N; j0 += 64) {
                const int j = j0 + lane;
                int v = 0x7fff;
                if (j < N) v = in_lds ? d[j] : desc_dist(q0, q1, rows + (long long)j * 32);
                const bool in = j < N && (v >> (bit + 1)) == (prefix >> (bit + 1)) && !((v >> bit) & 1);
                cnt0 += __popcll(__ballot(in));
            }
            if (rank >= cnt0) {
                rank -= cnt0;
                prefix |= 1 << bit;
            }
        }
        wave_lds_sync();
        if (prefix < bestMedian) {  // first strict minimum (MapPoint.cc:292-296)
            bestMedian = prefix;
            bestIdx = i;
        }
    }
    if (lane == 0) best_idx[p] = bestIdx;
    if (out_desc && lane < 8)
        ((uint32_t*)(out_desc + (long long)p * 32))[lane] = ((const uint32_t*)(rows + (long long)bestIdx * 32))[lane];
}

hipError_t launch_distinctive(int npoints, const int32_t* off, const uint8_t* desc, int32_t* best_idx,
                              uint8_t* out_desc, hipStream_t st) {
    if (npoints <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_distinctive, dim3((npoints + kDistinctWaves - 1) / kDistinctWaves), dim3(64 * kDistinctWaves),
                       0, st, npoints, off, desc, best_idx, out_desc);
    return hipGetLastError();
}

int stereo_lds_bytes(int cap, int nrows) { return StereoLds(cap, nrows).total; }

hipError_t stereo_setup(int lds_bytes) {
    hipError_t e = hipFuncSetAttribute((const void*)k_stereo<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute((const void*)k_stereo<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

hipError_t launch_stereo(const StereoArgs& a, int npairs, const int32_t* fl, const int32_t* fr, const orbx_kp* kpsL,
                         const uint8_t* descL, const int32_t* cntL, const orbx_kp* kpsR, const uint8_t* descR,
                         const int32_t* cntR, int stride, float* uright, float* depth, int32_t* nstereo, int32_t* sad,
                         int* err, hipStream_t st) {
    const int lds = stereo_lds_bytes(stride, a.nrows);
    // level-0 rows of both sides 4-byte aligned (the pyramid levels always are): the windows are staged as dwords
    auto rows_aligned = [](const PyrSide& s) {
        return (((uintptr_t)s.l0 | (uintptr_t)s.l0_fstride | (uintptr_t)s.l0_pitch) & 3) == 0;
    };
    if (rows_aligned(a.left) && rows_aligned(a.right))
        hipLaunchKernelGGL(k_stereo<true>, dim3(npairs * kStereoSplit), dim3(kStereoThreads), lds, st, a, fl, fr, kpsL,
                           descL, cntL, kpsR, descR, cntR, stride, uright, depth, sad, err);
    else
        hipLaunchKernelGGL(k_stereo<false>, dim3(npairs * kStereoSplit), dim3(kStereoThreads), lds, st, a, fl, fr, kpsL,
                           descL, cntL, kpsR, descR, cntR, stride, uright, depth, sad, err);
    hipLaunchKernelGGL(k_stereo_median, dim3(npairs), dim3(256), 0, st, fl, fr, cntL, cntR, a.left.nframes,
                       a.right.nframes, stride, a.thc, uright, depth, sad, nstereo);
    return hipGetLastError();
}

}  // namespace orbamd
