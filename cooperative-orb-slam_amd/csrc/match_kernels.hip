/*
 * match_kernels.hip -- gfx950 kernels for ORBmatcher (ORBmatcher.cc).
 *
 *   k_tri_mfma        SearchForTriangulation, one FeatureVector node holding every feature
 *                     (BASELINE "BF"), batch of frame pairs: Hamming distances as a +-1 fp4
 *                     GEMM on the matrix cores, then the reference's selection
 *                     -- ORBmatcher.cc:657-823, 1647-1663.
 *   k_tri_nodes       SearchForTriangulation over common BoW nodes (general form).
 *   k_tri_nodes_pairs the same for a batch of frame pairs, FeatureVectors on the device.
 *   k_bow_pairs       SearchByBoW (KF,F) / (KF,KF) for a batch of frame pairs, FeatureVectors on the device.
 *   k_bow             SearchByBoW(KF,F) / SearchByBoW(KF,KF): per common node, greedy over the
 *                     node's queries in order, wave-parallel best/second-best over candidates
 *                     (ORBmatcher.cc:159-288, 522-655).
 *   k_rot_filter      rotation-histogram consistency + ComputeThreeMaxima
 *                     (ORBmatcher.cc:236-246, 267-285, 1601-1642).
 * Candidate order / tie rules are the reference's (DESIGN.md "Matcher semantics").
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>

#include "../../include/orbslam_amd.h"
#include "orb_match.h"
#include "orb_wave.h"

namespace orbamd {

__device__ __forceinline__ int hamming8(const uint32_t* a, const uint32_t* b) {
    int d = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) d += __popc(a[k] ^ b[k]);
    return d;
}

/* CheckDistEpipolarLine (ORBmatcher.cc:140-157) with the line (a,b,c) of kp1 precomputed
 * (same float ops); compare in double like `dsqr < 3.84*sigma2`. */
__device__ __forceinline__ bool epi_ok(float a, float b, float c, float x2, float y2, double th384) {
    const float num = __fadd_rn(__fadd_rn(__fmul_rn(a, x2), __fmul_rn(b, y2)), c);
    const float den = __fadd_rn(__fmul_rn(a, a), __fmul_rn(b, b));
    if (den == 0.f) return false;
    const float dsqr = __fdiv_rn(__fmul_rn(num, num), den);
    return (double)dsqr < th384;
}

/* the same test against the float threshold thf = 3.84*sigma2 rounded up to a float (MatchGeom::th384f):
 * for a float dsqr, (double)dsqr < th384 <=> dsqr < thf, so the comparison is exact; thf < 0 rejects */
__device__ __forceinline__ bool epi_ok_f(float a, float b, float c, float x2, float y2, float thf) {
    const float num = __fadd_rn(__fadd_rn(__fmul_rn(a, x2), __fmul_rn(b, y2)), c);
    const float den = __fadd_rn(__fmul_rn(a, a), __fmul_rn(b, b));
    if (den == 0.f) return false;
    const float dsqr = __fdiv_rn(__fmul_rn(num, num), den);
    return dsqr < thf;
}

__device__ __forceinline__ void epi_line(const MatchGeom& g, float x1, float y1, float* a, float* b, float* c) {
    *a = __fadd_rn(__fadd_rn(__fmul_rn(x1, g.F[0]), __fmul_rn(y1, g.F[3])), g.F[6]);
    *b = __fadd_rn(__fadd_rn(__fmul_rn(x1, g.F[1]), __fmul_rn(y1, g.F[4])), g.F[7]);
    *c = __fadd_rn(__fadd_rn(__fmul_rn(x1, g.F[2]), __fmul_rn(y1, g.F[5])), g.F[8]);
}

/* epipole-radius rejection for mono-mono pairs (ORBmatcher.cc:743-749) */
__device__ __forceinline__ bool near_epipole(const MatchGeom& g, float x2, float y2, int oct2) {
    const float dx = __fsub_rn(g.ex, x2), dy = __fsub_rn(g.ey, y2);
    return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < g.th100[oct2];
}

/* Pair p: KF1 = (kps1, desc1, n1), KF2 = (kps2, desc2, n2) resolved by the caller-side
 * accessor; no MapPoints (BF bench configuration). ur1 / ur2: mvuRight of each keyframe (the stereo
 * form, k_tri_mfma<true>; unread by the mono form). */
struct PairSrc {
    const orbx_kp* kps1; const uint8_t* desc1; int n1;
    const orbx_kp* kps2; const uint8_t* desc2; int n2;
    const float* ur1; const float* ur2;
};

/* ----------------------------------------------------------------------------------- */
/* MFMA form of the BF SearchForTriangulation scan.                                      */
/*                                                                                       */
/* Hamming distance as a +-1 GEMM: with both operands mapped to (2b-1) in {-1,+1},        */
/*     dot' = sum_k (2a_k-1)(2b_k-1) = 256 - 2 D(a, b)                                    */
/* v_mfma_scale_f32_32x32x64_f8f6f4 on fp4 (e2m1) operands computes a 32 candidate x 32  */
/* query tile of dot' per 64 descriptor bits (exact in the f32 accumulator); 4 steps     */
/* cover 256 bits. Lane l holds query (l & 31) and candidates (reg&3) + 8(reg>>2) +     */
/* 4(l>>5) of the tile.                                                                  */
/*                                                                                       */
/* Selection: key = D << 16 | (65535 - idx2); the reference's scan (accept dist <= best,   */
/* geometric checks only for those) returns the valid candidate of minimum key             */
/* (DESIGN.md "Matcher semantics"). Per tile each lane takes its minimum key; only if it    */
/* beats the running best with D <= TH_LOW are the candidate's checks evaluated (epipole   */
/* radius, CheckDistEpipolarLine), walking up the lane's keys until one passes.           */
/* ----------------------------------------------------------------------------------- */
typedef int v4i __attribute__((ext_vector_type(4)));

/* fp4 form: both operands as +-1 (e2m1 nibbles: +1.0 = 0x2, -1.0 = 0xA, block scale 2^0), so the  */
/* 32x32x64 product gives dot' = sum (2a-1)(2b-1) = 256 - 2 D over 256 bits in 4 instructions    */
/* (the i8 form needs 8), exact in the f32 accumulator. 8 descriptor bits -> one dword of 8       */
/* nibbles: nibble 2i = bit i, nibble 2i+1 = bit 4+i (any fixed order serves: both operands use */
/* it, so the k order inside an instruction is irrelevant). The sign bit (nibble bit 3) is set   */
/* for a clear descriptor bit: spread of the inverted nibbles by one multiply each.             */
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
__device__ __forceinline__ uint32_t fp4_pm1_byte(uint32_t nb) {  // nb = the INVERTED byte in bits 0..7
    const uint32_t lo = nb & 15u, hi = (nb >> 4) & 15u;
    return ((hi * 0x10204080u) & 0x80808080u) | (((lo * 0x01020408u) & 0x08080808u) | 0x22222222u);
}
__device__ __forceinline__ v4i fp4_pm1_dword(uint32_t w) {  // 32 descriptor bits -> 128 bits of fp4
    const uint32_t n = ~w;
    return (v4i){(int)fp4_pm1_byte(n), (int)fp4_pm1_byte(n >> 8), (int)fp4_pm1_byte(n >> 16), (int)fp4_pm1_byte(n >> 24)};
}
__device__ __forceinline__ v8i fp4_operand(v4i a) {  // fp4 reads only the low 4 registers of an operand
    return __builtin_shufflevector(a, a, 0, 1, 2, 3, -1, -1, -1, -1);
}

constexpr int kMfChunk = 64;  // candidates staged per step (two 32-row tiles)
constexpr int kMfBufs = 2;   // LDS chunk buffers of k_tri_mfma (staging of chunk c+1 overlaps chunk c's MFMAs)
constexpr int kMfWaves = 8;    // query waves per workgroup (32 queries each); they share each chunk's expansion
constexpr int kMfThreads = 64 * kMfWaves;

/* Per 64-candidate chunk each thread expands descriptor dwords of one candidate (8 KB of fp4     */
/* fragments in LDS), each wave runs 4 MFMAs per 32-candidate tile, and the packed selection key   */
/* is the f32 accumulator's bit pattern (dot' is an even integer <= 256: its low 14 mantissa bits  */
/* are zero) OR the tile row, whose signed maximum is the first candidate of maximum dot' =        */
/* minimum D with ties to the later row.                                                          */
/* STEREO: keyframes with mvuRight (ORBmatcher.cc:703-749): the epipole-radius test applies only when both the
 * query and the candidate are monocular (!bStereo1 && !bStereo2), and with only_stereo a monocular query or
 * candidate takes no part. The candidate record's w is 1 for a monocular candidate near the epipole (rejected for
 * a monocular query only); the mono form folds that test into the threshold (-1) as before. */
template <bool STEREO>
__device__ __forceinline__ void tri_mfma_body_fp4(const PairSrc& s, const MatchGeom& g, int32_t* __restrict__ out,
                                                  int32_t* __restrict__ nmatch, int only_stereo) {
    static_assert(kMfWaves == 4 || kMfWaves == 8, "fp4 expansion roles: 4 waves (2 dwords per thread) or 8 (1)");
    constexpr int kDw = 512 / kMfThreads;  // descriptor dwords expanded per thread and chunk
    __shared__ v4i s_frag[kMfBufs][2][4][64];  // [buffer][tile][step][lane] candidate fragments (fp4 +-1)
    // per candidate (x, y, epipolar threshold thf or -1 when it is near the epipole / past n2): one
    // ds_read_b128 per geometric check in the key walk (instead of four b32 reads + a threshold gather)
    __shared__ float4 s_rec[kMfBufs][kMfChunk];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int qblk = blockIdx.x * (32 * kMfWaves);
    if (qblk >= s.n1) return;  // block-uniform
    const int h = lane >> 5;
    const int qi = qblk + wave * 32 + (lane & 31);
    const bool qon = qi < s.n1;
    // bStereo1 (ORBmatcher.cc:703); with bOnlyStereo a monocular query is skipped (:705-707): output -1
    const bool st1 = STEREO && qon && s.ur1[qi] >= 0.f;
    const bool qact = qon && (!STEREO || !only_stereo || st1);
    // query fragments: step st covers descriptor bits 64 st .. 64 st + 63, lane half h dword 2 st + h
    v4i bq[4];
    float la = 0.f, lb = 0.f, lc = 0.f;
    {
        const int qc = qon ? qi : 0;
        const uint4* qd = (const uint4*)(s.desc1 + (long long)qc * 32);
        const uint4 d0 = qd[0], d1 = qd[1];
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int st = 0; st < 4; st++) bq[st] = fp4_pm1_dword(h ? dw[2 * st + 1] : dw[2 * st]);
        const orbx_kp k1 = s.kps1[qc];
        epi_line(g, k1.x, k1.y, &la, &lb, &lc);
    }
    uint32_t best = 0xFFFFFFFFu;
    // expansion role: candidate ec of the chunk, descriptor dwords ed .. ed + kDw - 1 (dword d = step d / 2,
    // half d % 2). Lanes 8i..8i+7 (one lane group of ds_write_b128) take 8 consecutive candidates of one
    // dword, so their 16-byte fragment stores land on distinct banks (candidates in a group sharing a
    // dword would all hit the same four banks: 8-way conflicts)
    const int ec = (tid >> 6) * (64 / kMfWaves) + (tid & 7) + (kDw == 1 ? 0 : 8 * ((tid >> 5) & 1));
    const int ed = kDw == 1 ? (tid >> 3) & 7 : 2 * ((tid >> 3) & 3);
    struct DwT { uint32_t w[kDw]; };
    auto load_chunk = [&](int cb, DwT& d, orbx_kp& k2, float& u2) {
        const int c = min(cb + ec, s.n2 - 1);
        d = *(const DwT*)(s.desc2 + (long long)c * 32 + 4 * ed);
        const int c2 = min(cb + (tid & (kMfChunk - 1)), s.n2 - 1);
        k2 = s.kps2[c2];
        if (STEREO) u2 = s.ur2[c2];
    };
    DwT pd;
    orbx_kp pk;
    float pu = -1.f;
    load_chunk(0, pd, pk, pu);
    // chunk staging into LDS buffer bw (candidates cbw ..): expansion of the prefetched descriptor dwords and the
    // per-candidate geometry record
    auto stage = [&](int cbw, int bw) {
        const bool on = cbw + ec < s.n2;
        const int tile = ec >> 5, r = ec & 31;
#pragma unroll
        for (int k = 0; k < kDw; k++)
            s_frag[bw][tile][(ed + k) >> 1][32 * ((ed + k) & 1) + r] = fp4_pm1_dword(on ? pd.w[k] : 0u);
        if (tid < kMfChunk) {
            if (STEREO) {
                const bool st2 = pu >= 0.f;  // bStereo2 (:727); only_stereo skips a monocular candidate (:729-731)
                const bool on2 = cbw + tid < s.n2 && (!only_stereo || st2);
                const bool near = !st2 && near_epipole(g, pk.x, pk.y, pk.octave);
                s_rec[bw][tid] = make_float4(pk.x, pk.y, on2 ? g.th384f[pk.octave] : -1.0f, near ? 1.0f : 0.0f);
            } else {
                const bool on2 = cbw + tid < s.n2 && !near_epipole(g, pk.x, pk.y, pk.octave);
                s_rec[bw][tid] = make_float4(pk.x, pk.y, on2 ? g.th384f[pk.octave] : -1.0f, 0.0f);
            }
        }
    };
    // double-buffered: chunk c+1 is expanded into the other buffer before chunk c's MFMAs, so one barrier per chunk
    // (the one that publishes c+1 and retires c's reads) instead of two
    stage(0, 0);
    __syncthreads();
    if (kMfChunk < s.n2) load_chunk(kMfChunk, pd, pk, pu);
    for (int cb = 0, bf = 0; cb < s.n2; cb += kMfChunk, bf ^= 1) {
        if (cb + kMfChunk < s.n2) {
            stage(cb + kMfChunk, bf ^ 1);
            if (cb + 2 * kMfChunk < s.n2) load_chunk(cb + 2 * kMfChunk, pd, pk, pu);
        }
        v16f acc0 = (v16f)0.f, acc1 = (v16f)0.f;
#pragma unroll
        for (int st = 0; st < 4; st++) {
            // cbsz = blgp = 4: fp4 (e2m1) A and B; E8M0 scales 127 = 2^0
            acc0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fp4_operand(s_frag[bf][0][st][lane]), fp4_operand(bq[st]),
                                                                   acc0, 4, 4, 0, 127, 0, 127);
            acc1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fp4_operand(s_frag[bf][1][st][lane]), fp4_operand(bq[st]),
                                                                   acc1, 4, 4, 0, 127, 0, 127);
        }
#pragma unroll
        for (int tile = 0; tile < 2; tile++) {
            const v16f acc = tile ? acc1 : acc0;
            // key = D << 16 | (65535 - idx2) with D = (256 - dot') / 2 and idx2 = cb + 32 tile + 4 h + row
            const uint32_t kb = 65535u - (uint32_t)(cb + 32 * tile + 4 * h);
            auto pk = [&](int rg) { return __float_as_int(acc[rg]) | ((rg & 3) + 8 * (rg >> 2)); };
            auto key = [&](int p) {
                const float dp = __int_as_float(p & ~31);
                return ((uint32_t)(int)(256.f - dp) >> 1 << 16) + kb - (uint32_t)(p & 31);
            };
            int pmax = pk(0);
#pragma unroll
            for (int rg = 1; rg < 16; rg++) pmax = max(pmax, pk(rg));
            uint32_t km = key(pmax);
            while (km < best && (km >> 16) <= 50u) {  // TH_LOW (ORBmatcher.cc:715)
                const int jl = (int)(65535u - (km & 0xFFFFu)) - cb;
                const float4 c2 = s_rec[bf][jl];
                if ((!STEREO || st1 || c2.w == 0.0f) && epi_ok_f(la, lb, lc, c2.x, c2.y, c2.z)) {
                    best = km;
                    break;
                }
                // next key of the lane = largest packed value below the rejected one (rows are distinct);
                // a negative dot' (D > 128) ends the walk through the threshold test
                const int cur = pmax;
                int nx = INT_MIN;
#pragma unroll
                for (int rg = 0; rg < 16; rg++) nx = pk(rg) < cur ? max(nx, pk(rg)) : nx;
                pmax = nx;
                km = nx == INT_MIN ? 0xFFFFFFFFu : key(nx);
            }
        }
        __syncthreads();
    }
    best = min(best, (uint32_t)__shfl_xor((int)best, 32, 64));
    if (qon && h == 0) {
        const int idx2 = qact && (best >> 16) <= 50u ? (int)(65535u - (best & 0xFFFFu)) : -1;
        out[qi] = idx2;
        if (idx2 >= 0) atomicAdd(nmatch, 1);
    }
}

// 6 waves per SIMD: the compiler fits the kernel in 80 VGPRs (88 unconstrained: 5 waves) without scratch; match-only
// +19 % (C2 3.50M -> 4.18M pairs/s, 18.2 % -> 21.7 % of the fp4 peak), C2 step +0.5-1 %, C3 +-0, C4 -0.6 %
// (profiles/r05_ab_match_occupancy.log)
#ifndef ORBX_MF_WPE
#define ORBX_MF_WPE 6
#endif
#define ORBX_MF_ATTR __attribute__((amdgpu_waves_per_eu(ORBX_MF_WPE)))
template <bool STEREO>
__global__ __launch_bounds__(kMfThreads) ORBX_MF_ATTR void k_tri_mfma(const int32_t* __restrict__ q1, const int32_t* __restrict__ q2,
                                                  const orbx_kp* __restrict__ kps, const uint8_t* __restrict__ desc,
                                                  const int32_t* __restrict__ counts, const float* __restrict__ uright,
                                                  int kp_stride, MatchGeom g, int only_stereo,
                                                  int32_t* __restrict__ match12, int32_t* __restrict__ nmatches) {
    const int p = blockIdx.y;
    const int f1 = q1[p], f2 = q2[p];
    PairSrc s;
    s.kps1 = kps + (long long)f1 * kp_stride; s.desc1 = desc + (long long)f1 * kp_stride * 32; s.n1 = counts[f1];
    s.kps2 = kps + (long long)f2 * kp_stride; s.desc2 = desc + (long long)f2 * kp_stride * 32; s.n2 = counts[f2];
    s.ur1 = STEREO ? uright + (long long)f1 * kp_stride : nullptr;
    s.ur2 = STEREO ? uright + (long long)f2 * kp_stride : nullptr;
    tri_mfma_body_fp4<STEREO>(s, g, match12 + (long long)p * kp_stride, nmatches + p, only_stereo);
}

/* rotation bin of a match (ORBmatcher.cc:236-246): rot = angA[a] - angB[b], (a,b) = (i, j) or,
 * with swap, (j, i) */
__device__ __forceinline__ int rot_bin(const float* angA, const float* angB, int i, int j, int swap) {
    float rot = swap ? __fsub_rn(angA[j], angB[i]) : __fsub_rn(angA[i], angB[j]);
    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
    int bin = (int)roundf(__fmul_rn(rot, 1.0f / 30));
    return bin == 30 ? 0 : bin;
}

/* ComputeThreeMaxima (ORBmatcher.cc:1601-1642) over a 30-bin histogram, by one thread */
__device__ __forceinline__ void three_maxima(const int* hist, int* keep) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < 30; i++) {
        const int s = hist[i];
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
        else if (s > max3) { max3 = s; ind3 = i; }
    }
    if (max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
    else if (max3 < __fmul_rn(0.1f, (float)max1)) { ind3 = -1; }
    keep[0] = ind1; keep[1] = ind2; keep[2] = ind3;
}

/* Single host-API call (k_tri_nodes / k_bow), one launch: every accepted match is appended to a
 * compact device list with its rotation bin (ORBmatcher.cc:236-246), and the bin counted in a device
 * histogram, as it is made. The last workgroup of the launch to finish (a ticket; agent-scope fences
 * order every workgroup's list writes before it) takes ComputeThreeMaxima of the histogram
 * (ORBmatcher.cc:1601-1642) and writes the surviving matches and their count straight into the
 * caller's pinned host buffer, which the host filled with -1 (host_out[0] = count, host_out[1 + i]).
 * Its work is proportional to the matches, not to N. The state words are zero between calls. */
__device__ __forceinline__ void call_emit(const CallTail& t, int i, int j) {
    const int bin = t.check_ori ? rot_bin(t.angA, t.angB, i, j, t.swap) : 0;
    if (t.check_ori) atomicAdd(t.state + 2 + bin, 1);
    const int k = atomicAdd(t.state + 1, 1);
    ((int4*)t.list)[k] = make_int4(i, j, bin, 0);
}

__device__ void call_tail(const CallTail& t) {
    __shared__ int s_last, s_cnt, s_nl;
    __shared__ int hist[30], keep[3];
    __syncthreads();
    __threadfence();
    if (threadIdx.x == 0) s_last = atomicAdd(t.state, 1) == (int)(gridDim.x - 1);
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    if (threadIdx.x < 30) hist[threadIdx.x] = t.check_ori ? t.state[2 + threadIdx.x] : 0;
    if (threadIdx.x == 0) {
        s_cnt = 0;
        s_nl = t.state[1];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (t.check_ori) three_maxima(hist, keep);
        else keep[0] = keep[1] = keep[2] = -2;
    }
    __syncthreads();
    const int nl = s_nl;
    int local = 0;
    for (int k = threadIdx.x; k < nl; k += blockDim.x) {
        const int4 e = ((const int4*)t.list)[k];
        if (!t.check_ori || e.z == keep[0] || e.z == keep[1] || e.z == keep[2]) {
            t.host_out[1 + e.x] = e.y;
            local++;
        }
    }
    atomicAdd(&s_cnt, local);
    __threadfence_system();  // this wave's match writes reach host memory before the count
    __syncthreads();
    if (threadIdx.x < 30) t.state[2 + threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        t.state[1] = 0;
        t.state[0] = 0;
        // the count is the call's completion word: the host polls it (capi.cpp wait_call) instead of
        // synchronising the stream, so it is stored last, with release at system scope
        __hip_atomic_store(t.host_out, s_cnt, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* ----------------------------------------------------------------------------------- */
/* General node-based SearchForTriangulation (host API, one keyframe pair per call):     */
/* one 256-thread workgroup per (common node, 64 queries). The node's candidates are      */
/* staged through LDS kNodeStage at a time (descriptor, position, octave, eligibility:    */
/* one round of global-load latency per round instead of a dependent chain per candidate)  */
/* and the 4 waves scan interleaved quarters of each round for the same 64 queries. The    */
/* reference's scan (ORBmatcher.cc:704-776: skip dist > TH_LOW or > best, geometric checks, */
/* accept ties) returns the valid candidate of minimum distance, the later one on ties, so */
/* the quarters merge by (distance, node position).                                        */
/* ----------------------------------------------------------------------------------- */
constexpr int kNodeStage = 256;

__global__ __launch_bounds__(256) void k_tri_nodes(const DevView v1, const DevView v2, const NodeTask* __restrict__ tasks,
                                                   MatchGeom g, int only_stereo, CallTail tail) {
    __shared__ uint4 s_d[kNodeStage * 2];
    __shared__ float s_x[kNodeStage], s_y[kNodeStage];
    __shared__ int s_oct[kNodeStage];  // octave | 0x100 stereo; -1 = not a candidate (MapPoint / mono in stereo mode)
    __shared__ int s_idx[kNodeStage];
    __shared__ int s_bd[4][64], s_bp[4][64];
    const NodeTask t = tasks[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, part = tid >> 6;
    const int i1 = t.q_begin + lane;
    const int idx1 = i1 < t.q_end ? v1.node_feat[i1] : -1;
    const bool st1 = idx1 >= 0 && v1.uright ? v1.uright[idx1] >= 0.f : false;
    const bool active = idx1 >= 0 && !(v1.has_mp && v1.has_mp[idx1]) && (!only_stereo || st1);
    uint32_t q[8];
    float a = 0.f, b = 0.f, c = 0.f;
    if (active) {
        const uint4* qd = (const uint4*)(v1.desc + (long long)idx1 * 32);
        const uint4 qa = qd[0], qb = qd[1];
        q[0] = qa.x; q[1] = qa.y; q[2] = qa.z; q[3] = qa.w; q[4] = qb.x; q[5] = qb.y; q[6] = qb.z; q[7] = qb.w;
        epi_line(g, v1.x[idx1], v1.y[idx1], &a, &b, &c);
    }
    int bestDist = 50, bestPos = -1, bestIdx2 = -1;  // TH_LOW (ORBmatcher.cc:704)
    for (int cb = t.c_begin; cb < t.c_end; cb += kNodeStage) {
        const int nt = min(kNodeStage, t.c_end - cb);
        __syncthreads();
        if (tid < nt) {
            const int idx2 = v2.node_feat[cb + tid];
            const bool st2 = v2.uright ? v2.uright[idx2] >= 0.f : false;
            const bool ok = !(v2.has_mp && v2.has_mp[idx2]) && (!only_stereo || st2);
            const uint4* cd = (const uint4*)(v2.desc + (long long)idx2 * 32);
            s_d[2 * tid] = cd[0];
            s_d[2 * tid + 1] = cd[1];
            s_x[tid] = v2.x[idx2];
            s_y[tid] = v2.y[idx2];
            s_oct[tid] = ok ? (v2.octave[idx2] | (st2 ? 0x100 : 0)) : -1;
            s_idx[tid] = idx2;
        }
        __syncthreads();
        if (!active) continue;
        for (int j = part; j < nt; j += 4) {
            const int oc = s_oct[j];
            if (oc < 0) continue;
            const uint4 c0 = s_d[2 * j], c1 = s_d[2 * j + 1];
            const int dist = __popc(q[0] ^ c0.x) + __popc(q[1] ^ c0.y) + __popc(q[2] ^ c0.z) + __popc(q[3] ^ c0.w) +
                             __popc(q[4] ^ c1.x) + __popc(q[5] ^ c1.y) + __popc(q[6] ^ c1.z) + __popc(q[7] ^ c1.w);
            if (dist > 50 || dist > bestDist) continue;
            const float x2 = s_x[j], y2 = s_y[j];
            const int oct2 = oc & 0xFF;
            if (!st1 && !(oc & 0x100) && near_epipole(g, x2, y2, oct2)) continue;  // ORBmatcher.cc:743-749
            if (epi_ok(a, b, c, x2, y2, g.th384[oct2])) {
                bestDist = dist;
                bestPos = cb + j;
                bestIdx2 = s_idx[j];
            }
        }
    }
    s_bd[part][lane] = bestDist;
    s_bp[part][lane] = bestPos;
    __syncthreads();
    if (part == 0 && active) {
        for (int k = 1; k < 4; k++) {
            const int d = s_bd[k][lane], pos = s_bp[k][lane];
            if (pos >= 0 && (bestPos < 0 || d < bestDist || (d == bestDist && pos > bestPos))) {
                bestDist = d;
                bestPos = pos;
            }
        }
        if (bestPos >= 0) call_emit(tail, idx1, bestPos == s_bp[0][lane] ? bestIdx2 : v2.node_feat[bestPos]);
    }
    call_tail(tail);
}

/* ----------------------------------------------------------------------------------- */
/* SearchForTriangulation over common BoW nodes for a batch of frame pairs, with the       */
/* FeatureVectors of orbv_transform_batch_device (levelsup nodes) left on the device:       */
/* block (i, p) takes node i of KF1 = frame q1[p]; its partner in KF2 = frame q2[p] is      */
/* found by binary search over KF2's ascending node ids (the reference's merge walk,        */
/* ORBmatcher.cc:691-789, visits exactly the common ids). One lane per query of the node,   */
/* candidates scanned in node order with the reference's rule (dist > TH_LOW or > best:     */
/* skip; epipole radius and CheckDistEpipolarLine; accept = new best, ties to the later).   */
/* All keypoints mono, no MapPoints (the batch configuration of k_tri_mfma).               */
/* ----------------------------------------------------------------------------------- */
__global__ __launch_bounds__(64) void k_tri_nodes_pairs(const int32_t* __restrict__ q1, const int32_t* __restrict__ q2,
                                                        const orbx_kp* __restrict__ kps, const uint8_t* __restrict__ desc,
                                                        int kp_stride, const uint32_t* __restrict__ fv_node,
                                                        const int32_t* __restrict__ fv_off,
                                                        const int32_t* __restrict__ fv_feat,
                                                        const int32_t* __restrict__ nfv, MatchGeom g,
                                                        int32_t* __restrict__ match12, int32_t* __restrict__ nmatches) {
    const int p = blockIdx.y, i = blockIdx.x;
    const int f1 = q1[p], f2 = q2[p];
    if (i >= nfv[f1]) return;
    const uint32_t* nodes2 = fv_node + (long long)f2 * kp_stride;
    const uint32_t node = fv_node[(long long)f1 * kp_stride + i];
    int lo = 0, hi = nfv[f2];
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (nodes2[mid] < node) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= nfv[f2] || nodes2[lo] != node) return;  // not a common node: its queries stay -1
    const int32_t* off1 = fv_off + (long long)f1 * (kp_stride + 1);
    const int32_t* off2 = fv_off + (long long)f2 * (kp_stride + 1);
    const int32_t* feat1 = fv_feat + (long long)f1 * kp_stride;
    const int32_t* feat2 = fv_feat + (long long)f2 * kp_stride;
    const orbx_kp* k1 = kps + (long long)f1 * kp_stride;
    const orbx_kp* k2 = kps + (long long)f2 * kp_stride;
    const uint8_t* d1 = desc + (long long)f1 * kp_stride * 32;
    const uint8_t* d2 = desc + (long long)f2 * kp_stride * 32;
    const int cb = off2[lo], ce = off2[lo + 1];
    for (int qi = off1[i] + (int)threadIdx.x; qi < off1[i + 1]; qi += 64) {
        const int idx1 = feat1[qi];
        uint32_t q[8];
        const uint4* qd = (const uint4*)(d1 + (long long)idx1 * 32);
        const uint4 qa = qd[0], qb = qd[1];
        q[0] = qa.x; q[1] = qa.y; q[2] = qa.z; q[3] = qa.w; q[4] = qb.x; q[5] = qb.y; q[6] = qb.z; q[7] = qb.w;
        const orbx_kp kp1 = k1[idx1];
        float a, b, c;
        epi_line(g, kp1.x, kp1.y, &a, &b, &c);
        int bestDist = 50, bestIdx2 = -1;  // TH_LOW (ORBmatcher.cc:704)
        for (int ci = cb; ci < ce; ci++) {
            const int idx2 = feat2[ci];
            const int dist = hamming8(q, (const uint32_t*)(d2 + (long long)idx2 * 32));
            if (dist > 50 || dist > bestDist) continue;
            const orbx_kp kp2 = k2[idx2];
            if (near_epipole(g, kp2.x, kp2.y, kp2.octave)) continue;  // mono-mono (:743-749)
            if (epi_ok(a, b, c, kp2.x, kp2.y, g.th384[kp2.octave])) {
                bestIdx2 = idx2;
                bestDist = dist;
            }
        }
        match12[(long long)p * kp_stride + idx1] = bestIdx2;
        if (bestIdx2 >= 0) atomicAdd(&nmatches[p], 1);
    }
}

/* ----------------------------------------------------------------------------------- */
/* SearchByBoW: one wave per common node. Queries of node1 in order (greedy exclusion of */
/* already-matched candidates is node-local); per query the wave computes best/second   */
/* best over node2 with the sequential scan's semantics: best1 = first strict minimum,   */
/* best2 = second smallest of the multiset.                                              */
/* mode 0 = (KF,F): accept best1 <= TH_LOW, query needs a good MapPoint, candidates any  */
/* mode 1 = (KF,KF): accept best1 < TH_LOW, both sides need a good MapPoint.             */
/* out[idx of the side that is marked] as in the reference (F index / idx1).            */
/* ----------------------------------------------------------------------------------- */
struct Top2 { int b1, i1, b2; };
__device__ __forceinline__ Top2 top2_merge(Top2 A, Top2 B) {
    Top2 r;
    const bool takeB = (B.b1 < A.b1) || (B.b1 == A.b1 && B.i1 >= 0 && (A.i1 < 0 || B.i1 < A.i1));
    r.b1 = takeB ? B.b1 : A.b1;
    r.i1 = takeB ? B.i1 : A.i1;
    r.b2 = min(max(A.b1, B.b1), min(A.b2, B.b2));
    return r;
}


/* STAGED (node of <= kBowStage candidates, the common case: ~10 per node at levelsup 4): the node's
 * candidate descriptors and eligibility and, 64 at a time, its queries' descriptors are staged in LDS
 * first, so the greedy loop over queries runs without a global-load round trip per query */
constexpr int kBowStage = 512;

template <bool STAGED>
__global__ __launch_bounds__(64) void k_bow(const DevView vq, const DevView vc, const NodeTask* __restrict__ tasks,
                                            float nnratio, int mode, CallTail tail) {
    extern __shared__ uint8_t matched[];  // per candidate position in the node (unstaged form)
    __shared__ uint4 s_cd[STAGED ? kBowStage * 2 : 1];
    __shared__ uint8_t s_cok[STAGED ? kBowStage : 1], s_cm[STAGED ? kBowStage : 1];
    __shared__ uint4 s_qd[STAGED ? 128 : 1];
    __shared__ int s_qi[STAGED ? 64 : 1];
    __shared__ int s_cidx[STAGED ? kBowStage : 1];  // candidates' feature indices (node order)
    __shared__ int2 s_acc[STAGED ? 64 : 1];         // this query chunk's accepted (query idx, candidate idx)
    const NodeTask t = tasks[blockIdx.x];
    const int lane = threadIdx.x;
    const int nc = t.c_end - t.c_begin;
    uint8_t* mflag = STAGED ? s_cm : matched;
    if (STAGED && nc <= 64) {
        // candidate j = lane, its descriptor in registers; query k's descriptor broadcast by readlane. Per
        // query: best1 = the first strict minimum = min over eligible lanes of dist << 6 | j; best2 = min dist
        // of the other eligible lanes (ORBmatcher.cc:205-225); a claimed candidate drops out of its lane
        // (vpMapPointMatches / vbMatched2 within the node). The greedy chain never leaves registers.
        uint32_t cdw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        bool elig = false;
        int idxc = -1;
        if (lane < nc) {
            idxc = vc.node_feat[t.c_begin + lane];
            const uint4* cd = (const uint4*)(vc.desc + (long long)idxc * 32);
            const uint4 a = cd[0], b = cd[1];
            cdw[0] = a.x; cdw[1] = a.y; cdw[2] = a.z; cdw[3] = a.w; cdw[4] = b.x; cdw[5] = b.y; cdw[6] = b.z; cdw[7] = b.w;
            elig = mode == 0 || ((vc.has_mp && vc.has_mp[idxc]) && !(vc.mp_bad && vc.mp_bad[idxc]));
        }
        for (int qb = t.q_begin; qb < t.q_end; qb += 64) {
            const int nq = min(64, t.q_end - qb);
            int myq = -1;
            uint32_t qdw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (lane < nq) {
                const int iq = vq.node_feat[qb + lane];
                const bool ok = (vq.has_mp && vq.has_mp[iq]) && !(vq.mp_bad && vq.mp_bad[iq]);
                myq = ok ? iq : -1;
                const uint4* qd = (const uint4*)(vq.desc + (long long)iq * 32);
                const uint4 a = qd[0], b = qd[1];
                qdw[0] = a.x; qdw[1] = a.y; qdw[2] = a.z; qdw[3] = a.w; qdw[4] = b.x; qdw[5] = b.y; qdw[6] = b.z; qdw[7] = b.w;
            }
            int na = 0;
            for (int k = 0; k < nq; k++) {
                const int idxq = __builtin_amdgcn_readlane(myq, k);
                if (idxq < 0) continue;  // no good MapPoint (uniform)
                int dist = 0;
#pragma unroll
                for (int u = 0; u < 8; u++) dist += __popc(cdw[u] ^ (uint32_t)__builtin_amdgcn_readlane((int)qdw[u], k));
                const uint32_t m1 = wave_min_u32(elig ? ((uint32_t)dist << 6 | (uint32_t)lane) : 0xFFFFFFFFu);
                if (m1 == 0xFFFFFFFFu) continue;  // no eligible candidate left
                const int i1 = (int)(m1 & 63u), b1 = (int)(m1 >> 6);
                const int b2 = (int)wave_min_u32((elig && lane != i1) ? (uint32_t)dist : 256u);
                const bool ok_th = mode == 0 ? (b1 <= 50) : (b1 < 50);  // TH_LOW (ORBmatcher.cc:228 / :598)
                if (ok_th && __fmul_rn(1.0f, (float)b1) < __fmul_rn(nnratio, (float)b2)) {
                    const int idxc_w = __builtin_amdgcn_readlane(idxc, i1);
                    if (lane == i1) elig = false;
                    if (lane == 0) s_acc[na] = make_int2(idxq, idxc_w);
                    na++;
                }
            }
            __syncthreads();
            if (lane < na) {
                const int2 a = s_acc[lane];
                if (mode == 0) call_emit(tail, a.y, a.x);  // vpMapPointMatches[bestIdxF] = pMP(KF idx)
                else call_emit(tail, a.x, a.y);            // vpMatches12[idx1] = vpMapPoints2[bestIdx2]
            }
            __syncthreads();
        }
        call_tail(tail);
        return;
    }
    // STAGED: a chunk's queries: index (-1 = no good MapPoint) and descriptor; the first chunk is loaded
    // together with the candidates (one dependent load pair instead of two before the greedy loop)
    auto load_queries = [&](int qb) {
        if (lane < min(64, t.q_end - qb)) {
            const int idxq = vq.node_feat[qb + lane];
            const bool ok = (vq.has_mp && vq.has_mp[idxq]) && !(vq.mp_bad && vq.mp_bad[idxq]);
            s_qi[lane] = ok ? idxq : -1;
            const uint4* qd = (const uint4*)(vq.desc + (long long)idxq * 32);
            s_qd[2 * lane] = qd[0];
            s_qd[2 * lane + 1] = qd[1];
        }
    };
    if (STAGED) load_queries(t.q_begin);
    for (int j = lane; j < nc; j += 64) {
        mflag[j] = 0;
        if (STAGED) {
            const int idxc = vc.node_feat[t.c_begin + j];
            const uint4* cd = (const uint4*)(vc.desc + (long long)idxc * 32);
            s_cd[2 * j] = cd[0];
            s_cd[2 * j + 1] = cd[1];
            s_cok[j] = mode == 0 || ((vc.has_mp && vc.has_mp[idxc]) && !(vc.mp_bad && vc.mp_bad[idxc]));
            s_cidx[j] = idxc;
        }
    }
    __syncthreads();
    for (int qb = t.q_begin; qb < t.q_end; qb += 64) {
        const int nq = min(64, t.q_end - qb);
        int na = 0;  // STAGED: accepts of this chunk, emitted together after it
        if (STAGED && qb != t.q_begin) {
            load_queries(qb);
            __syncthreads();
        }
        for (int k = 0; k < nq; k++) {
            int idxq;
            uint32_t q[8];
            if (STAGED) {
                idxq = s_qi[k];
                if (idxq < 0) continue;
                const uint4 a0 = s_qd[2 * k], a1 = s_qd[2 * k + 1];
                q[0] = a0.x; q[1] = a0.y; q[2] = a0.z; q[3] = a0.w; q[4] = a1.x; q[5] = a1.y; q[6] = a1.z; q[7] = a1.w;
            } else {
                idxq = vq.node_feat[qb + k];
                if (!(vq.has_mp && vq.has_mp[idxq])) continue;
                if (vq.mp_bad && vq.mp_bad[idxq]) continue;
                const uint32_t* qd = (const uint32_t*)(vq.desc + (long long)idxq * 32);
#pragma unroll
                for (int u = 0; u < 8; u++) q[u] = qd[u];
            }
            Top2 r = {256, -1, 256};
            for (int j = lane; j < nc; j += 64) {
                if (mflag[j]) continue;
                int dist;
                if (STAGED) {
                    if (!s_cok[j]) continue;
                    const uint4 c0 = s_cd[2 * j], c1 = s_cd[2 * j + 1];
                    dist = __popc(q[0] ^ c0.x) + __popc(q[1] ^ c0.y) + __popc(q[2] ^ c0.z) + __popc(q[3] ^ c0.w) +
                           __popc(q[4] ^ c1.x) + __popc(q[5] ^ c1.y) + __popc(q[6] ^ c1.z) + __popc(q[7] ^ c1.w);
                } else {
                    const int idxc = vc.node_feat[t.c_begin + j];
                    if (mode == 1) {
                        if (!(vc.has_mp && vc.has_mp[idxc])) continue;
                        if (vc.mp_bad && vc.mp_bad[idxc]) continue;
                    }
                    dist = hamming8(q, (const uint32_t*)(vc.desc + (long long)idxc * 32));
                }
                if (dist < r.b1) { r.b2 = r.b1; r.b1 = dist; r.i1 = j; }
                else if (dist < r.b2) { r.b2 = dist; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                Top2 o2;
                o2.b1 = __shfl_xor(r.b1, o, 64);
                o2.i1 = __shfl_xor(r.i1, o, 64);
                o2.b2 = __shfl_xor(r.b2, o, 64);
                r = top2_merge(r, o2);
            }
            const bool ok_th = mode == 0 ? (r.b1 <= 50) : (r.b1 < 50);
            if (ok_th && r.i1 >= 0 && __fmul_rn(1.0f, (float)r.b1) < __fmul_rn(nnratio, (float)r.b2)) {
                if (STAGED) {
                    // the greedy chain touches LDS only: the match is recorded here and emitted (global
                    // atomics) after the chunk, so no accept waits for a global round trip
                    if (lane == 0) {
                        mflag[r.i1] = 1;
                        s_acc[na] = make_int2(idxq, s_cidx[r.i1]);
                    }
                    na++;
                    __syncthreads();
                } else {
                    const int idxc = vc.node_feat[t.c_begin + r.i1];
                    __syncthreads();
                    if (lane == 0) {
                        mflag[r.i1] = 1;
                        if (mode == 0) call_emit(tail, idxc, idxq);  // vpMapPointMatches[bestIdxF] = pMP(KF idx)
                        else call_emit(tail, idxq, idxc);            // vpMatches12[idx1] = vpMapPoints2[bestIdx2]
                    }
                    __syncthreads();
                }
            }
        }
        if (STAGED) {
            if (lane < na) {
                const int2 a = s_acc[lane];
                if (mode == 0) call_emit(tail, a.y, a.x);  // vpMapPointMatches[bestIdxF] = pMP(KF idx)
                else call_emit(tail, a.x, a.y);            // vpMatches12[idx1] = vpMapPoints2[bestIdx2]
            }
            __syncthreads();  // s_qi / s_qd / s_acc are rewritten by the next chunk
        }
    }
    call_tail(tail);
}

/* one accept of a small per-call matcher: a single 64-bit store to host memory that carries the call's seq
 * (orb_match.h small_entry), so the host can tell it has landed whatever order the stores arrive in; no
 * fence, no L2 write-back in the kernel */
__device__ __forceinline__ void small_emit(unsigned long long* slot, int x, int y, int bin, int seq) {
    __hip_atomic_store(slot, small_entry(x, y, bin, (uint32_t)seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* Small per-call SearchByBoW (BowSmall, orb_match.h): k_bow's lane-per-candidate greedy chain for nodes of
 * <= 64 candidates with every input in node order, no global atomics and no last-workgroup tail: a
 * workgroup emits its node's accepts (with their rotation bin) straight to host memory, then its done word
 * (the host waits for both). The rotation histogram over all nodes (ORBmatcher.cc:236-246, 1601-1642) is the host's (capi.cpp). */
__global__ __launch_bounds__(64) void k_bow_small(const BowSmall a) {
    const SmallTask t = a.tasks[blockIdx.x];
    const int lane = threadIdx.x;
    const int nc = t.c_end - t.c_begin;  // <= 64 (host checked)
    uint32_t cdw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool elig = false;
    int idxc = -1;
    float cang = 0.f;
    if (lane < nc) {
        const int p = t.c_begin + lane;
        const uint4 x0 = a.cd[2 * p], x1 = a.cd[2 * p + 1];
        cdw[0] = x0.x; cdw[1] = x0.y; cdw[2] = x0.z; cdw[3] = x0.w; cdw[4] = x1.x; cdw[5] = x1.y; cdw[6] = x1.z; cdw[7] = x1.w;
        idxc = a.cf[p];
        cang = a.ca[p * a.ca_stride];
        elig = a.mode == 0 || ((a.cgood[p >> 5] >> (p & 31)) & 1u);
    }
    int na = 0;
    for (int qb = t.q_begin; qb < t.q_end; qb += 64) {
        const int nq = min(64, t.q_end - qb);
        int myq = -1;
        float qang = 0.f;
        uint32_t qdw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (lane < nq) {
            const int p = qb + lane;
            const uint4 x0 = a.qd[2 * p], x1 = a.qd[2 * p + 1];
            qdw[0] = x0.x; qdw[1] = x0.y; qdw[2] = x0.z; qdw[3] = x0.w; qdw[4] = x1.x; qdw[5] = x1.y; qdw[6] = x1.z; qdw[7] = x1.w;
            myq = ((a.qgood[p >> 5] >> (p & 31)) & 1u) ? a.qf[p] : -1;
            qang = a.qa[p * a.qa_stride];
        }
        for (int k = 0; k < nq; k++) {
            const int idxq = __builtin_amdgcn_readlane(myq, k);
            if (idxq < 0) continue;  // no good MapPoint (uniform)
            int dist = 0;
#pragma unroll
            for (int u = 0; u < 8; u++) dist += __popc(cdw[u] ^ (uint32_t)__builtin_amdgcn_readlane((int)qdw[u], k));
            const uint32_t m1 = wave_min_u32(elig ? ((uint32_t)dist << 6 | (uint32_t)lane) : 0xFFFFFFFFu);
            if (m1 == 0xFFFFFFFFu) continue;  // no eligible candidate left
            const int i1 = (int)(m1 & 63u), b1 = (int)(m1 >> 6);
            const int b2 = (int)wave_min_u32((elig && lane != i1) ? (uint32_t)dist : 256u);
            const bool ok_th = a.mode == 0 ? (b1 <= 50) : (b1 < 50);  // TH_LOW (ORBmatcher.cc:228 / :598)
            if (ok_th && __fmul_rn(1.0f, (float)b1) < __fmul_rn(a.nnratio, (float)b2)) {
                const int idxc_w = __builtin_amdgcn_readlane(idxc, i1);
                int bin = 0;
                if (a.check_ori) {  // rot = angle(KF / KF1 keypoint) - angle(F / KF2 keypoint) in both modes
                    const float qa_k = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, qang), k));
                    const float ca_i = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cang), i1));
                    float rot = __fsub_rn(qa_k, ca_i);
                    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
                    bin = (int)roundf(__fmul_rn(rot, 1.0f / 30));
                    if (bin == 30) bin = 0;
                }
                if (lane == i1) elig = false;
                if (lane == 0)
                    small_emit(a.out + t.q_begin + na, a.mode == 0 ? idxc_w : idxq, a.mode == 0 ? idxq : idxc_w, bin,
                               a.seq);
                na++;
            }
        }
    }
    if (lane == 0)
        __hip_atomic_store(a.done + blockIdx.x, (unsigned long long)(uint32_t)a.seq | (unsigned long long)na << 32,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* Small per-call SearchForTriangulation over common BoW nodes (TriSmall, orb_match.h): a wave per 64-query
 * chunk of a common node, a lane per query; the node's candidates are loaded 64 at a time, one per lane, and
 * broadcast by readlane, so every lane scans them in node order with the reference's rule (ORBmatcher.cc:
 * 704-776: skip a MapPoint / non-stereo candidate, dist > TH_LOW or > best; epipole radius for mono pairs;
 * CheckDistEpipolarLine; accept = new best, ties to the later). Accepts are compacted by ballot into host
 * memory, then the chunk's done word; the rotation histogram is the host's. */
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

__global__ __launch_bounds__(64) void k_tri_small(const TriSmall a) {
    const SmallTask t = a.tasks[blockIdx.x];
    const int lane = threadIdx.x;
    const int p1 = t.q_begin + lane;
    bool active = false, st1 = false;
    int idx1 = -1;
    float ea = 0.f, eb = 0.f, ec = 0.f, ang1 = 0.f;
    uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (p1 < t.q_end) {
        const uint4 x0 = a.qd[2 * p1], x1 = a.qd[2 * p1 + 1];
        q[0] = x0.x; q[1] = x0.y; q[2] = x0.z; q[3] = x0.w; q[4] = x1.x; q[5] = x1.y; q[6] = x1.z; q[7] = x1.w;
        const NodeRec r = a.qr[p1];
        idx1 = a.qf[p1];
        st1 = a.q_ur && (r.oct & 0x100);
        active = !((a.qmp[p1 >> 5] >> (p1 & 31)) & 1u) && (!a.only_stereo || st1);
        ang1 = r.angle;
        epi_line(a.g, r.x, r.y, &ea, &eb, &ec);
    }
    int bestDist = 50, bestIdx2 = -1;  // TH_LOW (ORBmatcher.cc:704)
    float bestAng = 0.f;
    for (int cb = t.c_begin; cb < t.c_end; cb += 64) {
        const int nt = min(64, t.c_end - cb);
        uint32_t cdw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int coct = -1, cidx = -1;
        float cx = 0.f, cy = 0.f, cang = 0.f;
        if (lane < nt) {
            const int p2 = cb + lane;
            const uint4 x0 = a.cd[2 * p2], x1 = a.cd[2 * p2 + 1];
            cdw[0] = x0.x; cdw[1] = x0.y; cdw[2] = x0.z; cdw[3] = x0.w; cdw[4] = x1.x; cdw[5] = x1.y; cdw[6] = x1.z; cdw[7] = x1.w;
            const NodeRec r = a.cr[p2];
            cidx = a.cf[p2];
            const bool st2 = a.c_ur && (r.oct & 0x100);
            const bool ok = !((a.cmp[p2 >> 5] >> (p2 & 31)) & 1u) && (!a.only_stereo || st2);
            coct = ok ? ((r.oct & 0xFF) | (st2 ? 0x100 : 0)) : -1;
            cx = r.x;
            cy = r.y;
            cang = r.angle;
        }
        for (int j = 0; j < nt; j++) {
            const int oc = __builtin_amdgcn_readlane(coct, j);
            if (oc < 0) continue;  // a MapPoint (or mono in stereo mode): uniform
            int dist = 0;
#pragma unroll
            for (int u = 0; u < 8; u++) dist += __popc(q[u] ^ (uint32_t)__builtin_amdgcn_readlane((int)cdw[u], j));
            const float x2 = readlane_f(cx, j), y2 = readlane_f(cy, j), a2 = readlane_f(cang, j);
            const int i2 = __builtin_amdgcn_readlane(cidx, j);
            if (!active || dist > 50 || dist > bestDist) continue;
            const int oct2 = oc & 0xFF;
            if (!st1 && !(oc & 0x100) && near_epipole(a.g, x2, y2, oct2)) continue;  // ORBmatcher.cc:743-749
            if (epi_ok(ea, eb, ec, x2, y2, a.g.th384[oct2])) {
                bestDist = dist;
                bestIdx2 = i2;
                bestAng = a2;
            }
        }
    }
    const bool acc = active && bestIdx2 >= 0;
    int bin = 0;
    if (acc && a.check_ori) {  // rot = kp1.angle - kp2.angle (ORBmatcher.cc:784-792)
        float rot = __fsub_rn(ang1, bestAng);
        if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
        bin = (int)roundf(__fmul_rn(rot, 1.0f / 30));
        if (bin == 30) bin = 0;
    }
    const unsigned long long m = __ballot(acc);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    if (acc) small_emit(a.out + t.q_begin + rank, idx1, bestIdx2, bin, a.seq);
    if (lane == 0)
        __hip_atomic_store(a.done + blockIdx.x,
                           (unsigned long long)(uint32_t)a.seq | (unsigned long long)__popcll(m) << 32,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* SearchByBoW for a batch of frame pairs with the FeatureVectors of orbv_transform_batch_device on
 * the device: block (i, p) takes node i of the query frame qf[p] and, if the candidate frame cf[p]
 * has the same node (binary search), runs k_bow's node-local greedy (queries in order; best / second
 * over the not yet matched candidates). mp_flags[f * kp_stride + idx]: bit 0 = a MapPoint, bit 1 = it
 * is bad. mode 0 = (KF,F) (ORBmatcher.cc:159-288): qf = KF, out[cf index] = KF index;
 * mode 1 = (KF,KF) (:522-655): out[qf index] = cf index. */
__global__ __launch_bounds__(64) void k_bow_pairs(const int32_t* __restrict__ qf, const int32_t* __restrict__ cf,
                                                  const uint8_t* __restrict__ desc, int kp_stride,
                                                  const uint8_t* __restrict__ mp_flags,
                                                  const uint32_t* __restrict__ fv_node, const int32_t* __restrict__ fv_off,
                                                  const int32_t* __restrict__ fv_feat, const int32_t* __restrict__ nfv,
                                                  float nnratio, int mode, int32_t* __restrict__ out) {
    extern __shared__ uint8_t matched[];  // per candidate position in the node (<= kp_stride)
    const int p = blockIdx.y, i = blockIdx.x;
    const int fq = qf[p], fc = cf[p];
    if (i >= nfv[fq]) return;
    const uint32_t* nodes_c = fv_node + (long long)fc * kp_stride;
    const uint32_t node = fv_node[(long long)fq * kp_stride + i];
    int lo = 0, hi = nfv[fc];
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (nodes_c[mid] < node) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= nfv[fc] || nodes_c[lo] != node) return;
    const int32_t* offq = fv_off + (long long)fq * (kp_stride + 1);
    const int32_t* offc = fv_off + (long long)fc * (kp_stride + 1);
    const int32_t* featq = fv_feat + (long long)fq * kp_stride;
    const int32_t* featc = fv_feat + (long long)fc * kp_stride + offc[lo];
    const uint8_t* fq_flags = mp_flags + (long long)fq * kp_stride;
    const uint8_t* fc_flags = mp_flags + (long long)fc * kp_stride;
    const uint8_t* dq = desc + (long long)fq * kp_stride * 32;
    const uint8_t* dc = desc + (long long)fc * kp_stride * 32;
    int32_t* o = out + (long long)p * kp_stride;
    const int lane = threadIdx.x;
    const int nc = offc[lo + 1] - offc[lo];
    for (int j = lane; j < nc; j += 64) matched[j] = 0;
    __syncthreads();
    for (int i1 = offq[i]; i1 < offq[i + 1]; i1++) {
        const int idxq = featq[i1];
        if ((fq_flags[idxq] & 3) != 1) continue;  // a good MapPoint
        const uint32_t* qd = (const uint32_t*)(dq + (long long)idxq * 32);
        uint32_t q[8];
#pragma unroll
        for (int k = 0; k < 8; k++) q[k] = qd[k];
        Top2 r = {256, -1, 256};
        for (int j = lane; j < nc; j += 64) {
            if (matched[j]) continue;
            const int idxc = featc[j];
            if (mode == 1 && (fc_flags[idxc] & 3) != 1) continue;
            const int dist = hamming8(q, (const uint32_t*)(dc + (long long)idxc * 32));
            if (dist < r.b1) { r.b2 = r.b1; r.b1 = dist; r.i1 = j; }
            else if (dist < r.b2) { r.b2 = dist; }
        }
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            Top2 o2;
            o2.b1 = __shfl_xor(r.b1, sh, 64);
            o2.i1 = __shfl_xor(r.i1, sh, 64);
            o2.b2 = __shfl_xor(r.b2, sh, 64);
            r = top2_merge(r, o2);
        }
        const bool ok_th = mode == 0 ? (r.b1 <= 50) : (r.b1 < 50);
        if (ok_th && r.i1 >= 0 && __fmul_rn(1.0f, (float)r.b1) < __fmul_rn(nnratio, (float)r.b2)) {
            const int idxc = featc[r.i1];
            __syncthreads();
            if (lane == 0) {
                matched[r.i1] = 1;
                if (mode == 0) o[idxc] = idxq;
                else o[idxq] = idxc;
            }
            __syncthreads();
        }
    }
}

/* per-pair count of out >= 0 (after the optional rotation filter) */
__global__ __launch_bounds__(256) void k_count_pairs(const int32_t* __restrict__ out, int kp_stride,
                                                     int32_t* __restrict__ nmatches) {
    const int p = blockIdx.x;
    int local = 0;
    for (int i = threadIdx.x; i < kp_stride; i += 256) local += out[(long long)p * kp_stride + i] >= 0;
    atomicAdd(&nmatches[p], local);
}

/* Rotation consistency (ORBmatcher.cc:236-246 + 267-285): entries i with m[i] >= 0; rot =
 * angA[a] - angB[b] where (a,b) = (i, m[i]) or, with swap, (m[i], i). One workgroup. */
__global__ __launch_bounds__(256) void k_rot_filter(int n, int32_t* __restrict__ m, const float* __restrict__ angA,
                                                    const float* __restrict__ angB, int swap, int32_t* __restrict__ nout) {
    __shared__ int hist[30];
    __shared__ int keep[3];
    if (threadIdx.x < 30) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 256) {
        const int j = m[i];
        if (j >= 0) atomicAdd(&hist[rot_bin(angA, angB, i, j, swap)], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) three_maxima(hist, keep);
    __syncthreads();
    int local = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        const int j = m[i];
        if (j < 0) continue;
        const int bin = rot_bin(angA, angB, i, j, swap);
        if (bin != keep[0] && bin != keep[1] && bin != keep[2]) m[i] = -1;
        else local++;
    }
    if (nout) atomicAdd(nout, local);
}

/* batch form of the rotation filter for k_tri_mfma output: one workgroup per pair */
__global__ __launch_bounds__(256) void k_rot_filter_pairs(const int32_t* __restrict__ q1, const int32_t* __restrict__ q2,
                                                          const orbx_kp* __restrict__ kps, const int32_t* __restrict__ counts,
                                                          int kp_stride, int32_t* __restrict__ match12,
                                                          int32_t* __restrict__ nmatches, int swap) {
    __shared__ int hist[30];
    __shared__ int keep[3];
    const int p = blockIdx.x;
    const orbx_kp* k1 = kps + (long long)q1[p] * kp_stride;
    const orbx_kp* k2 = kps + (long long)q2[p] * kp_stride;
    int32_t* m = match12 + (long long)p * kp_stride;
    const int n = counts[q1[p]];
    if (threadIdx.x < 30) hist[threadIdx.x] = 0;
    __syncthreads();
    auto bin_of = [&](int i, int j) {
        float rot = swap ? __fsub_rn(k2[j].angle, k1[i].angle) : __fsub_rn(k1[i].angle, k2[j].angle);
        if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
        const int bin = (int)roundf(__fmul_rn(rot, 1.0f / 30));
        return bin == 30 ? 0 : bin;
    };
    for (int i = threadIdx.x; i < n; i += 256) {
        const int j = m[i];
        if (j >= 0) atomicAdd(&hist[bin_of(i, j)], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        three_maxima(hist, keep);
        nmatches[p] = 0;
    }
    __syncthreads();
    int local = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        const int j = m[i];
        if (j < 0) continue;
        const int bin = bin_of(i, j);
        if (bin != keep[0] && bin != keep[1] && bin != keep[2]) m[i] = -1;
        else local++;
    }
    atomicAdd(&nmatches[p], local);
}

}  // namespace orbamd

#include "launch.h"

namespace orbamd {

hipError_t launch_tri_bf(int npairs, const int32_t* q1, const int32_t* q2, const orbx_kp* kps, const uint8_t* desc,
                         const int32_t* counts, int kp_stride, const MatchGeom& g, int32_t* match12,
                         int32_t* nmatches, hipStream_t st, const float* uright, int only_stereo) {
    if (npairs == 0) return hipSuccess;
    dim3 grid((kp_stride + 32 * kMfWaves - 1) / (32 * kMfWaves), npairs);
    if (uright)
        hipLaunchKernelGGL(k_tri_mfma<true>, grid, dim3(kMfThreads), 0, st, q1, q2, kps, desc, counts, uright, kp_stride,
                           g, only_stereo, match12, nmatches);
    else
        hipLaunchKernelGGL(k_tri_mfma<false>, grid, dim3(kMfThreads), 0, st, q1, q2, kps, desc, counts, uright,
                           kp_stride, g, 0, match12, nmatches);
    return hipGetLastError();
}

hipError_t launch_tri_nodes_pairs(int npairs, int max_nodes, const int32_t* q1, const int32_t* q2, const orbx_kp* kps,
                                  const uint8_t* desc, int kp_stride, const uint32_t* fv_node, const int32_t* fv_off,
                                  const int32_t* fv_feat, const int32_t* nfv, const MatchGeom& g, int32_t* match12,
                                  int32_t* nmatches, hipStream_t st) {
    if (npairs == 0 || max_nodes <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_tri_nodes_pairs, dim3(max_nodes, npairs), dim3(64), 0, st, q1, q2, kps, desc, kp_stride,
                       fv_node, fv_off, fv_feat, nfv, g, match12, nmatches);
    return hipGetLastError();
}

hipError_t launch_rot_filter_pairs(int npairs, const int32_t* q1, const int32_t* q2, const orbx_kp* kps,
                                   const int32_t* counts, int kp_stride, int32_t* match12, int32_t* nmatches,
                                   hipStream_t st, int swap) {
    hipLaunchKernelGGL(k_rot_filter_pairs, dim3(npairs), dim3(256), 0, st, q1, q2, kps, counts, kp_stride, match12,
                       nmatches, swap);
    return hipGetLastError();
}

hipError_t launch_bow_pairs(int npairs, int max_nodes, const int32_t* qf, const int32_t* cf, const uint8_t* desc,
                            int kp_stride, const uint8_t* mp_flags, const uint32_t* fv_node, const int32_t* fv_off,
                            const int32_t* fv_feat, const int32_t* nfv, float nnratio, int mode, int32_t* out,
                            hipStream_t st) {
    if (npairs == 0 || max_nodes <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bow_pairs, dim3(max_nodes, npairs), dim3(64), (size_t)kp_stride, st, qf, cf, desc, kp_stride,
                       mp_flags, fv_node, fv_off, fv_feat, nfv, nnratio, mode, out);
    return hipGetLastError();
}

hipError_t launch_count_pairs(int npairs, const int32_t* out, int kp_stride, int32_t* nmatches, hipStream_t st) {
    if (npairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_count_pairs, dim3(npairs), dim3(256), 0, st, out, kp_stride, nmatches);
    return hipGetLastError();
}

hipError_t launch_tri_nodes(const DevView& v1, const DevView& v2, const NodeTask* tasks, int ntasks,
                            const MatchGeom& g, int only_stereo, const CallTail& tail, hipStream_t st) {
    if (ntasks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_tri_nodes, dim3(ntasks), dim3(256), 0, st, v1, v2, tasks, g, only_stereo, tail);
    return hipGetLastError();
}

hipError_t launch_bow(const DevView& vq, const DevView& vc, const NodeTask* tasks, int ntasks, int max_nc,
                      float nnratio, int mode, const CallTail& tail, hipStream_t st) {
    if (ntasks == 0) return hipSuccess;
    if (max_nc <= kBowStage)
        hipLaunchKernelGGL(k_bow<true>, dim3(ntasks), dim3(64), 0, st, vq, vc, tasks, nnratio, mode, tail);
    else
        hipLaunchKernelGGL(k_bow<false>, dim3(ntasks), dim3(64), (size_t)max_nc, st, vq, vc, tasks, nnratio, mode,
                           tail);
    return hipGetLastError();
}

hipError_t launch_bow_small(const BowSmall& a, hipStream_t st) {
    if (a.ntasks <= 0 || a.ntasks > kSmallTasks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_bow_small, dim3(a.ntasks), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_tri_small(const TriSmall& a, hipStream_t st) {
    if (a.ntasks <= 0 || a.ntasks > kSmallTasks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_tri_small, dim3(a.ntasks), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_rot_filter(int n, int32_t* m, const float* angA, const float* angB, int swap, int32_t* nout,
                             hipStream_t st) {
    hipLaunchKernelGGL(k_rot_filter, dim3(1), dim3(256), 0, st, n, m, angA, angB, swap, nout);
    return hipGetLastError();
}

}  // namespace orbamd
