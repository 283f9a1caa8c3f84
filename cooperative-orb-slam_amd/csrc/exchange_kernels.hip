/*
 * exchange_kernels.hip -- gfx950 kernels of the cross-agent keyframe exchange (SURVEY.md 8(e),
 * 8(f) row 4): the device pack of one keyframe into a slot (replacing the LCM KeyFrameexample
 * publisher, ORB_SLAM2.1/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:1907-2410) and
 * SearchForTriangulation of this agent's keyframe against received slots read straight from
 * the all-gather receive buffer (ORBmatcher.cc:657-823; the receiving agent inserts the
 * decoded keyframe into LocalMapping, whose CreateNewMapPoints calls it, LocalMapping.cc:268).
 *
 *   k_pack_slot     every section entry of the slot written by a grid-stride loop (entries past
 *                   the counts zeroed, so the device pack is byte-identical to the host packer)
 *   k_tri_slots_bf  one FeatureVector node holding every feature (BF), SIMT XOR + v_bcnt:
 *                   16 queries x 16 candidate slices per workgroup, candidate tiles in LDS
 *   k_tri_slots_bow the common BoW nodes of the query's and the slot's FeatureVectors: one
 *                   wave per query node, binary search for the slot's node, lane per query
 *   k_bow_slots     cross-agent SearchByBoW(KF,KF) (ORBmatcher.cc:522-655), the loop-candidate match
 *                   LoopClosing::ComputeSim3 runs on a received keyframe (LoopClosing.cc:265): one wave
 *                   per common node, the node's greedy chain over its queries in order, lane per
 *                   candidate, best / second best by DPP minima
 *   k_rot_slots     its rotation histogram + ComputeThreeMaxima filter and the per-slot count
 * Every received slot is validated on the device before use (header, sizes, counts, CSR
 * bounds); a bad slot yields no matches and raises the matcher's error flag.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbslam_amd.h"
#include "orb_slot.h"
#include "orb_wave.h"

namespace orbamd {

/* ----------------------------------------------------------------------------------- */
/* pack                                                                                 */
/* ----------------------------------------------------------------------------------- */
struct PackArgs {
    orbx_kf_source src;
    SlotLayout L;
    orbx_kf_meta meta;
};

__global__ __launch_bounds__(256) void k_pack_slot(const PackArgs a, uint8_t* __restrict__ slot,
                                                   int32_t* __restrict__ err) {
    const orbx_kf_source& s = a.src;
    const int cap = a.L.cap;
    const int n_in = *s.count;
    const int n = min(max(n_in, 0), cap);
    const int nb_in = s.nbow ? *s.nbow : 0;
    const int nbow = (s.bow_word && s.bow_value) ? min(max(nb_in, 0), cap) : 0;
    const int nf_in = s.nfv ? *s.nfv : 0;
    const bool has_fv = s.fv_node && s.fv_off && s.fv_feat;
    const int nfv = has_fv ? min(max(nf_in, 0), cap) : 0;
    const int nfeat = has_fv && nfv > 0 ? min(max(s.fv_off[nfv], 0), cap) : 0;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int nthr = gridDim.x * blockDim.x;
    if (tid == 0) {
        const bool clamped = n_in > cap || n_in < 0 || (has_fv && (nf_in > cap || (nfv > 0 && s.fv_off[nfv] > cap))) ||
                             ((s.bow_word && s.bow_value) && nb_in > cap);
        if (clamped && err) atomicOr(err, 1);
        orbx_slot_header* h = (orbx_slot_header*)slot;
        h->magic = ORBX_SLOT_MAGIC;
        h->version = ORBX_SLOT_VERSION;
        h->n = n;
        h->cap = cap;
        h->nbow = nbow;
        h->nfv = nfv;
        h->flags = (s.kun ? ORBX_SLOT_F_KUN : 0u) | ((s.uright && s.depth) ? ORBX_SLOT_F_STEREO : 0u) |
                   (s.mp_flags ? ORBX_SLOT_F_MP : 0u) | ((s.bow_word && s.bow_value) ? ORBX_SLOT_F_BOW : 0u) |
                   (has_fv ? ORBX_SLOT_F_FV : 0u);
        h->bytes = a.L.bytes;
        for (int k = 0; k < ORBX_SLOT_NSECTIONS; k++) h->off[k] = a.L.off[k];
        for (int k = 0; k < 12; k++) h->reserved[k] = 0;
    }
    // meta (704 B) and the zero gap up to the body: 224 dwords
    {
        const uint32_t* mw = (const uint32_t*)&a.meta;
        uint32_t* dst = (uint32_t*)(slot + kSlotMetaOff);
        constexpr int kMetaW = sizeof(orbx_kf_meta) / 4, kGapW = (kSlotBodyOff - kSlotMetaOff) / 4;
        for (int k = tid; k < kGapW; k += nthr) dst[k] = k < kMetaW ? mw[k] : 0u;
    }
    orbx_kp* o_kps = (orbx_kp*)(slot + a.L.off[ORBX_SLOT_KPS]);
    float2* o_kun = (float2*)(slot + a.L.off[ORBX_SLOT_KUN]);
    float* o_ur = (float*)(slot + a.L.off[ORBX_SLOT_URIGHT]);
    float* o_dp = (float*)(slot + a.L.off[ORBX_SLOT_DEPTH]);
    uint4* o_desc = (uint4*)(slot + a.L.off[ORBX_SLOT_DESC]);
    uint8_t* o_mpf = slot + a.L.off[ORBX_SLOT_MPFLAGS];
    float* o_mpp = (float*)(slot + a.L.off[ORBX_SLOT_MPPOS]);
    uint32_t* o_bw = (uint32_t*)(slot + a.L.off[ORBX_SLOT_BOWWORD]);
    double* o_bv = (double*)(slot + a.L.off[ORBX_SLOT_BOWVALUE]);
    uint32_t* o_fn = (uint32_t*)(slot + a.L.off[ORBX_SLOT_FVNODE]);
    int32_t* o_fo = (int32_t*)(slot + a.L.off[ORBX_SLOT_FVOFF]);
    int32_t* o_ff = (int32_t*)(slot + a.L.off[ORBX_SLOT_FVFEAT]);
    const uint4* i_desc = (const uint4*)s.desc;
    for (int i = tid; i <= cap; i += nthr) {
        if (i < cap) {
            const bool on = i < n;
            orbx_kp k = {0.f, 0.f, 0.f, 0.f, 0.f, 0};
            if (on) k = s.kps[i];
            o_kps[i] = k;
            float2 ku = {0.f, 0.f};
            if (on) ku = s.kun ? ((const float2*)s.kun)[i] : (float2){k.x, k.y};
            o_kun[i] = ku;
            const bool st = s.uright && s.depth;
            o_ur[i] = on ? (st ? s.uright[i] : -1.f) : 0.f;
            o_dp[i] = on ? (st ? s.depth[i] : -1.f) : 0.f;
            const uint4 z = {0u, 0u, 0u, 0u};
            o_desc[2 * i] = on ? i_desc[2 * i] : z;
            o_desc[2 * i + 1] = on ? i_desc[2 * i + 1] : z;
            o_mpf[i] = (on && s.mp_flags) ? s.mp_flags[i] : (uint8_t)0;
            const bool mp = on && s.mp_flags && s.mp_pos;
            o_mpp[3 * i] = mp ? s.mp_pos[3 * i] : 0.f;
            o_mpp[3 * i + 1] = mp ? s.mp_pos[3 * i + 1] : 0.f;
            o_mpp[3 * i + 2] = mp ? s.mp_pos[3 * i + 2] : 0.f;
            o_bw[i] = i < nbow ? s.bow_word[i] : 0u;
            o_bv[i] = i < nbow ? s.bow_value[i] : 0.0;
            o_fn[i] = i < nfv ? s.fv_node[i] : 0u;
            o_ff[i] = i < nfeat ? s.fv_feat[i] : 0;
        }
        o_fo[i] = (i <= nfv && nfv > 0) ? min(max(s.fv_off[i], 0), cap) : 0;
    }
    // the alignment padding after each section (< 256 bytes each) is zero too
    for (int k = tid; k < ORBX_SLOT_NSECTIONS * 256; k += nthr) {
        const int sec = k >> 8;
        const uint64_t pos = a.L.off[sec] + slot_section_bytes(sec, cap) + (uint64_t)(k & 255);
        const uint64_t end = sec + 1 < ORBX_SLOT_NSECTIONS ? a.L.off[sec + 1] : a.L.bytes;
        if (pos < end) slot[pos] = 0;
    }
}

/* ----------------------------------------------------------------------------------- */
/* received-slot validation (uniform per workgroup)                                     */
/* ----------------------------------------------------------------------------------- */
struct SlotRef {
    const orbx_kf_meta* meta;
    const orbx_kp* kps;
    const float2* kun;
    const float* uright;
    const uint8_t* desc;
    const uint8_t* mpf;
    const uint32_t* fv_node;
    const int32_t* fv_off;
    const int32_t* fv_feat;
    int n, nfv, cap, nlev;
};

__device__ __forceinline__ bool slot_open(const uint8_t* slot, long long slot_bytes, SlotRef& r) {
    const orbx_slot_header* h = (const orbx_slot_header*)slot;
    if (h->magic != ORBX_SLOT_MAGIC || h->version != ORBX_SLOT_VERSION) return false;
    uint32_t off[ORBX_SLOT_NSECTIONS], total;
    if (!slot_offsets(h->cap, off, &total)) return false;
    if (total != h->bytes || (long long)total > slot_bytes) return false;
    for (int k = 0; k < ORBX_SLOT_NSECTIONS; k++)
        if (h->off[k] != off[k]) return false;
    if (h->n < 0 || h->n > h->cap || h->nfv < 0 || h->nfv > h->cap || h->nbow < 0 || h->nbow > h->cap) return false;
    r.meta = (const orbx_kf_meta*)(slot + kSlotMetaOff);
    r.nlev = r.meta->mnScaleLevels;
    if (r.nlev < 1 || r.nlev > 16) return false;
    r.kps = (const orbx_kp*)(slot + off[ORBX_SLOT_KPS]);
    r.kun = (const float2*)(slot + off[ORBX_SLOT_KUN]);
    r.uright = (const float*)(slot + off[ORBX_SLOT_URIGHT]);
    r.desc = slot + off[ORBX_SLOT_DESC];
    r.mpf = slot + off[ORBX_SLOT_MPFLAGS];
    r.fv_node = (const uint32_t*)(slot + off[ORBX_SLOT_FVNODE]);
    r.fv_off = (const int32_t*)(slot + off[ORBX_SLOT_FVOFF]);
    r.fv_feat = (const int32_t*)(slot + off[ORBX_SLOT_FVFEAT]);
    r.n = h->n;
    r.nfv = h->nfv;
    r.cap = h->cap;
    return true;
}

/* per-slot geometry, by value (up to kMaxSlotsPerLaunch slots per launch) */
constexpr int kMaxSlotsPerLaunch = 16;
struct SlotGeoms {
    float F[kMaxSlotsPerLaunch][9];
    float ex[kMaxSlotsPerLaunch], ey[kMaxSlotsPerLaunch];
};

/* CheckDistEpipolarLine (ORBmatcher.cc:140-157) with kp1's line (a, b, c) precomputed in the
 * reference's float order; `dsqr < 3.84*sigma2` compared in double */
__device__ __forceinline__ bool slot_epi_ok(float a, float b, float c, float x2, float y2, float sigma2) {
    const float num = __fadd_rn(__fadd_rn(__fmul_rn(a, x2), __fmul_rn(b, y2)), c);
    const float den = __fadd_rn(__fmul_rn(a, a), __fmul_rn(b, b));
    if (den == 0.f) return false;
    const float dsqr = __fdiv_rn(__fmul_rn(num, num), den);
    return (double)dsqr < 3.84 * (double)sigma2;
}

__device__ __forceinline__ void slot_epi_line(const float* F, float x1, float y1, float* a, float* b, float* c) {
    *a = __fadd_rn(__fadd_rn(__fmul_rn(x1, F[0]), __fmul_rn(y1, F[3])), F[6]);
    *b = __fadd_rn(__fadd_rn(__fmul_rn(x1, F[1]), __fmul_rn(y1, F[4])), F[7]);
    *c = __fadd_rn(__fadd_rn(__fmul_rn(x1, F[2]), __fmul_rn(y1, F[5])), F[8]);
}

/* ----------------------------------------------------------------------------------- */
/* BF: 256 threads = 16 candidate slices x 16 queries. Slice k scans the k-th part of     */
/* every candidate tile with the reference's rule (accept dist <= best after the checks,  */
/* so ties go to the later idx2); slices merge by (min dist, then larger idx2) = the       */
/* sequential scan's result (DESIGN.md "Matcher semantics").                               */
/* ----------------------------------------------------------------------------------- */
constexpr int kSlotTile = 512;
constexpr int kSlotSplit = 16;
constexpr int kSlotQ = 256 / kSlotSplit;

__global__ __launch_bounds__(256) void k_tri_slots_bf(const QueryKF q, const uint8_t* __restrict__ slots,
                                                      long long slot_bytes, int slot0, const SlotGeoms G,
                                                      int32_t* __restrict__ match, int32_t* __restrict__ nmatches,
                                                      int32_t* __restrict__ err) {
    __shared__ uint4 s_desc[kSlotTile * 2];
    __shared__ float s_x[kSlotTile], s_y[kSlotTile];
    __shared__ int s_oct[kSlotTile];
    __shared__ uint8_t s_flag[kSlotTile];  // bit 0 skip (MapPoint), bit 1 stereo
    __shared__ float s_th100[16], s_sig2[16];
    __shared__ int s_bd[kSlotSplit][kSlotQ], s_bi[kSlotSplit][kSlotQ];
    const int tid = threadIdx.x;
    const int ql = tid % kSlotQ, part = tid / kSlotQ;
    const int gr = blockIdx.y;            // slot within this launch
    const int r = slot0 + gr;             // slot index in the buffer / output row
    const int idx1 = blockIdx.x * kSlotQ + ql;
    int32_t* out = match + (long long)r * q.cap;
    const int n1_in = *q.count;
    const int n1 = min(max(n1_in, 0), q.cap);
    if (blockIdx.x == 0 && tid == 0 && (n1_in > q.cap || n1_in < 0)) atomicOr(err, 2);
    SlotRef s;
    const bool ok = slot_open(slots + (long long)r * slot_bytes, slot_bytes, s);
    if (!ok) {
        if (blockIdx.x == 0 && tid == 0) atomicOr(err, 4);
        if (part == 0 && idx1 < q.cap) out[idx1] = -1;
        return;
    }
    if (tid < 16) {
        const int o = tid < s.nlev ? tid : 0;
        s_th100[tid] = __fmul_rn(100.f, s.meta->mvScaleFactors[o]);  // 100*mvScaleFactors[oct2] (:747)
        s_sig2[tid] = s.meta->mvLevelSigma2[o];
    }
    const bool active = idx1 < n1;
    uint32_t qd[8];
    float la = 0.f, lb = 0.f, lc = 0.f;
    bool st1 = false, skip1 = true;
    if (active) {
        const uint4* d = (const uint4*)(q.desc + (long long)idx1 * 32);
        const uint4 a0 = d[0], a1 = d[1];
        qd[0] = a0.x; qd[1] = a0.y; qd[2] = a0.z; qd[3] = a0.w; qd[4] = a1.x; qd[5] = a1.y; qd[6] = a1.z; qd[7] = a1.w;
        const float2 p1 = q.kun ? q.kun[idx1] : (float2){q.kps[idx1].x, q.kps[idx1].y};
        slot_epi_line(G.F[gr], p1.x, p1.y, &la, &lb, &lc);
        st1 = q.uright ? q.uright[idx1] >= 0.f : false;
        skip1 = q.mpf ? (q.mpf[idx1] & 1) != 0 : false;  // GetMapPoint(idx1) != NULL (:699-703)
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++) qd[k] = 0;
    }
    const float ex = G.ex[gr], ey = G.ey[gr];
    int bestDist = 50, bestIdx2 = -1;  // TH_LOW (:715)
    const int n2 = s.n;
    for (int t0 = 0; t0 < n2; t0 += kSlotTile) {
        const int nt = min(kSlotTile, n2 - t0);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kSlotTile / 256; u++) {
            const int j = tid + u * 256;
            if (j < nt) {
                const uint4* cd = (const uint4*)(s.desc + (long long)(t0 + j) * 32);
                s_desc[2 * j] = cd[0];
                s_desc[2 * j + 1] = cd[1];
                const float2 p = s.kun[t0 + j];
                s_x[j] = p.x;
                s_y[j] = p.y;
                // an octave outside [0, mnScaleLevels) fails the host parser's contract (orbx_slot_parse):
                // the candidate is skipped and the slot flagged, as k_tri_slots_bow does
                const int o2 = s.kps[t0 + j].octave;
                const bool obad = (unsigned)o2 >= (unsigned)s.nlev;
                if (obad) atomicOr(err, 4);
                s_oct[j] = obad ? 0 : o2;
                s_flag[j] = (uint8_t)((s.mpf[t0 + j] & 1) | (obad ? 1 : 0) | (s.uright[t0 + j] >= 0.f ? 2 : 0));
            }
        }
        __syncthreads();
        if (active && !skip1) {
            const int jb = part * (kSlotTile / kSlotSplit), je = min(nt, jb + kSlotTile / kSlotSplit);
            for (int j = jb; j < je; j++) {
                const int fl = s_flag[j];
                if (fl & 1) continue;  // vbMatched2 is never set; pMP2 != NULL skips (:722-726)
                const uint4 c0 = s_desc[2 * j], c1 = s_desc[2 * j + 1];
                const int dist = __popc(qd[0] ^ c0.x) + __popc(qd[1] ^ c0.y) + __popc(qd[2] ^ c0.z) +
                                 __popc(qd[3] ^ c0.w) + __popc(qd[4] ^ c1.x) + __popc(qd[5] ^ c1.y) +
                                 __popc(qd[6] ^ c1.z) + __popc(qd[7] ^ c1.w);
                if (dist > 50 || dist > bestDist) continue;
                const float x2 = s_x[j], y2 = s_y[j];
                const int oct2 = s_oct[j];
                if (!st1 && !(fl & 2)) {  // mono-mono: epipole radius (:743-749)
                    const float dx = __fsub_rn(ex, x2), dy = __fsub_rn(ey, y2);
                    if (__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < s_th100[oct2]) continue;
                }
                if (slot_epi_ok(la, lb, lc, x2, y2, s_sig2[oct2])) {
                    bestIdx2 = t0 + j;
                    bestDist = dist;
                }
            }
        }
    }
    s_bd[part][ql] = bestDist;
    s_bi[part][ql] = bestIdx2;
    __syncthreads();
    if (part != 0) return;
    for (int k = 1; k < kSlotSplit; k++) {
        const int d = s_bd[k][ql], i = s_bi[k][ql];
        if (i >= 0 && (bestIdx2 < 0 || d < bestDist || (d == bestDist && i > bestIdx2))) {
            bestDist = d;
            bestIdx2 = i;
        }
    }
    if (idx1 < q.cap) out[idx1] = active ? bestIdx2 : -1;
    if (active && bestIdx2 >= 0) atomicAdd(&nmatches[r], 1);
}

/* ----------------------------------------------------------------------------------- */
/* Common BoW nodes: block (i, slot) takes query node i; the reference's merge walk       */
/* (:691-789) visits exactly the node ids present in both FeatureVectors. Lane per query   */
/* of the node, candidates of the slot's node in order. Output rows preset to -1.         */
/* ----------------------------------------------------------------------------------- */
__global__ __launch_bounds__(64) void k_tri_slots_bow(const QueryKF q, const uint8_t* __restrict__ slots,
                                                      long long slot_bytes, int slot0, const SlotGeoms G,
                                                      int32_t* __restrict__ match, int32_t* __restrict__ nmatches,
                                                      int32_t* __restrict__ err) {
    const int gr = blockIdx.y, r = slot0 + gr, i = blockIdx.x;
    SlotRef s;
    if (!slot_open(slots + (long long)r * slot_bytes, slot_bytes, s)) {
        if (i == 0 && threadIdx.x == 0) atomicOr(err, 4);
        return;
    }
    const int nfv1 = min(max(*q.nfv, 0), q.cap);
    // query nodes at or above the grid's max_nodes would never be visited: flag it (the caller cannot
    // cheaply check the device count, as k_tri_slots_bf flags count > cap)
    if (i == 0 && threadIdx.x == 0 && nfv1 > (int)gridDim.x) atomicOr(err, 2);
    if (i >= nfv1) return;
    const int n1 = min(max(*q.count, 0), q.cap);
    const uint32_t node = q.fv_node[i];
    int lo = 0, hi = s.nfv;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s.fv_node[mid] < node) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= s.nfv || s.fv_node[lo] != node) return;  // not a common node
    const int cb = min(max(s.fv_off[lo], 0), s.cap);
    const int ce = min(max(s.fv_off[lo + 1], cb), s.cap);
    const int qb = min(max(q.fv_off[i], 0), q.cap);
    const int qe = min(max(q.fv_off[i + 1], qb), q.cap);
    const float* F = G.F[gr];
    const float ex = G.ex[gr], ey = G.ey[gr];
    int32_t* out = match + (long long)r * q.cap;
    for (int qi = qb + (int)threadIdx.x; qi < qe; qi += 64) {
        const int idx1 = q.fv_feat[qi];
        if ((unsigned)idx1 >= (unsigned)n1) { atomicOr(err, 8); continue; }
        if (q.mpf && (q.mpf[idx1] & 1)) continue;  // :699-703
        const bool st1 = q.uright ? q.uright[idx1] >= 0.f : false;
        uint32_t qd[8];
        const uint4* d = (const uint4*)(q.desc + (long long)idx1 * 32);
        const uint4 a0 = d[0], a1 = d[1];
        qd[0] = a0.x; qd[1] = a0.y; qd[2] = a0.z; qd[3] = a0.w; qd[4] = a1.x; qd[5] = a1.y; qd[6] = a1.z; qd[7] = a1.w;
        const float2 p1 = q.kun ? q.kun[idx1] : (float2){q.kps[idx1].x, q.kps[idx1].y};
        float la, lb, lc;
        slot_epi_line(F, p1.x, p1.y, &la, &lb, &lc);
        int bestDist = 50, bestIdx2 = -1;
        for (int ci = cb; ci < ce; ci++) {
            const int idx2 = s.fv_feat[ci];
            if ((unsigned)idx2 >= (unsigned)s.n) { atomicOr(err, 4); continue; }
            if (s.mpf[idx2] & 1) continue;  // :722-726
            const int oct2 = s.kps[idx2].octave;
            if ((unsigned)oct2 >= (unsigned)s.nlev) { atomicOr(err, 4); continue; }  // as orbx_slot_parse
            const bool st2 = s.uright[idx2] >= 0.f;
            const uint4* cd = (const uint4*)(s.desc + (long long)idx2 * 32);
            const uint4 c0 = cd[0], c1 = cd[1];
            const int dist = __popc(qd[0] ^ c0.x) + __popc(qd[1] ^ c0.y) + __popc(qd[2] ^ c0.z) +
                             __popc(qd[3] ^ c0.w) + __popc(qd[4] ^ c1.x) + __popc(qd[5] ^ c1.y) +
                             __popc(qd[6] ^ c1.z) + __popc(qd[7] ^ c1.w);
            if (dist > 50 || dist > bestDist) continue;
            const float2 p2 = s.kun[idx2];
            if (!st1 && !st2) {
                const float dx = __fsub_rn(ex, p2.x), dy = __fsub_rn(ey, p2.y);
                if (__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < __fmul_rn(100.f, s.meta->mvScaleFactors[oct2]))
                    continue;
            }
            if (slot_epi_ok(la, lb, lc, p2.x, p2.y, s.meta->mvLevelSigma2[oct2])) {
                bestIdx2 = idx2;
                bestDist = dist;
            }
        }
        out[idx1] = bestIdx2;
        if (bestIdx2 >= 0) atomicAdd(&nmatches[r], 1);
    }
}

/* ----------------------------------------------------------------------------------- */
/* Cross-agent SearchByBoW(KF1 = this agent's keyframe, KF2 = slot r) (ORBmatcher.cc:522-655). */
/* Block (i, slot) takes query node i; if the slot has the node (the reference's merge walk    */
/* visits exactly the common node ids), the node's queries run in order (:554): a query with   */
/* a good MapPoint (:558-562) takes the first strict minimum over the node's not yet matched   */
/* candidates with a good MapPoint (:571-592; vbMatched2 can only hold this node's candidates: */
/* a feature sits in one node), best2 = the minimum over the others; accept iff best1 < TH_LOW */
/* and (float)best1 < nnratio * (float)best2 (:594-598). The node's candidates are staged once */
/* in LDS (descriptor, feature index or -1 when it has no good MapPoint or is matched), 64     */
/* queries at a time sit one per lane and are broadcast by readlane, so the greedy walk's      */
/* per-query step reads only LDS. Lane j holds candidates j, j+64, ...; its local first        */
/* minimum and runner-up merge by two wave minima of (dist << 16 | position).                  */
/* match[r*cap1 + idx1] = the slot keyframe's feature idx2 (preset to -1 by the caller).       */
/* ----------------------------------------------------------------------------------- */
__device__ __forceinline__ uint32_t rl(uint32_t v, int t) { return (uint32_t)__builtin_amdgcn_readlane((int)v, t); }

__global__ __launch_bounds__(64) void k_bow_slots(const QueryKF q, const uint8_t* __restrict__ slots, long long slot_bytes,
                                                  int slot0, float nnratio, int lds_cap, int32_t* __restrict__ match,
                                                  int32_t* __restrict__ err) {
    extern __shared__ __align__(16) uint8_t lds[];  // [lds_cap] x 2 uint4 descriptors | [lds_cap] int candidates
    uint4* s_cd = (uint4*)lds;
    int* s_ci = (int*)(lds + 32 * (size_t)lds_cap);  // feature index, -1: no good MapPoint or matched (vbMatched2)
    const int gr = blockIdx.y, r = slot0 + gr, i = blockIdx.x, lane = threadIdx.x;
    SlotRef s;
    if (!slot_open(slots + (long long)r * slot_bytes, slot_bytes, s)) {
        if (i == 0 && lane == 0) atomicOr(err, 4);
        return;
    }
    const int nfv1 = min(max(*q.nfv, 0), q.cap);
    if (i == 0 && lane == 0 && nfv1 > (int)gridDim.x) atomicOr(err, 2);  // query nodes past max_nodes
    if (i >= nfv1) return;
    const uint32_t node = q.fv_node[i];
    int lo = 0, hi = s.nfv;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s.fv_node[mid] < node) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= s.nfv || s.fv_node[lo] != node) return;  // not a common node
    const int cb = min(max(s.fv_off[lo], 0), s.cap);
    const int ce = min(max(s.fv_off[lo + 1], cb), s.cap);
    const int nc = ce - cb;
    if (nc > lds_cap) {
        if (lane == 0) atomicOr(err, 8);
        return;
    }
    const int qb = min(max(q.fv_off[i], 0), q.cap);
    const int qe = min(max(q.fv_off[i + 1], qb), q.cap);
    const int n1 = min(max(*q.count, 0), q.cap);
    for (int j = lane; j < nc; j += 64) {
        const int idx2 = s.fv_feat[cb + j];
        int ci = -1;
        if ((unsigned)idx2 >= (unsigned)s.n) {
            atomicOr(err, 4);
        } else if ((s.mpf[idx2] & 3) == 1) {  // pMP2 NULL or bad (:575-579)
            const uint4* cd = (const uint4*)(s.desc + (long long)idx2 * 32);
            s_cd[2 * j] = cd[0];
            s_cd[2 * j + 1] = cd[1];
            ci = idx2;
        }
        s_ci[j] = ci;
    }
    __syncthreads();
    int32_t* out = match + (long long)r * q.cap;
    for (int q0 = qb; q0 < qe; q0 += 64) {
        // this lane's query of the next 64: feature index (-1: no good MapPoint, :558-562) and descriptor
        int idx1 = -1;
        uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
        if (q0 + lane < qe) {
            idx1 = q.fv_feat[q0 + lane];
            if ((unsigned)idx1 >= (unsigned)n1) {
                atomicOr(err, 8);
                idx1 = -1;
            } else if (!q.mpf || (q.mpf[idx1] & 3) != 1) {
                idx1 = -1;
            } else {
                const uint4* d = (const uint4*)(q.desc + (long long)idx1 * 32);
                a0 = d[0];
                a1 = d[1];
            }
        }
        const int nq = min(64, qe - q0);
        for (int t = 0; t < nq; t++) {  // the node's queries in order (wave-uniform)
            const int i1 = (int)rl((uint32_t)idx1, t);
            if (i1 < 0) continue;
            const uint32_t x0 = rl(a0.x, t), x1 = rl(a0.y, t), x2 = rl(a0.z, t), x3 = rl(a0.w, t);
            const uint32_t x4 = rl(a1.x, t), x5 = rl(a1.y, t), x6 = rl(a1.z, t), x7 = rl(a1.w, t);
            int b1 = 256, j1 = -1, b2 = 256;
            for (int j = lane; j < nc; j += 64) {
                if (s_ci[j] < 0) continue;
                const uint4 c0 = s_cd[2 * j], c1 = s_cd[2 * j + 1];
                const int dist = __popc(x0 ^ c0.x) + __popc(x1 ^ c0.y) + __popc(x2 ^ c0.z) + __popc(x3 ^ c0.w) +
                                 __popc(x4 ^ c1.x) + __popc(x5 ^ c1.y) + __popc(x6 ^ c1.z) + __popc(x7 ^ c1.w);
                if (dist < b1) {
                    b2 = b1;
                    b1 = dist;
                    j1 = j;
                } else if (dist < b2) {
                    b2 = dist;
                }
            }
            // the first strict minimum over all lanes = min of (dist << 16 | position); best2 = the minimum over
            // every other eligible candidate: the owner lane's runner-up, every other lane's own minimum
            const uint32_t k1 = j1 >= 0 ? ((uint32_t)b1 << 16) | (uint32_t)j1 : 0xFFFFFFFFu;
            const uint32_t kmin = wave_min_u32(k1);
            const bool owner = kmin != 0xFFFFFFFFu && k1 == kmin;
            const uint32_t bd2 = wave_min_u32(owner ? (uint32_t)b2 : (uint32_t)b1);
            if (kmin == 0xFFFFFFFFu) continue;
            const int best1 = (int)(kmin >> 16), pos = (int)(kmin & 0xFFFFu);
            if (best1 < 50 && __fmul_rn(1.0f, (float)best1) < __fmul_rn(nnratio, (float)bd2)) {  // TH_LOW, :594-598
                __syncthreads();  // every lane has read s_ci[pos] for this query
                if (lane == 0) {
                    out[i1] = s_ci[pos];
                    s_ci[pos] = -1;  // vbMatched2
                }
                __syncthreads();
            }
        }
    }
}

/* the rotation consistency of k_bow_slots' matches (ORBmatcher.cc:600-611, 633-650): rot = angle1 - angle2,
 * bin = round(rot / 30) mod 30, ComputeThreeMaxima (:1601-1642), every match outside the three bins dropped;
 * then nmatches[r] = the matches kept. One workgroup per slot. */
__global__ __launch_bounds__(256) void k_rot_slots(const QueryKF q, const uint8_t* __restrict__ slots,
                                                   long long slot_bytes, int slot0, int check_ori,
                                                   int32_t* __restrict__ match, int32_t* __restrict__ nmatches) {
    __shared__ int hist[32];
    __shared__ int keep[3];
    const int r = slot0 + blockIdx.x, tid = threadIdx.x;
    SlotRef s;
    if (!slot_open(slots + (long long)r * slot_bytes, slot_bytes, s)) return;  // flagged by k_bow_slots
    const int n1 = min(max(*q.count, 0), q.cap);
    int32_t* m = match + (long long)r * q.cap;
    auto bin_of = [&](int i, int j) {
        float rot = __fsub_rn(q.kps[i].angle, s.kps[j].angle);  // vKeysUn angle = vKeys angle
        if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
        const int bin = (int)roundf(__fmul_rn(rot, 1.0f / 30));
        return bin == 30 ? 0 : bin;
    };
    if (tid < 32) hist[tid] = 0;
    __syncthreads();
    if (check_ori) {
        for (int i = tid; i < n1; i += 256)
            if (m[i] >= 0) atomicAdd(&hist[bin_of(i, m[i])], 1);
        __syncthreads();
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int b = 0; b < 30; b++) {
                const int v = hist[b];
                if (v > max1) { max3 = max2; max2 = max1; max1 = v; ind3 = ind2; ind2 = ind1; ind1 = b; }
                else if (v > max2) { max3 = max2; max2 = v; ind3 = ind2; ind2 = b; }
                else if (v > max3) { max3 = v; ind3 = b; }
            }
            if (max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
            else if (max3 < __fmul_rn(0.1f, (float)max1)) { ind3 = -1; }
            keep[0] = ind1; keep[1] = ind2; keep[2] = ind3;
        }
        __syncthreads();
    }
    int local = 0;
    for (int i = tid; i < n1; i += 256) {
        const int j = m[i];
        if (j < 0) continue;
        if (check_ori) {
            const int bin = bin_of(i, j);
            if (bin != keep[0] && bin != keep[1] && bin != keep[2]) {
                m[i] = -1;
                continue;
            }
        }
        local++;
    }
    if (local) atomicAdd(&nmatches[r], local);
}

/* ----------------------------------------------------------------------------------- */
/* Read-and-clear of a sticky device error word in one atomic step (orbx_check_error,      */
/* orbm_check_error): a kernel on another stream that raises the flag after the exchange    */
/* leaves it set for the next check instead of racing a host-side clear.                   */
/* ----------------------------------------------------------------------------------- */
__global__ void k_flag_take(int32_t* flag, int32_t* out) {
    if (threadIdx.x == 0) *out = atomicExch(flag, 0);
}

hipError_t launch_flag_take(int32_t* flag, int32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_flag_take, dim3(1), dim3(64), 0, st, flag, out);
    return hipGetLastError();
}

/* The host extraction's last launch: takes the call's error word into mapped host memory like k_flag_take, then
 * stores the call's done word there (the device call counter + 1, never the value the host read before the
 * launch), last, with release at system scope: the host polls it instead of synchronising the stream. */
__global__ void k_call_done(int32_t* flag, int32_t* out_err, int32_t* seq, int32_t* out_done) {
    if (threadIdx.x == 0) {
        *out_err = atomicExch(flag, 0);
        const int32_t s = *seq >= (1 << 30) ? 1 : *seq + 1;
        *seq = s;
        __threadfence_system();
        __hip_atomic_store(out_done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_call_done(int32_t* flag, int32_t* out_err, int32_t* seq, int32_t* out_done, hipStream_t st) {
    hipLaunchKernelGGL(k_call_done, dim3(1), dim3(64), 0, st, flag, out_err, seq, out_done);
    return hipGetLastError();
}

/* ----------------------------------------------------------------------------------- */
hipError_t launch_pack_slot(const orbx_kf_source& src, const SlotLayout& L, const orbx_kf_meta& meta, uint8_t* slot,
                            int32_t* err, hipStream_t st) {
    PackArgs a;
    a.src = src;
    a.L = L;
    a.meta = meta;
    const int blocks = (L.cap + 1 + 255) / 256;
    hipLaunchKernelGGL(k_pack_slot, dim3(blocks), dim3(256), 0, st, a, slot, err);
    return hipGetLastError();
}

hipError_t launch_tri_slots(const QueryKF& q, const uint8_t* slots, long long slot_bytes, int nref,
                            const orbm_slot_geom* geom, int use_bow, int max_nodes, int32_t* match,
                            int32_t* nmatches, int32_t* err, hipStream_t st) {
    for (int s0 = 0; s0 < nref; s0 += kMaxSlotsPerLaunch) {
        const int ns = nref - s0 < kMaxSlotsPerLaunch ? nref - s0 : kMaxSlotsPerLaunch;
        SlotGeoms G;
        for (int k = 0; k < kMaxSlotsPerLaunch; k++) {
            const orbm_slot_geom& g = geom[k < ns ? s0 + k : s0];
            for (int e = 0; e < 9; e++) G.F[k][e] = g.F12[e];
            G.ex[k] = g.ex;
            G.ey[k] = g.ey;
        }
        if (use_bow) {
            if (max_nodes > 0)
                hipLaunchKernelGGL(k_tri_slots_bow, dim3(max_nodes, ns), dim3(64), 0, st, q, slots, slot_bytes, s0, G,
                                   match, nmatches, err);
        } else {
            hipLaunchKernelGGL(k_tri_slots_bf, dim3((q.cap + kSlotQ - 1) / kSlotQ, ns), dim3(256), 0, st, q, slots,
                               slot_bytes, s0, G, match, nmatches, err);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_bow_slots(const QueryKF& q, const uint8_t* slots, long long slot_bytes, int nref, float nnratio,
                            int check_ori, int max_nodes, int32_t* match, int32_t* nmatches, int32_t* err,
                            hipStream_t st) {
    if (nref == 0) return hipSuccess;
    if (max_nodes > 0) {
        // the node's candidates in LDS: 36 bytes each, up to the largest capacity a slot of slot_bytes can carry (a
        // node holds at most every feature of its slot, whatever the query keyframe's own capacity), bounded by the
        // 160 KB of a CU (4551 candidates; a node past the bound is flagged, error 8)
        int slot_cap = 0;
        for (int lo = 0, hi = kSlotMaxCap; lo <= hi;) {  // largest cap whose layout fits slot_bytes
            const int mid = (lo + hi) / 2;
            uint32_t off[ORBX_SLOT_NSECTIONS], total = 0;
            if (slot_offsets(mid, off, &total) && (long long)total <= slot_bytes) {
                slot_cap = mid;
                lo = mid + 1;
            } else {
                hi = mid - 1;
            }
        }
        const int lds_cap = std::min(std::max(q.cap, slot_cap), 160 * 1024 / 36);
        const size_t lds = 36 * (size_t)lds_cap;
        if (lds > 65536) {  // past the 64 KB default (a host-side attribute of the current device's function)
            const hipError_t e = hipFuncSetAttribute((const void*)k_bow_slots, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_bow_slots, dim3(max_nodes, nref), dim3(64), lds, st, q, slots, slot_bytes, 0, nnratio,
                           lds_cap, match, err);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_rot_slots, dim3(nref), dim3(256), 0, st, q, slots, slot_bytes, 0, check_ori, match, nmatches);
    return hipGetLastError();
}

}  // namespace orbamd
