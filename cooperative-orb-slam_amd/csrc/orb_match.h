/*
 * orb_match.h -- matcher argument structs shared by capi.cpp and match_kernels.hip.
 */
#pragma once
#include <stdint.h>

namespace orbamd {

/* F12 (row-major, F12.at<float>(r,c)), epipole and per-octave thresholds:
 * th100[o] = 100*mvScaleFactors[o] (float, ORBmatcher.cc:747),
 * th384[o] = 3.84*mvLevelSigma2[o] (double, ORBmatcher.cc:156). */
struct MatchGeom {
    float F[9];
    float ex, ey;
    float th100[16];
    double th384[16];
    float th384f[16];  // th384 rounded up to a float: (double)d < th384 <=> d < th384f for a float d
};

/* device-side copy of an orbm_kf_view */
struct DevView {
    const uint8_t* desc;
    const float* x;
    const float* y;
    const float* angle;
    const int32_t* octave;
    const float* uright;
    const uint8_t* has_mp;
    const uint8_t* mp_bad;
    const int32_t* node_feat;
    int32_t n;
};

/* one common BoW node (or a 64-query chunk of it): ranges into node_feat of each side */
struct NodeTask {
    int q_begin, q_end, c_begin, c_end;
};

/* one host-API match call (match_kernels.hip call_emit / call_tail): state = 32 zeroed device
 * words (ticket, list length, 30 rotation bins), list = device scratch for up to n matches,
 * host_out = the caller's pinned buffer (count, then n entries pre-filled with -1) */
struct CallTail {
    int32_t* state;
    int32_t* list;  // 4 words per match: index, partner, rotation bin, 0
    int32_t* host_out;
    const float* angA;
    const float* angB;
    int n, check_ori, swap;
};

/* One small per-call SearchByBoW (k_bow_small), passed whole in the kernel arguments: the per-call
 * inputs (common nodes, MapPoint eligibility bits) need no H2D copy, and both sides' descriptors and
 * angles are read in FeatureVector order (node position p), so a node's candidates are one contiguous
 * load. Each workgroup (one common node) writes its accepts into the host-mapped out[q_begin ..) and its
 * {seq, count} word; the host polls both (every store carries the call's seq) and applies the rotation
 * histogram. */
constexpr int kSmallTasks = 160;
constexpr uint32_t kSmallSeqMask = (1u << 27) - 1;  // call sequence numbers 1 .. 2^27-1
/* an accept in host memory: x (16 bits: the output index), y (16: its partner), the rotation bin (5) and the
 * call's seq (27), written with one 64-bit store; feature indices < 65536 (host checked) */
__host__ __device__ inline unsigned long long small_entry(int x, int y, int bin, uint32_t seq) {
    return (unsigned long long)(uint32_t)x | (unsigned long long)(uint32_t)y << 16 | (unsigned long long)bin << 32 |
           (unsigned long long)(seq & kSmallSeqMask) << 37;
}
constexpr int kSmallBitWords = 64;  // node positions < 2048 per side
struct SmallTask {
    uint16_t q_begin, q_end, c_begin, c_end;
};
/* one keypoint in FeatureVector order: position, octave (| 0x100 when mvuRight >= 0), angle */
struct NodeRec {
    float x, y;
    int32_t oct;
    float angle;
};
struct BowSmall {
    const uint4* qd;     // query side (the KeyFrame): 2 x uint4 per node position
    const float* qa;     // its keypoint angles: qa[p * qa_stride] (NodeRec::angle of a cached entry, stride 4)
    const int32_t* qf;   // its feature index per node position
    const uint4* cd;
    const float* ca;
    const int32_t* cf;
    int qa_stride, ca_stride;
    unsigned long long* out;   // host-mapped small_entry: mode 0 (F idx, KF idx) / mode 1 (KF1 idx, KF2 idx)
    unsigned long long* done;  // host-mapped: per task seq | count << 32
    int seq, ntasks, mode, check_ori;
    float nnratio;
    uint32_t qgood[kSmallBitWords];  // bit p: the query at node position p has a good MapPoint
    uint32_t cgood[kSmallBitWords];  // mode 1: the candidate at p has one (mode 0: every candidate is one)
    SmallTask tasks[kSmallTasks];
};

/* One small per-call SearchForTriangulation over common BoW nodes (k_tri_small): tasks are 64-query chunks
 * of a common node; the MapPoint bits say which node positions have a MapPoint (never matched) */
struct TriSmall {
    const uint4* qd;
    const NodeRec* qr;
    const int32_t* qf;
    const uint4* cd;
    const NodeRec* cr;
    const int32_t* cf;
    unsigned long long* out;  // small_entry (KF1 idx, KF2 idx)
    unsigned long long* done;
    int seq, ntasks, check_ori, only_stereo, q_ur, c_ur;  // q_ur / c_ur: the view has mvuRight
    MatchGeom g;
    uint32_t qmp[kSmallBitWords];
    uint32_t cmp[kSmallBitWords];
    SmallTask tasks[kSmallTasks];
};

}  // namespace orbamd
