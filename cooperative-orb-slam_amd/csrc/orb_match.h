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

}  // namespace orbamd
