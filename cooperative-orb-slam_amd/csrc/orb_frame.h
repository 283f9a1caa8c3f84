/*
 * orb_frame.h -- arguments of the Frame-level kernels (frame_kernels.hip): the consumers of
 * the extractor output that ORB-SLAM2's Frame runs next on the Tracking thread.
 */
#pragma once
#include <stdint.h>

#include "orb_device.h"

namespace orbamd {

/* one side (left or right extractor) of a stereo batch: the pyramid of its last extraction.
 * level 0 = the caller's frames (read in place), levels >= 1 = the handle's pyramid buffer */
struct PyrSide {
    const uint8_t* l0;
    long long l0_fstride;
    const uint8_t* pyr;
    long long pyr_fstride;
    int l0_pitch;
    int nframes;  // frames of that extraction (bounds of the frame-index arrays)
};

/* Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641) constants and the level
 * geometry of both pyramids (identical: same size and ORB parameters) */
struct StereoArgs {
    PyrSide left, right;
    int L;
    int nrows;      // mvImagePyramid[0].rows: size of vRowIndices (Frame.cc:477-483)
    int rspan;      // >= max over octaves of maxr - minr (Frame.cc:491-494)
    float maxD;     // mbf / minZ with minZ = mb (Frame.cc:501-503)
    float bf;       // mbf
    float thc;      // 1.5f*1.4f (Frame.cc:639), folded in float
    float scale[kMaxLevels], inv_scale[kMaxLevels];
    int lw[kMaxLevels], lh[kMaxLevels], lpitch[kMaxLevels];
    long long pyr_off[kMaxLevels];
};

/* SearchByProjection (ORBmatcher.cc:45-129, 290-403, 1328-1470, 1472-1599): one MapPoint after
 * the host prologue of its variant (projection, frustum and scale tests) */
constexpr int kGridCols = 64;  // FRAME_GRID_COLS (Frame.h:38)
constexpr int kGridRows = 48;  // FRAME_GRID_ROWS (Frame.h:37)
constexpr int kProjValid = 1, kProjClaims = 2, kProjStereo = 4;
// Fuse(pKF, vpMapPoints, th) (ORBmatcher.cc:904-929): reprojection-error test of each candidate,
// e2 * mvInvLevelSigma2[level] > 7.8 (stereo: u, v, ur) or > 5.99 (mono: u, v) rejects
constexpr int kProjChi2 = 8;

struct ProjQuery {
    float u, v, radius;        // GetFeaturesInArea(u, v, radius, min_level, max_level)
    int min_level, max_level;
    float ur, er_th;           // stereo check: fabs(ur - mvuRight[i]) > er_th rejects (kProjStereo); ur also
                               // feeds the kProjChi2 residual
    float angle;               // source keypoint angle (rotation histogram)
    int flags;                 // kProjValid | kProjClaims (a match occupies the feature) | kProjStereo
    int src;                   // MapPoint index reported in the output
};

/* one SearchByProjection call: the Frame/KeyFrame arrays, its queries, scratch and outputs */
struct ProjCall {
    const float *x, *y, *angle, *uright;
    const int32_t* octave;
    const uint8_t* occ0;       // initial occupancy (NULL = none)
    const uint8_t* desc;
    int n;
    float min_x, min_y, gw_inv, gh_inv;
    const ProjQuery* q;
    const uint8_t* qdesc;
    int nq;
    int accept_th;             // bestDist <= accept_th
    int ratio;                 // second-best ratio test when both on one level (ORBmatcher.cc:116-121)
    float nnratio;
    int check_ori;
    int* grid_start;           // [kGridCols*kGridRows + 1]
    uint16_t* grid_idx;        // [n]
    unsigned long long* scan;  // [4*nq] the 4 smallest candidate keys per query, ascending
    int* scan_cnt;             // [nq] candidates per query
    int* res;                  // [2*nq] accepted feature idx / rotation bin
    float inv_sigma2[kMaxLevels];  // mvInvLevelSigma2 (kProjChi2 queries)
    int32_t* match;            // [n]
    int32_t* nmatches;
    int direct;                // per-query results only, no claims / ratio / rotation (Fuse): k_proj_scan writes
                               // res[] from its best key and k_proj_resolve is not launched
    int n_out;                 // SearchForInitialization (k_init_resolve): F1's N, the length of match[] =
                               // vnMatches12
    unsigned long long* host_out;  // per-call host API (or nullptr): the results written straight to pinned host
                                   // memory, each entry (uint32 value | seq << 32): direct mode one per query,
                                   // otherwise match[0 .. n or n_out) then nmatches
    int seq;                       // this call's sequence number (> 0)
};

}  // namespace orbamd
