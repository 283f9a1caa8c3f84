/*
 * orbslam_amd.h -- C ABI of the MI355X-native ORB front-end + Hamming matcher.
 *
 * This is the drop-in boundary underneath the reference's two C++ class surfaces
 * (ORB_SLAM2/include/ORBextractor.h:45-111, ORB_SLAM2/include/ORBmatcher.h:37-102; the
 * files are byte-identical in ORB_SLAM2/ and ORB_SLAM2.1/). Every entry point below
 * names the reference member it replaces. Plain pointers and sizes only; no torch,
 * OpenCV or HIP types cross it (streams are passed as `void*` = hipStream_t).
 *
 * Conventions:
 *   return 0 = OK, negative = error (ORBX_E*). Nothing throws across the ABI.
 *   Host entry points take host memory; *_device entry points take device memory and a
 *   stream and do not synchronise.
 *   A handle (orbx_handle / orbm_ctx) must not be used by two threads at once; create one
 *   per thread (the reference creates one ORBextractor per Tracking instance and stack
 *   ORBmatcher objects per thread: Tracking.cc:119-125, LocalMapping.cc:215).
 */
#ifndef ORBSLAM_AMD_H
#define ORBSLAM_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBX_OK 0
#define ORBX_EARG (-1)     /* bad argument (null pointer, size out of range)          */
#define ORBX_EDEVICE (-2)  /* HIP runtime / kernel failure, or no usable device        */
#define ORBX_ECAPACITY (-3) /* caller buffer too small for the result                  */

/* ------------------------------------------------------------------------------------
 * Extractor -- replaces ORB_SLAM2::ORBextractor (ORBextractor.h:45-111, .cc:410-1132)
 * ---------------------------------------------------------------------------------- */

/* ctor arguments of ORBextractor::ORBextractor (ORBextractor.cc:410-411); the values the
 * reference runs with are my.yaml:31-43 = {1000, 1.2f, 8, 20, 7}. */
typedef struct orbx_params {
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
} orbx_params;

/* One output keypoint = cv::KeyPoint of ORBextractor::operator() (ORBextractor.cc:1043-1105)
 * minus class_id (always -1 in the reference). 24 bytes. Coordinates are level-0 pixels
 * (pt *= mvScaleFactor[level], ORBextractor.cc:1095-1101). */
typedef struct orbx_kp {
    float x, y;
    float size;      /* (int)(PATCH_SIZE * mvScaleFactor[level])  ORBextractor.cc:837,846 */
    float angle;     /* IC_Angle, degrees in [0,360]               ORBextractor.cc:77-104  */
    float response;  /* FAST score                                 ORBextractor.cc:809-816 */
    int32_t octave;  /* pyramid level                              ORBextractor.cc:845     */
} orbx_kp;

typedef struct orbx_handle orbx_handle;

/* ORBextractor::ORBextractor (ORBextractor.cc:410-470). Device buffers are sized for frames
 * up to max_width x max_height and batches up to max_batch frames. device = HIP ordinal. */
int orbx_create(const orbx_params* params, int device, int max_width, int max_height,
                int max_batch, orbx_handle** out);
void orbx_destroy(orbx_handle* h);

/* Upper bound on keypoints one frame can produce: sum over levels of
 * max(N_l + 3, 4*nIni_l) (DistributeOctTree overshoot, ORBextractor.cc:669-735). */
int orbx_max_keypoints(const orbx_handle* h, int width, int height);

/* ORBextractor::operator()(image, mask(ignored), keypoints, descriptors)
 * (ORBextractor.cc:1043-1105). Host image (8UC1, row pitch in bytes); outputs written to
 * host arrays kps[cap], desc[cap*32] in the reference's order (levels 0..L-1, each in
 * DistributeOctTree order). *n = keypoint count. Empty image (w or h == 0) -> *n = 0,
 * outputs untouched (ORBextractor.cc:1046-1047). */
int orbx_extract(orbx_handle* h, const uint8_t* img, int width, int height, size_t pitch,
                 orbx_kp* kps, uint8_t* desc, int cap, int* n);

/* Batched, device-resident form of operator(): nframes frames at d_frames + f*frame_stride
 * (each width x height, row pitch `pitch`). Per frame f: kps at d_kps + f*kp_stride,
 * descriptors at d_desc + f*kp_stride*32, count at d_counts[f]. kp_stride must be
 * >= orbx_max_keypoints(). Enqueued on `stream` (hipStream_t); no host sync. */
int orbx_extract_batch_device(orbx_handle* h, int nframes, const uint8_t* d_frames,
                              size_t frame_stride, int width, int height, size_t pitch,
                              orbx_kp* d_kps, uint8_t* d_desc, int32_t* d_counts,
                              int kp_stride, void* stream);

/* Waits for `stream` and reports a device-side consistency failure (octree capacity or
 * root-index overflow) of any batched extraction since the previous check: 0 = OK,
 * ORBX_EDEVICE otherwise (the flag is then cleared). */
int orbx_check_error(orbx_handle* h, void* stream);

/* public ORBextractor::mvImagePyramid (ORBextractor.h:85), materialised lazily: copies
 * level `level` of frame `frame` of the most recent extraction to host dst (pitch bytes).
 * Pass dst = NULL to query the size only. */
int orbx_pyramid_level(orbx_handle* h, int frame, int level, uint8_t* dst, size_t pitch,
                       int* width, int* height);

/* public ORBextractor::mvImagePyramid (ORBextractor.h:85, filled by ComputePyramid in every
 * operator() call, ORBextractor.cc:1107-1132) delivered eagerly for the host path without a
 * copy after the call: with on != 0 every subsequent orbx_extract on `h` also writes the frame's
 * levels 1..L-1 into pinned host memory from extra workgroups of its octree launch (they copy
 * while the octree runs, so the call's latency does not grow), and orbx_host_pyramid_level then
 * points at level `level` of the last orbx_extract (level 0: the call's pinned copy of the
 * input image). The memory belongs to the handle: valid until the next orbx_extract,
 * orbx_set_host_pyramid or orbx_destroy on it. ORBX_EARG when the last call delivered none
 * (host pyramid off, or a stage-profiled call). */
int orbx_set_host_pyramid(orbx_handle* h, int on);
int orbx_host_pyramid_level(orbx_handle* h, int level, const uint8_t** data, size_t* pitch,
                            int* width, int* height);

/* Caller-owned destination of that eager pyramid. The reference assigns every level a freshly
 * allocated Mat in each call (ORBextractor.cc:1114-1115), so a level a caller keeps is never
 * overwritten by a later call; the drop-in ORBextractor keeps that by handing each call storage no
 * caller holds (host/ORBextractor.cc). orbx_host_pyramid_bytes: bytes of one target for a
 * width x height frame (level 0 contiguous at offset 0, rounded up to 256, then levels 1..L-1 in
 * the device layout). orbx_host_register / orbx_host_unregister: make caller memory writable by
 * the device (mapped) and release it again. orbx_set_host_pyramid_target: subsequent
 * orbx_extract calls on `h` write their levels into `host` (registered, >= bytes of the frame;
 * ORBX_EARG from orbx_extract otherwise), and orbx_host_pyramid_level then points into the target
 * the last call filled; host = NULL returns to the handle's own pinned memory. The target stays
 * the caller's: the library never frees or unregisters it. */
int orbx_host_pyramid_bytes(orbx_handle* h, int width, int height, size_t* bytes);
int orbx_host_register(void* p, size_t bytes);
int orbx_host_unregister(void* p);
int orbx_set_host_pyramid_target(orbx_handle* h, uint8_t* host, size_t bytes);

/* ORBextractor getters (ORBextractor.h:63-81): GetLevels, GetScaleFactor,
 * GetScaleFactors, GetInverseScaleFactors, GetScaleSigmaSquares,
 * GetInverseScaleSigmaSquares. Arrays have nlevels entries. */
int orbx_get_levels(const orbx_handle* h);
float orbx_get_scale_factor(const orbx_handle* h);
int orbx_get_scale_tables(const orbx_handle* h, float* scale, float* inv_scale, float* sigma2,
                          float* inv_sigma2);
/* The same four tables from the ctor arguments alone, host-only (no device, no handle): the
 * drop-in ORBextractor answers its getters from these even when no device is usable. */
int orbx_compute_scale_tables(const orbx_params* params, float* scale, float* inv_scale, float* sigma2,
                              float* inv_sigma2);
/* mnFeaturesPerLevel (ORBextractor.cc:435-446) and umax (ORBextractor.cc:454-469, 16
 * entries) -- exposed for tests. */
int orbx_get_feature_split(const orbx_handle* h, int32_t* per_level, int32_t* umax16);

/* ------------------------------------------------------------------------------------
 * Matcher -- replaces ORB_SLAM2::ORBmatcher (ORBmatcher.h:37-102, ORBmatcher.cc)
 * ---------------------------------------------------------------------------------- */

/* One KeyFrame/Frame as the matcher sees it, gathered by the caller under its own
 * locks (KeyFrame::GetMapPoint/GetMapPointMatches, ORBmatcher.cc:526,699,722).
 * All arrays have n entries unless noted; host or device memory depending on the call. */
typedef struct orbm_kf_view {
    int32_t n;                 /* KeyFrame::N                                              */
    const uint8_t* desc;       /* mDescriptors, n x 32 contiguous rows                     */
    const float* x;            /* mvKeysUn[i].pt.x                                         */
    const float* y;            /* mvKeysUn[i].pt.y                                         */
    const float* angle;        /* mvKeysUn[i].angle (== mvKeys[i].angle)                   */
    const int32_t* octave;     /* mvKeysUn[i].octave                                       */
    const float* uright;       /* mvuRight; NULL = monocular (all -1)                      */
    const uint8_t* has_mp;     /* GetMapPoint(i) != NULL; NULL = none                      */
    const uint8_t* mp_bad;     /* that MapPoint's isBad(); NULL = none bad                 */
    int32_t n_nodes;           /* DBoW2::FeatureVector as CSR, node ids ascending          */
    const uint32_t* node_id;   /* [n_nodes]                                                */
    const int32_t* node_off;   /* [n_nodes+1] offsets into node_feat                       */
    const int32_t* node_feat;  /* feature indices, ascending within a node                 */
    int32_t nlevels;
    const float* scale_factors; /* mvScaleFactors[nlevels]                                 */
    const float* level_sigma2;  /* mvLevelSigma2[nlevels]                                  */
} orbm_kf_view;

typedef struct orbm_ctx orbm_ctx;

/* ORBmatcher::ORBmatcher(nnratio, checkOri) state lives in the call arguments; the ctx
 * only owns a device, a stream and scratch (one per thread). */
int orbm_create(int device, orbm_ctx** out);
void orbm_destroy(orbm_ctx* ctx);

/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:1647-1663): host, 32-byte rows. */
int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* ORBmatcher::SearchForTriangulation (ORBmatcher.cc:657-823). F12 = 3x3 row-major float
 * (F12.at<float>(r,c)); (ex,ey) = epipole of KF1's centre in KF2 (ORBmatcher.cc:664-670,
 * see orbm_epipole). match12[kf1.n] receives idx2 or -1; *nmatches = pair count. */
int orbm_search_for_triangulation(orbm_ctx* ctx, const orbm_kf_view* kf1, const orbm_kf_view* kf2,
                                  const float F12[9], float ex, float ey, int only_stereo,
                                  int check_ori, int32_t* match12, int* nmatches);

/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (ORBmatcher.cc:159-288).
 * match_f[f.n] receives the KF feature index whose MapPoint was assigned to that Frame
 * feature (vpMapPointMatches[i] = pKF->GetMapPointMatches()[match_f[i]]) or -1. */
int orbm_search_by_bow_kf_f(orbm_ctx* ctx, const orbm_kf_view* kf, const orbm_kf_view* f,
                            float nnratio, int check_ori, int32_t* match_f, int* nmatches);

/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (ORBmatcher.cc:522-655).
 * match12[kf1.n] receives idx2 (vpMatches12[idx1] = vpMapPoints2[idx2]) or -1. */
int orbm_search_by_bow_kf_kf(orbm_ctx* ctx, const orbm_kf_view* kf1, const orbm_kf_view* kf2,
                             float nnratio, int check_ori, int32_t* match12, int* nmatches);

/* Device batch of SearchForTriangulation with one FeatureVector node holding every
 * feature of both keyframes (the BASELINE "BF" configuration): pair p
 * matches frame q1[p] (KF1) against frame q2[p] (KF2) of an orbx_extract_batch_device
 * output (kps/desc/counts/kp_stride as produced there). All keypoints monocular, no
 * MapPoints, one F12/(ex,ey) and one scale table for all pairs. match12[p*kp_stride+i]. */
int orbm_triangulation_bf_batch_device(orbm_ctx* ctx, int npairs, const int32_t* d_q1,
                                       const int32_t* d_q2, const orbx_kp* d_kps,
                                       const uint8_t* d_desc, const int32_t* d_counts,
                                       int kp_stride, const float F12[9], float ex, float ey,
                                       int nlevels, const float* scale_factors,
                                       const float* level_sigma2, int check_ori,
                                       int32_t* d_match12, int32_t* d_nmatches, void* stream);
/* The stereo form of the same batch (ORBmatcher.cc:657-823 with mvuRight, as LocalMapping::CreateNewMapPoints
 * calls it between stereo keyframes): d_uright[f*kp_stride + i] = mvuRight of keypoint i of frame f (-1 =
 * monocular), e.g. the output of orbx_stereo_matches_batch_device for the left frames. The epipole-radius test
 * applies to monocular-monocular pairs only (:743-749); only_stereo = bOnlyStereo (:705-707, :729-731). No
 * MapPoints, one F12/(ex,ey) and scale table for all pairs, match12 / nmatches as above. */
int orbm_triangulation_bf_stereo_batch_device(orbm_ctx* ctx, int npairs, const int32_t* d_q1,
                                              const int32_t* d_q2, const orbx_kp* d_kps,
                                              const uint8_t* d_desc, const int32_t* d_counts,
                                              const float* d_uright, int kp_stride, const float F12[9],
                                              float ex, float ey, int nlevels,
                                              const float* scale_factors, const float* level_sigma2,
                                              int only_stereo, int check_ori, int32_t* d_match12,
                                              int32_t* d_nmatches, void* stream);
/* The same batch over common BoW nodes (SearchForTriangulation's own merge walk,
 * ORBmatcher.cc:691-789, as LocalMapping::CreateNewMapPoints calls it with a real vocabulary):
 * the FeatureVectors are orbv_transform_batch_device's device output for the same frames
 * (fv_node / fv_feat at f*kp_stride, fv_off at f*(kp_stride+1), nfv[f]); max_nodes bounds nfv
 * (e.g. min(kp_stride, k^(L-levelsup))). Mono, no MapPoints, as above. */
int orbm_triangulation_nodes_batch_device(orbm_ctx* ctx, int npairs, const int32_t* d_q1,
                                          const int32_t* d_q2, const orbx_kp* d_kps,
                                          const uint8_t* d_desc, const int32_t* d_counts,
                                          int kp_stride, const uint32_t* d_fv_node,
                                          const int32_t* d_fv_off, const int32_t* d_fv_feat,
                                          const int32_t* d_nfv, int max_nodes, const float F12[9],
                                          float ex, float ey, int nlevels,
                                          const float* scale_factors, const float* level_sigma2,
                                          int check_ori, int32_t* d_match12, int32_t* d_nmatches,
                                          void* stream);
/* SearchByBoW for a batch of frame pairs over the same device FeatureVectors: mode 1 =
 * SearchByBoW(KF1, KF2, vpMatches12) (ORBmatcher.cc:522-655; out[p*kp_stride + idx1] = idx2),
 * mode 0 = SearchByBoW(KF, F, vpMapPointMatches) (:159-288; qf = KF, cf = F,
 * out[p*kp_stride + idxF] = idxKF). mp_flags[f*kp_stride + idx]: bit 0 = the feature has a
 * MapPoint, bit 1 = that MapPoint is bad (the KF side, and in mode 1 both sides, need bit 0
 * without bit 1). Rotation histogram with check_ori. nmatches[p] = entries >= 0. */
int orbm_search_by_bow_batch_device(orbm_ctx* ctx, int npairs, int mode, const int32_t* d_qf,
                                    const int32_t* d_cf, const orbx_kp* d_kps,
                                    const uint8_t* d_desc, const int32_t* d_counts, int kp_stride,
                                    const uint8_t* d_mp_flags, const uint32_t* d_fv_node,
                                    const int32_t* d_fv_off, const int32_t* d_fv_feat,
                                    const int32_t* d_nfv, int max_nodes, float nnratio,
                                    int check_ori, int32_t* d_out, int32_t* d_nmatches,
                                    void* stream);

/* Waits for `stream` and reports (then clears) the ctx's device error flag, raised by the
 * *_device calls that validate device-resident input (orbm_search_for_triangulation_slots_device:
 * a malformed or foreign slot, a query count above its capacity): 0 = OK, ORBX_EDEVICE. */
int orbm_check_error(orbm_ctx* ctx, void* stream);

/* Epipole helper (ORBmatcher.cc:664-670): C2 = R2w*Cw + t2w with OpenCV's small-matrix gemm
 * semantics (float products/sums, + t in double, one rounding; DESIGN.md "Pinned semantics"),
 * ex = fx*C2.x*invz + cx, ey likewise. */
void orbm_epipole(const float R2w[9], const float t2w[3], const float Cw[3], float fx, float fy,
                  float cx, float cy, float* ex, float* ey);

/* ------------------------------------------------------------------------------------
 * SearchByProjection x4 (ORBmatcher.cc:45-129, 1328-1470, 1472-1599, 290-403) with
 * Frame/KeyFrame::GetFeaturesInArea over the 64x48 feature grid (Frame.cc:235-250,
 * 332-389; KeyFrame.cc:569-613). The per-MapPoint geometry prologue of each variant
 * (projection, frustum/scale tests, PredictScale) runs on the host with the reference's
 * float semantics (DESIGN.md "Pinned semantics"); the grid build, windowed Hamming search
 * (best / second best), the in-order claim resolution and the rotation histogram run on the
 * device.
 * ---------------------------------------------------------------------------------- */

/* The Frame (or KeyFrame) side. */
typedef struct orbm_frame_view {
    int32_t n;                    /* N                                                    */
    const uint8_t* desc;          /* mDescriptors, n x 32                                 */
    const float* x;               /* mvKeysUn[i].pt.x                                     */
    const float* y;               /* mvKeysUn[i].pt.y                                     */
    const int32_t* octave;        /* mvKeysUn[i].octave                                   */
    const float* angle;           /* mvKeysUn[i].angle (rotation histogram)               */
    const float* uright;          /* mvuRight; NULL = monocular (all -1)                  */
    const uint8_t* occupied;      /* the variant's "already matched" test on the state
                                     before the call (see each entry point); NULL = none  */
    float min_x, min_y, max_x, max_y;  /* mnMinX, mnMinY, mnMaxX, mnMaxY                  */
    float grid_w_inv, grid_h_inv;      /* mfGridElementWidthInv, mfGridElementHeightInv   */
    float fx, fy, cx, cy;              /* camera                                          */
    float bf, b;                       /* mbf, mb                                         */
    int32_t nlevels;                   /* mnScaleLevels                                   */
    const float* scale_factors;        /* mvScaleFactors[nlevels]                         */
    float log_scale_factor;            /* mfLogScaleFactor                                */
} orbm_frame_view;

/* The MapPoint side (one entry per candidate MapPoint, in the reference's loop order).
 * Each entry point documents which arrays it reads; the rest may be NULL. */
typedef struct orbm_mappoints {
    int32_t n;
    const uint8_t* desc;          /* GetDescriptor(), n x 32                              */
    const float* pos;             /* GetWorldPos(), n x 3                                 */
    const float* normal;          /* GetNormal(), n x 3                                   */
    const float* min_dist;        /* mfMinDistance (GetMinDistanceInvariance = 0.8f*it)   */
    const float* max_dist;        /* mfMaxDistance (GetMaxDistanceInvariance = 1.2f*it)   */
    const uint8_t* bad;           /* isBad()                                              */
    const uint8_t* has_obs;       /* Observations() > 0                                   */
    const uint8_t* skip;          /* entry excluded before any test (see entry points)    */
    const int32_t* octave;        /* source keypoint octave (SearchByProjection(F, LastF)) */
    const float* angle;           /* source keypoint angle (rotation histogram)           */
    /* Tracking fields set by Frame::isInFrustum (Frame.cc:274-330) */
    const uint8_t* track_in_view; /* mbTrackInView                                        */
    const float* track_proj_x;    /* mTrackProjX                                          */
    const float* track_proj_y;    /* mTrackProjY                                          */
    const float* track_proj_xr;   /* mTrackProjXR                                         */
    const int32_t* track_level;   /* mnTrackScaleLevel                                    */
    const float* track_view_cos;  /* mTrackViewCos                                        */
} orbm_mappoints;

/* Results of every variant: match[view.n] = index (into the orbm_mappoints) of the MapPoint
 * the call assigned to that feature (the last assignment wins, as in the reference), -1 if
 * the call left the feature untouched, -2 if the rotation-consistency filter reset it to
 * NULL; *nmatches = the reference's return value. */

/* ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, th) (ORBmatcher.cc:45-129).
 * F.occupied[i] = F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0. Reads mp: desc,
 * bad, has_obs, track_*. nnratio = mfNNratio. */
int orbm_search_by_projection_local(orbm_ctx* ctx, const orbm_frame_view* F, const orbm_mappoints* mp,
                                    float th, float nnratio, int32_t* match, int* nmatches);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 * (ORBmatcher.cc:1328-1470). mp = LastFrame's N entries: skip[i] = !LastFrame.mvpMapPoints[i]
 * || LastFrame.mvbOutlier[i]; pos, desc, has_obs of that MapPoint; octave = LastFrame.mvKeys[i]
 * .octave; angle = LastFrame.mvKeysUn[i].angle. F.occupied as in _local. Tcw_cur / Tcw_last =
 * the frames' mTcw (4x4 row-major float). */
int orbm_search_by_projection_last_frame(orbm_ctx* ctx, const orbm_frame_view* F, const float Tcw_cur[16],
                                         const orbm_mappoints* mp, const float Tcw_last[16], float th, int mono,
                                         int check_ori, int32_t* match, int* nmatches);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>&
 * sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1472-1599). mp = pKF->GetMapPointMatches():
 * skip[i] = NULL entry or in sAlreadyFound; pos, desc, bad, min_dist, max_dist; angle =
 * pKF->mvKeysUn[i].angle. F.occupied[i] = CurrentFrame.mvpMapPoints[i] != NULL. */
int orbm_search_by_projection_keyframe(orbm_ctx* ctx, const orbm_frame_view* F, const float Tcw_cur[16],
                                       const orbm_mappoints* mp, float th, int orb_dist, int check_ori,
                                       int32_t* match, int* nmatches);

/* ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints,
 * vector<MapPoint*>& vpMatched, th) (ORBmatcher.cc:290-403). KF.occupied[i] = vpMatched[i] !=
 * NULL; mp = vpPoints: skip[i] = in spAlreadyFound (the non-NULL entries of vpMatched); pos,
 * normal, desc, bad, min_dist, max_dist. Scw = 4x4 row-major float Sim3. */
int orbm_search_by_projection_sim3(orbm_ctx* ctx, const orbm_frame_view* KF, const float Scw[16],
                                   const orbm_mappoints* mp, int th, int32_t* match, int* nmatches);

/* ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, th) (ORBmatcher.cc:825-975,
 * called by LocalMapping::SearchInNeighbors, LocalMapping.cc:489,514): the per-MapPoint projection,
 * frustum / scale / viewing-angle tests, windowed search with the reprojection-error (chi2) test on
 * the device; best_idx[i] = the keypoint of pKF that MapPoint i fuses with (bestDist <= TH_LOW),
 * -1 otherwise, *nfused = the reference's return value. The caller then applies, for i in order,
 * the reference's update (:947-971: Replace by Observations() or AddObservation + AddMapPoint),
 * re-checking isBad() / IsInKeyFrame(pKF) at that point exactly as the reference loop does (an
 * entry that turns true there was changed by an earlier update and is skipped). mp: skip = NULL
 * entry or IsInKeyFrame(pKF), bad, pos, normal, desc, min_dist, max_dist. KF.occupied is ignored.
 * Tcw = pKF->GetPose() (4x4 row-major), Ow = pKF->GetCameraCenter(), inv_level_sigma2 =
 * pKF->mvInvLevelSigma2[nlevels]. */
int orbm_fuse(orbm_ctx* ctx, const orbm_frame_view* KF, const float Tcw[16], const float Ow[3],
              const orbm_mappoints* mp, float th, const float* inv_level_sigma2, int32_t* best_idx, int* nfused);

/* ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, th, vpReplacePoint)
 * (ORBmatcher.cc:977-1100, LoopClosing::SearchAndFuse): best_idx as in orbm_fuse (no reprojection
 * test); the caller sets vpReplacePoint[i] = pKF->GetMapPoint(best) when that is a good MapPoint,
 * else adds the observation (:1084-1096), in order. mp: skip = in pKF->GetMapPoints() at the call,
 * bad, pos, normal, desc, min_dist, max_dist. Scw = 4x4 row-major float Sim3. */
int orbm_fuse_sim3(orbm_ctx* ctx, const orbm_frame_view* KF, const float Scw[16], const orbm_mappoints* mp,
                   float th, int32_t* best_idx, int* nfused);

/* ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
 * vector<int>& vnMatches12, windowSize) (ORBmatcher.cc:405-520; Tracking::MonocularInitialization,
 * Tracking.cc:600, with ORBmatcher(0.9, true) and windowSize 100). F1: mvKeysUn octave / angle and
 * mDescriptors (n entries; x / y unused); F2: the grid side (F2.GetFeaturesInArea: x, y, octave, grid
 * bounds, angle, desc). prev_xy[2*F1.n] = vbPrevMatched (x, y), updated in place for every matched
 * keypoint; match12[F1.n] = vnMatches12; *nmatches = the reference's return value. Frames of at most
 * 8192 keypoints (ORBX_ECAPACITY above). */
int orbm_search_for_initialization(orbm_ctx* ctx, const orbm_frame_view* F1, const orbm_frame_view* F2,
                                   float* prev_xy, int window_size, float nnratio, int check_ori,
                                   int32_t* match12, int* nmatches);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:1102-1326;
 * LoopClosing::ComputeSim3). KF1 / KF2: the keyframes' grid views (mvKeysUn, descriptors, bounds, grid,
 * camera: both directions project with KF1's fx, fy, cx, cy as the reference does); T1w / T2w = their
 * poses (4x4 row-major). mp1 / mp2 = pKF1 / pKF2->GetMapPointMatches(): skip = NULL entry or
 * vbAlreadyMatched1 / 2 (:1129-1142: vpMatches12[i] != NULL, and that MapPoint's index in pKF2), bad, pos,
 * desc, min_dist, max_dist (mfMinDistance / mfMaxDistance). R12 row-major 3x3, t12[3].
 * match12[mp1.n] = idx2 where both directions agree (vpMatches12[i1] = vpMapPoints2[idx2]; other entries
 * of vpMatches12 are left as they were), else -1; *nfound = the reference's return value. */
int orbm_search_by_sim3(orbm_ctx* ctx, const orbm_frame_view* KF1, const float T1w[16], const orbm_mappoints* mp1,
                        const orbm_frame_view* KF2, const float T2w[16], const orbm_mappoints* mp2, float s12,
                        const float R12[9], const float t12[3], float th, int32_t* match12, int* nfound);

/* ------------------------------------------------------------------------------------
 * Keyframe cache: a KeyFrame's descriptors, mvKeysUn (x, y, angle, octave), mvuRight and
 * FeatureVector never change after KeyFrame::ComputeBoW, but the reference's matchers read them
 * again on every call (LocalMapping::CreateNewMapPoints matches one keyframe against up to 20
 * neighbours, LocalMapping.cc:207-268; SearchInNeighbors fuses into each of them, :454-520). The
 * cache keeps them in HBM across calls and threads (thread-safe, shared by every orbm_ctx of its
 * device), keyed by a caller-chosen 64-bit key (the drop-ins use the KeyFrame's address and mnId).
 * The *_cached matchers equal their uncached forms (same arguments, same results); the views must
 * still be complete: an absent or stale entry (different N, FeatureVector size or grid geometry)
 * is uploaded from them, and the per-call MapPoint flags (has_mp, mp_bad, occupied) are always
 * taken from the view. Least-recently-used entries are evicted above capacity_bytes (0 = 1 GiB).
 * ---------------------------------------------------------------------------------- */
typedef struct orbm_kf_cache orbm_kf_cache;
int orbm_kf_cache_create(int device, size_t capacity_bytes, orbm_kf_cache** out);
void orbm_kf_cache_destroy(orbm_kf_cache* cache);
/* drop a keyframe's entries (e.g. from KeyFrame::SetBadFlag); unknown keys are ignored */
int orbm_kf_cache_erase(orbm_kf_cache* cache, uint64_t key);
int orbm_kf_cache_stats(orbm_kf_cache* cache, int* entries, size_t* bytes, long long* hits, long long* misses);
int orbm_search_for_triangulation_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key1, const orbm_kf_view* kf1,
                                         uint64_t key2, const orbm_kf_view* kf2, const float F12[9], float ex,
                                         float ey, int only_stereo, int check_ori, int32_t* match12, int* nmatches);
int orbm_search_by_bow_kf_kf_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key1, const orbm_kf_view* kf1,
                                    uint64_t key2, const orbm_kf_view* kf2, float nnratio, int check_ori,
                                    int32_t* match12, int* nmatches);
/* the Frame side is not cached (a Frame is matched once) */
int orbm_search_by_bow_kf_f_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key, const orbm_kf_view* kf,
                                   const orbm_kf_view* f, float nnratio, int check_ori, int32_t* match_f,
                                   int* nmatches);
/* the keyframe's arrays and its feature grid (AssignFeaturesToGrid) are cached */
int orbm_fuse_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key, const orbm_frame_view* KF, const float Tcw[16],
                     const float Ow[3], const orbm_mappoints* mp, float th, const float* inv_level_sigma2,
                     int32_t* best_idx, int* nfused);

/* ------------------------------------------------------------------------------------
 * MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307) for a batch of MapPoints.
 * MapPoint p's observed descriptors (the rows pKF->mDescriptors.row(idx) of its non-bad
 * observing KeyFrames, in mObservations order) are desc[offsets[p] .. offsets[p+1]) (32 B
 * each). best_idx[p] = index within that list of the descriptor with the least median
 * Hamming distance to the others (first on ties), -1 if the list is empty (mDescriptor left
 * unchanged); out_desc[p] (optional) = that descriptor.
 * ---------------------------------------------------------------------------------- */
int orbm_compute_distinctive_descriptors(orbm_ctx* ctx, int npoints, const int32_t* offsets,
                                         const uint8_t* desc, int32_t* best_idx, uint8_t* out_desc);
int orbm_compute_distinctive_descriptors_device(orbm_ctx* ctx, int npoints, const int32_t* d_offsets,
                                                const uint8_t* d_desc, int32_t* d_best_idx,
                                                uint8_t* d_out_desc, void* stream);

/* ------------------------------------------------------------------------------------
 * DBoW2 vocabulary transform -- replaces ORBVocabulary::transform(features, BowVector&,
 * FeatureVector&, levelsup) as called by Frame::ComputeBoW (Frame.cc:400-407) and
 * KeyFrame::ComputeBoW (levelsup 4), with the vocabulary loaded by loadFromTextFile
 * (System.cc:64-65). DBoW2 is not vendored in the reference: the ORB-SLAM2 fork's published
 * algorithm is restated (parity unpinned).
 * ---------------------------------------------------------------------------------- */
typedef struct orbv_handle orbv_handle;

/* ORBvoc.txt text format: "k L scoring weighting", then "parent isLeaf d0..d31 weight" per node
 * (node ids = line order, root = 0). */
int orbv_load_text(const char* path, int device, orbv_handle** out);
/* the same from arrays of the node lines (nlines nodes after the root, in file order) */
int orbv_create(int k, int L, int scoring, int weighting, int nlines, const int32_t* parent,
                const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                orbv_handle** out);
void orbv_destroy(orbv_handle* h);
int orbv_info(const orbv_handle* h, int* k, int* L, int* nnodes, int* nwords);

/* n descriptors (32 B rows, n <= 4096) -> BowVector (bow_word ascending, bow_value; *nbow
 * entries) and FeatureVector as CSR (fv_node ascending, fv_off[*nfv+1], fv_feat ascending within
 * a node). Capacities: n entries each, fv_off n+1. */
int orbv_transform(orbv_handle* h, const uint8_t* desc, int n, int levelsup, uint32_t* bow_word,
                   double* bow_value, int* nbow, uint32_t* fv_node, int32_t* fv_off,
                   int32_t* fv_feat, int* nfv);
/* device batch over the frames of an orbx_extract_batch_device output (descriptors at f*kp_stride,
 * d_counts[f]; kp_stride <= 4096): per-feature word id / weight / node id at L-levelsup and per
 * frame the BowVector / FeatureVector (frame f's arrays at f*kp_stride, fv_off at
 * f*(kp_stride+1), counts d_nbow[f], d_nfv[f]). */
int orbv_transform_batch_device(orbv_handle* h, int nframes, const uint8_t* d_desc,
                                const int32_t* d_counts, int kp_stride, int levelsup,
                                int32_t* d_word, double* d_weight, uint32_t* d_nid,
                                uint32_t* d_bow_word, double* d_bow_value, int32_t* d_nbow,
                                uint32_t* d_fv_node, int32_t* d_fv_off, int32_t* d_fv_feat,
                                int32_t* d_nfv, void* stream);

/* ------------------------------------------------------------------------------------
 * Cross-agent keyframe slot -- replaces the LCM message lcmKeyFrame::lcmKeyFrameInfo
 * (ORB_SLAM2.1/include/lcmKeyFrame/lcmKeyFrameInfo.hpp:24-150), published by the sending
 * agent (ORB_SLAM2.1/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:1907-2410) and decoded into
 * receiveKeyframeInfo by the receiving one (ORB_SLAM2/Examples/ROS/ORB_SLAM2/src/
 * ros_mono.cc:88-166, 230-544) for Tracking::CreateNewKeyFrame (:2108-2192). One slot is a
 * fixed-size, self-describing byte block (so an RCCL all-gather of equal-sized slots is the
 * whole transport):
 *   [0, 128)      orbx_slot_header (magic, version, counts, section offsets)
 *   [128, 832)    orbx_kf_meta     (every scalar / matrix field of lcmKeyFrameInfo)
 *   [1024, ...)   sections, each 256-byte aligned, sized by the capacity `cap`:
 *     KPS      cap x orbx_kp        mvKeys (float coordinates; LCM truncated them to int16,
 *                                   lcmKeyPoint.hpp:19-24)
 *     KUN      cap x float[2]       mvKeysUn[i].pt (size/angle/octave equal mvKeys')
 *     URIGHT   cap x float          mvuRight (-1 = monocular)
 *     DEPTH    cap x float          mvDepth
 *     DESC     cap x 32 B           mDescriptors (bytes; LCM sent them as float rows)
 *     MPFLAGS  cap x u8             bit 0: mvpMapPoints[i] != NULL  (lcmKeyFrameMapPoints
 *                                   .ifMapPoints), bit 1: that MapPoint isBad()
 *     MPPOS    cap x float[3]       its world position (poseX/Y/Z)
 *     BOWWORD  cap x u32, BOWVALUE cap x f64   mBowVec (ascending word id), nbow entries
 *     FVNODE   cap x u32, FVOFF (cap+1) x i32, FVFEAT cap x i32   mFeatVec as CSR, nfv nodes
 * Entries past n (nbow, nfv) are zero. All-little-endian, no pointers.
 * ---------------------------------------------------------------------------------- */
#define ORBX_SLOT_MAGIC 0x4B42524Fu /* "ORBK" */
#define ORBX_SLOT_VERSION 2
enum {
    ORBX_SLOT_KPS = 0, ORBX_SLOT_KUN, ORBX_SLOT_URIGHT, ORBX_SLOT_DEPTH, ORBX_SLOT_DESC,
    ORBX_SLOT_MPFLAGS, ORBX_SLOT_MPPOS, ORBX_SLOT_BOWWORD, ORBX_SLOT_BOWVALUE, ORBX_SLOT_FVNODE,
    ORBX_SLOT_FVOFF, ORBX_SLOT_FVFEAT, ORBX_SLOT_NSECTIONS
};
/* header.flags: which optional fields the sender filled (the rest hold their defaults) */
#define ORBX_SLOT_F_KUN 1u     /* mvKeysUn differs from mvKeys (else KUN = mvKeys' pt)   */
#define ORBX_SLOT_F_STEREO 2u  /* mvuRight / mvDepth present (else -1)                   */
#define ORBX_SLOT_F_MP 4u      /* MapPoint records present (else none)                   */
#define ORBX_SLOT_F_BOW 8u     /* BowVector present                                      */
#define ORBX_SLOT_F_FV 16u     /* FeatureVector present                                  */

typedef struct orbx_slot_header {
    uint32_t magic, version;
    int32_t n;        /* N (keypoints)                                                    */
    int32_t cap;      /* capacity the section sizes were computed for                     */
    int32_t nbow;     /* BowVector entries                                                */
    int32_t nfv;      /* FeatureVector nodes                                              */
    uint32_t flags;   /* ORBX_SLOT_F_*                                                    */
    uint32_t bytes;   /* orbx_slot_bytes(cap)                                             */
    uint32_t off[ORBX_SLOT_NSECTIONS]; /* byte offset of each section                    */
    uint32_t reserved[12];
} orbx_slot_header; /* 128 bytes */

/* The scalar and matrix fields of lcmKeyFrameInfo (lcmKeyFrameInfo.hpp:24-100), grouped by
 * type; 4x4 / 3x3 matrices row-major (cv::Mat::at<float>(r,c)). 704 bytes. */
typedef struct orbx_kf_meta {
    int64_t nNextId, mnId, mnFrameId, mnGridCols, mnGridRows, mnTrackReferenceForFrame,
        mnFuseTargetForKF, mnBALocalForKF, mnBAFixedForKF, mnLoopQuery, mnLoopWords, mnRelocQuery,
        mnRelocWords, mnBAGlobalForKF, mnMinX, mnMinY, mnMaxX, mnMaxY;
    double mTimeStamp;
    int32_t agent;          /* sending agent (rank); not in the LCM message              */
    int32_t mnScaleLevels;
    float mfGridElementWidthInv, mfGridElementHeightInv, mLoopScore, mRelocScore;
    float fx, fy, cx, cy, invfx, invfy, mbf, mb, mThDepth;
    float mfScaleFactor, mfLogScaleFactor;
    float mvScaleFactors[16], mvLevelSigma2[16], mvInvLevelSigma2[16];
    float mK[9];
    float mTcw[16], mTcwGBA[16], mTcwBefGBA[16], mTcp[16];
} orbx_kf_meta;

/* One keyframe's per-feature arrays (device memory for the *_device calls, host memory for
 * orbx_pack_keyframe_host). count -> N. Optional arrays may be NULL (see ORBX_SLOT_F_*):
 * kun (n x 2 floats), uright + depth, mp_flags (+ mp_pos n x 3), bow_word + bow_value + nbow,
 * fv_node + fv_off + fv_feat + nfv. */
typedef struct orbx_kf_source {
    const orbx_kp* kps;
    const uint8_t* desc;
    const int32_t* count;
    const float* kun;
    const float* uright;
    const float* depth;
    const uint8_t* mp_flags;
    const float* mp_pos;
    const uint32_t* bow_word;
    const double* bow_value;
    const int32_t* nbow;
    const uint32_t* fv_node;
    const int32_t* fv_off;
    const int32_t* fv_feat;
    const int32_t* nfv;
} orbx_kf_source;

/* Fixed slot size for capacity cap (and the header with the section offsets, hdr optional). */
size_t orbx_slot_bytes(int cap);
int orbx_slot_layout(int cap, orbx_slot_header* hdr);

/* Pack one keyframe (device arrays, e.g. an orbx_extract_batch_device frame + its
 * orbv_transform_batch_device BoW) into d_slot (orbx_slot_bytes(cap) bytes), enqueued on
 * `stream`. Counts above cap are clamped to cap and raise bit 0 of *d_err (optional device int). */
int orbx_pack_keyframe_device(const orbx_kf_source* src, const orbx_kf_meta* meta, int cap,
                              uint8_t* d_slot, int32_t* d_err, void* stream);
/* The same from host arrays into a host slot (byte-identical to the device pack). ORBX_ECAPACITY
 * if a count exceeds cap. */
int orbx_pack_keyframe_host(const orbx_kf_source* src, const orbx_kf_meta* meta, int cap,
                            uint8_t* slot, size_t slot_bytes);

/* A validated view of a received slot in host memory: magic/version, cap vs slot_bytes, every
 * section offset, n/nbow/nfv <= cap, the FeatureVector CSR (offsets monotone, node ids and word
 * ids strictly ascending, feature indices < n and ascending within a node). ORBX_EARG if any
 * check fails. Pointers alias `slot`. */
typedef struct orbx_slot_view {
    const orbx_slot_header* hdr;
    const orbx_kf_meta* meta;
    const orbx_kp* kps;
    const float* kun;
    const float* uright;
    const float* depth;
    const uint8_t* desc;
    const uint8_t* mp_flags;
    const float* mp_pos;
    const uint32_t* bow_word;
    const double* bow_value;
    const uint32_t* fv_node;
    const int32_t* fv_off;
    const int32_t* fv_feat;
} orbx_slot_view;
int orbx_slot_parse(const uint8_t* slot, size_t slot_bytes, orbx_slot_view* out);

/* Geometry of one (query keyframe, slot keyframe) pair: F12 (LocalMapping::ComputeF12,
 * LocalMapping.cc:536-553) and the epipole (ex, ey) of the query's centre in the slot's
 * keyframe (ORBmatcher.cc:664-670). */
typedef struct orbm_slot_geom {
    float F12[9];
    float ex, ey;
} orbm_slot_geom;

/* Cross-agent ORBmatcher::SearchForTriangulation(query KF, slot KF, F12, vMatchedPairs,
 * bOnlyStereo = false) (ORBmatcher.cc:657-823) of this agent's keyframe (`query`, device
 * arrays: kps/desc/count, optional kun, uright, mp_flags and, with use_bow, its FeatureVector)
 * against nref received slots at d_slots + r*slot_bytes (e.g. the all-gather receive buffer),
 * straight from device memory. Per slot: geom[r] (host array), the slot keyframe's
 * mvScaleFactors / mvLevelSigma2 from its meta, its mvKeysUn / mvuRight / MapPoint flags.
 * use_bow = 0: one node holding every feature (brute force, the BASELINE configuration);
 * use_bow = 1: the common nodes of the two FeatureVectors (query nodes <= max_nodes).
 * Outputs d_match[r*cap1 + idx1] (idx2 or -1), d_nmatches[r]. A slot that fails validation
 * (magic, version, size, counts, CSR bounds) contributes no matches and raises the ctx's
 * device error flag (orbm_check_error). */
int orbm_search_for_triangulation_slots_device(orbm_ctx* ctx, const orbx_kf_source* query, int cap1,
                                               int nref, const uint8_t* d_slots, size_t slot_bytes,
                                               const orbm_slot_geom* geom, int use_bow, int max_nodes,
                                               int32_t* d_match, int32_t* d_nmatches, void* stream);

/* Cross-agent ORBmatcher::SearchByBoW(query KF, slot KF, vpMatches12) (ORBmatcher.cc:522-655):
 * the loop-candidate match the receiving agent runs on a received keyframe (it goes to
 * LoopClosing::InsertKeyFrame, ORB_SLAM2/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:3530, and
 * LoopClosing::ComputeSim3 calls SearchByBoW(mpCurrentKF, pKF) with ORBmatcher(0.75, true),
 * LoopClosing.cc:239, 265), of this agent's keyframe (`query`, device arrays: kps/desc/count,
 * mp_flags (bit 0 a MapPoint, bit 1 bad; NULL = none) and its FeatureVector) against nref
 * received slots at d_slots + r*slot_bytes, straight from device memory, over the common nodes
 * of the two FeatureVectors (query nodes <= max_nodes). Outputs d_match[r*cap1 + idx1] = the
 * slot keyframe's feature idx2 whose MapPoint vpMatches12[idx1] is (or -1), after the
 * rotation filter when check_ori, and d_nmatches[r]. A slot that fails validation contributes
 * no matches and raises the ctx's device error flag (orbm_check_error). Slots may carry a
 * larger capacity than the query (agents with other feature counts): a common node is matched
 * whole up to 4551 candidates (one CU's LDS); a node past that raises the error flag. */
int orbm_search_by_bow_slots_device(orbm_ctx* ctx, const orbx_kf_source* query, int cap1, int nref,
                                    const uint8_t* d_slots, size_t slot_bytes, float nnratio, int check_ori,
                                    int max_nodes, int32_t* d_match, int32_t* d_nmatches, void* stream);

/* ------------------------------------------------------------------------------------
 * Cross-agent collective -- replaces the LCM keyframe publish / subscribe between the agents
 * (ORB_SLAM2.1/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:2399, ORB_SLAM2/Examples/ROS/ORB_SLAM2/
 * src/ros_mono.cc:602): one RCCL all-gather over xGMI of every agent's keyframe slot
 * (orbx_pack_keyframe_device), enqueued on the caller's stream (no collective-owned stream), one
 * process = one agent = one GPU. RCCL is bound at run time (the process's librccl.so.1 if one
 * is loaded, else ROCm's); ORBX_EDEVICE without it.
 * ---------------------------------------------------------------------------------- */
#define ORBX_COMM_ID_BYTES 128
typedef struct orbx_comm orbx_comm;
/* rank 0 creates the id (ncclGetUniqueId); the caller hands it to every rank (any transport) */
int orbx_comm_unique_id(uint8_t* id);
/* collective over the world: every rank calls it with the same id, its rank and its device */
int orbx_comm_create(const uint8_t* id, int world, int rank, int device, orbx_comm** out);
/* d_recv[r*bytes .. (r+1)*bytes) = rank r's d_send[0 .. bytes), on `stream` (ncclAllGather, uint8) */
int orbx_comm_allgather(orbx_comm* c, const void* d_send, void* d_recv, size_t bytes, void* stream);
void orbx_comm_destroy(orbx_comm* c);

/* ------------------------------------------------------------------------------------
 * Stereo -- replaces Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641, the
 * stereo Frame constructor's step after ExtractORB(0/1), Frame.cc:80-98), reading the two
 * extractors' pyramids (mpORBextractorLeft/Right->mvImagePyramid) where they already live.
 * mvScaleFactors / mvInvScaleFactors come from `left`; both handles must have the same
 * frame size and ORB parameters. bf = mbf, b = mb (Frame.cc:501-503).
 * ---------------------------------------------------------------------------------- */

/* Host form: kpsL/descL (mvKeys, mDescriptors) and kpsR/descR (mvKeysRight,
 * mDescriptorsRight) are the outputs of the latest orbx_extract on `left` and `right`
 * (two distinct handles, like the two ORBextractor instances). Writes mvuRight and
 * mvDepth (nL floats, -1 = no stereo match) and the number of stereo matches kept.
 * ORBX_EARG where the reference would throw (an 11x11 correlation window outside the level:
 * cv::Mat::rowRange/colRange assert). */
int orbx_compute_stereo_matches(orbx_handle* left, orbx_handle* right, const orbx_kp* kpsL,
                                const uint8_t* descL, int nL, const orbx_kp* kpsR,
                                const uint8_t* descR, int nR, float bf, float b, float* uright,
                                float* depth, int* nstereo);

/* Device batch form: pair p = frame d_fl[p] of the latest orbx_extract_batch_device on
 * `left` with frame d_fr[p] of the latest one on `right` (left == right allowed, e.g. a
 * batch holding left and right images). Keypoints/descriptors/counts as produced by those
 * extractions (frame f at f*kp_stride). Outputs: d_uright/d_depth[p*kp_stride + i],
 * d_nstereo[p]. A window outside the level sets the device error flag (orbx_check_error on
 * `left`). Enqueued on `stream` after both extractions (the caller orders the streams). */
int orbx_stereo_matches_batch_device(orbx_handle* left, orbx_handle* right, int npairs,
                                     const int32_t* d_fl, const int32_t* d_fr,
                                     const orbx_kp* d_kpsL, const uint8_t* d_descL,
                                     const int32_t* d_cntL, const orbx_kp* d_kpsR,
                                     const uint8_t* d_descR, const int32_t* d_cntR, int kp_stride,
                                     float bf, float b, float* d_uright, float* d_depth,
                                     int32_t* d_nstereo, void* stream);

/* ------------------------------------------------------------------------------------
 * Synthetic input: deterministic frame t of agent a, width x height,
 * written to host out (pitch = width). Identical on every machine (integer-only).
 * ---------------------------------------------------------------------------------- */
int orbx_synth_frame(int agent, int t, int width, int height, uint8_t* out);
/* frames t0 .. t0+count-1 of agent a, back to back (frame stride width*height). */
int orbx_synth_frames(int agent, int t0, int count, int width, int height, uint8_t* out);
/* right image of a rectified stereo rig for the same frames: the crop shifted by +dx pixels
 * in x (0 <= dx <= 26), i.e. a fronto-parallel scene at disparity dx. */
int orbx_synth_frames_shifted(int agent, int t0, int count, int width, int height, int dx,
                              uint8_t* out);
/* shared-scene frames: view `view` (an agent) of the texture of `scene`, its crop 12*view pixels
 * further along the pan (mod 600), so several agents see overlapping parts of one environment as
 * A1 and A2 do; view 0 equals orbx_synth_frames_shifted(scene, ...). */
int orbx_synth_scene_frames(int scene, int view, int t0, int count, int width, int height, int dx,
                            uint8_t* out);

/* Stage profiling: a pair of HIP events brackets each stage's kernel on the stream it is
 * launched on (the overlapped schedule is kept, so a stage's time includes sharing the GPU
 * with the stage that runs beside it): stages = {pyramid, fast_cells, octree, blur, describe}.
 * orbx_profile_enable(h, mask) resets the accumulators and brackets the stages in `mask`
 * (bit k = stage k, 0x1F = all, 0 = off); orbx_profile_read waits for the recorded events and
 * returns the summed milliseconds per stage (ms[5], 0 for stages not in the mask) and the
 * number of profiled extraction calls. */
int orbx_profile_enable(orbx_handle* h, int on);
int orbx_profile_read(orbx_handle* h, double* ms, int* ncalls);

/* Schedule hook: every subsequent batched extraction of this handle records `event` (a hipEvent_t
 * created by the caller; NULL = off) on its stream right after the pyramid launch, so another stream
 * can start its own work once this batch's pyramid is done (bench schedules that stagger concurrent
 * extraction graphs by pyramid rather than by whole extraction). */
int orbx_set_pyramid_event(orbx_handle* h, void* event);
/* The same for any of the first two stages: stage 0 = after the pyramid launch (orbx_set_pyramid_event), 1 = after
 * the FAST launch; one event per stage, NULL = off. The bench staggers its graphs by FAST: graph p starts a step
 * once graph p-1's FAST is done, a third of the step apart at 3 graphs. */
int orbx_set_stage_event(orbx_handle* h, int stage, void* event);

/* Library/version and device probe. */
const char* orbx_version(void);
int orbx_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* ORBSLAM_AMD_H */
