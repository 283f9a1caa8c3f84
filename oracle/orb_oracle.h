/*
 * orb_oracle.h -- CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (liborbamd.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" at the OpenCV boundary. The reference
 * (ORB_SLAM2/src/ORBextractor.cc, ORBmatcher.cc) cannot be built here without writing
 * stand-ins for OpenCV/DBoW2 headers (forbidden), and it ships no tests or golden
 * vectors. Everything ORB-SLAM2 authored is restated literally with file:line
 * citations; the OpenCV 3.x primitives it calls (resize INTER_LINEAR, FAST-9/16 + NMS,
 * GaussianBlur 7x7 sigma 2, fastAtan2, cvRound) are restated from OpenCV 3.3's published
 * algorithm (DESIGN.md "Pinned semantics"). glibc cosf/sinf are called
 * directly (as the reference does). Pinned by: constant tables derived from the reference
 * source (tests/test_oracle_tables.py) and committed regression vectors (tests/golden/).
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/orbslam_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oc_extractor oc_extractor;

oc_extractor* oc_create(const orbx_params* p);
void oc_destroy(oc_extractor* e);
/* ORBextractor::operator() (ORBextractor.cc:1043-1105). Returns 0, or ORBX_ECAPACITY. */
int oc_extract(oc_extractor* e, const uint8_t* img, int w, int h, size_t pitch, orbx_kp* kps,
               uint8_t* desc, int cap, int* n);

/* accumulated per-stage wall time over all oc_extract calls of this extractor (seconds):
 * pyramid, FAST, octree, orientation, blur, descriptor; for bench.py's CPU breakdown */
void oc_stage_times(const oc_extractor* e, double* sec6, int* nframes);

/* stage access for stage-isolated parity tests (valid after oc_extract) */
int oc_level_size(const oc_extractor* e, int level, int* w, int* h);
const uint8_t* oc_pyramid(const oc_extractor* e, int level);
const uint8_t* oc_blurred(const oc_extractor* e, int level); /* NULL if level had no kps */
/* vToDistributeKeys of a level (ORBextractor.cc:778-829): xyr triplets (x, y relative to
 * minBorder, response). Returns the count (copies min(count, cap)). */
int oc_level_candidates(const oc_extractor* e, int level, float* xyr, int cap);
/* DistributeOctTree output of a level before orientation, level coordinates (+minBorder),
 * xyr triplets. Returns the count. */
int oc_level_octree(const oc_extractor* e, int level, float* xyr, int cap);

/* constructor tables (ORBextractor.cc:410-470) */
void oc_get_tables(const oc_extractor* e, float* scale, float* inv_scale, float* sigma2,
                   float* inv_sigma2, int32_t* nfeat_per_level, int32_t* umax16);

/* primitives, exposed for unit tests */
float oc_fast_atan2(float y, float x);
int oc_gauss_kernel_q8(int32_t* k7); /* fixed-point 7-tap kernel (sum returned) */
void oc_resize_linear(const uint8_t* src, int sw, int sh, size_t sstep, uint8_t* dst, int dw,
                      int dh, size_t dstep);
void oc_gauss7(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst, size_t dstep);
/* cv::FAST(img, kps, th, true) on a w x h view: xyr triplets, returns count */
int oc_fast(const uint8_t* img, int w, int h, size_t step, int threshold, float* xyr, int cap);
/* 1 (default): cv::FAST's vector form (AVX2, 32 pixels per step) where built; 0: scalar per pixel.
 * Same output either way. */
void oc_set_fast_simd(int on);

void oc_sincosf_batch(const float* in, float* s, float* c, int n);

/* matcher (ORBmatcher.cc) -- host views */
int oc_descriptor_distance(const uint8_t* a, const uint8_t* b);
int oc_search_for_triangulation(const orbm_kf_view* kf1, const orbm_kf_view* kf2,
                                const float F12[9], float ex, float ey, int only_stereo,
                                int check_ori, int32_t* match12);
int oc_search_by_bow_kf_f(const orbm_kf_view* kf, const orbm_kf_view* f, float nnratio,
                          int check_ori, int32_t* match_f);
int oc_search_by_bow_kf_kf(const orbm_kf_view* kf1, const orbm_kf_view* kf2, float nnratio,
                           int check_ori, int32_t* match12);

/* Frame-level consumers (orb_oracle_frame.c) */
int oc_compute_stereo_matches(const oc_extractor* left, const oc_extractor* right, const orbx_kp* kpsL,
                              const uint8_t* descL, int N, const orbx_kp* kpsR, const uint8_t* descR, int Nr,
                              float mbf, float mb, float* uright, float* depth);
int oc_search_by_projection_local(const orbm_frame_view* F, const orbm_mappoints* mp, float th, float nnratio,
                                  int32_t* match);
int oc_search_by_projection_last_frame(const orbm_frame_view* F, const float* Tcw_c, const orbm_mappoints* mp,
                                       const float* Tcw_l, float th, int bMono, int checkOri, int32_t* match);
int oc_search_by_projection_keyframe(const orbm_frame_view* F, const float* Tcw_c, const orbm_mappoints* mp, float th,
                                     int ORBdist, int checkOri, int32_t* match);
void oc_compute_distinctive_descriptors(int npoints, const int32_t* offsets, const uint8_t* desc,
                                        int32_t* best_idx);
int oc_search_by_projection_sim3(const orbm_frame_view* KF, const float* Scw, const orbm_mappoints* mp, int th,
                                 int32_t* match);
/* ORBmatcher::Fuse x2 (ORBmatcher.cc:825-975, 977-1100): per-MapPoint best_idx (-1 = no fuse) */
int oc_fuse(const orbm_frame_view* KF, const float* Tcw, const float* Ow, const orbm_mappoints* mp, float th,
            const float* inv_sigma2, int32_t* best_idx);
int oc_fuse_sim3(const orbm_frame_view* KF, const float* Scw, const orbm_mappoints* mp, float th, int32_t* best_idx);

/* ORBmatcher::SearchForInitialization (ORBmatcher.cc:405-520); prev_xy updated in place */
int oc_search_for_initialization(const orbm_frame_view* F1, const orbm_frame_view* F2, float* prev_xy, int windowSize,
                                 float nnratio, int checkOri, int32_t* match12);
/* ORBmatcher::SearchBySim3 (ORBmatcher.cc:1102-1326): match12[mp1->n] = agreeing idx2 or -1 */
int oc_search_by_sim3(const orbm_frame_view* KF1, const float* T1w, const orbm_mappoints* mp1,
                      const orbm_frame_view* KF2, const float* T2w, const orbm_mappoints* mp2, float s12,
                      const float* R12, const float* t12, float th, int32_t* match12);

/* DBoW2 vocabulary transform (orb_oracle_voc.c; parity unpinned: DBoW2 is not vendored) */
typedef struct oc_vocab oc_vocab;
oc_vocab* oc_vocab_create(int k, int L, int scoring, int weighting, int nlines, const int32_t* parent,
                          const uint8_t* is_leaf, const uint8_t* desc, const double* weight);
void oc_vocab_destroy(oc_vocab* v);
int oc_vocab_transform(const oc_vocab* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_word,
                       double* bow_value, int* nbow, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat, int* nfv);
void oc_vocab_descend(const oc_vocab* v, const uint8_t* desc, int n, int levelsup, int32_t* word, double* weight,
                      int32_t* nid);

#ifdef __cplusplus
}
#endif
#endif
