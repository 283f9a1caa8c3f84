/* launch.h -- host launchers of the gfx950 kernels (defined next to the kernels). */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbslam_amd.h"
#include "orb_device.h"
#include "orb_frame.h"
#include "orb_match.h"
#include "orb_slot.h"

namespace orbamd {

hipError_t launch_resize(const uint8_t* src, long long src_fstride, int src_pitch, int sw, int sh, uint8_t* dst,
                         long long dst_fstride, int dst_pitch, int dw, int dh, const int* coef, int xmax,
                         int simd_end, int nframes, hipStream_t st);
hipError_t launch_pyramid_frames(const uint8_t* frames, long long fstride, int pitch0, uint8_t* pyr,
                                 const ExtractParams& ep, const LevelDesc* levels, const int* ptab, int max_rows,
                                 int max_groups, int nframes, hipStream_t st,
                                 const int2* bands = nullptr, int nbands = 0);
hipError_t launch_resize_tiled(const uint8_t* src, long long src_fstride, int src_pitch, int sw, int sh, uint8_t* dst,
                               long long dst_fstride, int dst_pitch, int dw, int dh, const int* coef, int xmax,
                               int simd_end, int nframes, hipStream_t st);
int resize_tile_fits(const int* xofs, const int* yofs, int sw, int sh, int dw, int dh);
hipError_t launch_fast_cells2(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                              const ExtractParams& ep, const LevelDesc* levels, const CellDesc* cells,
                              uint32_t* cellkey, int* cellcnt, int RP, int RH, int max_pass, int cell_lo,
                              int cell_hi, int nframes, hipStream_t st);
hipError_t octree_setup(int lds_bytes);
hipError_t launch_sincos_selftest(const float* in, float* so, float* co, int n, hipStream_t st);
hipError_t launch_octree(const ExtractParams& ep, const LevelDesc* levels, const CellDesc* cells,
                         const uint32_t* cellkey, const int* cellcnt, uint32_t* lvkey, int* lvcnt,
                         uint8_t* gscratch, long long gscratch_frame_bytes, int NC, int KL, int lds_bytes,
                         int* err, int nframes, hipStream_t st, int level0 = 0, int nlevels = -1,
                         const HostCopy* copy = nullptr);
/* blur jobs [job0, job1) (ExtractParams::bjob_begin numbers every level's strips) */
/* FAST over every cell + the blur in kBlurRowsSmall-row chunks (job table eb) in one launch (small batches) */
hipError_t launch_fast_blur(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                            const ExtractParams& ep, const LevelDesc* levels, const CellDesc* cells, uint32_t* cellkey,
                            int* cellcnt, int RP, int RH, int max_pass, uint8_t* blur, const ExtractParams& eb,
                            int njobs, int nframes, hipStream_t st);
hipError_t launch_blur_strips(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr, uint8_t* blur,
                              const ExtractParams& ep, const LevelDesc* levels, int job0, int job1, const int* lvcnt,
                              int nframes, hipStream_t st, int rows = kBlurRows);
hipError_t launch_describe(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                           const uint8_t* blur, const ExtractParams& ep, const LevelDesc* levels,
                           const uint32_t* lvkey, const int* lvcnt, orbx_kp* out_kps, uint8_t* out_desc,
                           int* out_counts, int kp_stride, const int* ptab, int nframes, hipStream_t st);
/* the blur folded into describe (k_describe_blur): level-0 rows must be 4-aligned (describe_blur_ok) */
bool describe_blur_ok(const uint8_t* frames, long long fstride, int pitch0);
hipError_t launch_describe_blur(const uint8_t* frames, long long fstride, int pitch0, const uint8_t* pyr,
                                const ExtractParams& ep, const LevelDesc* levels, const uint32_t* lvkey,
                                const int* lvcnt, orbx_kp* out_kps, uint8_t* out_desc, int* out_counts, int kp_stride,
                                const int* ptab, int nframes, hipStream_t st);

/* uright: mvuRight of every frame (uright[f * kp_stride + i], -1 = monocular; nullptr = all monocular) */
hipError_t launch_tri_bf(int npairs, const int32_t* q1, const int32_t* q2, const orbx_kp* kps, const uint8_t* desc,
                         const int32_t* counts, int kp_stride, const MatchGeom& g, int32_t* match12,
                         int32_t* nmatches, hipStream_t st, const float* uright = nullptr, int only_stereo = 0);
hipError_t launch_tri_nodes_pairs(int npairs, int max_nodes, const int32_t* q1, const int32_t* q2, const orbx_kp* kps,
                                  const uint8_t* desc, int kp_stride, const uint32_t* fv_node, const int32_t* fv_off,
                                  const int32_t* fv_feat, const int32_t* nfv, const MatchGeom& g, int32_t* match12,
                                  int32_t* nmatches, hipStream_t st);
hipError_t launch_rot_filter_pairs(int npairs, const int32_t* q1, const int32_t* q2, const orbx_kp* kps,
                                   const int32_t* counts, int kp_stride, int32_t* match12, int32_t* nmatches,
                                   hipStream_t st, int swap = 0);
hipError_t launch_bow_pairs(int npairs, int max_nodes, const int32_t* qf, const int32_t* cf, const uint8_t* desc,
                            int kp_stride, const uint8_t* mp_flags, const uint32_t* fv_node, const int32_t* fv_off,
                            const int32_t* fv_feat, const int32_t* nfv, float nnratio, int mode, int32_t* out,
                            hipStream_t st);
hipError_t launch_count_pairs(int npairs, const int32_t* out, int kp_stride, int32_t* nmatches, hipStream_t st);
hipError_t launch_tri_nodes(const DevView& v1, const DevView& v2, const NodeTask* tasks, int ntasks,
                            const MatchGeom& g, int only_stereo, const CallTail& tail, hipStream_t st);
hipError_t launch_bow(const DevView& vq, const DevView& vc, const NodeTask* tasks, int ntasks, int max_nc,
                      float nnratio, int mode, const CallTail& tail, hipStream_t st);
hipError_t launch_bow_small(const BowSmall& a, hipStream_t st);
int proj_topk();  // candidate keys per query of k_proj_scan (ProjCall::scan holds proj_topk() x nq keys)
hipError_t launch_tri_small(const TriSmall& a, hipStream_t st);
hipError_t launch_rot_filter(int n, int32_t* m, const float* angA, const float* angB, int swap, int32_t* nout,
                             hipStream_t st);

hipError_t launch_flag_take(int32_t* flag, int32_t* out, hipStream_t st);
hipError_t launch_call_done(int32_t* flag, int32_t* out_err, int32_t* seq, int32_t* out_done, hipStream_t st);
hipError_t launch_pack_slot(const orbx_kf_source& src, const SlotLayout& L, const orbx_kf_meta& meta, uint8_t* slot,
                            int32_t* err, hipStream_t st);
hipError_t launch_bow_slots(const QueryKF& q, const uint8_t* slots, long long slot_bytes, int nref, float nnratio,
                            int check_ori, int max_nodes, int32_t* match, int32_t* nmatches, int32_t* err,
                            hipStream_t st);
hipError_t launch_tri_slots(const QueryKF& q, const uint8_t* slots, long long slot_bytes, int nref,
                            const orbm_slot_geom* geom, int use_bow, int max_nodes, int32_t* match,
                            int32_t* nmatches, int32_t* err, hipStream_t st);

hipError_t launch_projection(const ProjCall* d_calls, int ncalls, int max_nq, hipStream_t st, bool resolve = true,
                             bool init = false, bool grid = true);
int init_max_features();
hipError_t launch_distinctive(int npoints, const int32_t* off, const uint8_t* desc, int32_t* best_idx,
                              uint8_t* out_desc, hipStream_t st);
int stereo_lds_bytes(int cap, int nrows);
hipError_t stereo_setup(int lds_bytes);
hipError_t launch_stereo(const StereoArgs& a, int npairs, const int32_t* fl, const int32_t* fr, const orbx_kp* kpsL,
                         const uint8_t* descL, const int32_t* cntL, const orbx_kp* kpsR, const uint8_t* descR,
                         const int32_t* cntR, int stride, float* uright, float* depth, int32_t* nstereo, int32_t* sad,
                         int* err, hipStream_t st);  // sad: npairs * stride ints of scratch (k_stereo -> k_stereo_median)

}  // namespace orbamd
