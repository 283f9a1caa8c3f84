/*
 * orb_device.h -- geometry tables shared by the host launcher (capi.cpp) and the gfx950
 * kernels. Everything that depends only on (W, H, ORB params) -- pyramid sizes, resize
 * coefficients, the FAST cell grid, octree root split -- is computed ONCE on the host with
 * the reference's exact float semantics and uploaded; kernels do integer work on it.
 *
 * HBM layout per frame f of a batch (all offsets in bytes / elements):
 *   input   : caller's frames, level 0 read in place (frame_stride, pitch)
 *   pyr     : levels 1..L-1 at pyr + f*pyr_frame_bytes + lv.pyr_off, row pitch lv.pitch
 *   blur    : levels 0..L-1 at blur + f*blur_frame_bytes + lv.blur_off, row pitch lv.pitch
 *   cellkey : per FAST cell a fixed slot of `cap` u32 keys: cellkey + f*keys_per_frame +
 *             cell.slot; key = x_rel | y_rel << 12 | score << 24 (coords relative to the
 *             16-px border, ORBextractor.cc:822-823)
 *   cellcnt : cellcnt + f*ncells + c
 *   lvkey   : octree output per level, u32 key (level coords), lvkey + f*kp_per_frame +
 *             lv.kp_off, count lvcnt + f*L + l
 */
#pragma once
#include <stdint.h>

namespace orbamd {

constexpr int kMaxLevels = 16;
constexpr int kEdgeThreshold = 19;  // ORBextractor.cc:74
constexpr int kPatchSize = 31;      // ORBextractor.cc:72
constexpr int kHalfPatch = 15;      // ORBextractor.cc:73
constexpr int kRoiMax = 72;         // max FAST cell ROI side (cells are < 60+6 px)
constexpr int kRoiPitch = 72;
constexpr int kBlurRows = 63;  // blur strip chunk height: 9 x 7 (the 7-row window loop has no partial step)
static_assert(kBlurRows % 7 == 0, "blur chunk height must be a multiple of 7");
constexpr int kBlurRowsSmall = 14;  // small batches (run_extract_levels): short chunks, 4.5x the waves of one frame
static_assert(kBlurRowsSmall % 7 == 0, "blur chunk height must be a multiple of 7");
constexpr int kPyrMaxRows = 2048;   // k_pyramid_frames: LDS row table capacity (levels >= 1)
#ifndef ORBX_PYR_U
#define ORBX_PYR_U 6
#endif
// k_pyramid_frames: rows in flight per thread (round 5, with the v_mul_hi vertical pass: 6 beats 2/4/5/7/8 by
// 0.3-2.5 % at the bench step, pyramid alone -10 % against 4; profiles/r05_ab_pyr_rows.log)
constexpr int kPyrU = ORBX_PYR_U;
#ifndef ORBX_PYR_UMAX
#define ORBX_PYR_UMAX 4
#endif
// the same for the kPyrThreadsMax workgroups (wide levels: C4's 1241-column frames; row bands): 4, not 6, holds
// them at 59 VGPRs (C4 199.3-199.9k against 191-193k at 6, profiles/r05_ab_pyr_rows_c4.log)
constexpr int kPyrUMax = ORBX_PYR_UMAX;
// k_pyramid_frames: threads per frame's workgroup. kPyrThreads is used when every level's 4-column
// group count fits half of it (>= 2 rows per pass); wider levels take kPyrThreadsMax, the limit the
// whole-frame kernel accepts (>= column groups of every level)
#ifndef ORBX_PYR_THREADS
#define ORBX_PYR_THREADS 512
#endif
constexpr int kPyrThreads = ORBX_PYR_THREADS;  // 384-704 measured at 6 rows in flight: 512 best (profiles/r05_ab_pyr_threads.log)  // (1024 at the round-5 step: -4.5 %, profiles/r05_ab_pyr1024.log)
constexpr int kPyrThreadsMax = 1024;
constexpr int kPyrFramesMinBatch = 64;  // batches below this build the pyramid in row bands (below)
// small batches: k_pyramid_frames over kPyrBands row bands per frame, each band's workgroup computing every level's
// rows its band owns plus the rows its higher levels read (the band's dependency cone; overlapping rows are
// written by two workgroups with the same bytes): one launch instead of a dependent launch per level
constexpr int kPyrBands = 32;  // (batches in 2-8 bands measured slower in the overlapped schedule: whole frames)
constexpr int kRsTileW = 64, kRsTileH = 32;  // k_resize_tiled output tile

struct LevelDesc {
    int w, h, pitch;
    int pad0;
    long long pyr_off;   // byte offset inside a frame's pyramid area (levels >= 1)
    long long blur_off;  // byte offset inside a frame's blurred area
    int cell_begin, ncells;
    int N;               // mnFeaturesPerLevel[l]
    int nIni;            // DistributeOctTree root count
    float hX;            // root width (float, ORBextractor.cc:545)
    int minX, maxX, minY, maxY;  // octree bounds (ORBextractor.cc:773-776)
    int key_begin, key_cap;      // this level's cell-key range inside a frame
    int kp_off, kp_cap;          // octree output slots inside a frame
    int node_cap;                // max live octree nodes: max(N+3, 4*nIni)
    float scale;                 // mvScaleFactor[l]
    float patch_size;            // (float)(int)(31*scale)
    int blur_vec_end;            // w & ~3 (SSE2 column-filter span)
    int xmax, simd_end;          // resize: first column with sx+1>=sw; VResize SSE2 span
    int coef_off;                // offset of this level's resize tables
    int cg_off, rt_off;          // k_pyramid_frames tables (ints into ptab): column groups, rows
};

struct CellDesc {
    int level;
    int x0, y0;  // ROI origin in level coordinates
    int w, h;    // ROI size (before clipping to the band)
    int xoff, yoff;  // j*wCell, i*hCell (ORBextractor.cc:822-823)
    int slot;        // key slot offset inside a frame
    int cap;         // slot capacity
    // k_fast_cells2 lane schedules (wave-uniform divisions done on the host):
    // staging: D = dwords per ROI row, rpp = 64 / D rows per pass; pretest: G = dword groups per
    // band row, rpc = 64 / G rows per chunk; lane / n == (lane * mag_n) >> 16 (exact for lane < 64)
    int D, rpp, magD;
    int G, rpc, magG;
};

struct ExtractParams {
    int L;
    int ncells;
    int keys_per_frame;
    int kp_per_frame;
    int ini_th, min_th;
    long long pyr_frame_bytes;
    long long blur_frame_bytes;
    int umax[16];
    unsigned long long umax_packed;  // umax[v] in bits 4v..4v+3 (all values <= 15)
    int kp_off[kMaxLevels + 1];      // level l's octree output slots start (kp_off[L] = kp_per_frame)
    int bjob_begin[kMaxLevels + 1];  // blur strip jobs prefix
    int ic_off;                      // IC_Angle mask table (int2 pairs) inside the ptab buffer
    int host_out;                    // describe writes into mapped host memory: system-scope fence after the writes
};

/* extra workgroups of a launch that copy n16 16-byte words src -> dst (mapped pinned host memory): the host path's
 * delivery of mvImagePyramid (orbx_set_host_pyramid), carried by the one-frame octree launch */
struct HostCopy {
    const uint4* src;
    uint4* dst;
    long long n16;
    int nblocks;
    uint4* const* dst_ref;  // if set: the destination is read from this (host-mapped) word when the copy runs
};

/* level containing index g of a per-level prefix table (no dependent loads: unrolled compares
 * against kernel-argument values) */
__host__ __device__ inline int level_of(const int* begin, int L, int g) {
    int l = 0;
#pragma unroll
    for (int k = 1; k < kMaxLevels; k++) l += (k < L && g >= begin[k]) ? 1 : 0;
    return l;
}

}  // namespace orbamd
