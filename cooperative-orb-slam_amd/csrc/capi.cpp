/*
 * capi.cpp -- host side of the C ABI (include/orbslam_amd.h).
 *
 * Owns the per-handle device state, builds the geometry tables once per frame size with
 * the reference's exact float semantics (ORBextractor.cc:410-470, 765-787, 1107-1112 and
 * OpenCV 3.x resize coefficients), and sequences the gfx950 kernels on a HIP stream.
 * There is no CPU fallback: every compute entry point fails with ORBX_EDEVICE when the
 * device path is unavailable.
 */
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/orbslam_amd.h"
#include "orbslam_amd_testing.h"
#include "launch.h"
#include "orb_device.h"
#include "kf_cache.h"
#include "orb_match.h"

using namespace orbamd;

/* A failing HIP call is reported once, through the entry point's status (ORBX_EDEVICE), and then cleared from the
 * calling thread's HIP error state: hipGetLastError returns the last error of ANY runtime call on the thread, so a
 * failure left there would be raised again by the caller's next launch check, far from its cause (round 5's first GPU
 * run: hipEventElapsedTime over a never-recorded stage event pair in orbx_profile_read, whose status bench.py did not
 * read, surfaced as "HIP error: invalid resource handle" in torch's dist.barrier; tests/test_gpu_cache.py
 * ::test_library_hip_failure_does_not_leak pins this). */
#define HIPR(expr)                                                                    \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess) {                                                       \
            if (getenv("ORBX_DEBUG")) fprintf(stderr, "HIP error %s at %s:%d\n",     \
                                              hipGetErrorString(e_), __FILE__, __LINE__); \
            (void)hipGetLastError();                                                  \
            return ORBX_EDEVICE;                                                      \
        }                                                                             \
    } while (0)

namespace {

int cv_round_f(float v) { return (int)lrintf(v); }
int cv_floor_f(float v) { int i = (int)v; return i - (i > v); }
int cv_ceil_f(float v) { int i = (int)v; return i + (i < v); }
short sat_short(float v) {
    int i = cv_round_f(v);
    return (short)std::min(32767, std::max(-32768, i));
}
long long align_up(long long v, long long a) { return (v + a - 1) / a * a; }

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t need) {
        if (need <= bytes) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, need) != hipSuccess) { p = nullptr; return ORBX_EDEVICE; }
        bytes = need;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return (T*)p; }
};

/* ORBextractor constructor tables (ORBextractor.cc:410-470) */
struct Tables {
    int nfeatures, nlevels, ini_th, min_th;
    double scaleFactor;  // double member (ORBextractor.h:100)
    float scale[kMaxLevels], inv_scale[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
    int nfeat[kMaxLevels];
    int umax[16];
    void build(const orbx_params& p) {
        nfeatures = p.nfeatures;
        nlevels = p.nlevels;
        ini_th = p.ini_th_fast;
        min_th = p.min_th_fast;
        scaleFactor = p.scale_factor;
        scale[0] = 1.0f;
        sigma2[0] = 1.0f;
        for (int i = 1; i < nlevels; i++) {
            scale[i] = (float)(scale[i - 1] * scaleFactor);
            sigma2[i] = scale[i] * scale[i];
        }
        for (int i = 0; i < nlevels; i++) {
            inv_scale[i] = 1.0f / scale[i];
            inv_sigma2[i] = 1.0f / sigma2[i];
        }
        float factor = (float)(1.0f / scaleFactor);
        float nDesired = nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
        int sum = 0;
        for (int l = 0; l < nlevels - 1; l++) {
            nfeat[l] = cv_round_f(nDesired);
            sum += nfeat[l];
            nDesired *= factor;
        }
        nfeat[nlevels - 1] = std::max(nfeatures - sum, 0);
        int v, v0, vmax = cv_floor_f(kHalfPatch * sqrtf(2.f) / 2 + 1);
        int vmin = cv_ceil_f(kHalfPatch * sqrtf(2.f) / 2);
        const double hp2 = kHalfPatch * kHalfPatch;
        for (v = 0; v <= vmax; ++v) umax[v] = (int)lrint(sqrt(hp2 - v * v));
        for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }
};

/* Everything that depends on (W, H): host copies + device copies */
struct Geometry {
    /* k_pyramid_frames tables for one level (see PyrColGroup in extract_kernels.hip): per 4-column
     * group the 8-byte source window W and per output a v_perm selector + tap weights; per row
     * (r0, r1, beta). Returns false if some group's taps do not fit an 8-byte window. */
    bool build_pyr_tables(LevelDesc& d, const int* xofs, const short* alpha, const int* yofs, const short* beta,
                          int xmax, int sw, int sh, int dw, int dh) {
        bool ok = dh <= kPyrMaxRows && (dw + 3) / 4 <= kPyrThreadsMax && sw >= 12;
        const int AU = (int)align_up(sw, 4);
        const int gw = (dw + 3) / 4;
        d.cg_off = (int)ptab.size();
        for (int gi = 0; gi < gw; gi++) {
            int e[12] = {0};
            const int W = std::min(xofs[4 * gi], AU - 8);
            for (int i = 0; i < 4; i++) {
                const int x = std::min(4 * gi + i, dw - 1);
                const int o = xofs[x] - W;
                const bool two = x < xmax;  // second tap has a non-zero weight
                if (o < 0 || o > 7 || (two && o + 1 > 7)) ok = false;
                const int o1 = std::min(o + 1, 7);
                e[i] = (o & 7) | (0x0c << 8) | (o1 << 16) | (0x0c << 24);
                const short a0 = two ? alpha[2 * x] : (short)2048, a1 = two ? alpha[2 * x + 1] : (short)0;
                e[4 + i] = (int)(((uint32_t)(uint16_t)a1 << 16) | (uint16_t)a0);
            }
            e[8] = W;
            e[9] = AU - 4;  // last dword of the row (clamp of the window's third dword)
            ptab.insert(ptab.end(), e, e + 12);
        }
        d.rt_off = (int)ptab.size();
        for (int y = 0; y < dh; y++) {
            const int r0 = std::min(std::max(yofs[y], 0), sh - 1), r1 = std::min(std::max(yofs[y] + 1, 0), sh - 1);
            const int b = (int)(((uint32_t)(uint16_t)beta[2 * y + 1] << 16) | (uint16_t)beta[2 * y]);
            const int e[4] = {r0, r1, b, 0};
            ptab.insert(ptab.end(), e, e + 4);
        }
        return ok;
    }

    int W = 0, H = 0;
    ExtractParams ep{};
    std::vector<LevelDesc> lv;
    std::vector<CellDesc> cells;
    std::vector<int> coef;
    std::vector<int> bjob_begin;  // blur strip jobs (256 cols x kBlurRows rows) per level
    int nbjobs = 0;
    int bjob_small[kMaxLevels + 1] = {0};  // the same in kBlurRowsSmall-row chunks (run_extract_levels)
    int nbjobs_small = 0;
    int NC = 0, KL = 0, lds_bytes = 0;
    int oct_split = 0;                      // batches: levels [0, oct_split) use NC/KL, [oct_split, L) NC_lo/KL_lo
    int NC_lo = 0, KL_lo = 0, lds_lo = 0;
    int roi_pitch = 0, roi_rows = 0;  // FAST cell LDS staging (max cell ROI)
    int max_pass = 1;                 // ROI staging passes (rows per 64-lane dword pass)
    int tiled_ok[kMaxLevels] = {0};   // level's resize fits the LDS-tiled kernel
    std::vector<int> ptab;            // k_pyramid_frames column-group / row tables
    bool frames_ok = true;            // every level fits k_pyramid_frames
    int band_off = 0;                 // ptab offset of the small-batch row bands ([kPyrBands][kMaxLevels] int2)
    int pyr_rows = 1;                 // tallest level >= 1 (k_pyramid_frames' LDS row table rows)
    DevBuf d_lv, d_cells, d_coef, d_ptab;

    int build(const Tables& T, int W_, int H_) {
        W = W_;
        H = H_;
        const int L = T.nlevels;
        lv.assign(L, LevelDesc{});
        cells.clear();
        coef.clear();
        ptab.clear();
        frames_ok = true;
        long long pyr_off = 0, blur_off = 0;
        int key_begin = 0, kp_off = 0;
        int maxnode = 0;
        for (int l = 0; l < L; l++) {
            LevelDesc& d = lv[l];
            // ComputePyramid (ORBextractor.cc:1111-1112)
            d.w = cv_round_f((float)W * T.inv_scale[l]);
            d.h = cv_round_f((float)H * T.inv_scale[l]);
            if (d.w < 62 || d.h < 62 || d.w > 4096 || d.h > 4096) return ORBX_EARG;
            d.pitch = (int)align_up(d.w, 64);
            d.pyr_off = l == 0 ? 0 : pyr_off;
            if (l > 0) pyr_off += align_up((long long)d.pitch * d.h, 256);
            d.blur_off = blur_off;
            blur_off += align_up((long long)d.pitch * d.h, 256);
            d.scale = T.scale[l];
            d.patch_size = (float)(int)(kPatchSize * T.scale[l]);
            d.blur_vec_end = d.w & ~3;
            // resize tables from level l-1 (OpenCV resize(), INTER_LINEAR, 8U)
            if (l > 0) {
                const int sw = lv[l - 1].w, sh = lv[l - 1].h, dw = d.w, dh = d.h;
                d.coef_off = (int)coef.size();
                coef.resize(coef.size() + 2 * dw + 2 * dh);
                int* xofs = coef.data() + d.coef_off;
                short* alpha = (short*)(xofs + dw);
                int* yofs = xofs + 2 * dw;
                short* beta = (short*)(yofs + dh);
                const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
                int xmax = dw;
                for (int dx = 0; dx < dw; dx++) {
                    float fx = (float)((dx + 0.5) * scale_x - 0.5);
                    int sx = cv_floor_f(fx);
                    fx -= sx;
                    if (sx < 0) { fx = 0; sx = 0; }
                    if (sx + 1 >= sw) {
                        xmax = std::min(xmax, dx);
                        if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
                    }
                    xofs[dx] = sx;
                    alpha[2 * dx] = sat_short((1.f - fx) * 2048);
                    alpha[2 * dx + 1] = sat_short(fx * 2048);
                }
                for (int dy = 0; dy < dh; dy++) {
                    float fy = (float)((dy + 0.5) * scale_y - 0.5);
                    int sy = cv_floor_f(fy);
                    fy -= sy;
                    yofs[dy] = sy;
                    beta[2 * dy] = sat_short((1.f - fy) * 2048);
                    beta[2 * dy + 1] = sat_short(fy * 2048);
                }
                int se = 0;
                while (se <= dw - 16) se += 16;
                while (se < dw - 4) se += 4;
                d.xmax = xmax;
                d.simd_end = se;
                tiled_ok[l] = resize_tile_fits(xofs, yofs, sw, sh, dw, dh);
                frames_ok = frames_ok && build_pyr_tables(d, xofs, alpha, yofs, beta, xmax, sw, sh, dw, dh);
                // OpenCV switches INTER_LINEAR to INTER_AREA for exact 2x downscales; unsupported
                if (std::abs(scale_x - 2.0) < 1e-15 && std::abs(scale_y - 2.0) < 1e-15) return ORBX_EARG;
            }
            // FAST cell grid (ORBextractor.cc:769-806)
            const float Wc = 30;
            const int minBorderX = kEdgeThreshold - 3, minBorderY = minBorderX;
            const int maxBorderX = d.w - kEdgeThreshold + 3, maxBorderY = d.h - kEdgeThreshold + 3;
            const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
            const int nCols = (int)(width / Wc), nRows = (int)(height / Wc);
            if (nCols <= 0 || nRows <= 0) return ORBX_EARG;
            const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
            d.cell_begin = (int)cells.size();
            d.key_begin = key_begin;
            int kc = 0;
            for (int i = 0; i < nRows; i++) {
                const float iniY = (float)(minBorderY + i * hCell);
                float maxY = iniY + hCell + 6;
                if (iniY >= maxBorderY - 3) continue;
                if (maxY > maxBorderY) maxY = (float)maxBorderY;
                for (int j = 0; j < nCols; j++) {
                    const float iniX = (float)(minBorderX + j * wCell);
                    float maxX = iniX + wCell + 6;
                    if (iniX >= maxBorderX - 6) continue;
                    if (maxX > maxBorderX) maxX = (float)maxBorderX;
                    CellDesc c;
                    c.level = l;
                    c.x0 = (int)iniX;
                    c.y0 = (int)iniY;
                    c.w = (int)maxX - c.x0;
                    c.h = (int)maxY - c.y0;
                    if (c.w > kRoiMax || c.h > kRoiMax) return ORBX_EARG;
                    c.xoff = j * wCell;
                    c.yoff = i * hCell;
                    const int bw = std::max(c.w - 6, 0), bh = std::max(c.h - 6, 0);
                    c.cap = ((bw + 1) / 2) * ((bh + 1) / 2);
                    c.slot = key_begin + kc;
                    kc += c.cap;
                    c.D = (c.w + 3) / 4;
                    c.rpp = 64 / c.D;
                    c.magD = (65536 + c.D - 1) / c.D;
                    c.G = (bw + 6) / 4;
                    c.rpc = c.G > 0 ? 64 / c.G : 1;
                    c.magG = c.G > 0 ? (65536 + c.G - 1) / c.G : 0;
                    for (int ln = 0; ln < 64; ln++)  // the magic divisions are exact (checked)
                        if ((ln * c.magD) >> 16 != ln / c.D || (c.G > 0 && (ln * c.magG) >> 16 != ln / c.G))
                            return ORBX_EARG;
                    cells.push_back(c);
                }
            }
            d.ncells = (int)cells.size() - d.cell_begin;
            d.key_cap = kc;
            key_begin += (int)align_up(kc, 64);
            // DistributeOctTree roots (ORBextractor.cc:542-545)
            d.minX = minBorderX;
            d.maxX = maxBorderX;
            d.minY = minBorderY;
            d.maxY = maxBorderY;
            d.nIni = (int)roundf((float)(maxBorderX - minBorderX) / (maxBorderY - minBorderY));
            if (d.nIni <= 0) return ORBX_EARG;
            d.hX = (float)(maxBorderX - minBorderX) / d.nIni;
            d.N = T.nfeat[l];
            d.node_cap = std::max(d.N + 3, 4 * d.nIni);
            d.kp_off = kp_off;
            d.kp_cap = d.node_cap;
            kp_off += d.kp_cap;
            maxnode = std::max(maxnode, d.node_cap);
        }
        roi_pitch = 4;
        roi_rows = 1;
        max_pass = 1;
        for (const CellDesc& c : cells) {
            roi_pitch = std::max(roi_pitch, (int)align_up(c.w, 4));
            roi_rows = std::max(roi_rows, c.h);
            const int D = (c.w + 3) / 4, rpp = 64 / D;
            max_pass = std::max(max_pass, (c.h + rpp - 1) / rpp);
        }
        if (max_pass > 24) return ORBX_EARG;
        ep.L = L;
        ep.ncells = (int)cells.size();
        ep.keys_per_frame = key_begin;
        ep.kp_per_frame = kp_off;
        ep.ini_th = T.ini_th;
        ep.min_th = T.min_th;
        ep.pyr_frame_bytes = align_up(pyr_off, 256);
        ep.blur_frame_bytes = align_up(blur_off, 256);
        ep.umax_packed = 0;
        for (int v = 0; v < 16; v++) {
            ep.umax[v] = T.umax[v];
            ep.umax_packed |= (unsigned long long)(T.umax[v] & 15) << (4 * v);
        }
        // IC_Angle lane masks (k_describe): row ri = v + 15 (0..31), column group g (u = -15+4g+i):
        // {packed (u+15) inside the circular patch, packed 1 inside} (ORBextractor.cc:77-104)
        ep.ic_off = (int)ptab.size();
        for (int ri = 0; ri < 32; ri++) {
            const int v = ri - 15, av = v < 0 ? -v : v;
            for (int gq = 0; gq < 8; gq++) {
                uint32_t uw = 0, m1 = 0;
                for (int i = 0; i < 4; i++) {
                    const int u = -15 + 4 * gq + i, au = u < 0 ? -u : u;
                    if (av <= 15 && au <= 15 && au <= T.umax[av]) {
                        uw |= (uint32_t)(u + 15) << (8 * i);
                        m1 |= 1u << (8 * i);
                    }
                }
                ptab.push_back((int)uw);
                ptab.push_back((int)m1);
            }
        }
        bjob_begin.assign(L + 1, 0);
        for (int l = 0; l < L; l++)
            bjob_begin[l + 1] = bjob_begin[l] + ((lv[l].w + 255) / 256) * ((lv[l].h + kBlurRows - 1) / kBlurRows);
        nbjobs = bjob_begin[L];
        int bs = 0;  // the same jobs in kBlurRowsSmall-row chunks (small batches)
        for (int l = 0; l <= kMaxLevels; l++) {
            ep.kp_off[l] = l < L ? lv[l].kp_off : kp_off;
            ep.bjob_begin[l] = l <= L ? bjob_begin[l] : nbjobs;
            bjob_small[l] = bs;
            if (l < L) bs += ((lv[l].w + 255) / 256) * ((lv[l].h + kBlurRowsSmall - 1) / kBlurRowsSmall);
        }
        nbjobs_small = bjob_small[L];
        pyr_rows = 1;
        for (int l = 1; l < L; l++) pyr_rows = std::max(pyr_rows, lv[l].h);
        // row bands of the banded pyramid: band b of B owns rows [b h / B, (b + 1) h / B) of every level and also
        // makes the rows its own higher levels read (the (r0, r1) of k_pyramid_frames' row table), so each
        // workgroup only reads back rows it wrote itself
        auto band_table = [&](int B) {
            const int off = (int)ptab.size();
            std::vector<int> bt(2 * B * kMaxLevels, 0);
            for (int b = 0; b < B; b++) {
                int nlo = 0, nhi = 0;  // rows of level l that level l + 1's range reads ([nlo, nhi), empty at the top)
                for (int l = L - 1; l >= 1; l--) {
                    const int h = lv[l].h;
                    int lo = (int)((long long)b * h / B), hi = (int)((long long)(b + 1) * h / B);
                    if (nhi > nlo) {
                        lo = hi > lo ? std::min(lo, nlo) : nlo;
                        hi = std::max(hi, nhi);
                    }
                    bt[2 * (b * kMaxLevels + l)] = lo;
                    bt[2 * (b * kMaxLevels + l) + 1] = hi;
                    nlo = nhi = 0;
                    if (hi > lo && l > 1) {  // this range's source rows in level l - 1
                        const int* rt = &ptab[lv[l].rt_off];
                        nlo = rt[4 * lo];
                        nhi = rt[4 * (hi - 1) + 1] + 1;
                    }
                }
            }
            ptab.insert(ptab.end(), bt.begin(), bt.end());
            return off;
        };
        band_off = frames_ok ? band_table(kPyrBands) : 0;
        // octree LDS: node arrays (92 B/node, NC pow2) + keys (7 B/key)
        NC = 1;
        while (NC < maxnode) NC <<= 1;
        const int node_bytes = 76 * NC;
        // keys of a level stay in LDS up to KL, larger levels use global scratch. KL is sized so a workgroup
        // fits 32 KB when that still leaves >= 1024 keys (five octree workgroups per CU beside the other
        // graphs' kernels; 1888 keys at NC = 256 cover a 640x480 / 1000-feature level 0), else up to 2048.
        if (node_bytes + 7 * 256 > 160 * 1024) return ORBX_EARG;
        auto key_lds = [](int nc, int* kl, int* lds) {
            const int nb = 76 * nc;
            const int kl32 = ((32 * 1024 - nb - 64) / 7) & ~15;
            *kl = kl32 >= 1024 ? std::min(2048, kl32) : std::min(2048, ((160 * 1024 - nb) / 7) & ~15);
            *lds = nb + 7 * *kl;
        };
        key_lds(NC, &KL, &lds_bytes);
        // batches: the levels whose node tables fit 256 entries (all but level 0 of a 1200- or 2000-feature
        // extractor) take their own launch with 256-node tables and 256-thread workgroups, instead of every level
        // carrying the largest level's 512-node tables and 53 KB of LDS (C3 / C4: 2.4 ms per 1024-frame launch)
        oct_split = L;
        while (oct_split > 0 && lv[oct_split - 1].node_cap <= 256) oct_split--;
        NC_lo = NC;
        KL_lo = KL;
        lds_lo = lds_bytes;
        if (oct_split > 0 && oct_split < L) {
            int mx = 0;
            for (int l = oct_split; l < L; l++) mx = std::max(mx, lv[l].node_cap);
            NC_lo = 1;
            while (NC_lo < mx) NC_lo <<= 1;
            key_lds(NC_lo, &KL_lo, &lds_lo);
        } else {
            oct_split = 0;  // one launch: every level fits the same tables
        }
        // upload
        if (d_lv.ensure(sizeof(LevelDesc) * L) || d_cells.ensure(sizeof(CellDesc) * cells.size()) ||
            d_coef.ensure(sizeof(int) * std::max<size_t>(coef.size(), 1)) ||
            d_ptab.ensure(sizeof(int) * std::max<size_t>(ptab.size(), 4)))
            return ORBX_EDEVICE;
        HIPR(hipMemcpy(d_lv.p, lv.data(), sizeof(LevelDesc) * L, hipMemcpyHostToDevice));
        HIPR(hipMemcpy(d_cells.p, cells.data(), sizeof(CellDesc) * cells.size(), hipMemcpyHostToDevice));
        if (!coef.empty()) HIPR(hipMemcpy(d_coef.p, coef.data(), sizeof(int) * coef.size(), hipMemcpyHostToDevice));
        if (!ptab.empty()) HIPR(hipMemcpy(d_ptab.p, ptab.data(), sizeof(int) * ptab.size(), hipMemcpyHostToDevice));
        return 0;
    }
    void release() { d_lv.release(); d_cells.release(); d_coef.release(); d_ptab.release(); }
};

}  // namespace

struct orbx_handle {
    orbx_params params;
    Tables T;
    int device = 0;
    int max_w = 0, max_h = 0, max_batch = 1;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;  // branches of the extraction graph (run_extract)
    hipEvent_t ev_pyr = nullptr, ev_blur = nullptr;
    hipEvent_t user_ev_pyr = nullptr;   // orbx_set_stage_event(0) / orbx_set_pyramid_event (caller-owned)
    hipEvent_t user_ev_fast = nullptr;  // orbx_set_stage_event(1) (caller-owned)
    Geometry geo;
    DevBuf pyr, blur, cellkey, cellcnt, lvkey, lvcnt, gscratch, err;
    // host-path staging
    DevBuf in_frame, out_kps, out_desc, out_cnt;
    // orbx_compute_stereo_matches staging (host path) and k_stereo's LDS attribute
    DevBuf st_buf;
    DevBuf stereo_sad;  // orbx_stereo_matches_batch_device: each left keypoint's SAD for the median pass
    int stereo_lds_set = 0;
    // last extraction, for orbx_pyramid_level
    const uint8_t* last_frames = nullptr;
    long long last_fstride = 0;
    int last_pitch = 0, last_nframes = 0;
    hipStream_t last_stream = nullptr;  // stream of the last run_extract
    bool lds_attr_set = false;
    // host path as one captured hipGraph (orbx_extract): pinned staging in / out, replayed per frame
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    int graph_w = 0, graph_h = 0;
    unsigned graph_epoch = 0;   // geometry / buffer epoch the graph was captured at
    unsigned epoch = 1;         // bumped whenever ensure_geometry rebuilds or reallocates
    int graph_warm = 0;         // eager runs at the current epoch (the first one runs uncaptured)
    uint8_t* pin_in = nullptr;  // W*H frame
    uint8_t* pin_out = nullptr; // {cnt, err} + K orbx_kp + K x 32 descriptors
    uint8_t* pin_out_dev = nullptr;  // its device-mapped address: the graph's kernels write the results there
    size_t pin_in_bytes = 0, pin_out_bytes = 0;
    // orbx_set_host_pyramid: the host path also delivers levels 1..L-1 (device layout of one frame) into pin_pyr
    bool host_pyr = false;
    bool host_pyr_valid = false;  // pin_in / pin_pyr hold the last orbx_extract's levels
    uint8_t* pin_pyr = nullptr;
    uint8_t* pin_pyr_dev = nullptr;
    size_t pin_pyr_bytes = 0;
    // orbx_set_host_pyramid_target: caller-owned registered memory receiving the next calls' levels (level 0 at 0,
    // levels 1..L-1 from host_l0_bytes in the device layout) instead of pin_in / pin_pyr; last_target = the one the
    // last call filled (what orbx_host_pyramid_level points into)
    uint8_t* target = nullptr;
    uint8_t* target_dev = nullptr;
    size_t target_bytes = 0;
    uint8_t* last_target = nullptr;
    // stage profiling (orbx_profile_*)
    bool prof_on = false;
    int prof_mask = 0;  // stages with event pairs (bit k = stage k)
    std::vector<hipEvent_t> prof_ev;  // per profiled call: 5 stages x {start, end}
    int prof_calls = 0;
    double prof_ms[5] = {0, 0, 0, 0, 0};
    int skip_mask = 0;  // orbx_debug_skip_stages (test hook)
    bool serial = false;  // orbx_debug_serial (measurement hook): every stage in order on the caller's stream
    bool alias = false;   // orbx_debug_alias_frames (measurement hook): every frame of a batch is frame 0
};

static const int kProfMaxCalls = 4096;
static const int kHostCopyBlocks = 16;  // octree-launch workgroups (1024 threads) copying the host path's pyramid
// pin_out byte offset of the host copy's destination pointer: the captured graph's copy workgroups read it at run time,
// so a call can deliver its levels into another buffer (orbx_set_host_pyramid_target) without a new capture
static const int kPinOutCopyDst = 48;

/* bytes of a host pyramid target: level 0 (w x h, contiguous) rounded up to 256, then levels 1..L-1 as on the device */
static size_t host_l0_bytes(const orbx_handle* h) { return align_up((size_t)h->geo.W * h->geo.H, 256); }

/* stage k = {pyramid, fast_cells, octree, blur, describe}; e = 0 start / 1 end, recorded on the
 * stream the stage's kernel is launched on (the overlapped schedule is kept) */
static int prof_mark(orbx_handle* h, int k, int e, hipStream_t st) {
    if (!h->prof_on || !((h->prof_mask >> k) & 1)) return 0;
    if (h->prof_calls >= kProfMaxCalls) return 0;
    const size_t need = (size_t)(h->prof_calls + 1) * 10;
    while (h->prof_ev.size() < need) {
        hipEvent_t ev;
        HIPR(hipEventCreate(&ev));
        h->prof_ev.push_back(ev);
    }
    HIPR(hipEventRecord(h->prof_ev[(size_t)h->prof_calls * 10 + 2 * k + e], st));
    return 0;
}

static int ensure_geometry(orbx_handle* h, int W, int H, int nframes) {
    if (nframes < 1 || nframes > h->max_batch) return ORBX_EARG;
    if (h->geo.W != W || h->geo.H != H) {
        h->epoch++;
        int rc = h->geo.build(h->T, W, H);
        if (rc) { h->geo.W = h->geo.H = 0; return rc; }
    }
    const ExtractParams& ep = h->geo.ep;
    const size_t B = (size_t)h->max_batch;
    const void* before[7] = {h->pyr.p, h->blur.p, h->cellkey.p, h->cellcnt.p, h->lvkey.p, h->lvcnt.p, h->gscratch.p};
    const void* err_before = h->err.p;
    // the blurred pyramid is only for frames the fused describe cannot take (unaligned level-0 rows): allocated at the
    // first such call (ensure_blur), and kept sized here once it exists
    if (h->pyr.ensure(B * ep.pyr_frame_bytes) || (h->blur.p && h->blur.ensure(B * ep.blur_frame_bytes)) ||
        h->cellkey.ensure(B * ep.keys_per_frame * 4) || h->cellcnt.ensure(B * ep.ncells * 4) ||
        h->lvkey.ensure(B * ep.kp_per_frame * 4) || h->lvcnt.ensure((B * ep.L + kMaxLevels) * 4) ||
        h->gscratch.ensure(B * (size_t)ep.keys_per_frame * 8) || h->err.ensure(256))
        return ORBX_EDEVICE;
    if (h->err.p != err_before && hipMemset(h->err.p, 0, 256) != hipSuccess) return ORBX_EDEVICE;  // sticky flag starts clear
    const void* after[7] = {h->pyr.p, h->blur.p, h->cellkey.p, h->cellcnt.p, h->lvkey.p, h->lvcnt.p, h->gscratch.p};
    if (memcmp(before, after, sizeof(before))) h->epoch++;
    if (h->geo.lds_bytes > 64 * 1024 && !h->lds_attr_set) {
        HIPR(octree_setup(h->geo.lds_bytes));
        h->lds_attr_set = true;
    }
    return 0;
}

/* the separate blur's buffer (k_blur_strips / k_fast_blur + k_describe), allocated at the first extraction of frames whose
 * level-0 rows are not 4-byte aligned: every aligned frame blurs inside describe's LDS, so most handles never hold the
 * ~1 MB per 640x480 frame of max_batch (3 GB at the bench's 3 x 1024 frames). A host-call graph captured before holds no
 * blur launch, so a reallocation only bumps the epoch like any other buffer change. */
static int ensure_blur(orbx_handle* h) {
    const void* before = h->blur.p;
    if (h->blur.ensure((size_t)h->max_batch * h->geo.ep.blur_frame_bytes)) return ORBX_EDEVICE;
    if (h->blur.p != before) h->epoch++;
    return 0;
}

static int launch_pyramid(orbx_handle* h, const ExtractParams& ep, const uint8_t* d_frames, long long fstride,
                          int pitch, int nframes, hipStream_t st) {
    Geometry& g = h->geo;
    // pyramid levels 1..L-1 (ORBextractor.cc:1107-1132) of 4-byte-aligned frames: whole-frame workgroups for
    // large batches, row-band workgroups (kPyrBands per frame) for small ones; per-level kernels otherwise
    const bool aligned = ((uintptr_t)d_frames & 3) == 0 && (fstride & 3) == 0 && (pitch & 3) == 0;
    if (g.frames_ok && aligned && ep.L > 1) {
        int max_groups = 1;
        for (int l = 1; l < ep.L; l++) max_groups = std::max(max_groups, (g.lv[l].w + 3) / 4);
        const bool banded = nframes < kPyrFramesMinBatch;
        HIPR(launch_pyramid_frames(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), ep, g.d_lv.as<LevelDesc>(),
                                   g.d_ptab.as<int>(), g.pyr_rows, max_groups, nframes, st,
                                   banded ? (const int2*)(g.d_ptab.as<int>() + g.band_off) : nullptr,
                                   banded ? kPyrBands : 0));
        return 0;
    }
    for (int l = 1; l < ep.L; l++) {
        const LevelDesc& s = g.lv[l - 1];
        const LevelDesc& d = g.lv[l];
        const uint8_t* src = l == 1 ? d_frames : h->pyr.as<uint8_t>() + s.pyr_off;
        const long long sfs = l == 1 ? fstride : ep.pyr_frame_bytes;
        const int sp = l == 1 ? pitch : s.pitch;
        if (g.tiled_ok[l])
            HIPR(launch_resize_tiled(src, sfs, sp, s.w, s.h, h->pyr.as<uint8_t>() + d.pyr_off, ep.pyr_frame_bytes,
                                     d.pitch, d.w, d.h, g.d_coef.as<int>() + d.coef_off, d.xmax, d.simd_end, nframes,
                                     st));
        else
            HIPR(launch_resize(src, sfs, sp, s.w, s.h, h->pyr.as<uint8_t>() + d.pyr_off, ep.pyr_frame_bytes, d.pitch,
                               d.w, d.h, g.d_coef.as<int>() + d.coef_off, d.xmax, d.simd_end, nframes, st));
    }
    return 0;
}

static int launch_fast(orbx_handle* h, const ExtractParams& ep, const uint8_t* d_frames, long long fstride, int pitch,
                       int cell_lo, int cell_hi, int nframes, hipStream_t st) {
    Geometry& g = h->geo;
    HIPR(launch_fast_cells2(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), ep, g.d_lv.as<LevelDesc>(),
                            g.d_cells.as<CellDesc>(), h->cellkey.as<uint32_t>(), h->cellcnt.as<int>(), g.roi_pitch,
                            g.roi_rows, g.max_pass, cell_lo, cell_hi, nframes, st));
    return 0;
}

/* ORBextractor::operator() for a batch. Dependencies between the stages:
 *
 *   st   (caller): pyramid(1..L-1) -> [ev_pyr] FAST(all cells) -> octree -> [ev_blur] describe
 *   side         :                   [ev_pyr] blur(all levels) ---------> [ev_blur]
 *
 * The blur needs only the pyramid, so it runs beside FAST and the octree (whose workgroups are
 * barrier/latency-bound); describe joins both. (The reference blurs only levels that kept
 * keypoints (ORBextractor.cc:1081); blurring every level changes no output, since describe
 * reads only levels with keypoints.) h->serial (orbx_debug_serial, a measurement hook) runs every
 * stage in order on `st`, so each kernel runs alone. */
/* Error words of h->err: kErrSticky (word 0) collects the device batch paths' flags until orbx_check_error
 * takes them (kErrTake, word 32, receives the atomic read-and-clear); kErrExtract (word 2) is the host-buffer
 * extraction's per-call flag, read and cleared by the call's last launch (k_flag_take), so it is clean for the
 * next call; kErrCall (word 1) is the stereo host call's (zeroed and read by that call). A host call never
 * erases an unread batch error. */
constexpr int kErrWordSticky = 0, kErrWordCall = 1, kErrWordExtract = 2, kErrWordTake = 32, kErrWordExtractTake = 33;
constexpr int kErrWordExtractSeq = 40;  // the host extraction's call counter (k_call_done's done word)
/* Small batches (the Tracking thread's one frame per call, ORBextractor.cc:1043-1105): every stage in order on the
 * caller's queue -- the pyramid in kPyrBands row bands per frame (one launch); FAST over every cell; the octree over
 * every level; the blur inside describe (k_describe_blur). Unaligned frames run FAST and the blur in 14-row chunks
 * (4.5x the waves of the batch form's 63-row chunks: one frame's blur is one chunk's row chain) in one launch
 * (k_fast_blur), then describe. A single queue because the graph executor turns every edge between queues into a
 * marker behind all the work already submitted to the source queue (~10 us per hop in the kernel trace, and a
 * side branch started only once its marker came up), and streams share the process's 4 hardware queues; every
 * branch layout measured slower than the one queue (profiles/r04_latency_branches.log, r04_latency_lists.log,
 * r04m_latency_ab.log), and so did a single launch for levels 2.. whose tiles wait on each other's counters
 * (r04_latency_chain_reverted.log). */
/* the blur inside describe (k_describe_blur, no blurred pyramid in HBM) takes every frame whose level-0 rows are
 * 4-byte aligned; other frames blur each level in k_blur_strips and describe from it */
static bool use_describe_blur(const uint8_t* d_frames, long long fstride, int pitch) {
    return describe_blur_ok(d_frames, fstride, pitch);
}

static int run_extract_levels(orbx_handle* h, const ExtractParams& ep, int nframes, const uint8_t* d_frames,
                              long long fstride, int pitch, orbx_kp* d_kps, uint8_t* d_desc, int32_t* d_counts,
                              int kp_stride, hipStream_t st, int* errp, hipEvent_t ev_pyr, hipEvent_t ev_fast,
                              const HostCopy* copy) {
    Geometry& g = h->geo;
    const LevelDesc* dl = g.d_lv.as<LevelDesc>();
    if (!(h->skip_mask & 1) && launch_pyramid(h, ep, d_frames, fstride, pitch, nframes, st)) return ORBX_EDEVICE;
    if (ev_pyr) HIPR(hipEventRecord(ev_pyr, st));  // orbx_set_pyramid_event: right after the pyramid launch
    if (use_describe_blur(d_frames, fstride, pitch)) {  // FAST -> octree -> blur + describe
        if (!(h->skip_mask & 2) && launch_fast(h, ep, d_frames, fstride, pitch, 0, ep.ncells, nframes, st))
            return ORBX_EDEVICE;
        if (ev_fast) HIPR(hipEventRecord(ev_fast, st));
        if (!(h->skip_mask & 4))
            HIPR(launch_octree(ep, dl, g.d_cells.as<CellDesc>(), h->cellkey.as<uint32_t>(), h->cellcnt.as<int>(),
                               h->lvkey.as<uint32_t>(), h->lvcnt.as<int>(), h->gscratch.as<uint8_t>(),
                               (long long)ep.keys_per_frame * 8, g.NC, g.KL, g.lds_bytes, errp, nframes, st, 0, -1,
                               copy));
        if (!(h->skip_mask & 16))
            HIPR(launch_describe_blur(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), ep, dl, h->lvkey.as<uint32_t>(),
                                      h->lvcnt.as<int>(), d_kps, d_desc, d_counts, kp_stride, g.d_ptab.as<int>(),
                                      nframes, st));
        return 0;
    }
    if (ensure_blur(h)) return ORBX_EDEVICE;
    ExtractParams eb = ep;  // the blur's short-chunk job table
    for (int i = 0; i <= kMaxLevels; i++) eb.bjob_begin[i] = g.bjob_small[i];
    if (!(h->skip_mask & 2) && !(h->skip_mask & 8)) {  // FAST and the blur in one launch
        HIPR(launch_fast_blur(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), ep, dl, g.d_cells.as<CellDesc>(),
                              h->cellkey.as<uint32_t>(), h->cellcnt.as<int>(), g.roi_pitch, g.roi_rows, g.max_pass,
                              h->blur.as<uint8_t>(), eb, g.nbjobs_small, nframes, st));
        if (ev_fast) HIPR(hipEventRecord(ev_fast, st));
    } else {
        if (!(h->skip_mask & 2) && launch_fast(h, ep, d_frames, fstride, pitch, 0, ep.ncells, nframes, st))
            return ORBX_EDEVICE;
        if (!(h->skip_mask & 8))
            HIPR(launch_blur_strips(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), h->blur.as<uint8_t>(), eb, dl, 0,
                                    g.nbjobs_small, nullptr, nframes, st, kBlurRowsSmall));
    }
    if (!(h->skip_mask & 4))
        HIPR(launch_octree(ep, dl, g.d_cells.as<CellDesc>(), h->cellkey.as<uint32_t>(), h->cellcnt.as<int>(),
                           h->lvkey.as<uint32_t>(), h->lvcnt.as<int>(), h->gscratch.as<uint8_t>(),
                           (long long)ep.keys_per_frame * 8, g.NC, g.KL, g.lds_bytes, errp, nframes, st, 0, -1,
                           copy));
    if (!(h->skip_mask & 16))
        HIPR(launch_describe(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), h->blur.as<uint8_t>(), ep, dl,
                             h->lvkey.as<uint32_t>(), h->lvcnt.as<int>(), d_kps, d_desc, d_counts, kp_stride,
                             g.d_ptab.as<int>(), nframes, st));
    return 0;
}

/* a handle's own HIP stream (h->stream: host calls; h->side: the separate blur of frames the fused describe cannot
 * take), created on the handle's device at its first use */
static int ensure_stream(orbx_handle* h, hipStream_t* s) {
    if (*s) return 0;
    HIPR(hipSetDevice(h->device));
    if (hipStreamCreateWithFlags(s, hipStreamNonBlocking) != hipSuccess) {
        *s = nullptr;
        return ORBX_EDEVICE;
    }
    return 0;
}

static int run_extract(orbx_handle* h, int nframes, const uint8_t* d_frames, long long fstride, int pitch,
                       orbx_kp* d_kps, uint8_t* d_desc, int32_t* d_counts, int kp_stride, hipStream_t st,
                       bool host_call = true, bool mapped_out = false, const HostCopy* copy = nullptr) {
    Geometry& g = h->geo;
    // the L2-residency bound (orbx_debug_alias_frames): every frame of the batch reads frame 0's image and
    // shares one pyramid / blur buffer, so the stages read lines other workgroups of the launch keep in L2
    ExtractParams ep_alias = g.ep;
    if (h->alias) {
        ep_alias.pyr_frame_bytes = 0;
        ep_alias.blur_frame_bytes = 0;
        fstride = 0;
    }
    ep_alias.host_out = mapped_out ? 1 : 0;
    const ExtractParams& ep = ep_alias;
    const LevelDesc* dl = g.d_lv.as<LevelDesc>();
    // the host-buffer paths report their own per-call word; the device batch path leaves word 0 sticky
    // until orbx_check_error takes (and clears) it, so no fill kernel sits on the batch stream every call
    int* errp = h->err.as<int>() + (host_call ? kErrWordExtract : kErrWordSticky);
    if (nframes < kPyrFramesMinBatch && !h->serial && !h->prof_on && !h->alias) {
        if (run_extract_levels(h, ep, nframes, d_frames, fstride, pitch, d_kps, d_desc, d_counts, kp_stride, st, errp,
                               host_call ? nullptr : h->user_ev_pyr, host_call ? nullptr : h->user_ev_fast, copy))
            return ORBX_EDEVICE;
        h->last_frames = d_frames;
        h->last_fstride = fstride;
        h->last_pitch = pitch;
        h->last_nframes = nframes;
        h->last_stream = st;
        return 0;
    }
    const bool fused = use_describe_blur(d_frames, fstride, pitch);
    if (!fused && ensure_blur(h)) return ORBX_EDEVICE;
    if (!fused && !h->serial && ensure_stream(h, &h->side)) return ORBX_EDEVICE;
    const hipStream_t sd = h->serial ? st : h->side;
    if (prof_mark(h, 0, 0, st)) return ORBX_EDEVICE;
    if (!(h->skip_mask & 1) && launch_pyramid(h, ep, d_frames, fstride, pitch, nframes, st)) return ORBX_EDEVICE;
    if (prof_mark(h, 0, 1, st)) return ORBX_EDEVICE;
    if (!host_call && h->user_ev_pyr) HIPR(hipEventRecord(h->user_ev_pyr, st));
    if (!fused) {
        if (!h->serial) {
            HIPR(hipEventRecord(h->ev_pyr, st));
            HIPR(hipStreamWaitEvent(sd, h->ev_pyr, 0));
        }
        if (prof_mark(h, 3, 0, sd)) return ORBX_EDEVICE;
        if (!(h->skip_mask & 8))
            HIPR(launch_blur_strips(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), h->blur.as<uint8_t>(), ep, dl, 0,
                                    g.nbjobs, nullptr, nframes, sd));
        if (prof_mark(h, 3, 1, sd)) return ORBX_EDEVICE;
        if (!h->serial) HIPR(hipEventRecord(h->ev_blur, sd));
    } else if (prof_mark(h, 3, 0, st) || prof_mark(h, 3, 1, st)) {  // no blur stage: a zero-length pair
        return ORBX_EDEVICE;
    }
    if (prof_mark(h, 1, 0, st)) return ORBX_EDEVICE;
    if (!(h->skip_mask & 2) && launch_fast(h, ep, d_frames, fstride, pitch, 0, ep.ncells, nframes, st)) return ORBX_EDEVICE;
    if (!host_call && h->user_ev_fast) HIPR(hipEventRecord(h->user_ev_fast, st));
    if (prof_mark(h, 1, 1, st) || prof_mark(h, 2, 0, st)) return ORBX_EDEVICE;
    if (!(h->skip_mask & 4)) {
        const int split = g.oct_split;  // 0: one launch over every level
        HIPR(launch_octree(ep, dl, g.d_cells.as<CellDesc>(), h->cellkey.as<uint32_t>(), h->cellcnt.as<int>(),
                           h->lvkey.as<uint32_t>(), h->lvcnt.as<int>(), h->gscratch.as<uint8_t>(),
                           (long long)ep.keys_per_frame * 8, g.NC, g.KL, g.lds_bytes, errp, nframes, st, 0,
                           split ? split : -1));
        if (split)
            HIPR(launch_octree(ep, dl, g.d_cells.as<CellDesc>(), h->cellkey.as<uint32_t>(), h->cellcnt.as<int>(),
                               h->lvkey.as<uint32_t>(), h->lvcnt.as<int>(), h->gscratch.as<uint8_t>(),
                               (long long)ep.keys_per_frame * 8, g.NC_lo, g.KL_lo, g.lds_lo, errp, nframes, st,
                               split, ep.L - split));
    }
    if (prof_mark(h, 2, 1, st)) return ORBX_EDEVICE;
    if (!h->serial && !fused) HIPR(hipStreamWaitEvent(st, h->ev_blur, 0));
    if (prof_mark(h, 4, 0, st)) return ORBX_EDEVICE;
    if (!(h->skip_mask & 16)) {
        if (fused)
            HIPR(launch_describe_blur(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), ep, dl, h->lvkey.as<uint32_t>(),
                                      h->lvcnt.as<int>(), d_kps, d_desc, d_counts, kp_stride, g.d_ptab.as<int>(),
                                      nframes, st));
        else
            HIPR(launch_describe(d_frames, fstride, pitch, h->pyr.as<uint8_t>(), h->blur.as<uint8_t>(), ep, dl,
                                 h->lvkey.as<uint32_t>(), h->lvcnt.as<int>(), d_kps, d_desc, d_counts, kp_stride,
                                 g.d_ptab.as<int>(), nframes, st));
    }
    if (prof_mark(h, 4, 1, st)) return ORBX_EDEVICE;
    if (h->prof_on && h->prof_calls < kProfMaxCalls) h->prof_calls++;
    h->last_frames = d_frames;
    h->last_fstride = fstride;
    h->last_pitch = pitch;
    h->last_nframes = nframes;
    h->last_stream = st;
    return 0;
}

extern "C" {

const char* orbx_version(void) { return "orbslam-mi355x 0.1 (gfx950)"; }

int orbx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int orbx_create(const orbx_params* p, int device, int max_width, int max_height, int max_batch,
                orbx_handle** out) {
    if (!p || !out || p->nlevels < 1 || p->nlevels > kMaxLevels || p->nfeatures < 1 || p->scale_factor <= 1.0f ||
        max_width <= 0 || max_height <= 0 || max_batch < 1)
        return ORBX_EARG;
    *out = nullptr;
    int ndev = orbx_device_count();
    if (device < 0 || device >= ndev) return ORBX_EDEVICE;
    HIPR(hipSetDevice(device));
    orbx_handle* h = new orbx_handle();
    h->params = *p;
    h->T.build(*p);
    h->device = device;
    h->max_w = max_width;
    h->max_h = max_height;
    h->max_batch = max_batch;
    // no HIP stream here: the host-call stream and the blur's side stream are created at their first use
    // (ensure_stream), since every idle stream in the process costs the batch schedule's graph streams their step
    // rate (profiles/r04_idle_stream_cost.log) and a device batch on the caller's stream needs neither
    if (hipEventCreateWithFlags(&h->ev_pyr, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_blur, hipEventDisableTiming) != hipSuccess) {
        orbx_destroy(h);
        return ORBX_EDEVICE;
    }
    int rc = ensure_geometry(h, max_width, max_height, 1);
    if (rc) {
        orbx_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

void orbx_destroy(orbx_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->side) (void)hipStreamSynchronize(h->side);
    for (DevBuf* b : {&h->pyr, &h->blur, &h->cellkey, &h->cellcnt, &h->lvkey, &h->lvcnt, &h->gscratch, &h->err,
                      &h->in_frame, &h->out_kps, &h->out_desc, &h->out_cnt, &h->st_buf, &h->stereo_sad})
        b->release();
    h->geo.release();
    if (h->stream) (void)hipStreamDestroy(h->stream);
    if (h->side) (void)hipStreamDestroy(h->side);
    for (hipEvent_t e : {h->ev_pyr, h->ev_blur})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : h->prof_ev) (void)hipEventDestroy(e);
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    if (h->graph) (void)hipGraphDestroy(h->graph);
    if (h->pin_in) (void)hipHostFree(h->pin_in);
    if (h->pin_out) (void)hipHostFree(h->pin_out);
    if (h->pin_pyr) (void)hipHostFree(h->pin_pyr);
    delete h;
}

int orbx_check_error(orbx_handle* h, void* stream) {
    if (!h) return ORBX_EARG;
    HIPR(hipSetDevice(h->device));
    // read and clear in one device atomic (a batch on another stream that raises the flag afterwards
    // leaves it set for the next check)
    int flag = 0;
    int* w = h->err.as<int>();
    HIPR(launch_flag_take(w + kErrWordSticky, w + kErrWordTake, (hipStream_t)stream));
    HIPR(hipMemcpyAsync(&flag, w + kErrWordTake, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIPR(hipStreamSynchronize((hipStream_t)stream));
    return flag ? ORBX_EDEVICE : 0;
}

int orbx_selftest_sincosf(const float* d_in, float* d_sin, float* d_cos, int n, void* stream) {
    if (!d_in || !d_sin || !d_cos || n < 0) return ORBX_EARG;
    if (n == 0) return 0;
    HIPR(launch_sincos_selftest(d_in, d_sin, d_cos, n, (hipStream_t)stream));
    return 0;
}

int orbx_set_pyramid_event(orbx_handle* h, void* event) { return orbx_set_stage_event(h, 0, event); }

int orbx_set_stage_event(orbx_handle* h, int stage, void* event) {
    if (!h || stage < 0 || stage > 1) return ORBX_EARG;
    (stage == 0 ? h->user_ev_pyr : h->user_ev_fast) = (hipEvent_t)event;
    return 0;
}

int orbx_describe_blur_fused(const void* frames, size_t frame_stride, size_t pitch) {
    return use_describe_blur((const uint8_t*)frames, (long long)frame_stride, (int)pitch) ? 1 : 0;
}

int orbx_debug_hip_failure(void) {
    // two events that were never recorded: hipEventElapsedTime fails (invalid resource handle), as an unrecorded
    // stage pair did in round 5's orbx_profile_read
    hipEvent_t a = nullptr, b = nullptr;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        if (a) (void)hipEventDestroy(a);
        (void)hipGetLastError();
        return ORBX_EDEVICE;
    }
    float t = 0;
    const hipError_t e = hipEventElapsedTime(&t, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    HIPR(e);
    return 0;
}

int orbx_debug_skip_stages(orbx_handle* h, int mask) {
    if (!h || mask < 0 || mask > 0x1F) return ORBX_EARG;
    h->skip_mask = mask;
    h->epoch++;  // a captured host-call graph holds the schedule it was captured with
    return 0;
}

int orbx_debug_serial(orbx_handle* h, int on) {
    if (!h) return ORBX_EARG;
    h->serial = on != 0;
    h->epoch++;
    return 0;
}

int orbx_debug_alias_frames(orbx_handle* h, int on) {
    if (!h) return ORBX_EARG;
    h->alias = on != 0;
    h->epoch++;
    return 0;
}

int orbx_debug_raise_error(orbx_handle* h, int flag, void* stream) {
    if (!h || flag <= 0) return ORBX_EARG;
    HIPR(hipSetDevice(h->device));
    int cur = 0;
    hipStream_t st = (hipStream_t)stream;
    HIPR(hipMemcpyAsync(&cur, h->err.as<int>() + kErrWordSticky, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPR(hipStreamSynchronize(st));
    cur |= flag;
    HIPR(hipMemcpyAsync(h->err.as<int>() + kErrWordSticky, &cur, sizeof(int), hipMemcpyHostToDevice, st));
    HIPR(hipStreamSynchronize(st));
    return 0;
}

int orbx_profile_enable(orbx_handle* h, int on) {
    if (!h) return ORBX_EARG;
    h->prof_on = on != 0;
    h->prof_mask = on & 0x1F;
    h->prof_calls = 0;
    for (double& v : h->prof_ms) v = 0;
    return 0;
}

int orbx_profile_read(orbx_handle* h, double* ms, int* ncalls) {
    if (!h) return ORBX_EARG;
    HIPR(hipSetDevice(h->device));
    double acc[5] = {0, 0, 0, 0, 0};
    for (int c = 0; c < h->prof_calls; c++) {
        for (int k = 0; k < 5; k++) {
            const size_t e0 = (size_t)c * 10 + 2 * k;
            if (!((h->prof_mask >> k) & 1)) continue;
            HIPR(hipEventSynchronize(h->prof_ev[e0 + 1]));
            float t = 0;
            HIPR(hipEventElapsedTime(&t, h->prof_ev[e0], h->prof_ev[e0 + 1]));
            acc[k] += t;
        }
    }
    if (ms) for (int k = 0; k < 5; k++) ms[k] = acc[k];
    if (ncalls) *ncalls = h->prof_calls;
    return 0;
}

int orbx_max_keypoints(const orbx_handle* h, int width, int height) {
    if (!h) return ORBX_EARG;
    if (h->geo.W == width && h->geo.H == height) return h->geo.ep.kp_per_frame;
    // host-only computation of the cap (no upload): replicate build's kp accounting
    int total = 0;
    for (int l = 0; l < h->T.nlevels; l++) {
        const int w = cv_round_f((float)width * h->T.inv_scale[l]);
        const int hh = cv_round_f((float)height * h->T.inv_scale[l]);
        if (w - 32 <= 0 || hh - 32 <= 0) return ORBX_EARG;  // as Geometry::build rejects the level
        const int nIni = (int)roundf((float)(w - 32) / (hh - 32));
        total += std::max(h->T.nfeat[l] + 3, 4 * std::max(nIni, 1));
    }
    return total;
}

int orbx_extract_batch_device(orbx_handle* h, int nframes, const uint8_t* d_frames, size_t frame_stride, int width,
                              int height, size_t pitch, orbx_kp* d_kps, uint8_t* d_desc, int32_t* d_counts,
                              int kp_stride, void* stream) {
    if (!h || !d_frames || !d_kps || !d_desc || !d_counts || width <= 0 || height <= 0 || pitch < (size_t)width)
        return ORBX_EARG;
    HIPR(hipSetDevice(h->device));
    int rc = ensure_geometry(h, width, height, nframes);
    if (rc) return rc;
    if (kp_stride < h->geo.ep.kp_per_frame) return ORBX_ECAPACITY;
    return run_extract(h, nframes, d_frames, (long long)frame_stride, (int)pitch, d_kps, d_desc, d_counts, kp_stride,
                       (hipStream_t)stream, false);
}

extern "C++" {
namespace {

/* Wait for a per-call matcher launch: its last workgroup stores the match count (>= 0; the host
 * pre-filled it with -1) into pinned host memory last, with release at system scope (match_kernels.hip
 * call_tail), so polling that word ends the call ~5 us sooner than hipStreamSynchronize
 * (tools/latency_floor.hip, profiles/r03_latency_floor.jsonl). The launch needs no further wait: the
 * next call's copies and launches are ordered behind it on the stream. A stream that drains without
 * the word, or an error, is ORBX_EDEVICE. */
template <class Ready>
int wait_until(hipStream_t st, Ready ready) {
    {
        // spin (with a pause) for the first ~200 us, which covers a call that is not queued behind other GPU
        // work; after that yield the core to the other SLAM threads between polls instead of burning it
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned spins = 1;; spins++) {
            if (ready()) return 0;
            const bool late = (spins & 255) == 0 &&
                              std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200);
            if (late || (spins & 1023) == 0) {
                const hipError_t e = hipStreamQuery(st);
                if (e != hipErrorNotReady) {
                    if (e != hipSuccess) return ORBX_EDEVICE;
                    break;  // drained: the words are visible now if the kernel wrote them
                }
                if (late) {
                    sched_yield();
                    spins = 0;  // next check after another 256 polls
                }
            } else {
                __builtin_ia32_pause();
            }
        }
    }
    HIPR(hipStreamSynchronize(st));
    return ready() ? 0 : ORBX_EDEVICE;
}

}  // namespace
}  // extern "C++"

/* The captured host path: pinned H2D -> run_extract -> one pinned D2H of {count, error flag, K
 * keypoints, K descriptors}, as one hipGraph per geometry (replayed: no per-kernel launch cost on
 * the calling thread, one synchronisation per frame). The first call at a new geometry/buffer epoch
 * runs eagerly (it also performs one-time setup such as LDS attributes), the next one captures. */
static int extract_graph(orbx_handle* h, const uint8_t* img, int width, int height, size_t pitch, orbx_kp* kps,
                         uint8_t* desc, int cap, int* n) {
    const int K = h->geo.ep.kp_per_frame;
    const size_t in_bytes = (size_t)width * height;
    const size_t out_bytes = 64 + (sizeof(orbx_kp) + 32) * (size_t)K;
    if (h->pin_in_bytes < in_bytes) {
        if (h->pin_in) (void)hipHostFree(h->pin_in);
        h->pin_in = nullptr;
        h->pin_in_bytes = 0;
        HIPR(hipHostMalloc((void**)&h->pin_in, in_bytes, hipHostMallocDefault));
        h->pin_in_bytes = in_bytes;
        h->epoch++;
    }
    if (h->pin_out_bytes < out_bytes) {
        if (h->pin_out) (void)hipHostFree(h->pin_out);
        h->pin_out = nullptr;
        h->pin_out_bytes = 0;
        // fine-grained (coherent) like the matchers' polled buffers: the kernels' writes of the results and of the
        // done word are visible to the polling host without relying on an L2 writeback
        HIPR(hipHostMalloc((void**)&h->pin_out, out_bytes, hipHostMallocMapped | hipHostMallocCoherent));
        memset(h->pin_out, 0, out_bytes);  // done word 0: the device counter's first value is 1
        h->pin_out_bytes = out_bytes;
        HIPR(hipHostGetDevicePointer((void**)&h->pin_out_dev, h->pin_out, 0));
        h->epoch++;
    }
    // mvImagePyramid for the host (orbx_set_host_pyramid): extra workgroups of the octree launch copy levels 1..L-1
    // of this frame into mapped pinned memory while the octree runs; level 0 is pin_in itself
    const bool copies = h->host_pyr && !h->serial && !h->alias && h->geo.ep.L > 1;
    HostCopy hc{nullptr, nullptr, 0, 0};
    if (copies) {
        const size_t pb = (size_t)h->geo.ep.pyr_frame_bytes;
        if (h->pin_pyr_bytes < pb) {
            if (h->pin_pyr) (void)hipHostFree(h->pin_pyr);
            h->pin_pyr = h->pin_pyr_dev = nullptr;
            h->pin_pyr_bytes = 0;
            HIPR(hipHostMalloc((void**)&h->pin_pyr, pb, hipHostMallocMapped | hipHostMallocCoherent));
            h->pin_pyr_bytes = pb;
            HIPR(hipHostGetDevicePointer((void**)&h->pin_pyr_dev, h->pin_pyr, 0));
            h->epoch++;
        }
        hc = HostCopy{(const uint4*)h->pyr.p, nullptr, (long long)(pb / 16), kHostCopyBlocks,
                      (uint4* const*)(h->pin_out_dev + kPinOutCopyDst)};
        if (h->target && h->target_bytes < host_l0_bytes(h) + pb) return ORBX_EARG;
        // this call's destination of levels 1..L-1, read by the copy workgroups when they run
        uint8_t* dst = h->target ? h->target_dev + host_l0_bytes(h) : h->pin_pyr_dev;
        memcpy(h->pin_out + kPinOutCopyDst, &dst, sizeof(dst));
    }
    for (int y = 0; y < height; y++) memcpy(h->pin_in + (size_t)y * width, img + (size_t)y * pitch, width);
    uint8_t* o_kps = h->pin_out + 64;
    uint8_t* o_desc = o_kps + sizeof(orbx_kp) * (size_t)K;
    // describe writes the count, keypoints and descriptors straight into the pinned buffer (its device-mapped
    // address: 56 B per keypoint over PCIe inside the kernel, no D2H copies), and the last launch moves the
    // call's error word there and clears it for the next call
    uint8_t* d_out = h->pin_out_dev;
    auto enqueue = [&]() -> int {
        HIPR(hipMemcpyAsync(h->in_frame.p, h->pin_in, in_bytes, hipMemcpyHostToDevice, h->stream));
        int rc = run_extract(h, 1, h->in_frame.as<uint8_t>(), (long long)in_bytes, width, (orbx_kp*)(d_out + 64),
                             d_out + 64 + sizeof(orbx_kp) * (size_t)K, (int32_t*)d_out, K, h->stream, true, true,
                             copies ? &hc : nullptr);
        if (rc) return rc;
        HIPR(launch_call_done(h->err.as<int32_t>() + kErrWordExtract, (int32_t*)(d_out + 4),
                              h->err.as<int32_t>() + kErrWordExtractSeq, (int32_t*)(d_out + 8), h->stream));
        return 0;
    };
    // the done word before this call's launch (the previous call's value): the call is over when it changes
    const int32_t* done = (const int32_t*)(h->pin_out + 8);
    const int32_t done0 = __atomic_load_n(done, __ATOMIC_ACQUIRE);
    const bool valid = h->gexec && h->graph_w == width && h->graph_h == height && h->graph_epoch == h->epoch;
    if (!valid) {
        if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
        if (h->graph) (void)hipGraphDestroy(h->graph);
        h->gexec = nullptr;
        h->graph = nullptr;
        if (h->graph_epoch != h->epoch || h->graph_w != width || h->graph_h != height) h->graph_warm = 0;
        h->graph_w = width;
        h->graph_h = height;
        h->graph_epoch = h->epoch;
    }
    if (!h->gexec && h->graph_warm == 0) {
        // first frame at this epoch: eager
        int rc = enqueue();
        if (rc) return rc;
        h->graph_warm = 1;
    } else {
        if (!h->gexec) {
            HIPR(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
            int rc = enqueue();
            hipGraph_t g = nullptr;
            const hipError_t ce = hipStreamEndCapture(h->stream, &g);
            if (rc) {
                if (g) (void)hipGraphDestroy(g);
                return rc;
            }
            HIPR(ce);
            h->graph = g;
            HIPR(hipGraphInstantiate(&h->gexec, h->graph, nullptr, nullptr, 0));
        }
        HIPR(hipGraphLaunch(h->gexec, h->stream));
    }
    // level 0 of a caller-owned target: the staged input, copied on the host while the device works
    if (copies && h->target) memcpy(h->target, h->pin_in, in_bytes);
    if (const int rc = wait_until(h->stream, [&] { return __atomic_load_n(done, __ATOMIC_ACQUIRE) != done0; })) return rc;
    // the copy workgroups ride on the octree launch: a skipped octree (orbx_debug_skip_stages bit 2) delivers nothing
    h->host_pyr_valid = copies && !(h->skip_mask & 4);
    h->last_target = copies ? h->target : nullptr;
    h->last_frames = h->in_frame.as<uint8_t>();
    h->last_fstride = (long long)in_bytes;
    h->last_pitch = width;
    h->last_nframes = 1;
    int cnt = 0, errflag = 0;
    memcpy(&cnt, h->pin_out, sizeof(int));
    memcpy(&errflag, h->pin_out + 4, sizeof(int));
    if (errflag) return ORBX_EDEVICE;
    if (cnt > cap) return ORBX_ECAPACITY;
    if (cnt > 0) {
        if (kps) memcpy(kps, o_kps, sizeof(orbx_kp) * (size_t)cnt);
        if (desc) memcpy(desc, o_desc, 32 * (size_t)cnt);
    }
    *n = cnt;
    return 0;
}

int orbx_extract(orbx_handle* h, const uint8_t* img, int width, int height, size_t pitch, orbx_kp* kps,
                 uint8_t* desc, int cap, int* n) {
    if (!h || !n) return ORBX_EARG;
    *n = 0;
    if (width <= 0 || height <= 0 || !img) return 0;  // empty image: outputs untouched (:1046-1047)
    if (pitch < (size_t)width) return ORBX_EARG;
    HIPR(hipSetDevice(h->device));
    h->host_pyr_valid = false;
    if (ensure_stream(h, &h->stream)) return ORBX_EDEVICE;
    int rc = ensure_geometry(h, width, height, 1);
    if (rc) return rc;
    const int K = h->geo.ep.kp_per_frame;
    const void* before[4] = {h->in_frame.p, h->out_kps.p, h->out_desc.p, h->out_cnt.p};
    if (h->in_frame.ensure((size_t)width * height) || h->out_kps.ensure(sizeof(orbx_kp) * K) ||
        h->out_desc.ensure(32 * (size_t)K) || h->out_cnt.ensure(64))
        return ORBX_EDEVICE;
    const void* after[4] = {h->in_frame.p, h->out_kps.p, h->out_desc.p, h->out_cnt.p};
    if (memcmp(before, after, sizeof(before))) h->epoch++;
    // an unaligned frame (width not a multiple of 4) blurs into HBM: allocate that buffer here, never inside a capture
    if (!use_describe_blur(h->in_frame.as<uint8_t>(), (long long)width * height, width) && ensure_blur(h))
        return ORBX_EDEVICE;
    // captured graph, except while stage profiling (its events are recorded per call)
    if (!h->prof_on) return extract_graph(h, img, width, height, pitch, kps, desc, cap, n);
    HIPR(hipMemcpy2DAsync(h->in_frame.p, width, img, pitch, width, height, hipMemcpyHostToDevice, h->stream));
    rc = run_extract(h, 1, h->in_frame.as<uint8_t>(), (long long)width * height, width, h->out_kps.as<orbx_kp>(),
                     h->out_desc.as<uint8_t>(), h->out_cnt.as<int32_t>(), K, h->stream);
    if (rc) return rc;
    int cnt = 0, errflag = 0;
    HIPR(hipMemcpyAsync(&cnt, h->out_cnt.p, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HIPR(launch_flag_take(h->err.as<int32_t>() + kErrWordExtract, h->err.as<int32_t>() + kErrWordExtractTake, h->stream));
    HIPR(hipMemcpyAsync(&errflag, h->err.as<int>() + kErrWordExtractTake, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HIPR(hipStreamSynchronize(h->stream));
    if (errflag) return ORBX_EDEVICE;
    if (cnt > cap) return ORBX_ECAPACITY;
    if (cnt > 0) {
        if (kps) HIPR(hipMemcpyAsync(kps, h->out_kps.p, sizeof(orbx_kp) * cnt, hipMemcpyDeviceToHost, h->stream));
        if (desc) HIPR(hipMemcpyAsync(desc, h->out_desc.p, 32 * (size_t)cnt, hipMemcpyDeviceToHost, h->stream));
        HIPR(hipStreamSynchronize(h->stream));
    }
    *n = cnt;
    return 0;
}

int orbx_pyramid_level(orbx_handle* h, int frame, int level, uint8_t* dst, size_t pitch, int* width, int* height) {
    if (!h || level < 0 || level >= h->T.nlevels || !h->geo.W) return ORBX_EARG;
    const LevelDesc& d = h->geo.lv[level];
    if (width) *width = d.w;
    if (height) *height = d.h;
    if (!dst) return 0;
    if (!h->last_frames || frame < 0 || frame >= h->last_nframes || pitch < (size_t)d.w) return ORBX_EARG;
    HIPR(hipSetDevice(h->device));
    // wait for this handle's own last extraction only (the stream it was enqueued on and the handle's side
    // stream), not for every stream on the device (other extractor / matcher threads)
    HIPR(hipStreamSynchronize(h->last_stream));
    if (h->side) HIPR(hipStreamSynchronize(h->side));
    const uint8_t* src = level == 0 ? h->last_frames + frame * h->last_fstride
                                    : h->pyr.as<uint8_t>() + frame * h->geo.ep.pyr_frame_bytes + d.pyr_off;
    const size_t sp = level == 0 ? (size_t)h->last_pitch : (size_t)d.pitch;
    HIPR(hipMemcpy2D(dst, pitch, src, sp, d.w, d.h, hipMemcpyDeviceToHost));
    return 0;
}

int orbx_set_host_pyramid(orbx_handle* h, int on) {
    if (!h) return ORBX_EARG;
    h->host_pyr = on != 0;
    h->host_pyr_valid = false;
    h->epoch++;  // the captured host-call graph holds whether the octree launch carries the copy
    return 0;
}

int orbx_host_pyramid_level(orbx_handle* h, int level, const uint8_t** data, size_t* pitch, int* width, int* height) {
    if (!h || !data || !pitch || level < 0 || level >= h->T.nlevels || !h->geo.W || !h->host_pyr_valid)
        return ORBX_EARG;
    const LevelDesc& d = h->geo.lv[level];
    if (h->last_target)
        *data = level == 0 ? h->last_target : h->last_target + host_l0_bytes(h) + d.pyr_off;
    else
        *data = level == 0 ? h->pin_in : h->pin_pyr + d.pyr_off;
    *pitch = level == 0 ? (size_t)d.w : (size_t)d.pitch;
    if (width) *width = d.w;
    if (height) *height = d.h;
    return 0;
}

int orbx_host_pyramid_bytes(orbx_handle* h, int width, int height, size_t* bytes) {
    if (!h || !bytes || width <= 0 || height <= 0) return ORBX_EARG;
    *bytes = 0;
    HIPR(hipSetDevice(h->device));
    if (const int rc = ensure_geometry(h, width, height, 1)) return rc;
    *bytes = host_l0_bytes(h) + (size_t)h->geo.ep.pyr_frame_bytes;
    return 0;
}

int orbx_host_register(void* p, size_t bytes) {
    if (!p || !bytes) return ORBX_EARG;
    HIPR(hipHostRegister(p, bytes, hipHostRegisterMapped));
    return 0;
}

int orbx_host_unregister(void* p) {
    if (!p) return ORBX_EARG;
    HIPR(hipHostUnregister(p));
    return 0;
}

int orbx_set_host_pyramid_target(orbx_handle* h, uint8_t* host, size_t bytes) {
    if (!h || (host && !bytes)) return ORBX_EARG;
    if (!host) {
        h->target = h->target_dev = nullptr;
        h->target_bytes = 0;
        return 0;
    }
    if (host == h->target && bytes == h->target_bytes) return 0;  // the drop-in sets the same buffer every call
    HIPR(hipSetDevice(h->device));
    uint8_t* dev = nullptr;
    HIPR(hipHostGetDevicePointer((void**)&dev, host, 0));  // fails unless the memory is registered (or pinned) mapped
    h->target = host;
    h->target_dev = dev;
    h->target_bytes = bytes;
    return 0;
}

int orbx_get_levels(const orbx_handle* h) { return h ? h->T.nlevels : ORBX_EARG; }
float orbx_get_scale_factor(const orbx_handle* h) { return h ? (float)h->T.scaleFactor : 0.f; }

int orbx_get_scale_tables(const orbx_handle* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2) {
    if (!h) return ORBX_EARG;
    for (int l = 0; l < h->T.nlevels; l++) {
        if (scale) scale[l] = h->T.scale[l];
        if (inv_scale) inv_scale[l] = h->T.inv_scale[l];
        if (sigma2) sigma2[l] = h->T.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = h->T.inv_sigma2[l];
    }
    return 0;
}

int orbx_compute_scale_tables(const orbx_params* p, float* scale, float* inv_scale, float* sigma2,
                              float* inv_sigma2) {
    if (!p || p->nlevels < 1 || p->nlevels > kMaxLevels || p->nfeatures < 1 || p->scale_factor <= 1.0f)
        return ORBX_EARG;
    Tables T;
    T.build(*p);
    for (int l = 0; l < T.nlevels; l++) {
        if (scale) scale[l] = T.scale[l];
        if (inv_scale) inv_scale[l] = T.inv_scale[l];
        if (sigma2) sigma2[l] = T.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = T.inv_sigma2[l];
    }
    return 0;
}

int orbx_get_feature_split(const orbx_handle* h, int32_t* per_level, int32_t* umax16) {
    if (!h) return ORBX_EARG;
    for (int l = 0; l < h->T.nlevels; l++)
        if (per_level) per_level[l] = h->T.nfeat[l];
    for (int v = 0; v < 16; v++)
        if (umax16) umax16[v] = h->T.umax[v];
    return 0;
}

}  // extern "C"

/* ===================================================================================== */
/* Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641)                         */
/* ===================================================================================== */
static int stereo_args(orbx_handle* hl, orbx_handle* hr, float bf, float b, StereoArgs* a) {
    if (!hl || !hr || !hl->last_frames || !hr->last_frames || hl->geo.W != hr->geo.W || hl->geo.H != hr->geo.H ||
        hl->T.nlevels != hr->T.nlevels || hl->device != hr->device)
        return ORBX_EARG;
    for (int l = 0; l < hl->T.nlevels; l++)
        if (hl->T.scale[l] != hr->T.scale[l]) return ORBX_EARG;
    const Geometry& g = hl->geo;
    const int L = hl->T.nlevels;
    memset(a, 0, sizeof(*a));
    a->left = PyrSide{hl->last_frames, hl->last_fstride, hl->pyr.as<uint8_t>(), g.ep.pyr_frame_bytes, hl->last_pitch,
                      hl->last_nframes};
    a->right = PyrSide{hr->last_frames, hr->last_fstride, hr->pyr.as<uint8_t>(), hr->geo.ep.pyr_frame_bytes,
                       hr->last_pitch, hr->last_nframes};
    a->L = L;
    a->nrows = g.H;
    // maxr - minr = ceil(y + r) - floor(y - r) <= 2r + 2, r = 2*mvScaleFactors[octave]
    a->rspan = (int)std::ceil(4.0 * hl->T.scale[L - 1]) + 3;
    const float minZ = b;  // Frame.cc:501-503
    a->maxD = bf / minZ;
    a->bf = bf;
    volatile float c15 = 1.5f, c14 = 1.4f;
    a->thc = c15 * c14;  // 1.5f*1.4f (Frame.cc:639)
    for (int l = 0; l < L; l++) {
        a->scale[l] = hl->T.scale[l];
        a->inv_scale[l] = hl->T.inv_scale[l];
        a->lw[l] = g.lv[l].w;
        a->lh[l] = g.lv[l].h;
        a->lpitch[l] = g.lv[l].pitch;
        a->pyr_off[l] = g.lv[l].pyr_off;
    }
    return 0;
}

static int stereo_prepare(orbx_handle* hl, int stride) {
    if (stride < 1 || stride > 65535) return ORBX_EARG;
    const int lds = stereo_lds_bytes(stride, hl->geo.H);
    if (lds > 160 * 1024) return ORBX_EARG;
    if (lds > 64 * 1024 && lds > hl->stereo_lds_set) {
        HIPR(stereo_setup(lds));
        hl->stereo_lds_set = lds;
    }
    return 0;
}

extern "C" {

int orbx_stereo_matches_batch_device(orbx_handle* left, orbx_handle* right, int npairs, const int32_t* d_fl,
                                     const int32_t* d_fr, const orbx_kp* d_kpsL, const uint8_t* d_descL,
                                     const int32_t* d_cntL, const orbx_kp* d_kpsR, const uint8_t* d_descR,
                                     const int32_t* d_cntR, int kp_stride, float bf, float b, float* d_uright,
                                     float* d_depth, int32_t* d_nstereo, void* stream) {
    if (npairs < 0 || !d_fl || !d_fr || !d_kpsL || !d_descL || !d_cntL || !d_kpsR || !d_descR || !d_cntR ||
        !d_uright || !d_depth || !d_nstereo || !(b > 0.f))
        return ORBX_EARG;
    StereoArgs a;
    int rc = stereo_args(left, right, bf, b, &a);
    if (rc) return rc;
    if (npairs == 0) return 0;
    HIPR(hipSetDevice(left->device));
    if ((rc = stereo_prepare(left, kp_stride))) return rc;
    if (left->stereo_sad.ensure((size_t)npairs * kp_stride * 4)) return ORBX_EDEVICE;
    HIPR(launch_stereo(a, npairs, d_fl, d_fr, d_kpsL, d_descL, d_cntL, d_kpsR, d_descR, d_cntR, kp_stride, d_uright,
                       d_depth, d_nstereo, left->stereo_sad.as<int32_t>(), left->err.as<int>(), (hipStream_t)stream));
    return 0;
}

int orbx_compute_stereo_matches(orbx_handle* left, orbx_handle* right, const orbx_kp* kpsL, const uint8_t* descL,
                                int nL, const orbx_kp* kpsR, const uint8_t* descR, int nR, float bf, float b,
                                float* uright, float* depth, int* nstereo) {
    if (!left || !right || left == right || nL < 0 || nR < 0 || (nL && (!kpsL || !descL || !uright || !depth)) ||
        (nR && (!kpsR || !descR)) || !(b > 0.f))
        return ORBX_EARG;
    StereoArgs a;
    int rc = stereo_args(left, right, bf, b, &a);
    if (rc) return rc;
    if (left->last_nframes < 1 || right->last_nframes < 1) return ORBX_EARG;
    if (nstereo) *nstereo = 0;
    if (nL == 0) return 0;
    HIPR(hipSetDevice(left->device));
    const int stride = (int)align_up(std::max(nL, nR), 4);
    if ((rc = stereo_prepare(left, stride))) return rc;
    // staging: kpsL | kpsR | descL | descR | uright | depth | {fl=0, fr=0, cntL, cntR, nstereo} | sad scratch
    const size_t kb = sizeof(orbx_kp) * stride, db = 32 * (size_t)stride, fb = 4 * (size_t)stride;
    if (left->st_buf.ensure(2 * kb + 2 * db + 3 * fb + 64)) return ORBX_EDEVICE;
    uint8_t* base = left->st_buf.as<uint8_t>();
    orbx_kp* dkL = (orbx_kp*)base;
    orbx_kp* dkR = (orbx_kp*)(base + kb);
    uint8_t* ddL = base + 2 * kb;
    uint8_t* ddR = ddL + db;
    float* dur = (float*)(ddR + db);
    float* ddp = dur + stride;
    int32_t* misc = (int32_t*)(ddp + stride);
    const int32_t hm[4] = {0, 0, nL, nR};
    if (ensure_stream(left, &left->stream)) return ORBX_EDEVICE;
    hipStream_t st = left->stream;
    // the right extraction ran on the stream of the right handle's last call (its own, after a host call), and a
    // batch's blur on its side stream
    HIPR(hipStreamSynchronize(right->last_stream));
    if (right->side) HIPR(hipStreamSynchronize(right->side));
    HIPR(hipMemcpyAsync(dkL, kpsL, sizeof(orbx_kp) * nL, hipMemcpyHostToDevice, st));
    HIPR(hipMemcpyAsync(ddL, descL, 32 * (size_t)nL, hipMemcpyHostToDevice, st));
    if (nR) {
        HIPR(hipMemcpyAsync(dkR, kpsR, sizeof(orbx_kp) * nR, hipMemcpyHostToDevice, st));
        HIPR(hipMemcpyAsync(ddR, descR, 32 * (size_t)nR, hipMemcpyHostToDevice, st));
    }
    HIPR(hipMemcpyAsync(misc, hm, sizeof(hm), hipMemcpyHostToDevice, st));
    int* cerr = left->err.as<int>() + kErrWordCall;  // the host call's own word (the batch word stays sticky)
    HIPR(hipMemsetAsync(cerr, 0, sizeof(int), st));
    a.left.nframes = a.right.nframes = 1;
    HIPR(launch_stereo(a, 1, misc, misc + 1, dkL, ddL, misc + 2, dkR, ddR, misc + 3, stride, dur, ddp, misc + 4,
                       (int32_t*)((uint8_t*)misc + 64), cerr, st));
    int flag = 0, ns = 0;
    HIPR(hipMemcpyAsync(uright, dur, 4 * (size_t)nL, hipMemcpyDeviceToHost, st));
    HIPR(hipMemcpyAsync(depth, ddp, 4 * (size_t)nL, hipMemcpyDeviceToHost, st));
    HIPR(hipMemcpyAsync(&ns, misc + 4, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPR(hipMemcpyAsync(&flag, cerr, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPR(hipStreamSynchronize(st));
    if (flag & 2) return ORBX_EARG;
    if (flag) return ORBX_EDEVICE;
    if (nstereo) *nstereo = ns;
    return 0;
}

}  // extern "C"

/* ===================================================================================== */
/* Matcher                                                                               */
/* ===================================================================================== */
struct orbm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // the host calls' stream, created at the first one: the *_device paths run on the caller's stream, and an idle
    // HIP stream costs the bench's graph streams their step rate (profiles/r04_idle_stream_cost.log). Every host
    // entry point calls ready() first: it makes the context's device current (whatever the calling thread had) and
    // creates the stream there, or fails the call with ORBX_EDEVICE
    int ready() {
        HIPR(hipSetDevice(device));
        if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
            stream = nullptr;
            return ORBX_EDEVICE;
        }
        return 0;
    }
    hipStream_t s() const { return stream; }
    DevBuf scratch;
    DevBuf err;  // device error flag of the *_device calls that validate their input (orbm_check_error)
    std::vector<uint8_t> host;
    void* pinned = nullptr;  // host staging of one call's inputs (one H2D copy) and its results
    void* pinned_dev = nullptr;
    size_t pinned_bytes = 0;
    uint8_t* ensure_pinned(size_t need) {
        if (need <= pinned_bytes) return (uint8_t*)pinned;
        if (stream) (void)hipStreamSynchronize(stream);  // the previous call may still be retiring (wait_call)
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr;
        pinned_dev = nullptr;
        pinned_bytes = 0;
        // fine-grained: the per-call kernels' host writes are visible to the polling host at once
        if (hipHostMalloc(&pinned, need, hipHostMallocCoherent) != hipSuccess) return nullptr;
        if (hipHostGetDevicePointer(&pinned_dev, pinned, 0) != hipSuccess) {
            (void)hipHostFree(pinned);
            pinned = nullptr;
            return nullptr;
        }
        pinned_bytes = need;
        return (uint8_t*)pinned;
    }
    /* device address of byte `off` of the pinned buffer (kernels write results there directly) */
    int32_t* pinned_on_device(size_t off) const { return (int32_t*)((uint8_t*)pinned_dev + off); }
    uint32_t seq = 0;  // call sequence number of k_bow_small's done words (never 0)
    uint32_t next_seq() {
        seq = seq >= kSmallSeqMask ? 1u : seq + 1u;
        return seq;
    }
    /* the per-call state words (match_kernels.hip call_tail): ints 16..47 of the zeroed err buffer */
    int32_t* call_state() { return err.as<int32_t>() + 16; }
};

namespace {

int wait_call(hipStream_t st, const int32_t* word) {
    return wait_until(st, [word] { return __atomic_load_n(word, __ATOMIC_ACQUIRE) >= 0; });
}

/* ComputeThreeMaxima (ORBmatcher.cc:1601-1642) of a 30-bin rotation histogram, for the host-side tail of
 * k_bow_small (the same comparisons as match_kernels.hip three_maxima) */
void three_maxima_host(const int* hist, int keep[3]) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < 30; i++) {
        const int s = hist[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s; ind3 = i;
        }
    }
    const float tenth = 0.1f * (float)max1;
    if ((float)max2 < tenth) ind2 = ind3 = -1;
    else if ((float)max3 < tenth) ind3 = -1;
    keep[0] = ind1; keep[1] = ind2; keep[2] = ind3;
}

void make_geom(MatchGeom& g, const float F12[9], float ex, float ey, int nlevels, const float* scale,
               const float* sigma2) {
    for (int i = 0; i < 9; i++) g.F[i] = F12[i];
    g.ex = ex;
    g.ey = ey;
    for (int o = 0; o < 16; o++) {
        g.th100[o] = o < nlevels ? 100 * scale[o] : 0.f;
        g.th384[o] = o < nlevels ? 3.84 * (double)sigma2[o] : 0.0;
        // the smallest float >= th384: (double)d < th384 <=> d < th384f for every float d
        float t = (float)g.th384[o];
        if ((double)t < g.th384[o]) t = std::nextafter(t, INFINITY);
        g.th384f[o] = t;
    }
}

/* bump allocator over the ctx scratch buffer (sizes first, then carve) */
struct Carve {
    size_t off = 0;
    size_t take(size_t b) { size_t o = off; off += align_up((long long)b, 256); return o; }
};

/* merge-walk of two FeatureVectors (DBoW2 std::map iteration with lower_bound jumps,
 * ORBmatcher.cc:691-789): returns the common (node index 1, node index 2) pairs */
void common_nodes(const orbm_kf_view* a, const orbm_kf_view* b, std::vector<std::pair<int, int>>& out) {
    out.clear();
    int i = 0, j = 0;
    while (i < a->n_nodes && j < b->n_nodes) {
        if (a->node_id[i] == b->node_id[j]) {
            out.emplace_back(i, j);
            i++;
            j++;
        } else if (a->node_id[i] < b->node_id[j]) {
            i = (int)(std::lower_bound(a->node_id + i, a->node_id + a->n_nodes, b->node_id[j]) - a->node_id);
        } else {
            j = (int)(std::lower_bound(b->node_id + j, b->node_id + b->n_nodes, a->node_id[i]) - b->node_id);
        }
    }
}

bool view_ok(const orbm_kf_view* v) {
    return v && v->n >= 0 && (v->n == 0 || (v->desc && v->x && v->y && v->angle && v->octave)) && v->n_nodes >= 0 &&
           (v->n_nodes == 0 || (v->node_id && v->node_off && v->node_feat)) && v->nlevels > 0 && v->nlevels <= 16 &&
           v->scale_factors && v->level_sigma2;
}

/* One keyframe's immutable per-feature arrays in HBM (orbm_kf_cache): mDescriptors, mvKeysUn (x, y, angle,
 * octave), mvuRight, the FeatureVector's feature list and, for the projection matchers, its 64x48 feature
 * grid (k_grid output). A call holds a shared_ptr to the entries it reads until it has its results. Every
 * per-call kernel writes a result word only after the reads it depends on, and the call returns only once it
 * has seen every result word, so no read of the entry is outstanding when the call drops its reference; an
 * eviction on another thread then frees the buffer with hipFree, which in addition waits for the device. */
struct KfEntry {
    DevBuf buf;
    int n = 0, nfeat = 0, n_nodes = 0;
    bool has_ur = false, has_grid = false;
    size_t o_desc = 0, o_x = 0, o_y = 0, o_ang = 0, o_oct = 0, o_ur = 0, o_feat = 0, o_gs = 0, o_gi = 0;
    size_t o_dnode = 0, o_rnode = 0;  // descriptors / NodeRecs in FeatureVector order (k_bow_small, k_tri_small)
    float min_x = 0, min_y = 0, gw_inv = 0, gh_inv = 0;  // grid bounds / scale the grid was built with
    const uint8_t* at(size_t o) const { return buf.as<uint8_t>() + o; }
    size_t bytes() const { return buf.bytes; }  // what it holds against the cache's capacity (KfLru)
};

struct ViewPlan {
    size_t desc, x, y, angle, octave, uright, has_mp, mp_bad, feat;
    int nfeat;
};
/* geom = false (SearchByBoW): positions, octaves and mvuRight are not uploaded (the BoW matchers read
 * descriptors, MapPoint flags, angles and the node lists only) */
void plan_view(Carve& c, const orbm_kf_view* v, ViewPlan& p, bool geom = true, const KfEntry* ce = nullptr) {
    const size_t n = (size_t)std::max(v->n, 1);
    const size_t none = (size_t)-1;
    p.nfeat = v->n_nodes ? v->node_off[v->n_nodes] : 0;
    if (ce) {  // cached keyframe: only the MapPoint flags (they change between calls) are staged
        p.desc = p.x = p.y = p.angle = p.octave = p.uright = p.feat = none;
        p.has_mp = v->has_mp ? c.take(n) : none;
        p.mp_bad = v->mp_bad ? c.take(n) : none;
        return;
    }
    p.desc = c.take(32 * n);
    p.x = geom ? c.take(4 * n) : none;
    p.y = geom ? c.take(4 * n) : none;
    p.angle = c.take(4 * n);
    p.octave = geom ? c.take(4 * n) : none;
    p.uright = geom && v->uright ? c.take(4 * n) : none;
    p.has_mp = v->has_mp ? c.take(n) : (size_t)-1;
    p.mp_bad = v->mp_bad ? c.take(n) : (size_t)-1;
    p.feat = c.take(4 * (size_t)std::max(p.nfeat, 1));
}

/* stage one view into the pinned host image of the scratch (offsets from plan_view) and return
 * the device view of the same offsets: a call then uploads all its inputs with ONE H2D copy */
DevView stage_view(uint8_t* hbase, uint8_t* dbase, const orbm_kf_view* v, const ViewPlan& p,
                   const KfEntry* ce = nullptr) {
    DevView d;
    const size_t n = (size_t)v->n;
    d.n = v->n;
    if (ce) {
        d.desc = ce->at(ce->o_desc);
        d.x = (const float*)ce->at(ce->o_x);
        d.y = (const float*)ce->at(ce->o_y);
        d.angle = (const float*)ce->at(ce->o_ang);
        d.octave = (const int32_t*)ce->at(ce->o_oct);
        d.uright = v->uright && ce->has_ur ? (const float*)ce->at(ce->o_ur) : nullptr;
        d.node_feat = (const int32_t*)ce->at(ce->o_feat);
        d.has_mp = v->has_mp ? dbase + p.has_mp : nullptr;
        d.mp_bad = v->mp_bad ? dbase + p.mp_bad : nullptr;
        if (n && v->has_mp) memcpy(hbase + p.has_mp, v->has_mp, n);
        if (n && v->mp_bad) memcpy(hbase + p.mp_bad, v->mp_bad, n);
        return d;
    }
    d.desc = dbase + p.desc;
    const size_t none = (size_t)-1;
    d.x = p.x != none ? (const float*)(dbase + p.x) : nullptr;
    d.y = p.y != none ? (const float*)(dbase + p.y) : nullptr;
    d.angle = (const float*)(dbase + p.angle);
    d.octave = p.octave != none ? (const int32_t*)(dbase + p.octave) : nullptr;
    d.uright = p.uright != none ? (const float*)(dbase + p.uright) : nullptr;
    d.has_mp = v->has_mp ? dbase + p.has_mp : nullptr;
    d.mp_bad = v->mp_bad ? dbase + p.mp_bad : nullptr;
    d.node_feat = (const int32_t*)(dbase + p.feat);
    if (n) {
        memcpy(hbase + p.desc, v->desc, 32 * n);
        if (p.x != none) memcpy(hbase + p.x, v->x, 4 * n);
        if (p.y != none) memcpy(hbase + p.y, v->y, 4 * n);
        memcpy(hbase + p.angle, v->angle, 4 * n);
        if (p.octave != none) memcpy(hbase + p.octave, v->octave, 4 * n);
        if (p.uright != none) memcpy(hbase + p.uright, v->uright, 4 * n);
        if (v->has_mp) memcpy(hbase + p.has_mp, v->has_mp, n);
        if (v->mp_bad) memcpy(hbase + p.mp_bad, v->mp_bad, n);
    }
    if (p.nfeat) memcpy(hbase + p.feat, v->node_feat, 4 * (size_t)p.nfeat);
    return d;
}

}  // namespace

extern "C" {

int orbm_create(int device, orbm_ctx** out) {
    if (!out) return ORBX_EARG;
    *out = nullptr;
    if (device < 0 || device >= orbx_device_count()) return ORBX_EDEVICE;
    HIPR(hipSetDevice(device));
    orbm_ctx* c = new orbm_ctx();
    c->device = device;
    if (c->err.ensure(256) || hipMemset(c->err.p, 0, 256) != hipSuccess) {
        orbm_destroy(c);
        return ORBX_EDEVICE;
    }
    *out = c;
    return 0;
}

void orbm_destroy(orbm_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->scratch.release();
    c->err.release();
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:1647-1663) -- host scalar */
int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    if (!a || !b) return ORBX_EARG;
    int d = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

void orbm_epipole(const float R2w[9], const float t2w[3], const float Cw[3], float fx, float fy, float cx, float cy,
                  float* ex, float* ey) {
    // C2 = R2w*Cw + t2w: OpenCV's 3x3-by-3x1 gemm path (float products and sums, then
    // (float)(t*alpha + c*beta) in double), as pinned in DESIGN.md
    float C2[3];
    for (int i = 0; i < 3; i++) {
        const float* a = R2w + 3 * i;
        const float t0 = a[0] * Cw[0] + a[1] * Cw[1] + a[2] * Cw[2];
        C2[i] = (float)((double)t0 * 1.0 + (double)t2w[i] * 1.0);
    }
    const float invz = 1.0f / C2[2];
    *ex = fx * C2[0] * invz + cx;
    *ey = fy * C2[1] * invz + cy;
}

}  // extern "C"

static int node_feats(const orbm_kf_view* v) { return v->n_nodes ? v->node_off[v->n_nodes] : 0; }

/* ---- small per-call matchers (k_bow_small / k_tri_small): common nodes and per-call MapPoint bits in the
 * kernel arguments, node-ordered keyframe data from the keyframe cache or read by the kernel straight from
 * the pinned staging (zero copy: each element is read once, by one lane, so no H2D copy and no copy kernel
 * precede the launch), accepts + per-task done words written
 * to host memory, the rotation histogram on the host ---- */
struct SmallSide {
    const uint4* d = nullptr;
    const NodeRec* r = nullptr;  // k_tri_small
    const float* a = nullptr;    // k_bow_small: angles, a[p * a_stride]
    int a_stride = 1;
    const int32_t* f = nullptr;
};

/* carve + stage one side in node order (an uncached view), or take the cached entry's arrays */
struct SmallPlan {
    size_t od = 0, orec = 0, of = 0;
    int nf = 0;
    bool cached = false, bow = false;
};
/* bow: an uncached side stages its angles only (4 bytes a position instead of a NodeRec: the kernel reads
 * them across PCIe) */
static void small_plan(Carve& cv, const orbm_kf_view* v, const KfEntry* ce, SmallPlan& p, bool bow) {
    p.nf = node_feats(v);
    p.cached = ce != nullptr;
    p.bow = bow;
    if (ce) return;
    const size_t n = (size_t)std::max(p.nf, 1);
    p.od = cv.take(32 * n);
    p.orec = cv.take((bow ? 4 : sizeof(NodeRec)) * n);
    p.of = cv.take(4 * n);
}
static NodeRec node_rec(const float* x, const float* y, const float* ang, const int32_t* oct, const float* ur, int f) {
    NodeRec r;
    r.x = x ? x[f] : 0.f;
    r.y = y ? y[f] : 0.f;
    r.oct = (oct ? oct[f] : 0) | (ur && ur[f] >= 0.f ? 0x100 : 0);
    r.angle = ang ? ang[f] : 0.f;
    return r;
}
static SmallSide small_stage(const orbm_kf_view* v, const KfEntry* ce, const SmallPlan& p, uint8_t* hp,
                             uint8_t* dbase) {
    SmallSide s;
    if (ce) {
        s.d = (const uint4*)ce->at(ce->o_dnode);
        s.r = (const NodeRec*)ce->at(ce->o_rnode);
        s.a = &s.r->angle;
        s.a_stride = sizeof(NodeRec) / sizeof(float);
        s.f = (const int32_t*)ce->at(ce->o_feat);
        return s;
    }
    NodeRec* rec = (NodeRec*)(hp + p.orec);
    float* ang = (float*)(hp + p.orec);
    for (int q = 0; q < p.nf; q++) {
        const int f = v->node_feat[q];
        memcpy(hp + p.od + 32 * (size_t)q, v->desc + 32 * (size_t)f, 32);
        if (p.bow) ang[q] = v->angle ? v->angle[f] : 0.f;
        else rec[q] = node_rec(v->x, v->y, v->angle, v->octave, v->uright, f);
    }
    if (p.nf) memcpy(hp + p.of, v->node_feat, 4 * (size_t)p.nf);
    s.d = (const uint4*)(dbase + p.od);
    s.r = (const NodeRec*)(dbase + p.orec);
    s.a = (const float*)(dbase + p.orec);
    s.f = (const int32_t*)(dbase + p.of);
    return s;
}
/* per node position: bit set when pred(feature index) */
template <class Pred>
static void small_bits(const orbm_kf_view* v, uint32_t* bits, Pred pred) {
    const int nf = node_feats(v);
    for (int q = 0; q < nf; q++)
        if (pred(v->node_feat[q])) bits[q >> 5] |= 1u << (q & 31);
}

/* wait for every task's done word of this call, then the rotation histogram + ComputeThreeMaxima over the
 * accepts (ORBmatcher.cc:236-285 / 784-819) and the caller's output (out[x] = partner, -1 elsewhere) */
static int small_finish(orbm_ctx* ctx, const uint8_t* hp, size_t o_out, size_t o_done, const SmallTask* tasks, int nt,
                        uint32_t seq, int check_ori, int32_t* out, int nout, int* nmatches) {
    const unsigned long long* done = (const unsigned long long*)(hp + o_done);
    const unsigned long long* acc = (const unsigned long long*)(hp + o_out);
    // polled in task order: a done word, then its accepts, each final once it carries this call's seq (the
    // kernel's stores are unordered: no fence)
    int next = 0, k = 0;
    if (const int rc = wait_until(ctx->s(), [&] {
            for (; next < nt; next++, k = 0) {
                const unsigned long long d = __atomic_load_n(done + next, __ATOMIC_ACQUIRE);
                if ((uint32_t)d != seq) return false;
                for (const int na = (int)(d >> 32); k < na; k++)
                    if ((uint32_t)(__atomic_load_n(acc + tasks[next].q_begin + k, __ATOMIC_ACQUIRE) >> 37) != seq)
                        return false;
            }
            return true;
        }))
        return rc;
    int hist[30] = {0}, keep[3] = {-2, -2, -2};
    if (check_ori) {
        for (int i = 0; i < nt; i++) {
            const int na = (int)(done[i] >> 32);
            for (int j = 0; j < na; j++) hist[(acc[tasks[i].q_begin + j] >> 32) & 31]++;
        }
        three_maxima_host(hist, keep);
    }
    std::fill(out, out + nout, -1);
    int cnt = 0;
    for (int i = 0; i < nt; i++) {
        const int na = (int)(done[i] >> 32);
        for (int j = 0; j < na; j++) {
            const unsigned long long e = acc[tasks[i].q_begin + j];
            const int bin = (int)((e >> 32) & 31);
            if (check_ori && bin != keep[0] && bin != keep[1] && bin != keep[2]) continue;
            out[e & 0xFFFF] = (int32_t)((e >> 16) & 0xFFFF);
            cnt++;
        }
    }
    if (nmatches) *nmatches = cnt;
    return 0;
}

/* SearchByBoW through k_bow_small (every common node <= 64 candidates, <= kSmallTasks common nodes, <= 2048
 * FeatureVector entries a side) */
static int bow_small(orbm_ctx* ctx, const orbm_kf_view* vq, const orbm_kf_view* vc, const std::vector<NodeTask>& tasks,
                     float nnratio, int check_ori, int mode, int32_t* out, int nout, int* nmatches,
                     const KfEntry* cq, const KfEntry* cc) {
    const int nt = (int)tasks.size();
    Carve cv;
    SmallPlan pq, pc;
    small_plan(cv, vq, cq, pq, true);
    small_plan(cv, vc, cc, pc, true);
    const size_t o_out = cv.take(8 * (size_t)std::max(pq.nf, 1));
    const size_t o_done = cv.take(8 * (size_t)nt);
    uint8_t* hp = ctx->ensure_pinned(cv.off);
    if (!hp) return ORBX_EDEVICE;
    uint8_t* dbase = (uint8_t*)ctx->pinned_on_device(0);
    BowSmall a;
    memset(&a, 0, sizeof(a));
    const SmallSide sq = small_stage(vq, cq, pq, hp, dbase), sc = small_stage(vc, cc, pc, hp, dbase);
    a.qd = sq.d; a.qa = sq.a; a.qa_stride = sq.a_stride; a.qf = sq.f;
    a.cd = sc.d; a.ca = sc.a; a.ca_stride = sc.a_stride; a.cf = sc.f;
    auto good = [](const orbm_kf_view* v) {  // a good MapPoint: one, and not bad
        return [v](int f) { return v->has_mp && v->has_mp[f] && !(v->mp_bad && v->mp_bad[f]); };
    };
    small_bits(vq, a.qgood, good(vq));
    if (mode == 1) small_bits(vc, a.cgood, good(vc));
    for (int i = 0; i < nt; i++)
        a.tasks[i] = SmallTask{(uint16_t)tasks[i].q_begin, (uint16_t)tasks[i].q_end, (uint16_t)tasks[i].c_begin,
                               (uint16_t)tasks[i].c_end};
    a.out = (unsigned long long*)ctx->pinned_on_device(o_out);
    a.done = (unsigned long long*)ctx->pinned_on_device(o_done);
    a.seq = (int)ctx->next_seq();
    a.ntasks = nt;
    a.mode = mode;
    a.check_ori = check_ori ? 1 : 0;
    a.nnratio = nnratio;
    // the polled words start at 0, which no call carries (seq >= 1): a word left by an earlier call on this
    // context (another layout, or the same bits by chance) can never read as this call's
    memset(hp + o_out, 0, cv.off - o_out);
    HIPR(launch_bow_small(a, ctx->s()));
    return small_finish(ctx, hp, o_out, o_done, a.tasks, nt, (uint32_t)a.seq, check_ori, out, nout, nmatches);
}

/* SearchForTriangulation over common nodes through k_tri_small (<= kSmallTasks 64-query chunks, every common
 * node <= 256 candidates, <= 2048 FeatureVector entries a side) */
static int tri_small(orbm_ctx* ctx, const orbm_kf_view* kf1, const orbm_kf_view* kf2, const std::vector<NodeTask>& tasks,
                     const float F12[9], float ex, float ey, int only_stereo, int check_ori, int32_t* match12,
                     int* nmatches, const KfEntry* c1, const KfEntry* c2) {
    const int nt = (int)tasks.size();
    Carve cv;
    SmallPlan p1, p2;
    small_plan(cv, kf1, c1, p1, false);
    small_plan(cv, kf2, c2, p2, false);
    const size_t o_out = cv.take(8 * (size_t)std::max(p1.nf, 1));
    const size_t o_done = cv.take(8 * (size_t)nt);
    uint8_t* hp = ctx->ensure_pinned(cv.off);
    if (!hp) return ORBX_EDEVICE;
    uint8_t* dbase = (uint8_t*)ctx->pinned_on_device(0);
    TriSmall a;
    memset(&a, 0, sizeof(a));
    const SmallSide s1 = small_stage(kf1, c1, p1, hp, dbase), s2 = small_stage(kf2, c2, p2, hp, dbase);
    a.qd = s1.d; a.qr = s1.r; a.qf = s1.f;
    a.cd = s2.d; a.cr = s2.r; a.cf = s2.f;
    auto has_mp = [](const orbm_kf_view* v) { return [v](int f) { return v->has_mp && v->has_mp[f] != 0; }; };
    small_bits(kf1, a.qmp, has_mp(kf1));
    small_bits(kf2, a.cmp, has_mp(kf2));
    for (int i = 0; i < nt; i++)
        a.tasks[i] = SmallTask{(uint16_t)tasks[i].q_begin, (uint16_t)tasks[i].q_end, (uint16_t)tasks[i].c_begin,
                               (uint16_t)tasks[i].c_end};
    a.out = (unsigned long long*)ctx->pinned_on_device(o_out);
    a.done = (unsigned long long*)ctx->pinned_on_device(o_done);
    a.seq = (int)ctx->next_seq();
    a.ntasks = nt;
    a.check_ori = check_ori ? 1 : 0;
    a.only_stereo = only_stereo ? 1 : 0;
    a.q_ur = kf1->uright != nullptr;
    a.c_ur = kf2->uright != nullptr;
    make_geom(a.g, F12, ex, ey, kf2->nlevels, kf2->scale_factors, kf2->level_sigma2);
    memset(hp + o_out, 0, cv.off - o_out);  // polled words: 0 is no call's seq (bow_small)
    HIPR(launch_tri_small(a, ctx->s()));
    return small_finish(ctx, hp, o_out, o_done, a.tasks, nt, (uint32_t)a.seq, check_ori, match12, kf1->n, nmatches);
}


/* c1 / c2: the keyframes' cached device arrays (orbm_kf_cache), or nullptr to upload them with the call */
static int tri_common(orbm_ctx* ctx, const orbm_kf_view* kf1, const orbm_kf_view* kf2, const float F12[9], float ex,
                      float ey, int only_stereo, int check_ori, int32_t* match12, int* nmatches,
                      const KfEntry* c1 = nullptr, const KfEntry* c2 = nullptr) {
    if (const int rc_ = ctx->ready()) return rc_;
    std::vector<std::pair<int, int>> common;
    common_nodes(kf1, kf2, common);
    std::vector<NodeTask> tasks;
    for (auto& c : common) {
        const int qb = kf1->node_off[c.first], qe = kf1->node_off[c.first + 1];
        for (int q = qb; q < qe; q += 64)
            tasks.push_back({q, std::min(q + 64, qe), kf2->node_off[c.second], kf2->node_off[c.second + 1]});
    }
    const int n1 = kf1->n;
    if (tasks.empty()) {  // no common node: nothing to match
        std::fill(match12, match12 + n1, -1);
        if (nmatches) *nmatches = 0;
        return 0;
    }
    int max_nc = 0;
    for (const NodeTask& t : tasks) max_nc = std::max(max_nc, t.c_end - t.c_begin);
    if (max_nc <= 256 && tasks.size() <= (size_t)kSmallTasks && kf1->n <= 65535 && kf2->n <= 65535 &&
        node_feats(kf1) <= 32 * kSmallBitWords && node_feats(kf2) <= 32 * kSmallBitWords)
        return tri_small(ctx, kf1, kf2, tasks, F12, ex, ey, only_stereo, check_ori, match12, nmatches, c1, c2);
    // one H2D copy (views, tasks), one launch whose last workgroup writes the (rotation-filtered)
    // matches into pinned host memory pre-filled with -1, one synchronize
    Carve cv;
    ViewPlan p1, p2;
    plan_view(cv, kf1, p1, true, c1);
    plan_view(cv, kf2, p2, true, c2);
    const size_t o_tasks = cv.take(sizeof(NodeTask) * tasks.size());
    const size_t in_bytes = cv.off;
    const size_t o_list = cv.take(16 * (size_t)std::max(n1, 1));
    const size_t o_res = cv.take(4 * ((size_t)n1 + 1));
    if (ctx->scratch.ensure(cv.off)) return ORBX_EDEVICE;
    uint8_t* hp = ctx->ensure_pinned(cv.off);
    if (!hp) return ORBX_EDEVICE;
    uint8_t* base = ctx->scratch.as<uint8_t>();
    DevView d1 = stage_view(hp, base, kf1, p1, c1), d2 = stage_view(hp, base, kf2, p2, c2);
    memcpy(hp + o_tasks, tasks.data(), sizeof(NodeTask) * tasks.size());
    int32_t* res = (int32_t*)(hp + o_res);
    std::fill(res, res + n1 + 1, -1);
    HIPR(hipMemcpyAsync(base, hp, in_bytes, hipMemcpyHostToDevice, ctx->s()));
    MatchGeom g;
    make_geom(g, F12, ex, ey, kf2->nlevels, kf2->scale_factors, kf2->level_sigma2);
    const CallTail tail{ctx->call_state(), (int32_t*)(base + o_list), ctx->pinned_on_device(o_res), d1.angle, d2.angle,
                        n1, check_ori ? 1 : 0, 0};
    HIPR(launch_tri_nodes(d1, d2, (const NodeTask*)(base + o_tasks), (int)tasks.size(), g, only_stereo, tail,
                          ctx->s()));
    if (const int rc = wait_call(ctx->s(), res)) return rc;
    memcpy(match12, res + 1, 4 * (size_t)n1);
    if (nmatches) *nmatches = res[0];
    return 0;
}

extern "C" int orbm_search_for_triangulation(orbm_ctx* ctx, const orbm_kf_view* kf1, const orbm_kf_view* kf2,
                                             const float F12[9], float ex, float ey, int only_stereo, int check_ori,
                                             int32_t* match12, int* nmatches) {
    if (!ctx || !view_ok(kf1) || !view_ok(kf2) || !F12 || !match12) return ORBX_EARG;
    return tri_common(ctx, kf1, kf2, F12, ex, ey, only_stereo, check_ori, match12, nmatches);
}

extern "C" {

static int bow_common(orbm_ctx* ctx, const orbm_kf_view* vq, const orbm_kf_view* vc, float nnratio, int check_ori,
                      int mode, int32_t* out, int nout, int* nmatches, const KfEntry* cq = nullptr,
                      const KfEntry* cc = nullptr) {
    if (const int rc_ = ctx->ready()) return rc_;
    std::vector<std::pair<int, int>> common;
    common_nodes(vq, vc, common);
    std::vector<NodeTask> tasks;
    int max_nc = 1;
    for (auto& c : common) {
        NodeTask t{vq->node_off[c.first], vq->node_off[c.first + 1], vc->node_off[c.second],
                   vc->node_off[c.second + 1]};
        max_nc = std::max(max_nc, t.c_end - t.c_begin);
        tasks.push_back(t);
    }
    if (max_nc > 64 * 1024) return ORBX_EARG;
    if (tasks.empty()) {  // no common node: nothing to match
        std::fill(out, out + nout, -1);
        if (nmatches) *nmatches = 0;
        return 0;
    }
    if (max_nc <= 64 && vq->n <= 65535 && vc->n <= 65535 && tasks.size() <= (size_t)kSmallTasks && node_feats(vq) <= 32 * kSmallBitWords &&
        node_feats(vc) <= 32 * kSmallBitWords)
        return bow_small(ctx, vq, vc, tasks, nnratio, check_ori, mode, out, nout, nmatches, cq, cc);
    // one H2D copy, one launch (greedy per node; the last workgroup's rotation filter writes the
    // matches into pinned host memory pre-filled with -1), one synchronize
    Carve cv;
    ViewPlan pq, pc;
    plan_view(cv, vq, pq, false, cq);
    plan_view(cv, vc, pc, false, cc);
    const size_t o_tasks = cv.take(sizeof(NodeTask) * tasks.size());
    const size_t in_bytes = cv.off;
    const size_t o_list = cv.take(16 * (size_t)std::max(nout, 1));
    const size_t o_res = cv.take(4 * ((size_t)nout + 1));
    if (ctx->scratch.ensure(cv.off)) return ORBX_EDEVICE;
    uint8_t* hp = ctx->ensure_pinned(cv.off);
    if (!hp) return ORBX_EDEVICE;
    uint8_t* base = ctx->scratch.as<uint8_t>();
    DevView dq = stage_view(hp, base, vq, pq, cq), dc = stage_view(hp, base, vc, pc, cc);
    memcpy(hp + o_tasks, tasks.data(), sizeof(NodeTask) * tasks.size());
    int32_t* res = (int32_t*)(hp + o_res);
    std::fill(res, res + nout + 1, -1);
    HIPR(hipMemcpyAsync(base, hp, in_bytes, hipMemcpyHostToDevice, ctx->s()));
    // mode 0: out indexed by the F idx, partner = KF idx -> rot = angKF[m] - angF[i] (swap)
    const CallTail tail{ctx->call_state(), (int32_t*)(base + o_list), ctx->pinned_on_device(o_res), dq.angle,
                        dc.angle, nout, check_ori ? 1 : 0, mode == 0 ? 1 : 0};
    HIPR(launch_bow(dq, dc, (const NodeTask*)(base + o_tasks), (int)tasks.size(), max_nc, nnratio, mode, tail,
                    ctx->s()));
    if (const int rc = wait_call(ctx->s(), res)) return rc;
    memcpy(out, res + 1, 4 * (size_t)nout);
    if (nmatches) *nmatches = res[0];
    return 0;
}

int orbm_search_by_bow_kf_f(orbm_ctx* ctx, const orbm_kf_view* kf, const orbm_kf_view* f, float nnratio,
                            int check_ori, int32_t* match_f, int* nmatches) {
    if (!ctx || !view_ok(kf) || !view_ok(f) || !match_f) return ORBX_EARG;
    return bow_common(ctx, kf, f, nnratio, check_ori, 0, match_f, f->n, nmatches);
}

int orbm_search_by_bow_kf_kf(orbm_ctx* ctx, const orbm_kf_view* kf1, const orbm_kf_view* kf2, float nnratio,
                             int check_ori, int32_t* match12, int* nmatches) {
    if (!ctx || !view_ok(kf1) || !view_ok(kf2) || !match12) return ORBX_EARG;
    return bow_common(ctx, kf1, kf2, nnratio, check_ori, 1, match12, kf1->n, nmatches);
}

int orbm_triangulation_bf_batch_device(orbm_ctx* ctx, int npairs, const int32_t* d_q1, const int32_t* d_q2,
                                       const orbx_kp* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                                       int kp_stride, const float F12[9], float ex, float ey, int nlevels,
                                       const float* scale_factors, const float* level_sigma2, int check_ori,
                                       int32_t* d_match12, int32_t* d_nmatches, void* stream) {
    if (!ctx || npairs < 0 || !F12 || nlevels < 1 || nlevels > 16 || !scale_factors || !level_sigma2 ||
        kp_stride < 1)
        return ORBX_EARG;
    if (npairs == 0) return 0;
    HIPR(hipSetDevice(ctx->device));
    MatchGeom g;
    make_geom(g, F12, ex, ey, nlevels, scale_factors, level_sigma2);
    hipStream_t st = (hipStream_t)stream;
    HIPR(hipMemsetAsync(d_nmatches, 0, sizeof(int32_t) * npairs, st));
    HIPR(launch_tri_bf(npairs, d_q1, d_q2, d_kps, d_desc, d_counts, kp_stride, g, d_match12, d_nmatches, st));
    if (check_ori)
        HIPR(launch_rot_filter_pairs(npairs, d_q1, d_q2, d_kps, d_counts, kp_stride, d_match12, d_nmatches, st));
    return 0;
}

int orbm_triangulation_bf_stereo_batch_device(orbm_ctx* ctx, int npairs, const int32_t* d_q1, const int32_t* d_q2,
                                              const orbx_kp* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                                              const float* d_uright, int kp_stride, const float F12[9], float ex,
                                              float ey, int nlevels, const float* scale_factors,
                                              const float* level_sigma2, int only_stereo, int check_ori,
                                              int32_t* d_match12, int32_t* d_nmatches, void* stream) {
    if (!ctx || npairs < 0 || !F12 || nlevels < 1 || nlevels > 16 || !scale_factors || !level_sigma2 ||
        kp_stride < 1 || (npairs > 0 && !d_uright))
        return ORBX_EARG;
    if (npairs == 0) return 0;
    HIPR(hipSetDevice(ctx->device));
    MatchGeom g;
    make_geom(g, F12, ex, ey, nlevels, scale_factors, level_sigma2);
    hipStream_t st = (hipStream_t)stream;
    HIPR(hipMemsetAsync(d_nmatches, 0, sizeof(int32_t) * npairs, st));
    HIPR(launch_tri_bf(npairs, d_q1, d_q2, d_kps, d_desc, d_counts, kp_stride, g, d_match12, d_nmatches, st, d_uright,
                       only_stereo ? 1 : 0));
    if (check_ori)
        HIPR(launch_rot_filter_pairs(npairs, d_q1, d_q2, d_kps, d_counts, kp_stride, d_match12, d_nmatches, st));
    return 0;
}

int orbm_triangulation_nodes_batch_device(orbm_ctx* ctx, int npairs, const int32_t* d_q1, const int32_t* d_q2,
                                          const orbx_kp* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                                          int kp_stride, const uint32_t* d_fv_node, const int32_t* d_fv_off,
                                          const int32_t* d_fv_feat, const int32_t* d_nfv, int max_nodes,
                                          const float F12[9], float ex, float ey, int nlevels,
                                          const float* scale_factors, const float* level_sigma2, int check_ori,
                                          int32_t* d_match12, int32_t* d_nmatches, void* stream) {
    if (!ctx || npairs < 0 || !F12 || nlevels < 1 || nlevels > 16 || !scale_factors || !level_sigma2 ||
        kp_stride < 1 || max_nodes < 0 || max_nodes > kp_stride)
        return ORBX_EARG;
    if (npairs == 0) return 0;
    HIPR(hipSetDevice(ctx->device));
    MatchGeom g;
    make_geom(g, F12, ex, ey, nlevels, scale_factors, level_sigma2);
    hipStream_t st = (hipStream_t)stream;
    HIPR(hipMemsetAsync(d_match12, 0xFF, sizeof(int32_t) * (size_t)npairs * kp_stride, st));
    HIPR(hipMemsetAsync(d_nmatches, 0, sizeof(int32_t) * npairs, st));
    HIPR(launch_tri_nodes_pairs(npairs, max_nodes, d_q1, d_q2, d_kps, d_desc, kp_stride, d_fv_node, d_fv_off,
                                d_fv_feat, d_nfv, g, d_match12, d_nmatches, st));
    if (check_ori)
        HIPR(launch_rot_filter_pairs(npairs, d_q1, d_q2, d_kps, d_counts, kp_stride, d_match12, d_nmatches, st));
    return 0;
}

int orbm_search_by_bow_batch_device(orbm_ctx* ctx, int npairs, int mode, const int32_t* d_qf, const int32_t* d_cf,
                                    const orbx_kp* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                                    int kp_stride, const uint8_t* d_mp_flags, const uint32_t* d_fv_node,
                                    const int32_t* d_fv_off, const int32_t* d_fv_feat, const int32_t* d_nfv,
                                    int max_nodes, float nnratio, int check_ori, int32_t* d_out,
                                    int32_t* d_nmatches, void* stream) {
    if (!ctx || npairs < 0 || (mode != 0 && mode != 1) || kp_stride < 1 || max_nodes < 0 || max_nodes > kp_stride ||
        kp_stride > 64 * 1024)
        return ORBX_EARG;
    if (npairs == 0) return 0;
    HIPR(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    HIPR(hipMemsetAsync(d_out, 0xFF, sizeof(int32_t) * (size_t)npairs * kp_stride, st));
    HIPR(hipMemsetAsync(d_nmatches, 0, sizeof(int32_t) * npairs, st));
    HIPR(launch_bow_pairs(npairs, max_nodes, d_qf, d_cf, d_desc, kp_stride, d_mp_flags, d_fv_node, d_fv_off, d_fv_feat,
                          d_nfv, nnratio, mode, d_out, st));
    if (check_ori) {
        // rows of out: (KF,KF) the query frame's features, rot = angle1 - angle2; (KF,F) the Frame's,
        // rot = angleKF - angleF (ORBmatcher.cc:236-246, 616-627)
        if (mode == 1)
            HIPR(launch_rot_filter_pairs(npairs, d_qf, d_cf, d_kps, d_counts, kp_stride, d_out, d_nmatches, st, 0));
        else
            HIPR(launch_rot_filter_pairs(npairs, d_cf, d_qf, d_kps, d_counts, kp_stride, d_out, d_nmatches, st, 1));
    } else {
        HIPR(launch_count_pairs(npairs, d_out, kp_stride, d_nmatches, st));
    }
    return 0;
}

}  // extern "C"

/* ===================================================================================== */
/* Cross-agent keyframe slot (include/orbslam_amd.h; replaces lcmKeyFrameInfo,              */
/* lcmKeyFrameInfo.hpp:24-150) and the cross-agent SearchForTriangulation over slots        */
/* ===================================================================================== */
namespace {

SlotLayout slot_layout_of(int cap) {
    SlotLayout L;
    L.cap = cap;
    if (!slot_offsets(cap, L.off, &L.bytes)) L.bytes = 0;
    return L;
}

}  // namespace

extern "C" {

size_t orbx_slot_bytes(int cap) {
    uint32_t off[ORBX_SLOT_NSECTIONS], total = 0;
    if (!slot_offsets(cap, off, &total)) return 0;
    return total;
}

int orbx_slot_layout(int cap, orbx_slot_header* hdr) {
    const SlotLayout L = slot_layout_of(cap);
    if (!L.bytes) return ORBX_EARG;
    if (hdr) {
        memset(hdr, 0, sizeof(*hdr));
        hdr->magic = ORBX_SLOT_MAGIC;
        hdr->version = ORBX_SLOT_VERSION;
        hdr->cap = cap;
        hdr->bytes = L.bytes;
        for (int k = 0; k < ORBX_SLOT_NSECTIONS; k++) hdr->off[k] = L.off[k];
    }
    return 0;
}

int orbx_pack_keyframe_device(const orbx_kf_source* src, const orbx_kf_meta* meta, int cap, uint8_t* d_slot,
                              int32_t* d_err, void* stream) {
    if (!src || !meta || !src->kps || !src->desc || !src->count || !d_slot || cap < 1) return ORBX_EARG;
    const SlotLayout L = slot_layout_of(cap);
    if (!L.bytes) return ORBX_EARG;
    HIPR(launch_pack_slot(*src, L, *meta, d_slot, d_err, (hipStream_t)stream));
    return 0;
}

/* host restatement of k_pack_slot, byte for byte */
int orbx_pack_keyframe_host(const orbx_kf_source* s, const orbx_kf_meta* meta, int cap, uint8_t* slot,
                            size_t slot_bytes) {
    if (!s || !meta || !s->count || !slot || cap < 1) return ORBX_EARG;
    const SlotLayout L = slot_layout_of(cap);
    if (!L.bytes || slot_bytes < L.bytes) return ORBX_EARG;
    const int n = *s->count;
    if (n < 0) return ORBX_EARG;
    if (n > 0 && (!s->kps || !s->desc)) return ORBX_EARG;
    const bool has_bow = s->bow_word && s->bow_value;
    const int nbow = has_bow && s->nbow ? *s->nbow : 0;
    const bool has_fv = s->fv_node && s->fv_off && s->fv_feat;
    const int nfv = has_fv && s->nfv ? *s->nfv : 0;
    const int nfeat = has_fv && nfv > 0 ? s->fv_off[nfv] : 0;
    if (n > cap || nbow < 0 || nbow > cap || nfv < 0 || nfv > cap || nfeat < 0 || nfeat > cap) return ORBX_ECAPACITY;
    memset(slot, 0, L.bytes);
    orbx_slot_header* h = (orbx_slot_header*)slot;
    h->magic = ORBX_SLOT_MAGIC;
    h->version = ORBX_SLOT_VERSION;
    h->n = n;
    h->cap = cap;
    h->nbow = has_bow ? nbow : 0;
    h->nfv = nfv;
    h->flags = (s->kun ? ORBX_SLOT_F_KUN : 0u) | ((s->uright && s->depth) ? ORBX_SLOT_F_STEREO : 0u) |
               (s->mp_flags ? ORBX_SLOT_F_MP : 0u) | (has_bow ? ORBX_SLOT_F_BOW : 0u) | (has_fv ? ORBX_SLOT_F_FV : 0u);
    h->bytes = L.bytes;
    for (int k = 0; k < ORBX_SLOT_NSECTIONS; k++) h->off[k] = L.off[k];
    memcpy(slot + kSlotMetaOff, meta, sizeof(*meta));
    orbx_kp* kps = (orbx_kp*)(slot + L.off[ORBX_SLOT_KPS]);
    float* kun = (float*)(slot + L.off[ORBX_SLOT_KUN]);
    float* ur = (float*)(slot + L.off[ORBX_SLOT_URIGHT]);
    float* dp = (float*)(slot + L.off[ORBX_SLOT_DEPTH]);
    for (int i = 0; i < n; i++) {
        kps[i] = s->kps[i];
        kun[2 * i] = s->kun ? s->kun[2 * i] : s->kps[i].x;
        kun[2 * i + 1] = s->kun ? s->kun[2 * i + 1] : s->kps[i].y;
        const bool st = s->uright && s->depth;
        ur[i] = st ? s->uright[i] : -1.f;
        dp[i] = st ? s->depth[i] : -1.f;
    }
    if (n) memcpy(slot + L.off[ORBX_SLOT_DESC], s->desc, 32 * (size_t)n);
    if (s->mp_flags && n) {
        memcpy(slot + L.off[ORBX_SLOT_MPFLAGS], s->mp_flags, (size_t)n);
        if (s->mp_pos) memcpy(slot + L.off[ORBX_SLOT_MPPOS], s->mp_pos, 12 * (size_t)n);
    }
    if (has_bow && nbow) {
        memcpy(slot + L.off[ORBX_SLOT_BOWWORD], s->bow_word, 4 * (size_t)nbow);
        memcpy(slot + L.off[ORBX_SLOT_BOWVALUE], s->bow_value, 8 * (size_t)nbow);
    }
    if (has_fv && nfv) {
        memcpy(slot + L.off[ORBX_SLOT_FVNODE], s->fv_node, 4 * (size_t)nfv);
        int32_t* fo = (int32_t*)(slot + L.off[ORBX_SLOT_FVOFF]);
        for (int k = 0; k <= nfv; k++) fo[k] = std::min(std::max(s->fv_off[k], 0), cap);
        if (nfeat) memcpy(slot + L.off[ORBX_SLOT_FVFEAT], s->fv_feat, 4 * (size_t)nfeat);
    }
    return 0;
}

int orbx_slot_parse(const uint8_t* slot, size_t slot_bytes, orbx_slot_view* v) {
    if (!slot || !v || slot_bytes < kSlotBodyOff) return ORBX_EARG;
    const orbx_slot_header* h = (const orbx_slot_header*)slot;
    if (h->magic != ORBX_SLOT_MAGIC || h->version != ORBX_SLOT_VERSION) return ORBX_EARG;
    const SlotLayout L = slot_layout_of(h->cap);
    if (!L.bytes || h->bytes != L.bytes || (size_t)L.bytes > slot_bytes) return ORBX_EARG;
    for (int k = 0; k < ORBX_SLOT_NSECTIONS; k++)
        if (h->off[k] != L.off[k]) return ORBX_EARG;
    const int n = h->n, cap = h->cap;
    if (n < 0 || n > cap || h->nbow < 0 || h->nbow > cap || h->nfv < 0 || h->nfv > cap) return ORBX_EARG;
    const orbx_kf_meta* m = (const orbx_kf_meta*)(slot + kSlotMetaOff);
    if (m->mnScaleLevels < 1 || m->mnScaleLevels > 16) return ORBX_EARG;
    const orbx_kp* kps = (const orbx_kp*)(slot + L.off[ORBX_SLOT_KPS]);
    for (int i = 0; i < n; i++)
        if (kps[i].octave < 0 || kps[i].octave >= m->mnScaleLevels) return ORBX_EARG;
    const uint32_t* bw = (const uint32_t*)(slot + L.off[ORBX_SLOT_BOWWORD]);
    for (int k = 1; k < h->nbow; k++)
        if (bw[k] <= bw[k - 1]) return ORBX_EARG;
    const uint32_t* fn = (const uint32_t*)(slot + L.off[ORBX_SLOT_FVNODE]);
    const int32_t* fo = (const int32_t*)(slot + L.off[ORBX_SLOT_FVOFF]);
    const int32_t* ff = (const int32_t*)(slot + L.off[ORBX_SLOT_FVFEAT]);
    if (h->nfv > 0) {
        if (fo[0] != 0 || fo[h->nfv] > n) return ORBX_EARG;
        for (int k = 0; k < h->nfv; k++) {
            if (k && fn[k] <= fn[k - 1]) return ORBX_EARG;
            if (fo[k + 1] < fo[k]) return ORBX_EARG;
            for (int j = fo[k]; j < fo[k + 1]; j++)
                if (ff[j] < 0 || ff[j] >= n || (j > fo[k] && ff[j] <= ff[j - 1])) return ORBX_EARG;
        }
    }
    v->hdr = h;
    v->meta = m;
    v->kps = kps;
    v->kun = (const float*)(slot + L.off[ORBX_SLOT_KUN]);
    v->uright = (const float*)(slot + L.off[ORBX_SLOT_URIGHT]);
    v->depth = (const float*)(slot + L.off[ORBX_SLOT_DEPTH]);
    v->desc = slot + L.off[ORBX_SLOT_DESC];
    v->mp_flags = slot + L.off[ORBX_SLOT_MPFLAGS];
    v->mp_pos = (const float*)(slot + L.off[ORBX_SLOT_MPPOS]);
    v->bow_word = bw;
    v->bow_value = (const double*)(slot + L.off[ORBX_SLOT_BOWVALUE]);
    v->fv_node = fn;
    v->fv_off = fo;
    v->fv_feat = ff;
    return 0;
}

int orbm_check_error(orbm_ctx* ctx, void* stream) {
    if (!ctx) return ORBX_EARG;
    HIPR(hipSetDevice(ctx->device));
    // atomic read-and-clear on the device (word 0 -> word 56; the per-call state is words 16..47)
    int flag = 0;
    int32_t* w = ctx->err.as<int32_t>();
    HIPR(launch_flag_take(w, w + 56, (hipStream_t)stream));
    HIPR(hipMemcpyAsync(&flag, w + 56, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIPR(hipStreamSynchronize((hipStream_t)stream));
    return flag ? ORBX_EDEVICE : 0;
}

int orbm_search_by_bow_slots_device(orbm_ctx* ctx, const orbx_kf_source* query, int cap1, int nref,
                                    const uint8_t* d_slots, size_t slot_bytes, float nnratio, int check_ori,
                                    int max_nodes, int32_t* d_match, int32_t* d_nmatches, void* stream) {
    if (!ctx || !query || !query->kps || !query->desc || !query->count || !query->fv_node || !query->fv_off ||
        !query->fv_feat || !query->nfv || cap1 < 1 || cap1 > 65535 || nref < 0 || max_nodes < 0 || max_nodes > cap1 ||
        (nref > 0 && (!d_slots || !d_match || !d_nmatches)) || slot_bytes < kSlotBodyOff)
        return ORBX_EARG;
    if (nref == 0) return 0;
    HIPR(hipSetDevice(ctx->device));
    QueryKF q;
    memset(&q, 0, sizeof(q));
    q.kps = query->kps;
    q.mpf = query->mp_flags;
    q.desc = query->desc;
    q.count = query->count;
    q.fv_node = query->fv_node;
    q.fv_off = query->fv_off;
    q.fv_feat = query->fv_feat;
    q.nfv = query->nfv;
    q.cap = cap1;
    hipStream_t st = (hipStream_t)stream;
    HIPR(hipMemsetAsync(d_nmatches, 0, sizeof(int32_t) * (size_t)nref, st));
    HIPR(hipMemsetAsync(d_match, 0xFF, sizeof(int32_t) * (size_t)nref * cap1, st));
    HIPR(launch_bow_slots(q, d_slots, (long long)slot_bytes, nref, nnratio, check_ori ? 1 : 0, max_nodes, d_match,
                          d_nmatches, ctx->err.as<int32_t>(), st));
    return 0;
}

int orbm_search_for_triangulation_slots_device(orbm_ctx* ctx, const orbx_kf_source* query, int cap1, int nref,
                                               const uint8_t* d_slots, size_t slot_bytes, const orbm_slot_geom* geom,
                                               int use_bow, int max_nodes, int32_t* d_match, int32_t* d_nmatches,
                                               void* stream) {
    if (!ctx || !query || !query->kps || !query->desc || !query->count || cap1 < 1 || nref < 0 ||
        (nref > 0 && (!d_slots || !geom || !d_match || !d_nmatches)) || slot_bytes < kSlotBodyOff)
        return ORBX_EARG;
    if (use_bow && (!query->fv_node || !query->fv_off || !query->fv_feat || !query->nfv || max_nodes < 0 ||
                    max_nodes > cap1))
        return ORBX_EARG;
    if (nref == 0) return 0;
    HIPR(hipSetDevice(ctx->device));
    QueryKF q;
    q.kps = query->kps;
    q.kun = (const float2*)query->kun;
    q.uright = query->uright;
    q.mpf = query->mp_flags;
    q.desc = query->desc;
    q.count = query->count;
    q.fv_node = query->fv_node;
    q.fv_off = query->fv_off;
    q.fv_feat = query->fv_feat;
    q.nfv = query->nfv;
    q.cap = cap1;
    hipStream_t st = (hipStream_t)stream;
    HIPR(hipMemsetAsync(d_nmatches, 0, sizeof(int32_t) * (size_t)nref, st));
    if (use_bow) HIPR(hipMemsetAsync(d_match, 0xFF, sizeof(int32_t) * (size_t)nref * cap1, st));
    HIPR(launch_tri_slots(q, d_slots, (long long)slot_bytes, nref, geom, use_bow, max_nodes, d_match, d_nmatches,
                          ctx->err.as<int32_t>(), st));
    return 0;
}

}  // extern "C"

/* ===================================================================================== */
/* SearchByProjection x4: host prologues (per-MapPoint geometry with the reference's float  */
/* semantics) + the device grid / windowed search / claim resolution (frame_kernels.hip)    */
/* ===================================================================================== */
namespace {

/* cv::Mat float arithmetic as pinned in DESIGN.md (identical to the oracle's restatement):
 * A*x + c (3x3 by 3x1, flags 0) = OpenCV's small-matrix gemm path: float products and sums,
 * then (float)(t*alpha + c*beta) in double; A.t()*x (GEMM_1_T) = generic path, double
 * accumulation; norm/dot accumulate in double. */
void gemm33_fast(const float* A, int astep, const float* x, const float* c, float* d) {
    for (int i = 0; i < 3; i++) {
        const float* a = A + i * astep;
        const float t0 = a[0] * x[0] + a[1] * x[1] + a[2] * x[2];
        d[i] = (float)((double)t0 * 1.0 + (double)c[i] * 1.0);
    }
}
void gemm33t_neg(const float* A, int astep, const float* x, float* d) {
    for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += (double)A[k * astep + i] * (double)x[k];
        d[i] = (float)(-1.0 * s);
    }
}
float norm3(const float* v) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)v[k] * (double)v[k];
    return (float)std::sqrt(s);
}
double dot3(const float* a, const float* b) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)a[k] * (double)b[k];
    return s;
}
/* MapPoint::PredictScale (MapPoint.cc:385-417); log of a float = logf (pinned) */
int predict_scale(float max_dist, float currentDist, const orbm_frame_view* F) {
    const float ratio = max_dist / currentDist;
    int nScale = (int)std::ceil(logf(ratio) / F->log_scale_factor);
    if (nScale < 0)
        nScale = 0;
    else if (nScale >= F->nlevels)
        nScale = F->nlevels - 1;
    return nScale;
}
inline bool flag(const uint8_t* a, int i) { return a && a[i]; }

struct ProjBatch {
    std::vector<ProjQuery> q;
    std::vector<uint8_t> qdesc;
    void add(const ProjQuery& pq, const uint8_t* d) {
        q.push_back(pq);
        qdesc.insert(qdesc.end(), d, d + 32);
    }
};

bool frame_view_ok(const orbm_frame_view* F) {
    return F && F->n >= 0 && F->n < 65536 && F->nlevels >= 1 && F->nlevels <= 16 && F->scale_factors &&
           (F->n == 0 || (F->desc && F->x && F->y && F->octave));
}

/* uploads the Frame side + queries, runs k_grid / k_proj_scan / k_proj_resolve, downloads */
constexpr bool kProjDirect = true;  // Fuse: results written by the scan kernel (no k_proj_resolve wave)
/* init_n >= 0: SearchForInitialization (k_init_resolve) with F = F2 and match[] = vnMatches12 of F1's init_n
 * keypoints; otherwise match[] has F->n entries */
/* ce: the frame's cached device arrays and grid (orbm_kf_cache): only the queries travel, no k_grid */
int run_projection(orbm_ctx* ctx, const orbm_frame_view* F, const ProjBatch& pb, int accept_th, int ratio,
                   float nnratio, int check_ori, int32_t* match, int* nmatches, const float* inv_sigma2 = nullptr,
                   int32_t* qres = nullptr, int init_n = -1, const KfEntry* ce = nullptr) {
    if (const int rc_ = ctx->ready()) return rc_;
    const size_t n = (size_t)F->n, nq = pb.q.size();
    const size_t nout = init_n >= 0 ? (size_t)init_n : n;
    const size_t nF = ce ? 0 : n;  // per-feature arrays uploaded with the call
    // inputs first (staged in pinned memory, one H2D copy), then outputs (one D2H copy), then scratch
    Carve cv;
    const size_t o_call = cv.take(sizeof(ProjCall)), o_x = cv.take(4 * nF), o_y = cv.take(4 * nF),
                 o_ang = cv.take(4 * nF), o_ur = cv.take(4 * nF), o_oct = cv.take(4 * nF), o_occ = cv.take(n),
                 o_desc = cv.take(32 * nF), o_q = cv.take(sizeof(ProjQuery) * nq), o_qd = cv.take(32 * nq);
    const size_t in_bytes = cv.off;
    const size_t o_nm = cv.take(4 * nout + 4);  // nmatches, then match[nout]
    const size_t o_gs = cv.take(ce ? 0 : 4 * (kGridCols * kGridRows + 1)), o_gi = cv.take(2 * nF),
                 o_scan = cv.take(8 * (size_t)proj_topk() * nq), o_scnt = cv.take(4 * nq), o_res = cv.take(8 * nq);
    if (ctx->scratch.ensure(cv.off)) return ORBX_EDEVICE;
    // results: written by the kernels straight into the pinned buffer after the inputs (ProjCall::host_out)
    const size_t n_host = std::max(nout + 1, nq);
    uint8_t* hp = ctx->ensure_pinned(in_bytes + 8 * n_host);
    if (!hp) return ORBX_EDEVICE;
    uint8_t* base = ctx->scratch.as<uint8_t>();
    hipStream_t st = ctx->s();
    ProjCall c;
    memset(&c, 0, sizeof(c));
    c.x = (const float*)(base + o_x);
    c.y = (const float*)(base + o_y);
    c.angle = (const float*)(base + o_ang);
    c.uright = F->uright ? (const float*)(base + o_ur) : nullptr;
    c.octave = (const int32_t*)(base + o_oct);
    c.occ0 = F->occupied ? base + o_occ : nullptr;
    c.desc = base + o_desc;
    c.n = F->n;
    c.min_x = F->min_x;
    c.min_y = F->min_y;
    c.gw_inv = F->grid_w_inv;
    c.gh_inv = F->grid_h_inv;
    c.q = (const ProjQuery*)(base + o_q);
    c.qdesc = base + o_qd;
    c.nq = (int)nq;
    c.accept_th = accept_th;
    c.ratio = ratio;
    c.nnratio = nnratio;
    c.check_ori = check_ori && F->angle;
    // per-query results with nothing to arbitrate (Fuse): the scan writes them, no resolve wave
    bool claims = false;
    for (const ProjQuery& q : pb.q) claims |= (q.flags & kProjClaims) != 0;
    c.direct = kProjDirect && qres && !ratio && !c.check_ori && !claims;
    c.n_out = (int)nout;
    c.grid_start = (int*)(base + o_gs);
    c.grid_idx = (uint16_t*)(base + o_gi);
    if (ce) {
        c.x = (const float*)ce->at(ce->o_x);
        c.y = (const float*)ce->at(ce->o_y);
        c.angle = (const float*)ce->at(ce->o_ang);
        c.uright = F->uright && ce->has_ur ? (const float*)ce->at(ce->o_ur) : nullptr;
        c.octave = (const int32_t*)ce->at(ce->o_oct);
        c.desc = ce->at(ce->o_desc);
        c.grid_start = (int*)ce->at(ce->o_gs);
        c.grid_idx = (uint16_t*)ce->at(ce->o_gi);
    }
    c.scan = (unsigned long long*)(base + o_scan);
    c.scan_cnt = (int*)(base + o_scnt);
    c.res = (int*)(base + o_res);
    c.nmatches = (int32_t*)(base + o_nm);
    c.match = (int32_t*)(base + o_nm + 4);
    c.host_out = (unsigned long long*)ctx->pinned_on_device(in_bytes);
    c.seq = (int)ctx->next_seq();
    if (inv_sigma2)
        for (int l = 0; l < F->nlevels; l++) c.inv_sigma2[l] = inv_sigma2[l];
    memcpy(hp + o_call, &c, sizeof(c));
    if (n && F->occupied) memcpy(hp + o_occ, F->occupied, n);
    if (nF) {
        memcpy(hp + o_x, F->x, 4 * n);
        memcpy(hp + o_y, F->y, 4 * n);
        if (F->angle) memcpy(hp + o_ang, F->angle, 4 * n);
        if (F->uright) memcpy(hp + o_ur, F->uright, 4 * n);
        memcpy(hp + o_oct, F->octave, 4 * n);
        memcpy(hp + o_desc, F->desc, 32 * n);
    }
    if (nq) {
        memcpy(hp + o_q, pb.q.data(), sizeof(ProjQuery) * nq);
        memcpy(hp + o_qd, pb.qdesc.data(), 32 * nq);
    }
    const size_t nwait = c.direct ? nq : nout + 1;
    // the polled words start at 0, which no call carries (seq >= 1; see bow_small)
    memset(hp + in_bytes, 0, 8 * nwait);
    HIPR(hipMemcpyAsync(base, hp, in_bytes, hipMemcpyHostToDevice, st));
    HIPR(launch_projection((const ProjCall*)(base + o_call), 1, (int)nq, st, !c.direct, init_n >= 0, !ce));
    // poll the results (each carries this call's seq) instead of a D2H copy + stream synchronisation
    const unsigned long long* ho = (const unsigned long long*)(hp + in_bytes);
    const uint32_t seq = (uint32_t)c.seq;
    size_t next = 0;
    if (const int rc = wait_until(st, [&] {
            while (next < nwait && (uint32_t)(__atomic_load_n(ho + next, __ATOMIC_ACQUIRE) >> 32) == seq) next++;
            return next == nwait;
        }))
        return rc;
    if (qres) {
        // per-query results (Fuse): the accepted feature or -1, reported at the query's src
        if (c.direct)
            for (size_t qi = 0; qi < nq; qi++) qres[pb.q[qi].src] = (int32_t)(uint32_t)ho[qi];
        else {  // a resolve launch: per-query results stay on the device (res[2 qi])
            HIPR(hipMemcpyAsync(hp, base + o_res, 8 * nq, hipMemcpyDeviceToHost, st));
            HIPR(hipStreamSynchronize(st));
            for (size_t qi = 0; qi < nq; qi++) qres[pb.q[qi].src] = ((const int32_t*)hp)[2 * qi];
        }
        return 0;
    }
    for (size_t i = 0; i < nout; i++) match[i] = (int32_t)(uint32_t)ho[i];
    if (nmatches) *nmatches = (int)(uint32_t)ho[nout];
    return 0;
}

ProjQuery make_query(float u, float v, float radius, int minl, int maxl, float ur, float er_th, float angle, int flags,
                     int src) {
    ProjQuery q;
    q.u = u;
    q.v = v;
    q.radius = radius;
    q.min_level = minl;
    q.max_level = maxl;
    q.ur = ur;
    q.er_th = er_th;
    q.angle = angle;
    q.flags = flags | kProjValid;
    q.src = src;
    return q;
}

}  // namespace

extern "C" {

int orbm_search_by_projection_local(orbm_ctx* ctx, const orbm_frame_view* F, const orbm_mappoints* mp, float th,
                                    float nnratio, int32_t* match, int* nmatches) {
    if (!ctx || !frame_view_ok(F) || !mp || mp->n < 0 || (mp->n && (!mp->desc || !mp->track_in_view ||
        !mp->track_proj_x || !mp->track_proj_y || !mp->track_proj_xr || !mp->track_level || !mp->track_view_cos)) ||
        (F->n && !match))
        return ORBX_EARG;
    ProjBatch pb;
    const bool bFactor = th != 1.0;  // ORBmatcher.cc:49
    for (int iMP = 0; iMP < mp->n; iMP++) {
        if (!mp->track_in_view[iMP] || flag(mp->bad, iMP)) continue;
        const int lvl = mp->track_level[iMP];
        if (lvl < 0 || lvl >= F->nlevels) return ORBX_EARG;
        float r = mp->track_view_cos[iMP] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:131-137)
        if (bFactor) r *= th;
        const float radius = r * F->scale_factors[lvl];
        pb.add(make_query(mp->track_proj_x[iMP], mp->track_proj_y[iMP], radius, lvl - 1, lvl, mp->track_proj_xr[iMP],
                          radius, 0.f, kProjStereo | (flag(mp->has_obs, iMP) ? kProjClaims : 0), iMP),
               mp->desc + 32 * (size_t)iMP);
    }
    return run_projection(ctx, F, pb, 100 /*TH_HIGH*/, 1, nnratio, 0, match, nmatches);
}

int orbm_search_by_projection_last_frame(orbm_ctx* ctx, const orbm_frame_view* F, const float Tcw_c[16],
                                         const orbm_mappoints* mp, const float Tcw_l[16], float th, int bMono,
                                         int check_ori, int32_t* match, int* nmatches) {
    if (!ctx || !frame_view_ok(F) || !Tcw_c || !Tcw_l || !mp || mp->n < 0 ||
        (mp->n && (!mp->desc || !mp->pos || !mp->octave || (check_ori && !mp->angle))) || (F->n && !match) ||
        (check_ori && !F->angle))
        return ORBX_EARG;
    const float* Rcw = Tcw_c;  // ORBmatcher.cc:1339-1351
    const float tcw[3] = {Tcw_c[3], Tcw_c[7], Tcw_c[11]};
    float twc[3], tlc[3];
    gemm33t_neg(Rcw, 4, tcw, twc);
    const float tlw[3] = {Tcw_l[3], Tcw_l[7], Tcw_l[11]};
    gemm33_fast(Tcw_l, 4, twc, tlw, tlc);
    const bool bForward = tlc[2] > F->b && !bMono;
    const bool bBackward = -tlc[2] > F->b && !bMono;
    ProjBatch pb;
    for (int i = 0; i < mp->n; i++) {  // :1353-1405
        if (flag(mp->skip, i)) continue;
        float x3Dc[3];
        gemm33_fast(Rcw, 4, mp->pos + 3 * (size_t)i, tcw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = 1.0 / x3Dc[2];
        if (invzc < 0) continue;
        const float u = F->fx * xc * invzc + F->cx;
        const float v = F->fy * yc * invzc + F->cy;
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        const int nLastOctave = mp->octave[i];
        if (nLastOctave < 0 || nLastOctave >= F->nlevels) return ORBX_EARG;
        const float radius = th * F->scale_factors[nLastOctave];
        int minl, maxl;
        if (bForward) {
            minl = nLastOctave;
            maxl = -1;
        } else if (bBackward) {
            minl = 0;
            maxl = nLastOctave;
        } else {
            minl = nLastOctave - 1;
            maxl = nLastOctave + 1;
        }
        const float ur = u - F->bf * invzc;
        pb.add(make_query(u, v, radius, minl, maxl, ur, radius, mp->angle ? mp->angle[i] : 0.f,
                          kProjStereo | (flag(mp->has_obs, i) ? kProjClaims : 0), i),
               mp->desc + 32 * (size_t)i);
    }
    return run_projection(ctx, F, pb, 100 /*TH_HIGH*/, 0, 0.f, check_ori, match, nmatches);
}

int orbm_search_by_projection_keyframe(orbm_ctx* ctx, const orbm_frame_view* F, const float Tcw_c[16],
                                       const orbm_mappoints* mp, float th, int orb_dist, int check_ori,
                                       int32_t* match, int* nmatches) {
    if (!ctx || !frame_view_ok(F) || !Tcw_c || !mp || mp->n < 0 ||
        (mp->n && (!mp->desc || !mp->pos || !mp->min_dist || !mp->max_dist || (check_ori && !mp->angle))) ||
        (F->n && !match) || (check_ori && !F->angle))
        return ORBX_EARG;
    const float* Rcw = Tcw_c;  // ORBmatcher.cc:1476-1478
    const float tcw[3] = {Tcw_c[3], Tcw_c[7], Tcw_c[11]};
    float Ow[3];
    gemm33t_neg(Rcw, 4, tcw, Ow);
    ProjBatch pb;
    for (int i = 0; i < mp->n; i++) {  // :1488-1537
        if (flag(mp->skip, i) || flag(mp->bad, i)) continue;
        const float* x3Dw = mp->pos + 3 * (size_t)i;
        float x3Dc[3];
        gemm33_fast(Rcw, 4, x3Dw, tcw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = 1.0 / x3Dc[2];
        const float u = F->fx * xc * invzc + F->cx;
        const float v = F->fy * yc * invzc + F->cy;
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        const float PO[3] = {x3Dw[0] - Ow[0], x3Dw[1] - Ow[1], x3Dw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        const float maxDistance = 1.2f * mp->max_dist[i];
        const float minDistance = 0.8f * mp->min_dist[i];
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[i], dist3D, F);
        const float radius = th * F->scale_factors[nPredictedLevel];
        pb.add(make_query(u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1, 0.f, -1.f,
                          mp->angle ? mp->angle[i] : 0.f, kProjClaims, i),
               mp->desc + 32 * (size_t)i);
    }
    return run_projection(ctx, F, pb, orb_dist, 0, 0.f, check_ori, match, nmatches);
}

int orbm_search_by_projection_sim3(orbm_ctx* ctx, const orbm_frame_view* KF, const float Scw[16],
                                   const orbm_mappoints* mp, int th, int32_t* match, int* nmatches) {
    if (!ctx || !frame_view_ok(KF) || !Scw || !mp || mp->n < 0 ||
        (mp->n && (!mp->desc || !mp->pos || !mp->normal || !mp->min_dist || !mp->max_dist)) || (KF->n && !match))
        return ORBX_EARG;
    // decompose Scw (ORBmatcher.cc:298-304): sRcw/scw and t/scw are convertTo with scale (float)(1./scw)
    const float scw = (float)std::sqrt(dot3(Scw, Scw));
    const float inv = (float)(1. / (double)scw);
    float Rcw[9], tcw[3], Ow[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Rcw[3 * r + c] = Scw[4 * r + c] * inv;
        tcw[r] = Scw[4 * r + 3] * inv;
    }
    gemm33t_neg(Rcw, 3, tcw, Ow);
    ProjBatch pb;
    for (int iMP = 0; iMP < mp->n; iMP++) {  // :313-367
        if (flag(mp->bad, iMP) || flag(mp->skip, iMP)) continue;
        const float* p3Dw = mp->pos + 3 * (size_t)iMP;
        float p3Dc[3];
        gemm33_fast(Rcw, 3, p3Dw, tcw, p3Dc);
        if (p3Dc[2] < 0.0) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = KF->fx * x + KF->cx;
        const float v = KF->fy * y + KF->cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue;  // IsInImage
        const float maxDistance = 1.2f * mp->max_dist[iMP];
        const float minDistance = 0.8f * mp->min_dist[iMP];
        const float PO[3] = {p3Dw[0] - Ow[0], p3Dw[1] - Ow[1], p3Dw[2] - Ow[2]};
        const float dist = norm3(PO);
        if (dist < minDistance || dist > maxDistance) continue;
        if (dot3(PO, mp->normal + 3 * (size_t)iMP) < 0.5 * dist) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[iMP], dist, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        // KeyFrame::GetFeaturesInArea has no level test; the caller's kpLevel window (:385-388)
        pb.add(make_query(u, v, radius, nPredictedLevel - 1, nPredictedLevel, 0.f, -1.f, 0.f, kProjClaims, iMP),
               mp->desc + 32 * (size_t)iMP);
    }
    return run_projection(ctx, KF, pb, 50 /*TH_LOW*/, 0, 0.f, 0, match, nmatches);
}

}  // extern "C"

/* ===================================================================================== */
/* ORBmatcher::Fuse x2: the per-MapPoint projection + windowed search on the device (the    */
/* k_grid / k_proj_scan / k_proj_resolve pipeline without claims); the map updates that     */
/* follow each match stay with the caller, in the reference's loop order                    */
/* ===================================================================================== */
extern "C" {

}  // extern "C"

static int fuse_common(orbm_ctx* ctx, const orbm_frame_view* KF, const float Tcw[16], const float Ow[3],
                       const orbm_mappoints* mp, float th, const float* inv_level_sigma2, int32_t* best_idx,
                       int* nfused, const KfEntry* ce = nullptr) {
    const float* Rcw = Tcw;  // ORBmatcher.cc:827-837
    const float tcw[3] = {Tcw[3], Tcw[7], Tcw[11]};
    ProjBatch pb;
    for (int i = 0; i < mp->n; i++) {  // :843-892
        best_idx[i] = -1;
        if (flag(mp->skip, i) || flag(mp->bad, i)) continue;
        const float* p3Dw = mp->pos + 3 * (size_t)i;
        float p3Dc[3];
        gemm33_fast(Rcw, 4, p3Dw, tcw, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = KF->fx * x + KF->cx;
        const float v = KF->fy * y + KF->cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue;  // IsInImage
        const float ur = u - KF->bf * invz;
        const float maxDistance = 1.2f * mp->max_dist[i];
        const float minDistance = 0.8f * mp->min_dist[i];
        const float PO[3] = {p3Dw[0] - Ow[0], p3Dw[1] - Ow[1], p3Dw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        if (dot3(PO, mp->normal + 3 * (size_t)i) < 0.5 * dist3D) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[i], dist3D, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        // KeyFrame::GetFeaturesInArea has no level test; the caller's kpLevel window (:901-902)
        pb.add(make_query(u, v, radius, nPredictedLevel - 1, nPredictedLevel, ur, -1.f, 0.f, kProjChi2, i),
               mp->desc + 32 * (size_t)i);
    }
    orbm_frame_view K = *KF;
    K.occupied = nullptr;  // Fuse searches every feature
    const int rc = run_projection(ctx, &K, pb, 50 /*TH_LOW*/, 0, 0.f, 0, nullptr, nullptr, inv_level_sigma2, best_idx,
                                  -1, ce);
    if (rc) return rc;
    if (nfused) {
        int nf = 0;
        for (int i = 0; i < mp->n; i++) nf += best_idx[i] >= 0;
        *nfused = nf;
    }
    return 0;
}

static bool fuse_args_ok(orbm_ctx* ctx, const orbm_frame_view* KF, const float Tcw[16], const float Ow[3],
                         const orbm_mappoints* mp, const float* inv_level_sigma2, const int32_t* best_idx) {
    return ctx && frame_view_ok(KF) && Tcw && Ow && inv_level_sigma2 && mp && mp->n >= 0 &&
           !(mp->n && (!mp->desc || !mp->pos || !mp->normal || !mp->min_dist || !mp->max_dist || !best_idx));
}

extern "C" int orbm_fuse(orbm_ctx* ctx, const orbm_frame_view* KF, const float Tcw[16], const float Ow[3],
                         const orbm_mappoints* mp, float th, const float* inv_level_sigma2, int32_t* best_idx,
                         int* nfused) {
    if (!fuse_args_ok(ctx, KF, Tcw, Ow, mp, inv_level_sigma2, best_idx)) return ORBX_EARG;
    return fuse_common(ctx, KF, Tcw, Ow, mp, th, inv_level_sigma2, best_idx, nfused);
}

extern "C" {

int orbm_fuse_sim3(orbm_ctx* ctx, const orbm_frame_view* KF, const float Scw[16], const orbm_mappoints* mp, float th,
                   int32_t* best_idx, int* nfused) {
    if (!ctx || !frame_view_ok(KF) || !Scw || !mp || mp->n < 0 ||
        (mp->n && (!mp->desc || !mp->pos || !mp->normal || !mp->min_dist || !mp->max_dist || !best_idx)))
        return ORBX_EARG;
    // decompose Scw (ORBmatcher.cc:985-990) as in orbm_search_by_projection_sim3
    const float scw = (float)std::sqrt(dot3(Scw, Scw));
    const float inv = (float)(1. / (double)scw);
    float Rcw[9], tcw[3], Ow[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Rcw[3 * r + c] = Scw[4 * r + c] * inv;
        tcw[r] = Scw[4 * r + 3] * inv;
    }
    gemm33t_neg(Rcw, 3, tcw, Ow);
    ProjBatch pb;
    for (int iMP = 0; iMP < mp->n; iMP++) {  // :1000-1052
        best_idx[iMP] = -1;
        if (flag(mp->bad, iMP) || flag(mp->skip, iMP)) continue;
        const float* p3Dw = mp->pos + 3 * (size_t)iMP;
        float p3Dc[3];
        gemm33_fast(Rcw, 3, p3Dw, tcw, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = (float)(1.0 / (double)p3Dc[2]);  // 1.0/ here (:1019)
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = KF->fx * x + KF->cx;
        const float v = KF->fy * y + KF->cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue;  // IsInImage
        const float maxDistance = 1.2f * mp->max_dist[iMP];
        const float minDistance = 0.8f * mp->min_dist[iMP];
        const float PO[3] = {p3Dw[0] - Ow[0], p3Dw[1] - Ow[1], p3Dw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        if (dot3(PO, mp->normal + 3 * (size_t)iMP) < 0.5 * dist3D) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[iMP], dist3D, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        pb.add(make_query(u, v, radius, nPredictedLevel - 1, nPredictedLevel, 0.f, -1.f, 0.f, 0, iMP),
               mp->desc + 32 * (size_t)iMP);
    }
    orbm_frame_view K = *KF;
    K.occupied = nullptr;
    const int rc = run_projection(ctx, &K, pb, 50 /*TH_LOW*/, 0, 0.f, 0, nullptr, nullptr, nullptr, best_idx);
    if (rc) return rc;
    if (nfused) {
        int nf = 0;
        for (int i = 0; i < mp->n; i++) nf += best_idx[i] >= 0;
        *nfused = nf;
    }
    return 0;
}

}  // extern "C"

/* ===================================================================================== */
/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307), batched                 */
/* ===================================================================================== */
extern "C" {

/* ORBmatcher::SearchForInitialization (ORBmatcher.cc:405-520): one query per F1 keypoint of octave <= 0
 * (level1 > 0 skips, :421-423) over F2's grid, window prev_xy[i1] +- windowSize at level level1 (:425);
 * the in-order resolution on the device (k_init_resolve). prev_xy is updated for the matched i1 (:514-517). */
int orbm_search_for_initialization(orbm_ctx* ctx, const orbm_frame_view* F1, const orbm_frame_view* F2, float* prev_xy,
                                   int window_size, float nnratio, int check_ori, int32_t* match12, int* nmatches) {
    if (!ctx || !frame_view_ok(F1) || !frame_view_ok(F2) || (F1->n && (!prev_xy || !match12)) ||
        (check_ori && ((F1->n && !F1->angle) || (F2->n && !F2->angle))))
        return ORBX_EARG;
    if (F1->n > init_max_features() || F2->n > init_max_features()) return ORBX_ECAPACITY;
    ProjBatch pb;
    for (int i1 = 0; i1 < F1->n; i1++) {
        const int level1 = F1->octave[i1];
        if (level1 > 0) continue;
        pb.add(make_query(prev_xy[2 * i1], prev_xy[2 * i1 + 1], (float)window_size, level1, level1, 0.f, 0.f,
                          check_ori ? F1->angle[i1] : 0.f, 0, i1),
               F1->desc + 32 * (size_t)i1);
    }
    int nm = 0;
    int rc = run_projection(ctx, F2, pb, 50 /*TH_LOW*/, 1, nnratio, check_ori, match12, &nm, nullptr, nullptr, F1->n);
    if (rc) return rc;
    for (int i1 = 0; i1 < F1->n; i1++)  // :514-517
        if (match12[i1] >= 0) {
            prev_xy[2 * i1] = F2->x[match12[i1]];
            prev_xy[2 * i1 + 1] = F2->y[match12[i1]];
        }
    if (nmatches) *nmatches = nm;
    return 0;
}

/* one direction of SearchBySim3 (ORBmatcher.cc:1148-1225, 1228-1305): the prologue of each MapPoint of the
 * source keyframe on the host (reference float semantics), the windowed first-strict-minimum search with
 * the octave band [nPredictedLevel-1, nPredictedLevel] on the device (per-query results, no claims) */
static int sim3_direction(orbm_ctx* ctx, const orbm_frame_view* KF, const float* Tsw, const orbm_mappoints* mp,
                          const float* sR, const float* t, float fx, float fy, float cx, float cy, float th,
                          int32_t* vnMatch) {
    const float Rsw[9] = {Tsw[0], Tsw[1], Tsw[2], Tsw[4], Tsw[5], Tsw[6], Tsw[8], Tsw[9], Tsw[10]};
    const float tsw[3] = {Tsw[3], Tsw[7], Tsw[11]};
    ProjBatch pb;
    for (int i = 0; i < mp->n; i++) {
        vnMatch[i] = -1;
        if (flag(mp->skip, i) || flag(mp->bad, i)) continue;  // :1152-1156
        const float* p3Dw = mp->pos + 3 * (size_t)i;
        float p3Dcs[3], p3Dct[3];
        gemm33_fast(Rsw, 3, p3Dw, tsw, p3Dcs);
        gemm33_fast(sR, 3, p3Dcs, t, p3Dct);
        if (p3Dct[2] < 0.0) continue;
        const float invz = 1.0 / p3Dct[2];
        const float x = p3Dct[0] * invz;
        const float y = p3Dct[1] * invz;
        const float u = fx * x + cx;
        const float v = fy * y + cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue;  // IsInImage
        const float maxDistance = 1.2f * mp->max_dist[i];
        const float minDistance = 0.8f * mp->min_dist[i];
        const float dist3D = norm3(p3Dct);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[i], dist3D, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        pb.add(make_query(u, v, radius, nPredictedLevel - 1, nPredictedLevel, 0.f, 0.f, 0.f, 0, i),
               mp->desc + 32 * (size_t)i);
    }
    if (pb.q.empty()) return 0;
    return run_projection(ctx, KF, pb, 100 /*TH_HIGH*/, 0, 0.f, 0, nullptr, nullptr, nullptr, vnMatch);
}

/* ORBmatcher::SearchBySim3 (ORBmatcher.cc:1102-1326) */
int orbm_search_by_sim3(orbm_ctx* ctx, const orbm_frame_view* KF1, const float T1w[16], const orbm_mappoints* mp1,
                        const orbm_frame_view* KF2, const float T2w[16], const orbm_mappoints* mp2, float s12,
                        const float R12[9], const float t12[3], float th, int32_t* match12, int* nfound) {
    auto mp_ok = [](const orbm_mappoints* m) {
        return m && m->n >= 0 && (m->n == 0 || (m->desc && m->pos && m->min_dist && m->max_dist));
    };
    if (!ctx || !frame_view_ok(KF1) || !frame_view_ok(KF2) || !T1w || !T2w || !mp_ok(mp1) || !mp_ok(mp2) || !R12 ||
        !t12 || (mp1->n && !match12) || !(s12 != 0.f))
        return ORBX_EARG;
    // sR12 = s12*R12, sR21 = (1.0/s12)*R12.t() (convertTo with a float scale), t21 = -sR21*t12 (small-matrix
    // gemm, alpha = -1) (:1119-1121)
    float sR12[9], sR21[9], t21[3];
    const float inv_s = (float)(1.0 / (double)s12);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[3 * r + c] = R12[3 * r + c] * s12;
            sR21[3 * r + c] = R12[3 * c + r] * inv_s;
        }
    for (int r = 0; r < 3; r++) {
        const float t0 = sR21[3 * r] * t12[0] + sR21[3 * r + 1] * t12[1] + sR21[3 * r + 2] * t12[2];
        t21[r] = (float)((double)t0 * -1.0);
    }
    std::vector<int32_t> m1((size_t)mp1->n + 1), m2((size_t)mp2->n + 1);
    // both directions project with pKF1's camera (:1105-1108, 1250-1251)
    int rc = sim3_direction(ctx, KF2, T1w, mp1, sR21, t21, KF1->fx, KF1->fy, KF1->cx, KF1->cy, th, m1.data());
    if (!rc) rc = sim3_direction(ctx, KF1, T2w, mp2, sR12, t12, KF1->fx, KF1->fy, KF1->cx, KF1->cy, th, m2.data());
    if (rc) return rc;
    int nFound = 0;
    for (int i1 = 0; i1 < mp1->n; i1++) {  // :1310-1323
        const int idx2 = m1[i1];
        match12[i1] = -1;
        if (idx2 >= 0 && idx2 < mp2->n && m2[idx2] == i1) {
            match12[i1] = idx2;
            nFound++;
        }
    }
    if (nfound) *nfound = nFound;
    return 0;
}

int orbm_compute_distinctive_descriptors_device(orbm_ctx* ctx, int npoints, const int32_t* d_offsets,
                                                const uint8_t* d_desc, int32_t* d_best_idx, uint8_t* d_out_desc,
                                                void* stream) {
    if (!ctx || npoints < 0 || (npoints && (!d_offsets || !d_desc || !d_best_idx))) return ORBX_EARG;
    if (npoints == 0) return 0;
    HIPR(hipSetDevice(ctx->device));
    HIPR(launch_distinctive(npoints, d_offsets, d_desc, d_best_idx, d_out_desc, (hipStream_t)stream));
    return 0;
}

int orbm_compute_distinctive_descriptors(orbm_ctx* ctx, int npoints, const int32_t* offsets, const uint8_t* desc,
                                         int32_t* best_idx, uint8_t* out_desc) {
    if (!ctx || npoints < 0 || (npoints && (!offsets || !best_idx))) return ORBX_EARG;
    if (npoints == 0) return 0;
    if (offsets[0] != 0) return ORBX_EARG;
    for (int p = 0; p < npoints; p++)
        if (offsets[p + 1] < offsets[p]) return ORBX_EARG;
    const size_t nrows = (size_t)offsets[npoints];
    if (nrows && !desc) return ORBX_EARG;
    if (const int rc_ = ctx->ready()) return rc_;
    Carve cv;
    const size_t o_off = cv.take(4 * ((size_t)npoints + 1)), o_desc = cv.take(32 * nrows), o_best = cv.take(4 * (size_t)npoints),
                 o_out = cv.take(32 * (size_t)npoints);
    if (ctx->scratch.ensure(cv.off)) return ORBX_EDEVICE;
    uint8_t* base = ctx->scratch.as<uint8_t>();
    hipStream_t st = ctx->s();
    HIPR(hipMemcpyAsync(base + o_off, offsets, 4 * ((size_t)npoints + 1), hipMemcpyHostToDevice, st));
    if (nrows) HIPR(hipMemcpyAsync(base + o_desc, desc, 32 * nrows, hipMemcpyHostToDevice, st));
    HIPR(launch_distinctive(npoints, (const int32_t*)(base + o_off), base + o_desc, (int32_t*)(base + o_best),
                            out_desc ? base + o_out : nullptr, st));
    HIPR(hipMemcpyAsync(best_idx, base + o_best, 4 * (size_t)npoints, hipMemcpyDeviceToHost, st));
    if (out_desc) HIPR(hipMemcpyAsync(out_desc, base + o_out, 32 * (size_t)npoints, hipMemcpyDeviceToHost, st));
    HIPR(hipStreamSynchronize(st));
    return 0;
}

}  // extern "C"

/* ===================================================================================== */
/* DBoW2 vocabulary transform (Frame::ComputeBoW, Frame.cc:400-407)                       */
/* ===================================================================================== */
#include <fstream>
#include <sstream>
#include <string>

#include "orb_bow.h"

struct orbv_handle {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0, nnodes = 0, nwords = 0;
    // the host transform's stream, created at its first call: the device paths run on the caller's stream, and one
    // more HIP stream in the process costs the bench's four graph streams 3.7 % of their step rate even idle
    // (profiles/r04_idle_stream_cost.log)
    hipStream_t stream = nullptr;
    std::mutex mu;   // the host transform's stream and staging
    DevBuf nodes;    // child-slot descriptors | child-slot records (VocChild)
    DevBuf scratch;  // per-call staging
    VocDev v{};
};

extern "C" {

int orbv_create(int k, int L, int scoring, int weighting, int nlines, const int32_t* parent, const uint8_t* is_leaf,
                const uint8_t* desc, const double* weight, int device, orbv_handle** out) {
    if (!out || k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3 ||
        nlines < 0 || (nlines && (!parent || !is_leaf || !desc || !weight)))
        return ORBX_EARG;
    *out = nullptr;
    if (device < 0 || device >= orbx_device_count()) return ORBX_EDEVICE;
    const int n = nlines + 1;
    std::vector<int32_t> word(n, 0), child_off(n + 1, 0), child(std::max(n, 1), 0), fill(n, 0);
    std::vector<double> w(n, 0.0);
    std::vector<uint8_t> d(32 * (size_t)n, 0);
    int nwords = 0;
    for (int i = 1; i < n; i++) {  // loadFromTextFile's node loop: ids in file order
        const int pid = parent[i - 1];
        if (pid < 0 || pid >= i) return ORBX_EARG;
        memcpy(&d[32 * (size_t)i], desc + 32 * (size_t)(i - 1), 32);
        w[i] = weight[i - 1];
        if (is_leaf[i - 1] > 0) word[i] = nwords++;
        child_off[pid + 1]++;
    }
    for (int i = 0; i < n; i++) child_off[i + 1] += child_off[i];
    for (int i = 1; i < n; i++) child[child_off[parent[i - 1]] + fill[parent[i - 1]]++] = i;  // push_back order
    // child-slot order: slot c holds node child[c]'s descriptor and record (the kernels never read by node id)
    const int ns = std::max(n - 1, 1);
    std::vector<uint8_t> cd(32 * (size_t)ns, 0);
    std::vector<VocChild> cr(ns);
    for (int c = 0; c < n - 1; c++) {
        const int id = child[c];
        memcpy(&cd[32 * (size_t)c], &d[32 * (size_t)id], 32);
        VocChild r{};
        r.id = id, r.c0 = child_off[id], r.nc = child_off[id + 1] - child_off[id], r.word = word[id], r.weight = w[id];
        cr[c] = r;
    }
    HIPR(hipSetDevice(device));
    orbv_handle* h = new orbv_handle();
    h->device = device;
    h->k = k, h->L = L, h->scoring = scoring, h->weighting = weighting, h->nnodes = n, h->nwords = nwords;
    Carve cv;
    const size_t o_d = cv.take(32 * (size_t)ns), o_r = cv.take(sizeof(VocChild) * (size_t)ns);
    if (h->nodes.ensure(cv.off)) {
        orbv_destroy(h);
        return ORBX_EDEVICE;
    }
    uint8_t* b = h->nodes.as<uint8_t>();
    if (hipMemcpy(b + o_d, cd.data(), 32 * (size_t)ns, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b + o_r, cr.data(), sizeof(VocChild) * (size_t)ns, hipMemcpyHostToDevice) != hipSuccess) {
        orbv_destroy(h);
        return ORBX_EDEVICE;
    }
    h->v.cdesc = b + o_d;
    h->v.crec = (const VocChild*)(b + o_r);
    h->v.root_c0 = child_off[0], h->v.root_nc = child_off[1] - child_off[0];
    h->v.n = n, h->v.L = L, h->v.scoring = scoring, h->v.weighting = weighting;
    *out = h;
    return 0;
}

/* TemplatedVocabulary::loadFromTextFile of the ORB-SLAM2 DBoW2 fork (System.cc:64-65 loads
 * ORBvoc.txt with it): "k L scoring weighting", then one line per node "parent isLeaf d0 .. d31
 * weight". Blank lines are skipped (the reference turns a trailing one into a node with an
 * indeterminate descriptor). */
int orbv_load_text(const char* path, int device, orbv_handle** out) {
    if (!path || !out) return ORBX_EARG;
    std::ifstream f(path);
    if (!f) return ORBX_EARG;
    std::string s;
    if (!std::getline(f, s)) return ORBX_EARG;
    std::stringstream ss(s);
    int k = -1, L = -1, n1 = -1, n2 = -1;
    ss >> k >> L >> n1 >> n2;
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) return ORBX_EARG;
    std::vector<int32_t> parent;
    std::vector<uint8_t> leaf, desc;
    std::vector<double> weight;
    while (std::getline(f, s)) {
        if (s.find_first_not_of(" \t\r") == std::string::npos) continue;
        std::stringstream sn(s);
        int pid = 0, isleaf = 0;
        sn >> pid >> isleaf;
        uint8_t d[32];
        for (int i = 0; i < 32; i++) {  // FORB::fromString: ints, one per byte
            int v = 0;
            sn >> v;
            d[i] = (uint8_t)v;
        }
        double w = 0;
        sn >> w;
        if (sn.fail()) return ORBX_EARG;
        parent.push_back(pid);
        leaf.push_back((uint8_t)(isleaf > 0));
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
    }
    return orbv_create(k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(), desc.data(), weight.data(),
                       device, out);
}

void orbv_destroy(orbv_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    h->nodes.release();
    h->scratch.release();
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int orbv_info(const orbv_handle* h, int* k, int* L, int* nnodes, int* nwords) {
    if (!h) return ORBX_EARG;
    if (k) *k = h->k;
    if (L) *L = h->L;
    if (nnodes) *nnodes = h->nnodes;
    if (nwords) *nwords = h->nwords;
    return 0;
}

int orbv_transform_batch_device(orbv_handle* h, int nframes, const uint8_t* d_desc, const int32_t* d_counts,
                                int kp_stride, int levelsup, int32_t* d_word, double* d_weight, uint32_t* d_nid,
                                uint32_t* d_bow_word, double* d_bow_value, int32_t* d_nbow, uint32_t* d_fv_node,
                                int32_t* d_fv_off, int32_t* d_fv_feat, int32_t* d_nfv, void* stream) {
    if (!h || nframes < 0 || kp_stride < 1 || kp_stride > kVocMaxFeatures || !d_desc || !d_counts || !d_word ||
        !d_weight || !d_nid || !d_bow_word || !d_bow_value || !d_nbow || !d_fv_node || !d_fv_off || !d_fv_feat ||
        !d_nfv)
        return ORBX_EARG;
    if (nframes == 0) return 0;
    HIPR(hipSetDevice(h->device));
    HIPR(launch_voc_transform(h->v, levelsup, nframes, d_desc, d_counts, kp_stride, kp_stride, d_word, d_weight, d_nid,
                              d_bow_word, d_bow_value, d_nbow, d_fv_node, d_fv_off, d_fv_feat, d_nfv,
                              (hipStream_t)stream));
    return 0;
}

int orbv_transform(orbv_handle* h, const uint8_t* desc, int n, int levelsup, uint32_t* bow_word, double* bow_value,
                   int* nbow, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat, int* nfv) {
    if (!h || n < 0 || n > kVocMaxFeatures || (n && !desc) || !bow_word || !bow_value || !nbow || !fv_node ||
        !fv_off || !fv_feat || !nfv)
        return ORBX_EARG;
    *nbow = 0;
    *nfv = 0;
    fv_off[0] = 0;
    // TemplatedVocabulary::empty(): no nodes under the root
    if (n == 0 || h->nnodes <= 1) return 0;
    HIPR(hipSetDevice(h->device));
    std::lock_guard<std::mutex> lock(h->mu);
    if (!h->stream) HIPR(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    const size_t N = (size_t)n;
    Carve cv;
    const size_t o_desc = cv.take(32 * N), o_cnt = cv.take(4), o_word = cv.take(4 * N), o_w = cv.take(8 * N),
                 o_nid = cv.take(4 * N), o_bw = cv.take(4 * N), o_bv = cv.take(8 * N), o_nb = cv.take(4),
                 o_fn = cv.take(4 * N), o_fo = cv.take(4 * (N + 1)), o_ff = cv.take(4 * N), o_nf = cv.take(4);
    if (h->scratch.ensure(cv.off)) return ORBX_EDEVICE;
    uint8_t* b = h->scratch.as<uint8_t>();
    hipStream_t st = h->stream;
    const int32_t cnt = n;
    HIPR(hipMemcpyAsync(b + o_desc, desc, 32 * N, hipMemcpyHostToDevice, st));
    HIPR(hipMemcpyAsync(b + o_cnt, &cnt, 4, hipMemcpyHostToDevice, st));
    HIPR(launch_voc_transform(h->v, levelsup, 1, b + o_desc, (const int32_t*)(b + o_cnt), n, n, (int32_t*)(b + o_word),
                              (double*)(b + o_w), (uint32_t*)(b + o_nid), (uint32_t*)(b + o_bw), (double*)(b + o_bv),
                              (int32_t*)(b + o_nb), (uint32_t*)(b + o_fn), (int32_t*)(b + o_fo), (int32_t*)(b + o_ff),
                              (int32_t*)(b + o_nf), st));
    int nb = 0, nf = 0;
    HIPR(hipMemcpyAsync(&nb, b + o_nb, 4, hipMemcpyDeviceToHost, st));
    HIPR(hipMemcpyAsync(&nf, b + o_nf, 4, hipMemcpyDeviceToHost, st));
    HIPR(hipStreamSynchronize(st));
    if (nb) {
        HIPR(hipMemcpyAsync(bow_word, b + o_bw, 4 * (size_t)nb, hipMemcpyDeviceToHost, st));
        HIPR(hipMemcpyAsync(bow_value, b + o_bv, 8 * (size_t)nb, hipMemcpyDeviceToHost, st));
    }
    HIPR(hipMemcpyAsync(fv_off, b + o_fo, 4 * ((size_t)nf + 1), hipMemcpyDeviceToHost, st));
    if (nf) HIPR(hipMemcpyAsync(fv_node, b + o_fn, 4 * (size_t)nf, hipMemcpyDeviceToHost, st));
    HIPR(hipStreamSynchronize(st));
    const int nfeat = fv_off[nf];
    if (nfeat) HIPR(hipMemcpy(fv_feat, b + o_ff, 4 * (size_t)nfeat, hipMemcpyDeviceToHost));
    *nbow = nb;
    *nfv = nf;
    return 0;
}

}  // extern "C"

/* ===================================================================================== */
/* Keyframe cache (orbm_kf_cache): KeyFrames' immutable per-feature arrays kept in HBM     */
/* across the per-call matchers (LocalMapping::CreateNewMapPoints matches one KF1 against  */
/* up to 20 neighbours, LocalMapping.cc:207-268; SearchInNeighbors fuses into them)        */
/* ===================================================================================== */
struct orbm_kf_cache {
    int device = 0;
    hipStream_t stream = nullptr;
    // kind 0: matcher views (orbm_kf_view: + FeatureVector), kind 1: projection views (orbm_frame_view: + grid); the
    // LRU books and their mutex are csrc/kf_cache.h's (also run under ThreadSanitizer by tests/test_sanitizers.py)
    orbamd::KfLru<KfEntry> lru;
    explicit orbm_kf_cache(size_t capacity) : lru(capacity) {}
};

namespace {

/* the cached entry for (kind, key) matching this call's view, uploading (or replacing) it when absent or
 * stale (a different N, FeatureVector size, stereo presence or grid geometry); LRU eviction over the
 * capacity (KfLru). The lookup and the insertion hold the cache's mutex; a miss builds and uploads its entry on the
 * calling context's stream with the mutex released, so calls of other threads are not held behind the upload
 * (two threads missing on the same key both upload; the second insertion keeps the first one's entry).
 * Returns nullptr on a device error. */
std::shared_ptr<KfEntry> cache_get(orbm_kf_cache* c, int kind, uint64_t key, const orbm_kf_view* kv,
                                   const orbm_frame_view* fv, hipStream_t st) {
    const int n = kv ? kv->n : fv->n;
    const int n_nodes = kv ? kv->n_nodes : 0;
    const int nfeat = kv && kv->n_nodes ? kv->node_off[kv->n_nodes] : 0;
    const bool has_ur = kv ? kv->uright != nullptr : fv->uright != nullptr;
    auto matches = [&](const KfEntry& e) {
        return e.n == n && e.n_nodes == n_nodes && e.nfeat == nfeat && (e.has_ur || !has_ur) &&
               (kind == 0 || (e.min_x == fv->min_x && e.min_y == fv->min_y && e.gw_inv == fv->grid_w_inv &&
                              e.gh_inv == fv->grid_h_inv));
    };
    if (std::shared_ptr<KfEntry> hit = c->lru.find(kind, key, matches)) return hit;
    auto e = std::make_shared<KfEntry>();
    e->n = n;
    e->n_nodes = n_nodes;
    e->nfeat = nfeat;
    e->has_ur = has_ur;
    const size_t N = (size_t)std::max(n, 1);
    Carve cv;
    e->o_desc = cv.take(32 * N);
    e->o_x = cv.take(4 * N);
    e->o_y = cv.take(4 * N);
    e->o_ang = cv.take(4 * N);
    e->o_oct = cv.take(4 * N);
    e->o_ur = cv.take(has_ur ? 4 * N : 0);
    e->o_feat = cv.take(4 * (size_t)std::max(nfeat, 1));
    if (kind == 0) {
        e->o_dnode = cv.take(32 * (size_t)std::max(nfeat, 1));
        e->o_rnode = cv.take(sizeof(NodeRec) * (size_t)std::max(nfeat, 1));
    }
    size_t o_call = 0;
    if (kind == 1) {
        e->has_grid = true;
        e->min_x = fv->min_x;
        e->min_y = fv->min_y;
        e->gw_inv = fv->grid_w_inv;
        e->gh_inv = fv->grid_h_inv;
        e->o_gs = cv.take(4 * (kGridCols * kGridRows + 1));
        e->o_gi = cv.take(2 * N);
        o_call = cv.take(sizeof(ProjCall));
    }
    if (hipSetDevice(c->device) != hipSuccess || e->buf.ensure(cv.off)) return nullptr;
    std::vector<uint8_t> h(cv.off, 0);
    const uint8_t* desc = kv ? kv->desc : fv->desc;
    const float* x = kv ? kv->x : fv->x;
    const float* y = kv ? kv->y : fv->y;
    const float* ang = kv ? kv->angle : fv->angle;
    const int32_t* oct = kv ? kv->octave : fv->octave;
    const float* ur = kv ? kv->uright : fv->uright;
    if (n) {
        memcpy(h.data() + e->o_desc, desc, 32 * (size_t)n);
        memcpy(h.data() + e->o_x, x, 4 * (size_t)n);
        memcpy(h.data() + e->o_y, y, 4 * (size_t)n);
        if (ang) memcpy(h.data() + e->o_ang, ang, 4 * (size_t)n);
        memcpy(h.data() + e->o_oct, oct, 4 * (size_t)n);
        if (has_ur) memcpy(h.data() + e->o_ur, ur, 4 * (size_t)n);
    }
    if (nfeat) memcpy(h.data() + e->o_feat, kv->node_feat, 4 * (size_t)nfeat);
    if (kind == 0)
        for (int p = 0; p < nfeat; p++) {
            const int f = kv->node_feat[p];
            memcpy(h.data() + e->o_dnode + 32 * (size_t)p, desc + 32 * (size_t)f, 32);
            const NodeRec r = node_rec(x, y, ang, oct, has_ur ? ur : nullptr, f);
            memcpy(h.data() + e->o_rnode + sizeof(NodeRec) * (size_t)p, &r, sizeof(r));
        }
    if (kind == 1) {  // the KeyFrame's grid (AssignFeaturesToGrid), built once by k_grid
        ProjCall pc;
        memset(&pc, 0, sizeof(pc));
        pc.x = (const float*)e->at(e->o_x);
        pc.y = (const float*)e->at(e->o_y);
        pc.n = n;
        pc.min_x = fv->min_x;
        pc.min_y = fv->min_y;
        pc.gw_inv = fv->grid_w_inv;
        pc.gh_inv = fv->grid_h_inv;
        pc.grid_start = (int*)e->at(e->o_gs);
        pc.grid_idx = (uint16_t*)e->at(e->o_gi);
        memcpy(h.data() + o_call, &pc, sizeof(pc));
    }
    if (hipMemcpyAsync(e->buf.p, h.data(), cv.off, hipMemcpyHostToDevice, st) != hipSuccess) return nullptr;
    if (kind == 1 && launch_projection((const ProjCall*)e->at(o_call), 1, 0, st, false) != hipSuccess) return nullptr;
    if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
    return c->lru.insert(kind, key, e, matches);  // another thread's matching entry, if it inserted one meanwhile
}

}  // namespace

extern "C" {

int orbm_kf_cache_create(int device, size_t capacity_bytes, orbm_kf_cache** out) {
    if (!out) return ORBX_EARG;
    *out = nullptr;
    if (device < 0 || device >= orbx_device_count()) return ORBX_EDEVICE;
    HIPR(hipSetDevice(device));
    orbm_kf_cache* c = new orbm_kf_cache(capacity_bytes ? capacity_bytes : (size_t)1 << 30);
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return ORBX_EDEVICE;
    }
    *out = c;
    return 0;
}

void orbm_kf_cache_destroy(orbm_kf_cache* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->lru.clear();
    (void)hipStreamDestroy(c->stream);
    delete c;
}

int orbm_kf_cache_erase(orbm_kf_cache* c, uint64_t key) {
    if (!c) return ORBX_EARG;
    c->lru.erase(key);
    return 0;
}

int orbm_kf_cache_stats(orbm_kf_cache* c, int* entries, size_t* bytes, long long* hits, long long* misses) {
    if (!c) return ORBX_EARG;
    c->lru.stats(entries, bytes, hits, misses);
    return 0;
}

int orbm_search_for_triangulation_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key1, const orbm_kf_view* kf1,
                                         uint64_t key2, const orbm_kf_view* kf2, const float F12[9], float ex, float ey,
                                         int only_stereo, int check_ori, int32_t* match12, int* nmatches) {
    if (!ctx || !cache || cache->device != ctx->device || !view_ok(kf1) || !view_ok(kf2) || !F12 || !match12)
        return ORBX_EARG;
    if (const int rc_ = ctx->ready()) return rc_;
    const std::shared_ptr<KfEntry> c1 = cache_get(cache, 0, key1, kf1, nullptr, ctx->s());
    const std::shared_ptr<KfEntry> c2 = c1 ? cache_get(cache, 0, key2, kf2, nullptr, ctx->s()) : nullptr;
    if (!c1 || !c2) return ORBX_EDEVICE;
    return tri_common(ctx, kf1, kf2, F12, ex, ey, only_stereo, check_ori, match12, nmatches, c1.get(), c2.get());
}

int orbm_search_by_bow_kf_kf_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key1, const orbm_kf_view* kf1,
                                    uint64_t key2, const orbm_kf_view* kf2, float nnratio, int check_ori,
                                    int32_t* match12, int* nmatches) {
    if (!ctx || !cache || cache->device != ctx->device || !view_ok(kf1) || !view_ok(kf2) || !match12)
        return ORBX_EARG;
    if (const int rc_ = ctx->ready()) return rc_;
    const std::shared_ptr<KfEntry> c1 = cache_get(cache, 0, key1, kf1, nullptr, ctx->s());
    const std::shared_ptr<KfEntry> c2 = c1 ? cache_get(cache, 0, key2, kf2, nullptr, ctx->s()) : nullptr;
    if (!c1 || !c2) return ORBX_EDEVICE;
    return bow_common(ctx, kf1, kf2, nnratio, check_ori, 1, match12, kf1->n, nmatches, c1.get(), c2.get());
}

int orbm_search_by_bow_kf_f_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key, const orbm_kf_view* kf,
                                   const orbm_kf_view* f, float nnratio, int check_ori, int32_t* match_f,
                                   int* nmatches) {
    if (!ctx || !cache || cache->device != ctx->device || !view_ok(kf) || !view_ok(f) || !match_f) return ORBX_EARG;
    if (const int rc_ = ctx->ready()) return rc_;
    const std::shared_ptr<KfEntry> ck = cache_get(cache, 0, key, kf, nullptr, ctx->s());
    if (!ck) return ORBX_EDEVICE;
    return bow_common(ctx, kf, f, nnratio, check_ori, 0, match_f, f->n, nmatches, ck.get(), nullptr);
}

int orbm_fuse_cached(orbm_ctx* ctx, orbm_kf_cache* cache, uint64_t key, const orbm_frame_view* KF, const float Tcw[16],
                     const float Ow[3], const orbm_mappoints* mp, float th, const float* inv_level_sigma2,
                     int32_t* best_idx, int* nfused) {
    if (!cache || !fuse_args_ok(ctx, KF, Tcw, Ow, mp, inv_level_sigma2, best_idx) || cache->device != ctx->device)
        return ORBX_EARG;
    if (const int rc_ = ctx->ready()) return rc_;
    const std::shared_ptr<KfEntry> ck = cache_get(cache, 1, key, nullptr, KF, ctx->s());
    if (!ck) return ORBX_EDEVICE;
    return fuse_common(ctx, KF, Tcw, Ow, mp, th, inv_level_sigma2, best_idx, nfused, ck.get());
}

}  // extern "C"
