/*
 * orb_oracle_frame.c -- CPU restatement of the Frame-level consumers of the extractor and
 * matcher on the hot path's "next" rows. TEST INFRASTRUCTURE ONLY (see
 * orb_oracle.h for who may load it and the parity status).
 *
 *   oc_compute_stereo_matches  Frame::ComputeStereoMatches
 *                              (ORB_SLAM2.1/src/Frame.cc:470-641)
 *   oc_search_by_projection_*  ORBmatcher::SearchByProjection x4 (ORBmatcher.cc:45-129,
 *                              1328-1470, 1472-1599, 290-403) with Frame/KeyFrame::
 *                              GetFeaturesInArea and AssignFeaturesToGrid
 */
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

static int imax(int a, int b) { return a > b ? a : b; }
static int imin(int a, int b) { return a < b ? a : b; }

#define TH_HIGH 100 /* ORBmatcher.cc:37 */
#define TH_LOW 50   /* ORBmatcher.cc:38 */

typedef struct { int* v; int n, cap; } rowvec;
static void rowvec_push(rowvec* r, int x) {
    if (r->n == r->cap) {
        r->cap = r->cap ? 2 * r->cap : 8;
        r->v = (int*)realloc(r->v, sizeof(int) * (size_t)r->cap);
    }
    r->v[r->n++] = x;
}

typedef struct { int first, second; } dist_idx; /* vector<pair<int,int>> vDistIdx (Frame.cc:504) */
static int dist_idx_cmp(const void* a, const void* b) {
    const dist_idx* p = (const dist_idx*)a;
    const dist_idx* q = (const dist_idx*)b;
    if (p->first != q->first) return p->first < q->first ? -1 : 1;
    return p->second < q->second ? -1 : (p->second > q->second);
}

/* cv::norm(IL, IR, NORM_L1) of two continuous 11x11 CV_32F mats: OpenCV 3.x normDiffL1_32f
 * accumulates |a-b| (float difference) in double. */
static double norm_l1_f32(const float* a, const float* b, int n) {
    double s = 0;
    for (int i = 0; i < n; i++) s += fabs((double)(a[i] - b[i]));
    return s;
}

/* Frame::ComputeStereoMatches (Frame.cc:470-641). left/right hold the pyramids of the last
 * extraction of the two images (mpORBextractorLeft/Right->mvImagePyramid); kps are the
 * extractor outputs (mvKeys / mvKeysRight, level-0 coordinates). uright/depth: N floats.
 * Returns the number of keypoints left with a stereo match. ORBX_EARG where the reference
 * would throw (a correlation window outside the level: cv::Mat::colRange asserts). */
int oc_compute_stereo_matches(const oc_extractor* left, const oc_extractor* right, const orbx_kp* kpsL,
                              const uint8_t* descL, int N, const orbx_kp* kpsR, const uint8_t* descR, int Nr,
                              float mbf, float mb, float* uright, float* depth) {
    float scale[32], inv_scale[32], sigma2[32], inv_sigma2[32];
    int32_t nfeat[32], umax[16];
    oc_get_tables(left, scale, inv_scale, sigma2, inv_sigma2, nfeat, umax);
    for (int i = 0; i < N; i++) { /* :472-473 */
        uright[i] = -1.0f;
        depth[i] = -1.0f;
    }
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2; /* :475 */
    int nRows = 0, w0 = 0;
    oc_level_size(left, 0, &w0, &nRows); /* :477 */
    rowvec* vRowIndices = (rowvec*)calloc((size_t)nRows, sizeof(rowvec));
    for (int iR = 0; iR < Nr; iR++) { /* :487-498 */
        const float kpY = kpsR[iR].y;
        const float r = 2.0f * scale[kpsR[iR].octave];
        const int maxr = (int)ceilf(kpY + r);
        const int minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rowvec_push(&vRowIndices[yi], iR); /* out of range is UB there */
    }
    const float minZ = mb; /* :501-503 */
    const float minD = 0;
    const float maxD = mbf / minZ;
    dist_idx* vDistIdx = (dist_idx*)malloc(sizeof(dist_idx) * (size_t)(N > 0 ? N : 1));
    int nDist = 0;
    int rc = 0;
    for (int iL = 0; iL < N; iL++) { /* :508-622 */
        const orbx_kp* kpL = &kpsL[iL];
        const int levelL = kpL->octave;
        const float vL = kpL->y;
        const float uL = kpL->x;
        const size_t row = (size_t)vL;
        if (row >= (size_t)nRows) continue;
        const rowvec* vCandidates = &vRowIndices[row];
        if (vCandidates->n == 0) continue;
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH;
        size_t bestIdxR = 0;
        const uint8_t* dL = descL + 32 * (size_t)iL;
        for (int iC = 0; iC < vCandidates->n; iC++) { /* :531-550 */
            const int iR = vCandidates->v[iC];
            const orbx_kp* kpR = &kpsR[iR];
            if (kpR->octave < levelL - 1 || kpR->octave > levelL + 1) continue;
            const float uR = kpR->x;
            if (uR >= minU && uR <= maxU) {
                const int dist = oc_descriptor_distance(dL, descR + 32 * (size_t)iR);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = (size_t)iR;
                }
            }
        }
        if (bestDist >= thOrbDist) continue; /* :553 */
        /* subpixel match by correlation (:555-621) */
        const float uR0 = kpsR[bestIdxR].x;
        const float scaleFactor = inv_scale[kpL->octave];
        const float scaleduL = roundf(kpL->x * scaleFactor);
        const float scaledvL = roundf(kpL->y * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const int w = 5;
        int lw, lh, rw, rh;
        oc_level_size(left, kpL->octave, &lw, &lh);
        oc_level_size(right, kpL->octave, &rw, &rh);
        const uint8_t* PL = oc_pyramid(left, kpL->octave);
        const uint8_t* PR = oc_pyramid(right, kpL->octave);
        const int r0 = (int)(scaledvL - w), r1 = (int)(scaledvL + w + 1);
        const int c0 = (int)(scaleduL - w), c1 = (int)(scaleduL + w + 1);
        if (r0 < 0 || r1 > lh || r1 > rh || c0 < 0 || c1 > lw) { rc = ORBX_EARG; continue; }
        float IL[11 * 11];
        for (int y = 0; y < 11; y++)
            for (int x = 0; x < 11; x++) IL[11 * y + x] = (float)PL[(size_t)(r0 + y) * lw + c0 + x];
        {
            const float cL = IL[11 * w + w];
            for (int k = 0; k < 121; k++) IL[k] = IL[k] - cL * 1.0f;
        }
        int bestDistS = INT_MAX;
        int bestincR = 0;
        const int L = 5;
        float vDists[2 * 5 + 1];
        const float iniu = scaleduR0 + L - w;
        const float endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= rw) continue;
        int bad = 0;
        for (int incR = -L; incR <= +L; incR++) { /* :590-603 */
            const int cc0 = (int)(scaleduR0 + incR - w);
            if (cc0 < 0 || cc0 + 11 > rw) { bad = 1; break; }
            float IR[11 * 11];
            for (int y = 0; y < 11; y++)
                for (int x = 0; x < 11; x++) IR[11 * y + x] = (float)PR[(size_t)(r0 + y) * rw + cc0 + x];
            const float cR = IR[11 * w + w];
            for (int k = 0; k < 121; k++) IR[k] = IR[k] - cR * 1.0f;
            const float dist = (float)norm_l1_f32(IL, IR, 121);
            if (dist < bestDistS) {
                bestDistS = (int)dist;
                bestincR = incR;
            }
            vDists[L + incR] = dist;
        }
        if (bad) { rc = ORBX_EARG; continue; }
        if (bestincR == -L || bestincR == L) continue;
        const float dist1 = vDists[L + bestincR - 1]; /* parabola fit (:609-616) */
        const float dist2 = vDists[L + bestincR];
        const float dist3 = vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[kpL->octave] * ((float)scaleduR0 + (float)bestincR + deltaR); /* :619 */
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) { /* :623-633 */
            if (disparity <= 0) {
                disparity = 0.01;
                bestuR = uL - 0.01;
            }
            depth[iL] = mbf / disparity;
            uright[iL] = bestuR;
            vDistIdx[nDist].first = bestDistS;
            vDistIdx[nDist].second = iL;
            nDist++;
        }
    }
    int nkept = nDist;
    if (nDist > 0) { /* :636-650 (an empty vDistIdx is UB there) */
        qsort(vDistIdx, (size_t)nDist, sizeof(dist_idx), dist_idx_cmp);
        const float median = (float)vDistIdx[nDist / 2].first;
        const float thDist = 1.5f * 1.4f * median;
        for (int i = nDist - 1; i >= 0; i--) {
            if (vDistIdx[i].first < thDist) break;
            uright[vDistIdx[i].second] = -1;
            depth[vDistIdx[i].second] = -1;
            nkept--;
        }
    }
    for (int i = 0; i < nRows; i++) free(vRowIndices[i].v);
    free(vRowIndices);
    free(vDistIdx);
    return rc ? rc : nkept;
}

/* ===================================================================================== */
/* SearchByProjection x4 + Frame/KeyFrame::GetFeaturesInArea                             */
/* ===================================================================================== */
#define FRAME_GRID_ROWS 48 /* Frame.h:37 */
#define FRAME_GRID_COLS 64 /* Frame.h:38 */
#define HISTO_LENGTH 30    /* ORBmatcher.cc:39 */

/* its own push (not rowvec_push through a cast: the two struct types may not alias under -O3's strict
 * aliasing, which let GCC keep the memset's zero counts of a local ivec2 array across the pushes) */
typedef struct { int* v; int n, cap; } ivec2;
static void iv_push(ivec2* s, int x) {
    if (s->n == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 8;
        s->v = (int*)realloc(s->v, sizeof(int) * (size_t)s->cap);
    }
    s->v[s->n++] = x;
}

/* Frame::AssignFeaturesToGrid + PosInGrid (Frame.cc:235-250, 391-401): mGrid[ix][iy] lists in
 * feature order. round() of a float (half away from zero). */
typedef struct { ivec2 cell[FRAME_GRID_COLS][FRAME_GRID_ROWS]; } ogrid;
static ogrid* grid_build(const orbm_frame_view* F) {
    ogrid* g = (ogrid*)calloc(1, sizeof(ogrid));
    for (int i = 0; i < F->n; i++) {
        const int posX = (int)roundf((F->x[i] - F->min_x) * F->grid_w_inv);
        const int posY = (int)roundf((F->y[i] - F->min_y) * F->grid_h_inv);
        if (posX < 0 || posX >= FRAME_GRID_COLS || posY < 0 || posY >= FRAME_GRID_ROWS) continue;
        iv_push(&g->cell[posX][posY], i);
    }
    return g;
}
static void grid_free(ogrid* g) {
    for (int i = 0; i < FRAME_GRID_COLS; i++)
        for (int j = 0; j < FRAME_GRID_ROWS; j++) free(g->cell[i][j].v);
    free(g);
}

/* Frame::GetFeaturesInArea (Frame.cc:332-389); KeyFrame::GetFeaturesInArea (KeyFrame.cc:569-608)
 * is the same with minLevel = maxLevel = -1. Appends to out (cleared first). */
static void features_in_area(const orbm_frame_view* F, const ogrid* g, float x, float y, float r, int minLevel,
                             int maxLevel, ivec2* out) {
    out->n = 0;
    const int nMinCellX = imax(0, (int)floorf((x - F->min_x - r) * F->grid_w_inv));
    if (nMinCellX >= FRAME_GRID_COLS) return;
    const int nMaxCellX = imin(FRAME_GRID_COLS - 1, (int)ceilf((x - F->min_x + r) * F->grid_w_inv));
    if (nMaxCellX < 0) return;
    const int nMinCellY = imax(0, (int)floorf((y - F->min_y - r) * F->grid_h_inv));
    if (nMinCellY >= FRAME_GRID_ROWS) return;
    const int nMaxCellY = imin(FRAME_GRID_ROWS - 1, (int)ceilf((y - F->min_y + r) * F->grid_h_inv));
    if (nMaxCellY < 0) return;
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const ivec2* vCell = &g->cell[ix][iy];
            for (int j = 0; j < vCell->n; j++) {
                const int k = vCell->v[j];
                if (bCheckLevels) {
                    if (F->octave[k] < minLevel) continue;
                    if (maxLevel >= 0)
                        if (F->octave[k] > maxLevel) continue;
                }
                const float distx = F->x[k] - x;
                const float disty = F->y[k] - y;
                if (fabsf(distx) < r && fabsf(disty) < r) iv_push(out, k);
            }
        }
    }
}

/* cv::Mat float arithmetic as pinned in DESIGN.md: A*x+c with A 3x3 and x 3x1 is OpenCV's
 * small-matrix gemm path (float products and sums, then (float)(t*alpha + c*beta) in double);
 * A.t()*x (GEMM_1_T) is the generic path (double accumulation); norm / dot accumulate in double. */
static void gemm33_fast(const float* A, int astep, const float* x, const float* c, float* d) {
    for (int i = 0; i < 3; i++) {
        const float* a = A + i * astep;
        const float t0 = a[0] * x[0] + a[1] * x[1] + a[2] * x[2];
        d[i] = (float)((double)t0 * 1.0 + (double)c[i] * 1.0);
    }
}
static void gemm33t_neg(const float* A, int astep, const float* x, float* d) {
    for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += (double)A[k * astep + i] * (double)x[k];
        d[i] = (float)(-1.0 * s);
    }
}
static float norm3(const float* v) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)v[k] * (double)v[k];
    return (float)sqrt(s);
}
static double dot3(const float* a, const float* b) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)a[k] * (double)b[k];
    return s;
}

/* MapPoint::PredictScale (MapPoint.cc:385-417): log of a float = logf (pinned) */
static int predict_scale(float max_dist, float currentDist, const orbm_frame_view* F) {
    const float ratio = max_dist / currentDist;
    int nScale = (int)ceilf(logf(ratio) / F->log_scale_factor);
    if (nScale < 0)
        nScale = 0;
    else if (nScale >= F->nlevels)
        nScale = F->nlevels - 1;
    return nScale;
}

static void three_maxima2(const ivec2* histo, int L, int* ind1, int* ind2, int* ind3) { /* ORBmatcher.cc:1601-1642 */
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = histo[i].n;
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            *ind3 = *ind2; *ind2 = i;
        } else if (s > max3) {
            max3 = s; *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        *ind2 = -1; *ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        *ind3 = -1;
    }
}

/* the rotation-consistency block shared by ORBmatcher.cc:1437-1467 and 1578-1596 */
static int rot_push_bin(float a1, float a2) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}
static int rot_filter(ivec2* rotHist, int32_t* match, int nmatches) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima2(rotHist, HISTO_LENGTH, &ind1, &ind2, &ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
        if (i != ind1 && i != ind2 && i != ind3) {
            for (int j = 0; j < rotHist[i].n; j++) {
                match[rotHist[i].v[j]] = -2; /* = NULL */
                nmatches--;
            }
        }
    }
    return nmatches;
}

static int has(const uint8_t* a, int i) { return a ? a[i] != 0 : 0; }

/* ORBmatcher::RadiusByViewingCos (ORBmatcher.cc:131-137) */
static float radius_by_viewing_cos(float viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) (ORBmatcher.cc:45-129) */
int oc_search_by_projection_local(const orbm_frame_view* F, const orbm_mappoints* mp, float th, float nnratio,
                                  int32_t* match) {
    int nmatches = 0;
    const int bFactor = th != 1.0;
    ogrid* g = grid_build(F);
    uint8_t* occ = (uint8_t*)malloc((size_t)F->n + 1);
    for (int i = 0; i < F->n; i++) {
        occ[i] = (uint8_t)has(F->occupied, i);
        match[i] = -1;
    }
    ivec2 vIndices = {0};
    for (int iMP = 0; iMP < mp->n; iMP++) {
        if (!mp->track_in_view[iMP]) continue;
        if (has(mp->bad, iMP)) continue;
        const int nPredictedLevel = mp->track_level[iMP];
        float r = radius_by_viewing_cos(mp->track_view_cos[iMP]);
        if (bFactor) r *= th;
        features_in_area(F, g, mp->track_proj_x[iMP], mp->track_proj_y[iMP], r * F->scale_factors[nPredictedLevel],
                         nPredictedLevel - 1, nPredictedLevel, &vIndices);
        if (vIndices.n == 0) continue;
        const uint8_t* MPdescriptor = mp->desc + 32 * (size_t)iMP;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int k = 0; k < vIndices.n; k++) {
            const int idx = vIndices.v[k];
            if (occ[idx]) continue; /* mvpMapPoints[idx] && Observations() > 0 */
            if (F->uright && F->uright[idx] > 0) {
                const float er = fabsf(mp->track_proj_xr[iMP] - F->uright[idx]);
                if (er > r * F->scale_factors[nPredictedLevel]) continue;
            }
            const int dist = oc_descriptor_distance(MPdescriptor, F->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = F->octave[idx];
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F->octave[idx];
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            match[bestIdx] = iMP;
            occ[bestIdx] = (uint8_t)has(mp->has_obs, iMP);
            nmatches++;
        }
    }
    free(vIndices.v);
    free(occ);
    grid_free(g);
    return nmatches;
}

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 * (ORBmatcher.cc:1328-1470) */
int oc_search_by_projection_last_frame(const orbm_frame_view* F, const float* Tcw_c, const orbm_mappoints* mp,
                                       const float* Tcw_l, float th, int bMono, int checkOri, int32_t* match) {
    int nmatches = 0;
    ivec2 rotHist[HISTO_LENGTH];
    memset(rotHist, 0, sizeof(rotHist));
    const float* Rcw = Tcw_c; /* rowRange(0,3).colRange(0,3) of a 4x4: row step 4 */
    const float tcw[3] = {Tcw_c[3], Tcw_c[7], Tcw_c[11]};
    float twc[3];
    gemm33t_neg(Rcw, 4, tcw, twc);
    const float* Rlw = Tcw_l;
    const float tlw[3] = {Tcw_l[3], Tcw_l[7], Tcw_l[11]};
    float tlc[3];
    gemm33_fast(Rlw, 4, twc, tlw, tlc);
    const int bForward = tlc[2] > F->b && !bMono;
    const int bBackward = -tlc[2] > F->b && !bMono;
    ogrid* g = grid_build(F);
    uint8_t* occ = (uint8_t*)malloc((size_t)F->n + 1);
    for (int i = 0; i < F->n; i++) {
        occ[i] = (uint8_t)has(F->occupied, i);
        match[i] = -1;
    }
    ivec2 vIndices2 = {0};
    for (int i = 0; i < mp->n; i++) {
        if (has(mp->skip, i)) continue; /* !pMP || mvbOutlier[i] */
        float x3Dc[3];
        gemm33_fast(Rcw, 4, mp->pos + 3 * (size_t)i, tcw, x3Dc);
        const float xc = x3Dc[0];
        const float yc = x3Dc[1];
        const float invzc = 1.0 / x3Dc[2];
        if (invzc < 0) continue;
        const float u = F->fx * xc * invzc + F->cx;
        const float v = F->fy * yc * invzc + F->cy;
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        const int nLastOctave = mp->octave[i];
        const float radius = th * F->scale_factors[nLastOctave];
        if (bForward)
            features_in_area(F, g, u, v, radius, nLastOctave, -1, &vIndices2);
        else if (bBackward)
            features_in_area(F, g, u, v, radius, 0, nLastOctave, &vIndices2);
        else
            features_in_area(F, g, u, v, radius, nLastOctave - 1, nLastOctave + 1, &vIndices2);
        if (vIndices2.n == 0) continue;
        const uint8_t* dMP = mp->desc + 32 * (size_t)i;
        int bestDist = 256, bestIdx2 = -1;
        for (int k = 0; k < vIndices2.n; k++) {
            const int i2 = vIndices2.v[k];
            if (occ[i2]) continue;
            if (F->uright && F->uright[i2] > 0) {
                const float ur = u - F->bf * invzc;
                const float er = fabsf(ur - F->uright[i2]);
                if (er > radius) continue;
            }
            const int dist = oc_descriptor_distance(dMP, F->desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            match[bestIdx2] = i;
            occ[bestIdx2] = (uint8_t)has(mp->has_obs, i);
            nmatches++;
            if (checkOri) iv_push(&rotHist[rot_push_bin(mp->angle[i], F->angle[bestIdx2])], bestIdx2);
        }
    }
    if (checkOri) nmatches = rot_filter(rotHist, match, nmatches);
    for (int i = 0; i < HISTO_LENGTH; i++) free(rotHist[i].v);
    free(vIndices2.v);
    free(occ);
    grid_free(g);
    return nmatches;
}

/* ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
 * (ORBmatcher.cc:1472-1599) */
int oc_search_by_projection_keyframe(const orbm_frame_view* F, const float* Tcw_c, const orbm_mappoints* mp, float th,
                                     int ORBdist, int checkOri, int32_t* match) {
    int nmatches = 0;
    const float* Rcw = Tcw_c;
    const float tcw[3] = {Tcw_c[3], Tcw_c[7], Tcw_c[11]};
    float Ow[3];
    gemm33t_neg(Rcw, 4, tcw, Ow);
    ivec2 rotHist[HISTO_LENGTH];
    memset(rotHist, 0, sizeof(rotHist));
    ogrid* g = grid_build(F);
    uint8_t* occ = (uint8_t*)malloc((size_t)F->n + 1);
    for (int i = 0; i < F->n; i++) {
        occ[i] = (uint8_t)has(F->occupied, i);
        match[i] = -1;
    }
    ivec2 vIndices2 = {0};
    for (int i = 0; i < mp->n; i++) {
        if (has(mp->skip, i) || has(mp->bad, i)) continue; /* !pMP, isBad, sAlreadyFound.count */
        const float* x3Dw = mp->pos + 3 * (size_t)i;
        float x3Dc[3];
        gemm33_fast(Rcw, 4, x3Dw, tcw, x3Dc);
        const float xc = x3Dc[0];
        const float yc = x3Dc[1];
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
        features_in_area(F, g, u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1, &vIndices2);
        if (vIndices2.n == 0) continue;
        const uint8_t* dMP = mp->desc + 32 * (size_t)i;
        int bestDist = 256, bestIdx2 = -1;
        for (int k = 0; k < vIndices2.n; k++) {
            const int i2 = vIndices2.v[k];
            if (occ[i2]) continue;
            const int dist = oc_descriptor_distance(dMP, F->desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= ORBdist) {
            match[bestIdx2] = i;
            occ[bestIdx2] = 1;
            nmatches++;
            if (checkOri) iv_push(&rotHist[rot_push_bin(mp->angle[i], F->angle[bestIdx2])], bestIdx2);
        }
    }
    if (checkOri) nmatches = rot_filter(rotHist, match, nmatches);
    for (int i = 0; i < HISTO_LENGTH; i++) free(rotHist[i].v);
    free(vIndices2.v);
    free(occ);
    grid_free(g);
    return nmatches;
}

/* ORBmatcher::SearchByProjection(KeyFrame*, cv::Mat Scw, vpPoints, vpMatched, th)
 * (ORBmatcher.cc:290-403) */
int oc_search_by_projection_sim3(const orbm_frame_view* KF, const float* Scw, const orbm_mappoints* mp, int th,
                                 int32_t* match) {
    /* Decompose Scw: scw = sqrt(row0.dot(row0)); Rcw = sRcw/scw and tcw = t/scw are
     * convertTo with scale (float)(1./scw); Ow = -Rcw.t()*tcw */
    const double d0 = dot3(Scw, Scw);
    const float scw = (float)sqrt(d0);
    const float inv = (float)(1. / (double)scw);
    float Rcw[9], tcw[3], Ow[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Rcw[3 * r + c] = Scw[4 * r + c] * inv;
        tcw[r] = Scw[4 * r + 3] * inv;
    }
    gemm33t_neg(Rcw, 3, tcw, Ow);
    int nmatches = 0;
    ogrid* g = grid_build(KF);
    uint8_t* occ = (uint8_t*)malloc((size_t)KF->n + 1);
    for (int i = 0; i < KF->n; i++) {
        occ[i] = (uint8_t)has(KF->occupied, i);
        match[i] = -1;
    }
    ivec2 vIndices = {0};
    for (int iMP = 0; iMP < mp->n; iMP++) {
        if (has(mp->bad, iMP) || has(mp->skip, iMP)) continue;
        const float* p3Dw = mp->pos + 3 * (size_t)iMP;
        float p3Dc[3];
        gemm33_fast(Rcw, 3, p3Dw, tcw, p3Dc);
        if (p3Dc[2] < 0.0) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = KF->fx * x + KF->cx;
        const float v = KF->fy * y + KF->cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue; /* IsInImage */
        const float maxDistance = 1.2f * mp->max_dist[iMP];
        const float minDistance = 0.8f * mp->min_dist[iMP];
        const float PO[3] = {p3Dw[0] - Ow[0], p3Dw[1] - Ow[1], p3Dw[2] - Ow[2]};
        const float dist = norm3(PO);
        if (dist < minDistance || dist > maxDistance) continue;
        if (dot3(PO, mp->normal + 3 * (size_t)iMP) < 0.5 * dist) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[iMP], dist, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        features_in_area(KF, g, u, v, radius, -1, -1, &vIndices);
        if (vIndices.n == 0) continue;
        const uint8_t* dMP = mp->desc + 32 * (size_t)iMP;
        int bestDist = 256, bestIdx = -1;
        for (int k = 0; k < vIndices.n; k++) {
            const int idx = vIndices.v[k];
            if (occ[idx]) continue;
            const int kpLevel = KF->octave[idx];
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int dist2 = oc_descriptor_distance(dMP, KF->desc + 32 * (size_t)idx);
            if (dist2 < bestDist) {
                bestDist = dist2;
                bestIdx = idx;
            }
        }
        if (bestDist <= TH_LOW) {
            match[bestIdx] = iMP;
            occ[bestIdx] = 1;
            nmatches++;
        }
    }
    free(vIndices.v);
    free(occ);
    grid_free(g);
    return nmatches;
}

/* ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, th) (ORBmatcher.cc:825-975),
 * the per-MapPoint search: best_idx[i] = bestIdx when bestDist <= TH_LOW (the reference then fuses or
 * adds the observation, :947-971, on the caller's side), else -1. mp: skip = NULL entry or
 * IsInKeyFrame(pKF), bad, pos, normal, desc, min_dist, max_dist. Tcw = pKF's pose (4x4 row-major),
 * Ow = pKF->GetCameraCenter(), inv_sigma2 = mvInvLevelSigma2. Returns nFused. */
int oc_fuse(const orbm_frame_view* KF, const float* Tcw, const float* Ow, const orbm_mappoints* mp, float th,
            const float* inv_sigma2, int32_t* best_idx) {
    const float tcw[3] = {Tcw[3], Tcw[7], Tcw[11]};
    int nFused = 0;
    ogrid* g = grid_build(KF);
    ivec2 vIndices = {0};
    for (int i = 0; i < mp->n; i++) {
        best_idx[i] = -1;
        if (has(mp->skip, i) || has(mp->bad, i)) continue; /* :844-850 */
        const float* p3Dw = mp->pos + 3 * (size_t)i;
        float p3Dc[3];
        gemm33_fast(Tcw, 4, p3Dw, tcw, p3Dc); /* Rcw*p3Dw + tcw */
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = KF->fx * x + KF->cx;
        const float v = KF->fy * y + KF->cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue; /* IsInImage */
        const float ur = u - KF->bf * invz;
        const float maxDistance = 1.2f * mp->max_dist[i];
        const float minDistance = 0.8f * mp->min_dist[i];
        const float PO[3] = {p3Dw[0] - Ow[0], p3Dw[1] - Ow[1], p3Dw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        if (dot3(PO, mp->normal + 3 * (size_t)i) < 0.5 * dist3D) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[i], dist3D, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        features_in_area(KF, g, u, v, radius, -1, -1, &vIndices);
        if (vIndices.n == 0) continue;
        const uint8_t* dMP = mp->desc + 32 * (size_t)i;
        int bestDist = 256, bestIdx = -1;
        for (int k = 0; k < vIndices.n; k++) {
            const int idx = vIndices.v[k];
            const int kpLevel = KF->octave[idx];
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const float kpx = KF->x[idx], kpy = KF->y[idx];
            const float ex = u - kpx, ey = v - kpy;
            if (KF->uright && KF->uright[idx] >= 0) { /* reprojection error, stereo (:907-918) */
                const float er = ur - KF->uright[idx];
                const float e2 = ex * ex + ey * ey + er * er;
                if (e2 * inv_sigma2[kpLevel] > 7.8) continue;
            } else { /* mono (:920-929) */
                const float e2 = ex * ex + ey * ey;
                if (e2 * inv_sigma2[kpLevel] > 5.99) continue;
            }
            const int dist = oc_descriptor_distance(dMP, KF->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        if (bestDist <= TH_LOW) {
            best_idx[i] = bestIdx;
            nFused++;
        }
    }
    free(vIndices.v);
    grid_free(g);
    return nFused;
}

/* ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, th, vpReplacePoint)
 * (ORBmatcher.cc:977-1100), the per-MapPoint search: best_idx[i] as in oc_fuse (the caller then sets
 * vpReplacePoint[i] or adds the observation, :1084-1096). mp: skip = in spAlreadyFound
 * (pKF->GetMapPoints() at the call), bad, pos, normal, desc, min_dist, max_dist. Returns nFused. */
int oc_fuse_sim3(const orbm_frame_view* KF, const float* Scw, const orbm_mappoints* mp, float th, int32_t* best_idx) {
    const double d0 = dot3(Scw, Scw); /* :987-991, decomposition as in oc_search_by_projection_sim3 */
    const float scw = (float)sqrt(d0);
    const float inv = (float)(1. / (double)scw);
    float Rcw[9], tcw[3], Ow[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Rcw[3 * r + c] = Scw[4 * r + c] * inv;
        tcw[r] = Scw[4 * r + 3] * inv;
    }
    gemm33t_neg(Rcw, 3, tcw, Ow);
    int nFused = 0;
    ogrid* g = grid_build(KF);
    ivec2 vIndices = {0};
    for (int iMP = 0; iMP < mp->n; iMP++) {
        best_idx[iMP] = -1;
        if (has(mp->bad, iMP) || has(mp->skip, iMP)) continue; /* :1005-1006 */
        const float* p3Dw = mp->pos + 3 * (size_t)iMP;
        float p3Dc[3];
        gemm33_fast(Rcw, 3, p3Dw, tcw, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = (float)(1.0 / (double)p3Dc[2]); /* 1.0/ (double) here, 1/ (float) in :322 */
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = KF->fx * x + KF->cx;
        const float v = KF->fy * y + KF->cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue; /* IsInImage */
        const float maxDistance = 1.2f * mp->max_dist[iMP];
        const float minDistance = 0.8f * mp->min_dist[iMP];
        const float PO[3] = {p3Dw[0] - Ow[0], p3Dw[1] - Ow[1], p3Dw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        if (dot3(PO, mp->normal + 3 * (size_t)iMP) < 0.5 * dist3D) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[iMP], dist3D, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        features_in_area(KF, g, u, v, radius, -1, -1, &vIndices);
        if (vIndices.n == 0) continue;
        const uint8_t* dMP = mp->desc + 32 * (size_t)iMP;
        int bestDist = INT_MAX, bestIdx = -1;
        for (int k = 0; k < vIndices.n; k++) {
            const int idx = vIndices.v[k];
            const int kpLevel = KF->octave[idx];
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int dist = oc_descriptor_distance(dMP, KF->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        if (bestDist <= TH_LOW) {
            best_idx[iMP] = bestIdx;
            nFused++;
        }
    }
    free(vIndices.v);
    grid_free(g);
    return nFused;
}

/* ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.cc:405-520).
 * F1: mvKeysUn octave / angle and mDescriptors (x, y unused); F2: the grid side (F2.GetFeaturesInArea,
 * mvKeysUn, mDescriptors). prev_xy[2*i1] = vbPrevMatched[i1] (x, y), overwritten with F2.mvKeysUn[match].pt
 * for every matched i1 (:514-517). match12[F1->n] = vnMatches12. Returns nmatches. */
int oc_search_for_initialization(const orbm_frame_view* F1, const orbm_frame_view* F2, float* prev_xy, int windowSize,
                                 float nnratio, int checkOri, int32_t* match12) {
    int nmatches = 0;
    for (int i = 0; i < F1->n; i++) match12[i] = -1; /* :408 */
    ivec2 rotHist[HISTO_LENGTH];
    memset(rotHist, 0, sizeof(rotHist));
    const float factor = 1.0f / HISTO_LENGTH; /* :413 */
    int* vMatchedDistance = (int*)malloc(sizeof(int) * ((size_t)F2->n + 1));
    int* vnMatches21 = (int*)malloc(sizeof(int) * ((size_t)F2->n + 1));
    for (int i = 0; i < F2->n; i++) {
        vMatchedDistance[i] = INT_MAX; /* :415-416 */
        vnMatches21[i] = -1;
    }
    ogrid* g = grid_build(F2);
    ivec2 vIndices2 = {0};
    for (int i1 = 0; i1 < F1->n; i1++) { /* :418 */
        const int level1 = F1->octave[i1];
        if (level1 > 0) continue;
        features_in_area(F2, g, prev_xy[2 * i1], prev_xy[2 * i1 + 1], (float)windowSize, level1, level1, &vIndices2);
        if (vIndices2.n == 0) continue;
        const uint8_t* d1 = F1->desc + 32 * (size_t)i1;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int k = 0; k < vIndices2.n; k++) { /* :436-457 */
            const int i2 = vIndices2.v[k];
            const int dist = oc_descriptor_distance(d1, F2->desc + 32 * (size_t)i2);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) { /* :459-485 */
            if ((float)bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    match12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                match12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) {
                    float rot = F1->angle[i1] - F2->angle[bestIdx2];
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == HISTO_LENGTH) bin = 0;
                    iv_push(&rotHist[bin], i1);
                }
            }
        }
    }
    if (checkOri) { /* :489-512: the bins keep matches that a later i1 took away (counted by ComputeThreeMaxima) */
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima2(rotHist, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j = 0; j < rotHist[i].n; j++) {
                const int idx1 = rotHist[i].v[j];
                if (match12[idx1] >= 0) {
                    match12[idx1] = -1;
                    nmatches--;
                }
            }
        }
    }
    for (int i1 = 0; i1 < F1->n; i1++) /* :514-517 */
        if (match12[i1] >= 0) {
            prev_xy[2 * i1] = F2->x[match12[i1]];
            prev_xy[2 * i1 + 1] = F2->y[match12[i1]];
        }
    for (int i = 0; i < HISTO_LENGTH; i++) free(rotHist[i].v);
    free(vIndices2.v);
    free(vMatchedDistance);
    free(vnMatches21);
    grid_free(g);
    return nmatches;
}

/* one direction of SearchBySim3 (ORBmatcher.cc:1148-1225 / 1228-1305): MapPoints of the source keyframe
 * (mp: skip = NULL or vbAlreadyMatched, bad, pos, desc, min_dist, max_dist) through Tsw = (Rsw, tsw) into the
 * source camera, then (sR, t) into the target keyframe KF, projected with the camera (fx, fy, cx, cy) of pKF1
 * (the reference reads pKF1's intrinsics for both directions, :1105-1108); vnMatch[i] = best KF keypoint
 * (first strict minimum, octave in [nPredictedLevel-1, nPredictedLevel]) if bestDist <= TH_HIGH, else -1 */
static void sim3_direction(const orbm_frame_view* KF, const float* Tsw, const orbm_mappoints* mp, const float* sR,
                           const float* t, float fx, float fy, float cx, float cy, float th, int32_t* vnMatch) {
    const float Rsw[9] = {Tsw[0], Tsw[1], Tsw[2], Tsw[4], Tsw[5], Tsw[6], Tsw[8], Tsw[9], Tsw[10]};
    const float tsw[3] = {Tsw[3], Tsw[7], Tsw[11]};
    ogrid* g = grid_build(KF);
    ivec2 vIndices = {0};
    for (int i = 0; i < mp->n; i++) {
        vnMatch[i] = -1;
        if (has(mp->skip, i) || has(mp->bad, i)) continue; /* :1152-1156 */
        const float* p3Dw = mp->pos + 3 * (size_t)i;
        float p3Dcs[3], p3Dct[3];
        gemm33_fast(Rsw, 3, p3Dw, tsw, p3Dcs); /* R1w*p3Dw + t1w */
        gemm33_fast(sR, 3, p3Dcs, t, p3Dct);  /* sR21*p3Dc1 + t21 */
        if (p3Dct[2] < 0.0) continue;
        const float invz = (float)(1.0 / (double)p3Dct[2]);
        const float x = p3Dct[0] * invz;
        const float y = p3Dct[1] * invz;
        const float u = fx * x + cx;
        const float v = fy * y + cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue; /* IsInImage */
        const float maxDistance = 1.2f * mp->max_dist[i];
        const float minDistance = 0.8f * mp->min_dist[i];
        const float dist3D = norm3(p3Dct);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = predict_scale(mp->max_dist[i], dist3D, KF);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        features_in_area(KF, g, u, v, radius, -1, -1, &vIndices);
        if (vIndices.n == 0) continue;
        const uint8_t* dMP = mp->desc + 32 * (size_t)i;
        int bestDist = INT_MAX, bestIdx = -1;
        for (int k = 0; k < vIndices.n; k++) {
            const int idx = vIndices.v[k];
            const int oct = KF->octave[idx];
            if (oct < nPredictedLevel - 1 || oct > nPredictedLevel) continue;
            const int dist = oc_descriptor_distance(dMP, KF->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        if (bestDist <= TH_HIGH) vnMatch[i] = bestIdx;
    }
    free(vIndices.v);
    grid_free(g);
}

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:1102-1326).
 * T1w / T2w: the keyframes' poses (4x4 row-major; GetRotation / GetTranslation); mp1 / mp2: their
 * GetMapPointMatches() with skip = NULL entry or vbAlreadyMatched1/2 (:1129-1142). match12[mp1->n] = idx2
 * where both directions agree (vpMatches12[i1] = vpMapPoints2[idx2], :1310-1323), else -1. Returns nFound. */
int oc_search_by_sim3(const orbm_frame_view* KF1, const float* T1w, const orbm_mappoints* mp1,
                      const orbm_frame_view* KF2, const float* T2w, const orbm_mappoints* mp2, float s12,
                      const float* R12, const float* t12, float th, int32_t* match12) {
    /* sR12 = s12*R12 and sR21 = (1.0/s12)*R12.t() are MatExpr scalings evaluated by convertTo with a float
     * scale; t21 = -sR21*t12 is the small-matrix gemm with alpha = -1 (:1119-1121) */
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
    int32_t* vnMatch1 = (int32_t*)malloc(sizeof(int32_t) * ((size_t)mp1->n + 1));
    int32_t* vnMatch2 = (int32_t*)malloc(sizeof(int32_t) * ((size_t)mp2->n + 1));
    sim3_direction(KF2, T1w, mp1, sR21, t21, KF1->fx, KF1->fy, KF1->cx, KF1->cy, th, vnMatch1);
    sim3_direction(KF1, T2w, mp2, sR12, t12, KF1->fx, KF1->fy, KF1->cx, KF1->cy, th, vnMatch2);
    int nFound = 0;
    for (int i1 = 0; i1 < mp1->n; i1++) { /* :1310-1323 */
        match12[i1] = -1;
        const int idx2 = vnMatch1[i1];
        if (idx2 >= 0 && idx2 < mp2->n && vnMatch2[idx2] == i1) {
            match12[i1] = idx2;
            nFound++;
        }
    }
    free(vnMatch1);
    free(vnMatch2);
    return nFound;
}

/* ===================================================================================== */
/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307)                          */
/* ===================================================================================== */
static int int_cmp(const void* a, const void* b) {
    const int x = *(const int*)a, y = *(const int*)b;
    return (x > y) - (x < y);
}

/* one MapPoint: vDescriptors = desc[0..N) (32 B rows); returns BestIdx, -1 if N == 0 */
static int distinctive_one(const uint8_t* desc, int N) {
    if (N <= 0) return -1;
    float* Distances = (float*)malloc(sizeof(float) * (size_t)N * N);
    for (int i = 0; i < N; i++) {
        Distances[(size_t)i * N + i] = 0;
        for (int j = i + 1; j < N; j++) {
            const int distij = oc_descriptor_distance(desc + 32 * (size_t)i, desc + 32 * (size_t)j);
            Distances[(size_t)i * N + j] = distij;
            Distances[(size_t)j * N + i] = distij;
        }
    }
    int BestMedian = INT_MAX, BestIdx = 0;
    int* vDists = (int*)malloc(sizeof(int) * (size_t)N);
    for (int i = 0; i < N; i++) {
        for (int j = 0; j < N; j++) vDists[j] = (int)Distances[(size_t)i * N + j];
        qsort(vDists, (size_t)N, sizeof(int), int_cmp);
        const int median = vDists[(size_t)(0.5 * (N - 1))];
        if (median < BestMedian) {
            BestMedian = median;
            BestIdx = i;
        }
    }
    free(vDists);
    free(Distances);
    return BestIdx;
}

void oc_compute_distinctive_descriptors(int npoints, const int32_t* offsets, const uint8_t* desc, int32_t* best_idx) {
    for (int p = 0; p < npoints; p++)
        best_idx[p] = distinctive_one(desc + 32 * (size_t)offsets[p], offsets[p + 1] - offsets[p]);
}
