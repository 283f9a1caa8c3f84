/*
 * orb_oracle_frame.c -- CPU restatement of the Frame-level consumers of the extractor and
 * matcher on the hot path's "next" rows. TEST INFRASTRUCTURE ONLY (see
 * orb_oracle.h for who may load it and the parity status).
 *
 *   oc_compute_stereo_matches  Frame::ComputeStereoMatches
 *                              (ORB_SLAM2.1/src/Frame.cc:470-641)
 */
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

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
