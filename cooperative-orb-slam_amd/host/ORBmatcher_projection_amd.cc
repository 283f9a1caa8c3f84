/*
 * ORBmatcher_projection_amd.cc -- MI355X definitions of the four ORBmatcher::SearchByProjection
 * overloads (replace the same definitions in ORB_SLAM2/src/ORBmatcher.cc):
 *   SearchByProjection(Frame&, const vector<MapPoint*>&, th)                 ORBmatcher.cc:45-129
 *   SearchByProjection(Frame&, const Frame&, th, bMono)                      ORBmatcher.cc:1328-1470
 *   SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist) ORBmatcher.cc:1472-1599
 *   SearchByProjection(KeyFrame*, cv::Mat Scw, vpPoints, vpMatched, th)      ORBmatcher.cc:290-403
 * and the two Fuse overloads:
 *   Fuse(KeyFrame*, const vector<MapPoint*>&, th)                            ORBmatcher.cc:825-975
 *   Fuse(KeyFrame*, cv::Mat Scw, vpPoints, th, vpReplacePoint)               ORBmatcher.cc:977-1100
 * and SearchForInitialization (ORBmatcher.cc:405-520) and SearchBySim3 (ORBmatcher.cc:1102-1326).
 * Each call gathers what the reference reads (keypoints, descriptors, mvuRight, grid bounds, the
 * MapPoint state through the same accessors), runs orbm_search_by_projection_* (geometry prologue
 * on the host with the reference's float semantics; grid, windowed Hamming search, in-order claims
 * and the rotation histogram on the device) and writes the assignments back. MapPoint's private
 * mfMinDistance / mfMaxDistance are read through GetMinDistance() / GetMaxDistance(), two getters
 * the maintainer adds to MapPoint.h. A device failure does not throw (orbamd_status.h): the call
 * returns 0 and leaves the caller's containers and the map untouched.
 * Fuse: the device returns each MapPoint's fused keypoint (orbm_fuse*); the map updates (Replace,
 * AddObservation, AddMapPoint / vpReplacePoint) then run here in the reference's loop order, with the
 * reference's per-iteration isBad() / IsInKeyFrame() test, so an entry changed by an earlier update is
 * skipped exactly as in ORBmatcher.cc.
 */
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <set>
#include <vector>

#include "ORBmatcher.h"
#include "orbamd_status.h"
#include "orbslam_amd.h"

namespace ORB_SLAM2 {

namespace {

template <class F>
bool run(const char* what, F f) {
    orbm_ctx* c = amd::ThreadMatcher();
    return c && amd::StatusOk(f(c), what);
}

/* the Frame / KeyFrame side of a call */
struct FrameSide {
    std::vector<float> x, y, angle;
    std::vector<int32_t> octave;
    std::vector<uint8_t> occ;
    cv::Mat desc;
    orbm_frame_view v;
    template <class FK>
    void gather(FK& F, const std::vector<float>* uright, float bf, float b) {
        const size_t n = F.mvKeysUn.size();
        x.resize(n); y.resize(n); angle.resize(n); octave.resize(n);
        for (size_t i = 0; i < n; i++) {
            x[i] = F.mvKeysUn[i].pt.x;
            y[i] = F.mvKeysUn[i].pt.y;
            angle[i] = F.mvKeysUn[i].angle;
            octave[i] = F.mvKeysUn[i].octave;
        }
        desc = F.mDescriptors.isContinuous() ? F.mDescriptors : F.mDescriptors.clone();
        memset(&v, 0, sizeof(v));
        v.n = (int32_t)n;
        v.desc = n ? desc.data : nullptr;
        v.x = x.data(); v.y = y.data(); v.octave = octave.data(); v.angle = angle.data();
        v.uright = uright && !uright->empty() ? uright->data() : nullptr;
        v.min_x = F.mnMinX; v.min_y = F.mnMinY; v.max_x = F.mnMaxX; v.max_y = F.mnMaxY;
        v.grid_w_inv = F.mfGridElementWidthInv; v.grid_h_inv = F.mfGridElementHeightInv;
        v.fx = F.fx; v.fy = F.fy; v.cx = F.cx; v.cy = F.cy;
        v.bf = bf; v.b = b;
        v.nlevels = (int32_t)F.mvScaleFactors.size();
        v.scale_factors = F.mvScaleFactors.data();
        v.log_scale_factor = F.mfLogScaleFactor;
    }
    void occupied(const std::vector<uint8_t>& o) {
        occ = o;
        v.occupied = occ.data();
    }
};

/* the MapPoint side */
struct PointSide {
    std::vector<uint8_t> desc, bad, has_obs, skip, in_view;
    std::vector<float> pos, normal, mind, maxd, angle, px, py, pxr, vcos;
    std::vector<int32_t> octave, level;
    orbm_mappoints m;
    void reserve(size_t n) {
        desc.assign(32 * n, 0); bad.assign(n, 0); has_obs.assign(n, 0); skip.assign(n, 0);
        pos.assign(3 * n, 0.f); normal.assign(3 * n, 0.f); mind.assign(n, 0.f); maxd.assign(n, 0.f);
        angle.assign(n, 0.f); octave.assign(n, 0);
    }
    void point(size_t i, MapPoint* p, bool geometry) {
        bad[i] = p->isBad();
        has_obs[i] = p->Observations() > 0;
        cv::Mat d = p->GetDescriptor();
        memcpy(&desc[32 * i], d.ptr<unsigned char>(), 32);
        if (geometry) {
            cv::Mat w = p->GetWorldPos();
            for (int k = 0; k < 3; k++) pos[3 * i + k] = w.at<float>(k, 0);
            mind[i] = p->GetMinDistance();
            maxd[i] = p->GetMaxDistance();
        }
    }
    void finish(size_t n) {
        memset(&m, 0, sizeof(m));
        m.n = (int32_t)n;
        m.desc = desc.data(); m.pos = pos.data(); m.normal = normal.data(); m.min_dist = mind.data();
        m.max_dist = maxd.data(); m.bad = bad.data(); m.has_obs = has_obs.data(); m.skip = skip.data();
        m.octave = octave.data(); m.angle = angle.data();
        if (!in_view.empty()) {
            m.track_in_view = in_view.data(); m.track_proj_x = px.data(); m.track_proj_y = py.data();
            m.track_proj_xr = pxr.data(); m.track_level = level.data(); m.track_view_cos = vcos.data();
        }
    }
};

std::vector<uint8_t> occupied_obs(const std::vector<MapPoint*>& mps) {
    std::vector<uint8_t> o(mps.size());
    for (size_t i = 0; i < mps.size(); i++) o[i] = mps[i] && mps[i]->Observations() > 0;
    return o;
}

std::vector<uint8_t> occupied_any(const std::vector<MapPoint*>& mps) {
    std::vector<uint8_t> o(mps.size());
    for (size_t i = 0; i < mps.size(); i++) o[i] = mps[i] != NULL;
    return o;
}

const float* mat44(const cv::Mat& T, cv::Mat& keep) {
    keep = T.isContinuous() ? T : T.clone();
    return keep.ptr<float>();
}

/* match[i] >= 0: assign src[match[i]]; -2: the rotation filter reset it to NULL */
void apply(std::vector<MapPoint*>& dst, const std::vector<int32_t>& m, const std::vector<MapPoint*>& src) {
    for (size_t i = 0; i < dst.size(); i++) {
        if (m[i] >= 0) dst[i] = src[m[i]];
        else if (m[i] == -2) dst[i] = static_cast<MapPoint*>(NULL);
    }
}

}  // namespace

// ORBmatcher.cc:45-129
int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th) {
    FrameSide fs;
    fs.gather(F, &F.mvuRight, F.mbf, F.mb);
    fs.occupied(occupied_obs(F.mvpMapPoints));
    const size_t n = vpMapPoints.size();
    PointSide ps;
    ps.reserve(n);
    ps.in_view.assign(n, 0); ps.px.assign(n, 0.f); ps.py.assign(n, 0.f); ps.pxr.assign(n, 0.f);
    ps.level.assign(n, 0); ps.vcos.assign(n, 0.f);
    for (size_t i = 0; i < n; i++) {
        MapPoint* p = vpMapPoints[i];
        ps.in_view[i] = p->mbTrackInView;
        if (!p->mbTrackInView) continue;
        ps.point(i, p, false);
        ps.px[i] = p->mTrackProjX; ps.py[i] = p->mTrackProjY; ps.pxr[i] = p->mTrackProjXR;
        ps.level[i] = p->mnTrackScaleLevel; ps.vcos[i] = p->mTrackViewCos;
    }
    ps.finish(n);
    std::vector<int32_t> m((size_t)std::max(F.N, 1));
    int nm = 0;
    if (!run("orbm_search_by_projection_local", [&](orbm_ctx* c) {
            return orbm_search_by_projection_local(c, &fs.v, &ps.m, th, mfNNratio, m.data(), &nm);
        }))
        return 0;
    apply(F.mvpMapPoints, m, vpMapPoints);
    return nm;
}

// ORBmatcher.cc:1328-1470
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
    FrameSide fs;
    fs.gather(CurrentFrame, &CurrentFrame.mvuRight, CurrentFrame.mbf, CurrentFrame.mb);
    fs.occupied(occupied_obs(CurrentFrame.mvpMapPoints));
    const size_t n = (size_t)LastFrame.N;
    PointSide ps;
    ps.reserve(n);
    for (size_t i = 0; i < n; i++) {
        MapPoint* p = LastFrame.mvpMapPoints[i];
        ps.skip[i] = !p || LastFrame.mvbOutlier[i];
        if (ps.skip[i]) continue;
        ps.point(i, p, true);
        ps.octave[i] = LastFrame.mvKeys[i].octave;
        ps.angle[i] = LastFrame.mvKeysUn[i].angle;
    }
    ps.finish(n);
    cv::Mat kc, kl;
    std::vector<int32_t> m((size_t)std::max(CurrentFrame.N, 1));
    int nm = 0;
    if (!run("orbm_search_by_projection_last_frame", [&](orbm_ctx* c) {
            return orbm_search_by_projection_last_frame(c, &fs.v, mat44(CurrentFrame.mTcw, kc), &ps.m,
                                                       mat44(LastFrame.mTcw, kl), th, bMono ? 1 : 0,
                                                       mbCheckOrientation ? 1 : 0, m.data(), &nm);
        }))
        return 0;
    apply(CurrentFrame.mvpMapPoints, m, LastFrame.mvpMapPoints);
    return nm;
}

// ORBmatcher.cc:1472-1599
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist) {
    FrameSide fs;
    fs.gather(CurrentFrame, &CurrentFrame.mvuRight, CurrentFrame.mbf, CurrentFrame.mb);
    fs.occupied(occupied_any(CurrentFrame.mvpMapPoints));
    const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
    const size_t n = vpMPs.size();
    PointSide ps;
    ps.reserve(n);
    for (size_t i = 0; i < n; i++) {
        MapPoint* p = vpMPs[i];
        ps.skip[i] = !p || sAlreadyFound.count(p);
        if (ps.skip[i]) continue;
        ps.point(i, p, true);
        ps.angle[i] = pKF->mvKeysUn[i].angle;
    }
    ps.finish(n);
    cv::Mat kc;
    std::vector<int32_t> m((size_t)std::max(CurrentFrame.N, 1));
    int nm = 0;
    if (!run("orbm_search_by_projection_keyframe", [&](orbm_ctx* c) {
            return orbm_search_by_projection_keyframe(c, &fs.v, mat44(CurrentFrame.mTcw, kc), &ps.m, th, ORBdist,
                                                     mbCheckOrientation ? 1 : 0, m.data(), &nm);
        }))
        return 0;
    apply(CurrentFrame.mvpMapPoints, m, vpMPs);
    return nm;
}

// ORBmatcher.cc:290-403
int ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                                   std::vector<MapPoint*>& vpMatched, int th) {
    FrameSide fs;
    fs.gather(*pKF, nullptr, 0.f, 0.f);
    fs.occupied(occupied_any(vpMatched));
    std::set<MapPoint*> spAlreadyFound(vpMatched.begin(), vpMatched.end());
    spAlreadyFound.erase(static_cast<MapPoint*>(NULL));
    const size_t n = vpPoints.size();
    PointSide ps;
    ps.reserve(n);
    for (size_t i = 0; i < n; i++) {
        MapPoint* p = vpPoints[i];
        ps.skip[i] = spAlreadyFound.count(p) > 0;
        if (ps.skip[i]) continue;
        ps.point(i, p, true);
        cv::Mat nv = p->GetNormal();
        for (int k = 0; k < 3; k++) ps.normal[3 * i + k] = nv.at<float>(k, 0);
    }
    ps.finish(n);
    cv::Mat ks;
    std::vector<int32_t> m(vpMatched.size() ? vpMatched.size() : 1);
    int nm = 0;
    if (!run("orbm_search_by_projection_sim3", [&](orbm_ctx* c) {
            return orbm_search_by_projection_sim3(c, &fs.v, mat44(Scw, ks), &ps.m, th, m.data(), &nm);
        }))
        return 0;
    apply(vpMatched, m, vpPoints);
    return nm;
}

// ORBmatcher.cc:825-975
int ORBmatcher::Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th) {
    FrameSide fs;
    fs.gather(*pKF, &pKF->mvuRight, pKF->mbf, 0.f);
    const size_t n = vpMapPoints.size();
    PointSide ps;
    ps.reserve(n);
    for (size_t i = 0; i < n; i++) {  // :843-850
        MapPoint* p = vpMapPoints[i];
        ps.skip[i] = !p || p->isBad() || p->IsInKeyFrame(pKF);
        if (ps.skip[i]) continue;
        ps.point(i, p, true);
        cv::Mat nv = p->GetNormal();
        for (int k = 0; k < 3; k++) ps.normal[3 * i + k] = nv.at<float>(k, 0);
    }
    ps.finish(n);
    cv::Mat R = pKF->GetRotation(), t = pKF->GetTranslation(), Ow = pKF->GetCameraCenter();
    float T[16] = {0}, O[3];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) T[4 * r + c] = R.at<float>(r, c);
        T[4 * r + 3] = t.at<float>(r, 0);
        O[r] = Ow.at<float>(r, 0);
    }
    T[15] = 1.f;
    std::vector<int32_t> best(n ? n : 1);
    int nf = 0;
    orbm_kf_cache* kc = amd::KeyFrameCache();
    if (!run("orbm_fuse", [&](orbm_ctx* c) {
            if (kc)  // the keyframe's arrays and feature grid stay in HBM across SearchInNeighbors' calls
                return orbm_fuse_cached(c, kc, amd::KeyFrameKey(pKF, pKF->mnId), &fs.v, T, O, &ps.m, th,
                                        pKF->mvInvLevelSigma2.data(), best.data(), &nf);
            return orbm_fuse(c, &fs.v, T, O, &ps.m, th, pKF->mvInvLevelSigma2.data(), best.data(), &nf);
        }))
        return 0;
    // the reference's updates, in order (:947-971)
    int nFused = 0;
    for (size_t i = 0; i < n; i++) {
        MapPoint* pMP = vpMapPoints[i];
        if (!pMP || best[i] < 0) continue;
        if (pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;  // changed by an earlier update
        const size_t bestIdx = (size_t)best[i];
        MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations())
                    pMP->Replace(pMPinKF);
                else
                    pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, bestIdx);
            pKF->AddMapPoint(pMP, bestIdx);
        }
        nFused++;
    }
    return nFused;
}

// ORBmatcher.cc:977-1100
int ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
                     std::vector<MapPoint*>& vpReplacePoint) {
    FrameSide fs;
    fs.gather(*pKF, nullptr, 0.f, 0.f);
    const std::set<MapPoint*> spAlreadyFound = pKF->GetMapPoints();  // :993
    const size_t n = vpPoints.size();
    PointSide ps;
    ps.reserve(n);
    for (size_t i = 0; i < n; i++) {
        MapPoint* p = vpPoints[i];
        ps.skip[i] = p->isBad() || spAlreadyFound.count(p) > 0;  // :1005-1006
        if (ps.skip[i]) continue;
        ps.point(i, p, true);
        cv::Mat nv = p->GetNormal();
        for (int k = 0; k < 3; k++) ps.normal[3 * i + k] = nv.at<float>(k, 0);
    }
    ps.finish(n);
    cv::Mat ks;
    std::vector<int32_t> best(n ? n : 1);
    int nf = 0;
    if (!run("orbm_fuse_sim3", [&](orbm_ctx* c) {
            return orbm_fuse_sim3(c, &fs.v, mat44(Scw, ks), &ps.m, th, best.data(), &nf);
        }))
        return 0;
    int nFused = 0;
    for (size_t i = 0; i < n; i++) {  // :1082-1097, in order
        if (best[i] < 0) continue;
        MapPoint* pMP = vpPoints[i];
        if (pMP->isBad()) continue;
        const size_t bestIdx = (size_t)best[i];
        MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
        } else {
            pMP->AddObservation(pKF, bestIdx);
            pKF->AddMapPoint(pMP, bestIdx);
        }
        nFused++;
    }
    return nFused;
}

// ORBmatcher.cc:405-520 (Tracking::MonocularInitialization, Tracking.cc:600)
int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
    const size_t n1 = F1.mvKeysUn.size();
    vnMatches12 = std::vector<int>(n1, -1);  // :408
    FrameSide f1, f2;
    f1.gather(F1, nullptr, 0.f, 0.f);
    f2.gather(F2, nullptr, 0.f, 0.f);
    std::vector<float> prev(2 * n1 + 2);
    for (size_t i = 0; i < n1; i++) {
        prev[2 * i] = vbPrevMatched[i].x;
        prev[2 * i + 1] = vbPrevMatched[i].y;
    }
    std::vector<int32_t> m(n1 + 1);
    int nm = 0;
    if (!run("orbm_search_for_initialization", [&](orbm_ctx* c) {
            return orbm_search_for_initialization(c, &f1.v, &f2.v, prev.data(), windowSize, mfNNratio,
                                                  mbCheckOrientation ? 1 : 0, m.data(), &nm);
        }))
        return 0;
    for (size_t i = 0; i < n1; i++) {  // :514-517 (the updated positions come back in prev)
        vnMatches12[i] = m[i];
        if (m[i] >= 0) vbPrevMatched[i] = cv::Point2f(prev[2 * i], prev[2 * i + 1]);
    }
    return nm;
}

// ORBmatcher.cc:1102-1326 (LoopClosing::ComputeSim3)
int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                             const cv::Mat& R12, const cv::Mat& t12, const float th) {
    FrameSide k1, k2;
    k1.gather(*pKF1, nullptr, 0.f, 0.f);
    k2.gather(*pKF2, nullptr, 0.f, 0.f);
    const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
    const size_t N1 = vpMapPoints1.size(), N2 = vpMapPoints2.size();
    std::vector<uint8_t> already1(N1, 0), already2(N2, 0);  // :1129-1142
    for (size_t i = 0; i < N1; i++) {
        MapPoint* pMP = vpMatches12[i];
        if (pMP) {
            already1[i] = 1;
            const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
            if (idx2 >= 0 && idx2 < (int)N2) already2[idx2] = 1;
        }
    }
    PointSide p1, p2;
    p1.reserve(N1);
    p2.reserve(N2);
    for (size_t i = 0; i < N1; i++) {
        p1.skip[i] = !vpMapPoints1[i] || already1[i];
        if (!p1.skip[i]) p1.point(i, vpMapPoints1[i], true);
    }
    for (size_t i = 0; i < N2; i++) {
        p2.skip[i] = !vpMapPoints2[i] || already2[i];
        if (!p2.skip[i]) p2.point(i, vpMapPoints2[i], true);
    }
    p1.finish(N1);
    p2.finish(N2);
    float T1[16] = {0}, T2[16] = {0}, R[9], t[3];
    const cv::Mat R1w = pKF1->GetRotation(), t1w = pKF1->GetTranslation();
    const cv::Mat R2w = pKF2->GetRotation(), t2w = pKF2->GetTranslation();
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) {
            T1[4 * r + c] = R1w.at<float>(r, c);
            T2[4 * r + c] = R2w.at<float>(r, c);
            R[3 * r + c] = R12.at<float>(r, c);
        }
        T1[4 * r + 3] = t1w.at<float>(r, 0);
        T2[4 * r + 3] = t2w.at<float>(r, 0);
        t[r] = t12.at<float>(r, 0);
    }
    T1[15] = T2[15] = 1.f;
    std::vector<int32_t> m(N1 + 1);
    int nFound = 0;
    if (!run("orbm_search_by_sim3", [&](orbm_ctx* c) {
            return orbm_search_by_sim3(c, &k1.v, T1, &p1.m, &k2.v, T2, &p2.m, s12, R, t, th, m.data(), &nFound);
        }))
        return 0;
    for (size_t i1 = 0; i1 < N1; i1++)  // :1310-1323
        if (m[i1] >= 0) vpMatches12[i1] = vpMapPoints2[m[i1]];
    return nFound;
}

}  // namespace ORB_SLAM2
