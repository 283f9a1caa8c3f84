/*
 * ORBmatcher_amd.cc -- MI355X definitions of the ORBmatcher hot-path members (replace the
 * same definitions in ORB_SLAM2/src/ORBmatcher.cc):
 *   DescriptorDistance          ORBmatcher.cc:1647-1663
 *   SearchForTriangulation      ORBmatcher.cc:657-823
 *   SearchByBoW(KF*, Frame&)    ORBmatcher.cc:159-288
 *   SearchByBoW(KF*, KF*)       ORBmatcher.cc:522-655
 * Each call gathers the KeyFrame/Frame state the reference reads (under the same accessor
 * locks: GetMapPointMatches, GetRotation/GetTranslation/GetCameraCenter) into an
 * orbm_kf_view and runs the matcher kernels; results are converted back to the reference's
 * containers. One orbm_ctx per calling thread (Tracking, LocalMapping, LoopClosing call
 * concurrently). KeyFrames' immutable arrays are kept in HBM across calls (the process-wide
 * orbm_kf_cache of orbamd_status.h; ORBAMD_KF_CACHE_MB=0 turns it off). A device failure does not
 * throw (orbamd_status.h): the call returns 0 with the reference's empty result (no pairs / a
 * NULL-filled match vector) and logs the status.
 */
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ORBmatcher.h"
#include "orbamd_status.h"
#include "orbslam_amd.h"

namespace ORB_SLAM2 {

namespace {

/* the call's status through the thread's matcher context (nullptr ctx: the creation failure was
 * already recorded) */
template <class F>
bool run(const char* what, F f) {
    orbm_ctx* c = amd::ThreadMatcher();
    return c && amd::StatusOk(f(c), what);
}

/* host staging of one KeyFrame / Frame (ORBmatcher.cc reads exactly these members) */
struct ViewData {
    std::vector<float> x, y, angle, uright;
    std::vector<int32_t> octave, node_off, node_feat;
    std::vector<uint32_t> node_id;
    std::vector<uint8_t> has_mp, mp_bad;
    cv::Mat desc;
    orbm_kf_view v;

    void keys(const std::vector<cv::KeyPoint>& kps, const std::vector<cv::KeyPoint>& angles_from) {
        const size_t n = kps.size();
        x.resize(n); y.resize(n); angle.resize(n); octave.resize(n);
        for (size_t i = 0; i < n; i++) {
            x[i] = kps[i].pt.x;
            y[i] = kps[i].pt.y;
            angle[i] = angles_from[i].angle;
            octave[i] = kps[i].octave;
        }
    }
    void featvec(const DBoW2::FeatureVector& fv) {
        node_off.assign(1, 0);
        for (DBoW2::FeatureVector::const_iterator it = fv.begin(); it != fv.end(); ++it) {
            node_id.push_back((uint32_t)it->first);
            for (size_t k = 0; k < it->second.size(); k++) node_feat.push_back((int32_t)it->second[k]);
            node_off.push_back((int32_t)node_feat.size());
        }
    }
    void mappoints(const std::vector<MapPoint*>& mps) {
        has_mp.resize(mps.size());
        mp_bad.resize(mps.size());
        for (size_t i = 0; i < mps.size(); i++) {
            has_mp[i] = mps[i] != nullptr;
            mp_bad[i] = mps[i] ? (uint8_t)mps[i]->isBad() : 0;
        }
    }
    void finish(int n, const cv::Mat& d, const std::vector<float>& ur, const std::vector<float>& scale,
                const std::vector<float>& sigma2, bool with_mp) {
        desc = d.isContinuous() ? d : d.clone();
        uright = ur;
        memset(&v, 0, sizeof(v));
        v.n = n;
        v.desc = n ? desc.data : nullptr;
        v.x = x.data(); v.y = y.data(); v.angle = angle.data(); v.octave = octave.data();
        v.uright = uright.empty() ? nullptr : uright.data();
        v.has_mp = with_mp ? has_mp.data() : nullptr;
        v.mp_bad = with_mp ? mp_bad.data() : nullptr;
        v.n_nodes = (int32_t)node_id.size();
        v.node_id = node_id.data();
        v.node_off = node_off.data();
        v.node_feat = node_feat.data();
        v.nlevels = (int32_t)scale.size();
        v.scale_factors = scale.data();
        v.level_sigma2 = sigma2.data();
    }
};

void gather_kf(KeyFrame* pKF, ViewData& d) {
    d.keys(pKF->mvKeysUn, pKF->mvKeysUn);
    d.featvec(pKF->mFeatVec);
    d.mappoints(pKF->GetMapPointMatches());
    d.finish(pKF->N, pKF->mDescriptors, pKF->mvuRight, pKF->mvScaleFactors, pKF->mvLevelSigma2, true);
}

}  // namespace

// ORBmatcher.cc:1647-1663
int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
    return orbm_descriptor_distance(a.ptr<unsigned char>(), b.ptr<unsigned char>());
}

// ORBmatcher.cc:657-823
int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                                       std::vector<std::pair<size_t, size_t> >& vMatchedPairs,
                                       const bool bOnlyStereo) {
    cv::Mat Cw = pKF1->GetCameraCenter().clone();
    cv::Mat R2w = pKF2->GetRotation().clone();
    cv::Mat t2w = pKF2->GetTranslation().clone();
    float ex = 0, ey = 0;
    orbm_epipole(R2w.ptr<float>(), t2w.ptr<float>(), Cw.ptr<float>(), pKF2->fx, pKF2->fy, pKF2->cx, pKF2->cy, &ex,
                 &ey);
    ViewData v1, v2;
    gather_kf(pKF1, v1);
    gather_kf(pKF2, v2);
    cv::Mat F = F12.isContinuous() ? F12 : F12.clone();
    std::vector<int32_t> m12((size_t)std::max(pKF1->N, 1));
    int n = 0;
    vMatchedPairs.clear();
    orbm_kf_cache* kc = amd::KeyFrameCache();
    if (!run("orbm_search_for_triangulation", [&](orbm_ctx* c) {
            if (kc)  // both keyframes' arrays stay in HBM across LocalMapping's ~20 calls per keyframe
                return orbm_search_for_triangulation_cached(c, kc, amd::KeyFrameKey(pKF1, pKF1->mnId), &v1.v,
                                                            amd::KeyFrameKey(pKF2, pKF2->mnId), &v2.v, F.ptr<float>(),
                                                            ex, ey, bOnlyStereo ? 1 : 0, mbCheckOrientation ? 1 : 0,
                                                            m12.data(), &n);
            return orbm_search_for_triangulation(c, &v1.v, &v2.v, F.ptr<float>(), ex, ey, bOnlyStereo ? 1 : 0,
                                                 mbCheckOrientation ? 1 : 0, m12.data(), &n);
        }))
        return 0;
    vMatchedPairs.reserve(n);
    for (int i = 0; i < pKF1->N; i++)
        if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)m12[i]));
    return n;
}

// ORBmatcher.cc:159-288
int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
    const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
    ViewData vk, vf;
    vk.keys(pKF->mvKeysUn, pKF->mvKeysUn);
    vk.featvec(pKF->mFeatVec);
    vk.mappoints(vpMapPointsKF);
    vk.finish(pKF->N, pKF->mDescriptors, std::vector<float>(), pKF->mvScaleFactors, pKF->mvLevelSigma2, true);
    vf.keys(F.mvKeysUn, F.mvKeys);  // rotation uses F.mvKeys[..].angle (ORBmatcher.cc:238)
    vf.featvec(F.mFeatVec);
    vf.finish(F.N, F.mDescriptors, std::vector<float>(), F.mvScaleFactors, F.mvLevelSigma2, false);
    std::vector<int32_t> mf((size_t)std::max(F.N, 1));
    int n = 0;
    vpMapPointMatches = std::vector<MapPoint*>(F.N, static_cast<MapPoint*>(NULL));  // :163
    orbm_kf_cache* kc = amd::KeyFrameCache();
    if (!run("orbm_search_by_bow_kf_f", [&](orbm_ctx* c) {
            if (kc)
                return orbm_search_by_bow_kf_f_cached(c, kc, amd::KeyFrameKey(pKF, pKF->mnId), &vk.v, &vf.v, mfNNratio,
                                                      mbCheckOrientation ? 1 : 0, mf.data(), &n);
            return orbm_search_by_bow_kf_f(c, &vk.v, &vf.v, mfNNratio, mbCheckOrientation ? 1 : 0, mf.data(), &n);
        }))
        return 0;
    for (int i = 0; i < F.N; i++)
        if (mf[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[mf[i]];
    return n;
}

// ORBmatcher.cc:522-655
int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
    const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
    ViewData v1, v2;
    v1.keys(pKF1->mvKeysUn, pKF1->mvKeysUn);
    v1.featvec(pKF1->mFeatVec);
    v1.mappoints(vpMapPoints1);
    v1.finish(pKF1->N, pKF1->mDescriptors, std::vector<float>(), pKF1->mvScaleFactors, pKF1->mvLevelSigma2, true);
    v2.keys(pKF2->mvKeysUn, pKF2->mvKeysUn);
    v2.featvec(pKF2->mFeatVec);
    v2.mappoints(vpMapPoints2);
    v2.finish(pKF2->N, pKF2->mDescriptors, std::vector<float>(), pKF2->mvScaleFactors, pKF2->mvLevelSigma2, true);
    std::vector<int32_t> m12(vpMapPoints1.size() ? vpMapPoints1.size() : 1);
    int n = 0;
    vpMatches12 = std::vector<MapPoint*>(vpMapPoints1.size(), static_cast<MapPoint*>(NULL));  // :536
    orbm_kf_cache* kc = amd::KeyFrameCache();
    if (!run("orbm_search_by_bow_kf_kf", [&](orbm_ctx* c) {
            if (kc)
                return orbm_search_by_bow_kf_kf_cached(c, kc, amd::KeyFrameKey(pKF1, pKF1->mnId), &v1.v,
                                                       amd::KeyFrameKey(pKF2, pKF2->mnId), &v2.v, mfNNratio,
                                                       mbCheckOrientation ? 1 : 0, m12.data(), &n);
            return orbm_search_by_bow_kf_kf(c, &v1.v, &v2.v, mfNNratio, mbCheckOrientation ? 1 : 0, m12.data(), &n);
        }))
        return 0;
    for (size_t i = 0; i < vpMapPoints1.size(); i++)
        if (m12[i] >= 0) vpMatches12[i] = vpMapPoints2[m12[i]];
    return n;
}

}  // namespace ORB_SLAM2
