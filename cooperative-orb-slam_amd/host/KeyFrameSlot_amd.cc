/*
 * KeyFrameSlot_amd.cc -- decode / encode of the cross-agent keyframe slot into / from the
 * receiving agent's receiveKeyframeInfo (see KeyFrameSlot_amd.h). All validation is the C ABI's
 * (orbx_slot_parse); this file only moves fields between the slot and the ORB-SLAM2 containers,
 * in the order the LCM handler filled them (ORB_SLAM2/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:246-540).
 */
#include "KeyFrameSlot_amd.h"

#include <cstring>

namespace ORB_SLAM2 {
namespace amd {

namespace {

cv::Mat mat_from(const float* v, int rows, int cols) {
    cv::Mat m(rows, cols, CV_32F);
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) m.at<float>(r, c) = v[r * cols + c];
    return m;
}

void mat_to(const cv::Mat& m, float* v, int rows, int cols) {
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) v[r * cols + c] = m.empty() ? (r == c ? 1.f : 0.f) : m.at<float>(r, c);
}

}  // namespace

bool DecodeKeyFrameSlot(const uint8_t* slot, size_t slot_bytes, ReceivedKeyFrame& out) {
    orbx_slot_view v;
    if (orbx_slot_parse(slot, slot_bytes, &v) != ORBX_OK) return false;
    const orbx_kf_meta& m = *v.meta;
    const int N = v.hdr->n;
    ReceivedKeyFrame kf;
    kf.nNextId = (long unsigned int)m.nNextId;
    kf.mnId = (long unsigned int)m.mnId;
    kf.mnFrameId = (long unsigned int)m.mnFrameId;
    kf.mTimeStamp = m.mTimeStamp;
    kf.mnGridCols = (int)m.mnGridCols;
    kf.mnGridRows = (int)m.mnGridRows;
    kf.mfGridElementWidthInv = m.mfGridElementWidthInv;
    kf.mfGridElementHeightInv = m.mfGridElementHeightInv;
    kf.mnTrackReferenceForFrame = (long unsigned int)m.mnTrackReferenceForFrame;
    kf.mnFuseTargetForKF = (long unsigned int)m.mnFuseTargetForKF;
    kf.mnBALocalForKF = (long unsigned int)m.mnBALocalForKF;
    kf.mnBAFixedForKF = (long unsigned int)m.mnBAFixedForKF;
    kf.mnLoopQuery = (long unsigned int)m.mnLoopQuery;
    kf.mnLoopWords = (int)m.mnLoopWords;
    kf.mLoopScore = m.mLoopScore;
    kf.mnRelocQuery = (long unsigned int)m.mnRelocQuery;
    kf.mnRelocWords = (int)m.mnRelocWords;
    kf.mRelocScore = m.mRelocScore;
    kf.mTcwGBA = mat_from(m.mTcwGBA, 4, 4);
    kf.mTcwBefGBA = mat_from(m.mTcwBefGBA, 4, 4);
    kf.mnBAGlobalForKF = (long unsigned int)m.mnBAGlobalForKF;
    kf.fx = m.fx; kf.fy = m.fy; kf.cx = m.cx; kf.cy = m.cy;
    kf.invfx = m.invfx; kf.invfy = m.invfy;
    kf.mbf = m.mbf; kf.mb = m.mb; kf.mThDepth = m.mThDepth;
    kf.N = N;
    kf.mvKeys.resize(N);
    kf.mvKeysUn.resize(N);
    for (int i = 0; i < N; i++) {
        const orbx_kp& k = v.kps[i];
        kf.mvKeys[i] = cv::KeyPoint(k.x, k.y, k.size, k.angle, k.response, k.octave, -1);
        kf.mvKeysUn[i] = cv::KeyPoint(v.kun[2 * i], v.kun[2 * i + 1], k.size, k.angle, k.response, k.octave, -1);
    }
    kf.mvuRight.assign(v.uright, v.uright + N);
    kf.mvDepth.assign(v.depth, v.depth + N);
    kf.mDescriptors.create(N, 32, CV_8U);
    if (N) memcpy(kf.mDescriptors.data, v.desc, 32 * (size_t)N);
    for (int k = 0; k < v.hdr->nbow; k++) kf.mBowVec[v.bow_word[k]] = v.bow_value[k];
    for (int k = 0; k < v.hdr->nfv; k++) {
        std::vector<unsigned int>& f = kf.mFeatVec[v.fv_node[k]];
        for (int j = v.fv_off[k]; j < v.fv_off[k + 1]; j++) f.push_back((unsigned int)v.fv_feat[j]);
    }
    kf.mTcp = mat_from(m.mTcp, 4, 4);
    kf.mnScaleLevels = m.mnScaleLevels;
    kf.mfScaleFactor = m.mfScaleFactor;
    kf.mfLogScaleFactor = m.mfLogScaleFactor;
    kf.mvScaleFactors.assign(m.mvScaleFactors, m.mvScaleFactors + m.mnScaleLevels);
    kf.mvLevelSigma2.assign(m.mvLevelSigma2, m.mvLevelSigma2 + m.mnScaleLevels);
    kf.mvInvLevelSigma2.assign(m.mvInvLevelSigma2, m.mvInvLevelSigma2 + m.mnScaleLevels);
    kf.mnMinX = (int)m.mnMinX;
    kf.mnMinY = (int)m.mnMinY;
    kf.mnMaxX = (int)m.mnMaxX;
    kf.mnMaxY = (int)m.mnMaxY;
    kf.mK = mat_from(m.mK, 3, 3);
    kf.mTcw = mat_from(m.mTcw, 4, 4);
    if (v.hdr->flags & ORBX_SLOT_F_MP) {
        // one record per keypoint, as the sender emits them (ros_mono.cc:2353-2382)
        kf.receiveMapPoints.resize(N);
        for (int i = 0; i < N; i++) {
            const bool has = (v.mp_flags[i] & 1) != 0;
            kf.receiveMapPoints[i] = receivePoints{has, i, v.mp_pos[3 * i], v.mp_pos[3 * i + 1], v.mp_pos[3 * i + 2]};
        }
    }
    kf.agent = m.agent;
    kf.flags = v.hdr->flags;
    out = kf;
    return true;
}

int EncodeKeyFrameSlot(const ReceivedKeyFrame& kf, int cap, std::vector<uint8_t>& slot) {
    const int N = (int)kf.mvKeys.size();
    if (cap < 1) return ORBX_EARG;
    if ((!kf.mvKeysUn.empty() && (int)kf.mvKeysUn.size() != N) || (!kf.mvuRight.empty() && (int)kf.mvuRight.size() != N) ||
        (!kf.mvDepth.empty() && (int)kf.mvDepth.size() != N) || (N && (kf.mDescriptors.rows != N || kf.mDescriptors.cols != 32)))
        return ORBX_EARG;
    orbx_kf_meta m;
    memset(&m, 0, sizeof(m));
    m.nNextId = (int64_t)kf.nNextId;
    m.mnId = (int64_t)kf.mnId;
    m.mnFrameId = (int64_t)kf.mnFrameId;
    m.mTimeStamp = kf.mTimeStamp;
    m.mnGridCols = kf.mnGridCols;
    m.mnGridRows = kf.mnGridRows;
    m.mfGridElementWidthInv = kf.mfGridElementWidthInv;
    m.mfGridElementHeightInv = kf.mfGridElementHeightInv;
    m.mnTrackReferenceForFrame = (int64_t)kf.mnTrackReferenceForFrame;
    m.mnFuseTargetForKF = (int64_t)kf.mnFuseTargetForKF;
    m.mnBALocalForKF = (int64_t)kf.mnBALocalForKF;
    m.mnBAFixedForKF = (int64_t)kf.mnBAFixedForKF;
    m.mnLoopQuery = (int64_t)kf.mnLoopQuery;
    m.mnLoopWords = kf.mnLoopWords;
    m.mLoopScore = kf.mLoopScore;
    m.mnRelocQuery = (int64_t)kf.mnRelocQuery;
    m.mnRelocWords = kf.mnRelocWords;
    m.mRelocScore = kf.mRelocScore;
    mat_to(kf.mTcwGBA, m.mTcwGBA, 4, 4);
    mat_to(kf.mTcwBefGBA, m.mTcwBefGBA, 4, 4);
    m.mnBAGlobalForKF = (int64_t)kf.mnBAGlobalForKF;
    m.fx = kf.fx; m.fy = kf.fy; m.cx = kf.cx; m.cy = kf.cy;
    m.invfx = kf.invfx; m.invfy = kf.invfy;
    m.mbf = kf.mbf; m.mb = kf.mb; m.mThDepth = kf.mThDepth;
    mat_to(kf.mTcp, m.mTcp, 4, 4);
    m.mnScaleLevels = kf.mnScaleLevels;
    m.mfScaleFactor = kf.mfScaleFactor;
    m.mfLogScaleFactor = kf.mfLogScaleFactor;
    for (int l = 0; l < kf.mnScaleLevels && l < 16; l++) {
        m.mvScaleFactors[l] = l < (int)kf.mvScaleFactors.size() ? kf.mvScaleFactors[l] : 0.f;
        m.mvLevelSigma2[l] = l < (int)kf.mvLevelSigma2.size() ? kf.mvLevelSigma2[l] : 0.f;
        m.mvInvLevelSigma2[l] = l < (int)kf.mvInvLevelSigma2.size() ? kf.mvInvLevelSigma2[l] : 0.f;
    }
    m.mnMinX = kf.mnMinX;
    m.mnMinY = kf.mnMinY;
    m.mnMaxX = kf.mnMaxX;
    m.mnMaxY = kf.mnMaxY;
    mat_to(kf.mK, m.mK, 3, 3);
    mat_to(kf.mTcw, m.mTcw, 4, 4);
    m.agent = kf.agent;

    std::vector<orbx_kp> kps(N);
    std::vector<float> kun;
    for (int i = 0; i < N; i++) {
        const cv::KeyPoint& k = kf.mvKeys[i];
        kps[i] = orbx_kp{k.pt.x, k.pt.y, k.size, k.angle, k.response, k.octave};
    }
    if (!kf.mvKeysUn.empty()) {
        kun.resize(2 * (size_t)N);
        for (int i = 0; i < N; i++) {
            kun[2 * i] = kf.mvKeysUn[i].pt.x;
            kun[2 * i + 1] = kf.mvKeysUn[i].pt.y;
        }
    }
    std::vector<uint8_t> mpf;
    std::vector<float> mpp;
    if (!kf.receiveMapPoints.empty()) {
        mpf.assign(N, 0);
        mpp.assign(3 * (size_t)N, 0.f);
        for (const receivePoints& p : kf.receiveMapPoints) {
            if (!p.ifMapPoints || p.x < 0 || p.x >= N) continue;
            mpf[p.x] = 1;
            mpp[3 * p.x] = p.poseX;
            mpp[3 * p.x + 1] = p.poseY;
            mpp[3 * p.x + 2] = p.poseZ;
        }
    }
    std::vector<uint32_t> bw, fn;
    std::vector<double> bv;
    std::vector<int32_t> fo, ff;
    for (DBoW2::BowVector::const_iterator it = kf.mBowVec.begin(); it != kf.mBowVec.end(); ++it) {
        bw.push_back((uint32_t)it->first);
        bv.push_back((double)it->second);
    }
    fo.push_back(0);
    for (DBoW2::FeatureVector::const_iterator it = kf.mFeatVec.begin(); it != kf.mFeatVec.end(); ++it) {
        fn.push_back((uint32_t)it->first);
        for (unsigned int f : it->second) ff.push_back((int32_t)f);
        fo.push_back((int32_t)ff.size());
    }
    const int32_t n = N, nb = (int32_t)bw.size(), nf = (int32_t)fn.size();
    const cv::Mat desc = kf.mDescriptors.isContinuous() ? kf.mDescriptors : kf.mDescriptors.clone();
    orbx_kf_source s;
    memset(&s, 0, sizeof(s));
    s.kps = kps.data();
    s.desc = N ? desc.data : nullptr;
    s.count = &n;
    s.kun = kun.empty() ? nullptr : kun.data();
    if (!kf.mvuRight.empty() && !kf.mvDepth.empty()) {
        s.uright = kf.mvuRight.data();
        s.depth = kf.mvDepth.data();
    }
    if (!mpf.empty()) {
        s.mp_flags = mpf.data();
        s.mp_pos = mpp.data();
    }
    if (nb) {
        s.bow_word = bw.data();
        s.bow_value = bv.data();
        s.nbow = &nb;
    }
    if (nf) {
        s.fv_node = fn.data();
        s.fv_off = fo.data();
        s.fv_feat = ff.data();
        s.nfv = &nf;
    }
    const size_t bytes = orbx_slot_bytes(cap);
    if (!bytes) return ORBX_EARG;
    slot.assign(bytes, 0);
    return orbx_pack_keyframe_host(&s, &m, cap, slot.data(), bytes);
}

}  // namespace amd
}  // namespace ORB_SLAM2
