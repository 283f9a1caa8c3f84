/* test_slot.cpp -- CPU test of the C++ keyframe-slot codec (host/KeyFrameSlot_amd.*): a keyframe in
 * receiveKeyframeInfo form (ORB_SLAM2/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:79-166) survives
 * EncodeKeyFrameSlot -> DecodeKeyFrameSlot field for field; malformed slots are rejected.
 * No GPU needed. Prints "ALL PASS". Build: tests/cpp/build.sh */
#include <cmath>
#include <cstdio>
#include <cstring>

#include "KeyFrameSlot_amd.h"

using namespace ORB_SLAM2;
using namespace ORB_SLAM2::amd;

static int failures = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            printf("FAIL %s:%d ", __FILE__, __LINE__);     \
            printf(__VA_ARGS__);                           \
            printf("\n");                                  \
            failures++;                                    \
        }                                                  \
    } while (0)

static uint32_t lcg(uint32_t& s) { s = s * 1664525u + 1013904223u; return s >> 8; }
static float frand(uint32_t& s) { return (float)(lcg(s) & 0xFFFFF) / (float)0x100000; }

static bool same_mat(const cv::Mat& a, const cv::Mat& b) {
    if (a.rows != b.rows || a.cols != b.cols || a.type() != b.type()) return false;
    for (int r = 0; r < a.rows; r++)
        if (memcmp(a.ptr<unsigned char>(r), b.ptr<unsigned char>(r), a.cols * cv::Mat::esz(a.type()))) return false;
    return true;
}

static ReceivedKeyFrame make_kf(int N, uint32_t seed, bool full) {
    ReceivedKeyFrame kf;
    kf.nNextId = 44; kf.mnId = 43; kf.mnFrameId = 1200; kf.mTimeStamp = 1403636579.763555;
    kf.mnGridCols = 64; kf.mnGridRows = 48; kf.mfGridElementWidthInv = 0.1f; kf.mfGridElementHeightInv = 0.1f;
    kf.mnTrackReferenceForFrame = 5; kf.mnFuseTargetForKF = 6; kf.mnBALocalForKF = 7; kf.mnBAFixedForKF = 8;
    kf.mnLoopQuery = 9; kf.mnLoopWords = 10; kf.mLoopScore = 0.5f; kf.mnRelocQuery = 11; kf.mnRelocWords = 12;
    kf.mRelocScore = 0.25f; kf.mnBAGlobalForKF = 13;
    kf.fx = 458.654f; kf.fy = 457.296f; kf.cx = 367.215f; kf.cy = 248.375f;
    kf.invfx = 1.f / kf.fx; kf.invfy = 1.f / kf.fy; kf.mbf = 47.9f; kf.mb = 0.11f; kf.mThDepth = 35.f;
    kf.mnScaleLevels = 8; kf.mfScaleFactor = 1.2f; kf.mfLogScaleFactor = logf(1.2f);
    float s = 1.f;
    for (int l = 0; l < 8; l++) {
        kf.mvScaleFactors.push_back(s);
        kf.mvLevelSigma2.push_back(s * s);
        kf.mvInvLevelSigma2.push_back(1.f / (s * s));
        s *= 1.2f;
    }
    kf.mnMinX = 0; kf.mnMinY = 0; kf.mnMaxX = 752; kf.mnMaxY = 480;
    kf.mK = cv::Mat(3, 3, CV_32F);
    kf.mTcw = cv::Mat(4, 4, CV_32F);
    kf.mTcwGBA = cv::Mat(4, 4, CV_32F);
    kf.mTcwBefGBA = cv::Mat(4, 4, CV_32F);
    kf.mTcp = cv::Mat(4, 4, CV_32F);
    for (int i = 0; i < 9; i++) kf.mK.at<float>(i / 3, i % 3) = frand(seed);
    for (int i = 0; i < 16; i++) {
        kf.mTcw.at<float>(i / 4, i % 4) = frand(seed);
        kf.mTcwGBA.at<float>(i / 4, i % 4) = frand(seed);
        kf.mTcwBefGBA.at<float>(i / 4, i % 4) = frand(seed);
        kf.mTcp.at<float>(i / 4, i % 4) = frand(seed);
    }
    kf.N = N;
    kf.mDescriptors.create(N, 32, CV_8U);
    for (int i = 0; i < N; i++) {
        cv::KeyPoint k(frand(seed) * 752, frand(seed) * 480, 31.f * (1 + (lcg(seed) & 3)), frand(seed) * 360,
                       frand(seed) * 100, (int)(lcg(seed) % 8), -1);
        kf.mvKeys.push_back(k);
        for (int j = 0; j < 32; j++) kf.mDescriptors.at<unsigned char>(i, j) = (unsigned char)lcg(seed);
    }
    kf.agent = 1;
    if (!full) return kf;
    for (int i = 0; i < N; i++) {
        cv::KeyPoint u = kf.mvKeys[i];
        u.pt.x += frand(seed) - 0.5f;
        u.pt.y += frand(seed) - 0.5f;
        kf.mvKeysUn.push_back(u);
        const bool st = (lcg(seed) & 1) != 0;
        kf.mvuRight.push_back(st ? u.pt.x - 20 * frand(seed) : -1.f);
        kf.mvDepth.push_back(st ? 5 * frand(seed) : -1.f);
        const bool mp = (lcg(seed) % 3) == 0;
        kf.receiveMapPoints.push_back(receivePoints{mp, i, mp ? frand(seed) : 0.f, mp ? frand(seed) : 0.f,
                                                    mp ? frand(seed) : 0.f});
    }
    for (int w = 0; w < N / 3; w++) kf.mBowVec[(unsigned)(w * 977 + 3)] = frand(seed);
    for (int i = 0; i < N; i++) kf.mFeatVec[(unsigned)(lcg(seed) % 37) * 11].push_back((unsigned)i);
    return kf;
}

static void check_roundtrip(const ReceivedKeyFrame& a, const ReceivedKeyFrame& b, bool full) {
    CHECK(a.mnId == b.mnId && a.nNextId == b.nNextId && a.mnFrameId == b.mnFrameId, "ids");
    CHECK(a.mTimeStamp == b.mTimeStamp, "timestamp");
    CHECK(a.mnGridCols == b.mnGridCols && a.mnGridRows == b.mnGridRows, "grid");
    CHECK(a.mfGridElementWidthInv == b.mfGridElementWidthInv && a.mfGridElementHeightInv == b.mfGridElementHeightInv,
          "grid inv");
    CHECK(a.mnTrackReferenceForFrame == b.mnTrackReferenceForFrame && a.mnFuseTargetForKF == b.mnFuseTargetForKF &&
              a.mnBALocalForKF == b.mnBALocalForKF && a.mnBAFixedForKF == b.mnBAFixedForKF &&
              a.mnLoopQuery == b.mnLoopQuery && a.mnLoopWords == b.mnLoopWords && a.mLoopScore == b.mLoopScore &&
              a.mnRelocQuery == b.mnRelocQuery && a.mnRelocWords == b.mnRelocWords && a.mRelocScore == b.mRelocScore &&
              a.mnBAGlobalForKF == b.mnBAGlobalForKF,
          "bookkeeping ids");
    CHECK(a.fx == b.fx && a.fy == b.fy && a.cx == b.cx && a.cy == b.cy && a.invfx == b.invfx && a.invfy == b.invfy &&
              a.mbf == b.mbf && a.mb == b.mb && a.mThDepth == b.mThDepth,
          "calibration");
    CHECK(a.N == b.N && a.mvKeys.size() == b.mvKeys.size(), "N");
    for (size_t i = 0; i < a.mvKeys.size() && i < b.mvKeys.size(); i++) {
        const cv::KeyPoint &p = a.mvKeys[i], &q = b.mvKeys[i];
        CHECK(p.pt.x == q.pt.x && p.pt.y == q.pt.y && p.size == q.size && p.angle == q.angle &&
                  p.response == q.response && p.octave == q.octave && q.class_id == -1,
              "mvKeys[%zu]", i);
        const cv::KeyPoint& u = full ? a.mvKeysUn[i] : p;
        CHECK(u.pt.x == b.mvKeysUn[i].pt.x && u.pt.y == b.mvKeysUn[i].pt.y && b.mvKeysUn[i].octave == p.octave,
              "mvKeysUn[%zu]", i);
        CHECK(b.mvuRight[i] == (full ? a.mvuRight[i] : -1.f) && b.mvDepth[i] == (full ? a.mvDepth[i] : -1.f),
              "stereo[%zu]", i);
    }
    CHECK(same_mat(a.mDescriptors, b.mDescriptors), "descriptors");
    CHECK(a.mBowVec == b.mBowVec, "BowVector (%zu vs %zu)", a.mBowVec.size(), b.mBowVec.size());
    CHECK(a.mFeatVec == b.mFeatVec, "FeatureVector (%zu vs %zu)", a.mFeatVec.size(), b.mFeatVec.size());
    CHECK(same_mat(a.mTcp, b.mTcp) && same_mat(a.mK, b.mK) && same_mat(a.mTcw, b.mTcw) &&
              same_mat(a.mTcwGBA, b.mTcwGBA) && same_mat(a.mTcwBefGBA, b.mTcwBefGBA),
          "matrices");
    CHECK(a.mnScaleLevels == b.mnScaleLevels && a.mfScaleFactor == b.mfScaleFactor &&
              a.mfLogScaleFactor == b.mfLogScaleFactor && a.mvScaleFactors == b.mvScaleFactors &&
              a.mvLevelSigma2 == b.mvLevelSigma2 && a.mvInvLevelSigma2 == b.mvInvLevelSigma2,
          "scale tables");
    CHECK(a.mnMinX == b.mnMinX && a.mnMinY == b.mnMinY && a.mnMaxX == b.mnMaxX && a.mnMaxY == b.mnMaxY, "bounds");
    CHECK(a.agent == b.agent, "agent");
    CHECK(b.receiveMapPoints.size() == (full ? a.receiveMapPoints.size() : 0u), "map point records");
    for (size_t i = 0; full && i < a.receiveMapPoints.size() && i < b.receiveMapPoints.size(); i++) {
        const receivePoints &p = a.receiveMapPoints[i], &q = b.receiveMapPoints[i];
        CHECK(p.ifMapPoints == q.ifMapPoints && p.x == q.x && p.poseX == q.poseX && p.poseY == q.poseY &&
                  p.poseZ == q.poseZ,
              "map point %zu", i);
    }
}

int main() {
    for (int full = 0; full < 2; full++) {
        for (int N : {0, 1, 777, 1200}) {
            ReceivedKeyFrame a = make_kf(N, 7u + N, full != 0);
            std::vector<uint8_t> slot;
            int rc = EncodeKeyFrameSlot(a, 1200, slot);
            CHECK(rc == ORBX_OK, "encode rc %d (N=%d)", rc, N);
            ReceivedKeyFrame b;
            CHECK(DecodeKeyFrameSlot(slot.data(), slot.size(), b), "decode (N=%d)", N);
            check_roundtrip(a, b, full != 0);
            // the decoded keyframe re-encodes to the same bytes (full form)
            if (full) {
                std::vector<uint8_t> again;
                CHECK(EncodeKeyFrameSlot(b, 1200, again) == ORBX_OK && again == slot, "re-encode N=%d", N);
            }
        }
    }
    ReceivedKeyFrame a = make_kf(300, 99, true);
    std::vector<uint8_t> slot;
    CHECK(EncodeKeyFrameSlot(a, 200, slot) == ORBX_ECAPACITY, "capacity");
    CHECK(EncodeKeyFrameSlot(a, 400, slot) == ORBX_OK, "encode");
    ReceivedKeyFrame untouched;
    untouched.mnId = 12345;
    std::vector<uint8_t> bad = slot;
    bad[0] ^= 1;  // magic
    CHECK(!DecodeKeyFrameSlot(bad.data(), bad.size(), untouched) && untouched.mnId == 12345, "bad magic");
    bad = slot;
    ((int32_t*)bad.data())[2] = 401;  // n > cap
    CHECK(!DecodeKeyFrameSlot(bad.data(), bad.size(), untouched), "n > cap");
    CHECK(!DecodeKeyFrameSlot(slot.data(), slot.size() - 256, untouched), "truncated");
    if (failures == 0) printf("ALL PASS\n");
    return failures ? 1 : 0;
}
