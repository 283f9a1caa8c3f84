/* test_nodevice.cpp -- the C++ drop-ins when the device is unusable (run with ORBAMD_DEVICE=99, so
 * every orbx_create / orbm_create returns ORBX_EDEVICE even on a GPU box). The reference never throws
 * on these paths (ORBextractor.cc:1043-1105, ORBmatcher.cc), so each call must return normally with
 * the reference's "nothing found" result: keypoints cleared and descriptors released
 * (ORBextractor.cc:1064-1065), zero matches with the match containers in their initial state, no map
 * update, no stereo match, mDescriptor unchanged. The getters still answer (host-side tables).
 * Prints "ALL PASS" on success. Build: tests/cpp/build.sh */
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <exception>
#include <set>
#include <vector>

#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "orbamd_status.h"
#include "orbslam_amd.h"

using namespace ORB_SLAM2;

static int failures = 0;
#define CHECK(cond, ...)                               \
    do {                                               \
        if (!(cond)) {                                 \
            printf("FAIL %s:%d ", __FILE__, __LINE__); \
            printf(__VA_ARGS__);                       \
            printf("\n");                              \
            failures++;                                \
        }                                              \
    } while (0)

static void make_kf(KeyFrame& kf, int n, std::vector<MapPoint>& pool) {
    kf.N = n;
    kf.mvKeys.clear();
    for (int i = 0; i < n; i++) kf.mvKeys.push_back(cv::KeyPoint(20.f + 3 * i, 30.f + 2 * i, 31.f, 10.f * i, 20.f, 0, -1));
    kf.mvKeysUn = kf.mvKeys;
    kf.mDescriptors = cv::Mat(n, 32, CV_8U);
    for (int i = 0; i < n; i++)
        for (int b = 0; b < 32; b++) kf.mDescriptors.at<unsigned char>(i, b) = (unsigned char)(i * 7 + b);
    kf.mvScaleFactors.assign(8, 1.f);
    kf.mvLevelSigma2.assign(8, 1.f);
    kf.mvInvLevelSigma2.assign(8, 1.f);
    kf.mvuRight.assign(n, -1.f);
    kf.fx = kf.fy = 500.f;
    kf.cx = 320.f;
    kf.cy = 240.f;
    kf.mnMaxX = 640.f;
    kf.mnMaxY = 480.f;
    kf.mfGridElementWidthInv = 0.1f;
    kf.mfGridElementHeightInv = 0.1f;
    for (int i = 0; i < n; i++) kf.mFeatVec[5].push_back(i);
    pool.resize(n);
    kf.mvpMapPoints.assign(n, nullptr);
    for (int i = 0; i < n; i += 2) {
        pool[i].mWorldPos = cv::Mat(3, 1, CV_32F);
        pool[i].mNormalVector = cv::Mat(3, 1, CV_32F);
        pool[i].mDescriptor = cv::Mat(1, 32, CV_8U);
        for (int k = 0; k < 3; k++) {
            pool[i].mWorldPos.at<float>(k, 0) = k == 2 ? 2.f : 0.f;
            pool[i].mNormalVector.at<float>(k, 0) = k == 2 ? 1.f : 0.f;
        }
        kf.mvpMapPoints[i] = &pool[i];
    }
    kf.Rcw = cv::Mat(3, 3, CV_32F);
    kf.tcw = cv::Mat(3, 1, CV_32F);
    kf.Ow = cv::Mat(3, 1, CV_32F);
    for (int i = 0; i < 9; i++) kf.Rcw.at<float>(i / 3, i % 3) = (i % 4 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; i++) kf.tcw.at<float>(i) = kf.Ow.at<float>(i) = 0.f;
}

int main() {
    try {
        const int W = 640, H = 480;
        std::vector<uint8_t> img((size_t)W * H);
        orbx_synth_frame(0, 0, W, H, img.data());
        ORBextractor ext(1000, 1.2f, 8, 20, 7);
        // getters from the host-side tables (ORBextractor.cc:415-431)
        const std::vector<float> sc = ext.GetScaleFactors();
        CHECK(ext.GetLevels() == 8 && sc.size() == 8 && sc[0] == 1.f && sc[1] == 1.2f, "scale tables without a device");
        CHECK(ext.GetScaleSigmaSquares()[1] == sc[1] * sc[1], "sigma2 table");
        // operator(): the zero-keypoint result, for every frame (the next frame retries the device)
        for (int f = 0; f < 2; f++) {
            std::vector<cv::KeyPoint> kps(3, cv::KeyPoint(1.f, 1.f, 31.f, 0.f, 1.f, 0, -1));
            cv::Mat desc(3, 32, CV_8U);
            ext(cv::Mat(H, W, CV_8U, img.data(), W), cv::Mat(), kps, desc);
            CHECK(kps.empty() && desc.empty(), "extractor must return no keypoints and released descriptors");
            CHECK(ext.LastStatus() == ORBX_EDEVICE, "LastStatus %d", ext.LastStatus());
        }
        CHECK(amd::LastStatus() == ORBX_EDEVICE, "thread status");
        CHECK(amd::LastStatus() == ORBX_OK, "thread status is reset by the read");
        ext.SyncImagePyramid();
        // matchers: 0 with the reference's initial containers
        std::vector<MapPoint> pool1, pool2;
        KeyFrame kf1, kf2;
        make_kf(kf1, 40, pool1);
        make_kf(kf2, 40, pool2);
        ORBmatcher m(0.6f, true);
        cv::Mat F12(3, 3, CV_32F);
        for (int i = 0; i < 9; i++) F12.at<float>(i / 3, i % 3) = 0.001f * (i + 1);
        std::vector<std::pair<size_t, size_t> > pairs(2, std::make_pair((size_t)1, (size_t)2));
        CHECK(m.SearchForTriangulation(&kf1, &kf2, F12, pairs, false) == 0 && pairs.empty(), "SearchForTriangulation");
        std::vector<MapPoint*> v12(3, &pool1[0]);
        CHECK(m.SearchByBoW(&kf1, &kf2, v12) == 0 && v12.size() == 40u &&
                  std::count(v12.begin(), v12.end(), (MapPoint*)nullptr) == 40,
              "SearchByBoW(KF,KF)");
        Frame F;
        F.N = kf2.N; F.mvKeys = kf2.mvKeys; F.mvKeysUn = kf2.mvKeysUn; F.mDescriptors = kf2.mDescriptors;
        F.mFeatVec = kf2.mFeatVec; F.mvScaleFactors = kf2.mvScaleFactors; F.mvLevelSigma2 = kf2.mvLevelSigma2;
        F.mvuRight = kf2.mvuRight; F.mvpMapPoints.assign(F.N, nullptr); F.mvbOutlier.assign(F.N, false);
        F.fx = F.fy = 500.f; F.cx = 320.f; F.cy = 240.f; F.mnMaxX = 640.f; F.mnMaxY = 480.f;
        F.mfGridElementWidthInv = F.mfGridElementHeightInv = 0.1f;
        F.mTcw = cv::Mat(4, 4, CV_32F);
        for (int i = 0; i < 16; i++) F.mTcw.at<float>(i / 4, i % 4) = (i % 5 == 0) ? 1.f : 0.f;
        std::vector<MapPoint*> vf;
        CHECK(m.SearchByBoW(&kf1, F, vf) == 0 && vf.size() == (size_t)F.N &&
                  std::count(vf.begin(), vf.end(), (MapPoint*)nullptr) == F.N,
              "SearchByBoW(KF,F)");
        std::vector<MapPoint*> local;
        for (int i = 0; i < kf1.N; i += 2) {
            pool1[i].mbTrackInView = true;
            local.push_back(&pool1[i]);
        }
        CHECK(m.SearchByProjection(F, local, 3.f) == 0, "SearchByProjection(F, MapPoints)");
        CHECK(std::count(F.mvpMapPoints.begin(), F.mvpMapPoints.end(), (MapPoint*)nullptr) == F.N, "no assignment");
        Frame last = F;
        last.mvpMapPoints = kf1.mvpMapPoints;
        CHECK(m.SearchByProjection(F, last, 7.f, true) == 0, "SearchByProjection(F, LastF)");
        CHECK(m.SearchByProjection(F, &kf1, std::set<MapPoint*>(), 10.f, 100) == 0, "SearchByProjection(F, KF)");
        cv::Mat Scw(4, 4, CV_32F);
        for (int i = 0; i < 16; i++) Scw.at<float>(i / 4, i % 4) = (i % 5 == 0) ? 1.f : 0.f;
        std::vector<MapPoint*> matched(kf2.N, nullptr);
        CHECK(m.SearchByProjection(&kf2, Scw, local, matched, 10) == 0 &&
                  std::count(matched.begin(), matched.end(), (MapPoint*)nullptr) == kf2.N,
              "SearchByProjection(KF, Scw)");
        std::vector<MapPoint*> before = kf2.mvpMapPoints;
        CHECK(m.Fuse(&kf2, local, 3.f) == 0 && kf2.mvpMapPoints == before, "Fuse leaves the map untouched");
        std::vector<MapPoint*> repl(local.size(), nullptr);
        CHECK(m.Fuse(&kf2, Scw, local, 4.f, repl) == 0 && kf2.mvpMapPoints == before, "Fuse(Scw)");
        // MapPoint::ComputeDistinctiveDescriptors: mDescriptor unchanged
        pool1[0].mObservations[&kf1] = 0;
        pool1[0].mObservations[&kf2] = 2;
        cv::Mat d0 = pool1[0].mDescriptor.clone();
        pool1[0].ComputeDistinctiveDescriptors();
        CHECK(memcmp(d0.data, pool1[0].mDescriptor.data, 32) == 0, "ComputeDistinctiveDescriptors");
        CHECK(amd::LastStatus() == ORBX_EDEVICE, "matchers recorded the device status");
    } catch (const std::exception& e) {
        printf("FAIL: a drop-in threw: %s\n", e.what());
        return 1;
    } catch (...) {
        printf("FAIL: a drop-in threw\n");
        return 1;
    }
    if (failures) {
        printf("%d FAILURES\n", failures);
        return 1;
    }
    printf("ALL PASS\n");
    return 0;
}
