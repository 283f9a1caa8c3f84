/*
 * ORBextractor.cc -- drop-in ORB_SLAM2::ORBextractor over the C ABI (include/orbslam_amd.h).
 * Replaces ORB_SLAM2/src/ORBextractor.cc; same outputs (bit-exact vs tests' oracle): keypoints
 * level by level in DistributeOctTree order, N x 32 CV_8U descriptors (ORBextractor.cc:1043-1105).
 */
#include "ORBextractor.h"

#include <cassert>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "orbslam_amd.h"

namespace ORB_SLAM2 {

static void orbx_ok(int rc, const char* what) {
    if (rc != ORBX_OK) throw std::runtime_error(std::string("orbslam_amd: ") + what + " failed rc=" + std::to_string(rc));
}

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST), mpHandle(nullptr), mHandleW(0), mHandleH(0), mDevice(0), mbHostPyramid(false),
      mbPyramidStale(false) {
    const char* dev = getenv("ORBAMD_DEVICE");
    if (dev) mDevice = atoi(dev);
    const char* hp = getenv("ORBAMD_HOST_PYRAMID");
    if (hp && atoi(hp) != 0) mbHostPyramid = true;
    // the tables are computed by the library with the reference's float semantics
    // (ORBextractor.cc:415-431); a probe handle at 640x480 answers the getters.
    ensureHandle(640, 480);
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    orbx_ok(orbx_get_scale_tables(mpHandle, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                                  mvInvLevelSigma2.data()),
            "orbx_get_scale_tables");
    mvImagePyramid.resize(nlevels);
}

ORBextractor::~ORBextractor() {
    if (mpHandle) orbx_destroy(mpHandle);
}

void ORBextractor::ensureHandle(int width, int height) {
    if (mpHandle && width <= mHandleW && height <= mHandleH) return;
    if (mpHandle) orbx_destroy(mpHandle);
    mpHandle = nullptr;
    orbx_params p;
    p.nfeatures = nfeatures;
    p.scale_factor = (float)scaleFactor;
    p.nlevels = nlevels;
    p.ini_th_fast = iniThFAST;
    p.min_th_fast = minThFAST;
    orbx_ok(orbx_create(&p, mDevice, width, height, 1, &mpHandle), "orbx_create");
    mHandleW = width;
    mHandleH = height;
}

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint>& _keypoints,
                              cv::OutputArray _descriptors) {
    (void)_mask;
    if (_image.empty()) return;  // ORBextractor.cc:1046-1047
    cv::Mat image = _image.getMat();
    assert(image.type() == CV_8UC1);  // ORBextractor.cc:1050
    ensureHandle(image.cols, image.rows);
    const int cap = orbx_max_keypoints(mpHandle, image.cols, image.rows);
    mKpBuf.resize(sizeof(orbx_kp) * (size_t)cap);
    mDescBuf.resize(32 * (size_t)cap);
    int n = 0;
    orbx_ok(orbx_extract(mpHandle, image.data, image.cols, image.rows, image.step, (orbx_kp*)mKpBuf.data(),
                         mDescBuf.data(), cap, &n),
            "orbx_extract");
    if (n == 0) {
        _descriptors.release();  // ORBextractor.cc:1064-1065
    } else {
        _descriptors.create(n, 32, CV_8U);
        cv::Mat d = _descriptors.getMat();
        for (int i = 0; i < n; i++) memcpy(d.ptr<unsigned char>(i), mDescBuf.data() + 32 * (size_t)i, 32);
    }
    _keypoints.clear();
    _keypoints.reserve(n);
    const orbx_kp* k = (const orbx_kp*)mKpBuf.data();
    for (int i = 0; i < n; i++)
        _keypoints.push_back(cv::KeyPoint(k[i].x, k[i].y, k[i].size, k[i].angle, k[i].response, k[i].octave, -1));
    mbPyramidStale = true;
    if (mbHostPyramid) SyncImagePyramid();
}

const std::vector<cv::Mat>& ORBextractor::SyncImagePyramid() {
    if (!mbPyramidStale) return mvImagePyramid;
    for (int l = 0; l < nlevels; l++) {
        int w = 0, h = 0;
        orbx_ok(orbx_pyramid_level(mpHandle, 0, l, nullptr, 0, &w, &h), "orbx_pyramid_level");
        mvImagePyramid[l].create(h, w, CV_8U);
        orbx_ok(orbx_pyramid_level(mpHandle, 0, l, mvImagePyramid[l].data, mvImagePyramid[l].step, &w, &h),
                "orbx_pyramid_level");
    }
    mbPyramidStale = false;
    return mvImagePyramid;
}

}  // namespace ORB_SLAM2
