/*
 * ORBextractor.cc -- drop-in ORB_SLAM2::ORBextractor over the C ABI (include/orbslam_amd.h).
 * Replaces ORB_SLAM2/src/ORBextractor.cc; same outputs (bit-exact vs tests' oracle): keypoints
 * level by level in DistributeOctTree order, N x 32 CV_8U descriptors (ORBextractor.cc:1043-1105).
 */
#include "ORBextractor.h"

#include <cassert>
#include <cstdlib>
#include <cstring>

#include "orbamd_status.h"
#include "orbslam_amd.h"

namespace ORB_SLAM2 {

namespace {

// references to a Mat's storage (the extractor's own one included)
int storageRefs(const cv::Mat& m) {
#ifdef CVMIN_CORE_HPP
    return (int)m.store.use_count();
#else
    return m.u ? m.u->refcount : 0;
#endif
}

// an h x w header at p inside buf's storage that shares buf's reference count (as Mat(const Mat&, Rect) does)
cv::Mat storageView(const cv::Mat& buf, const uint8_t* p, int h, int w, size_t step) {
    cv::Mat m(h, w, CV_8U, (void*)p, step);
#ifdef CVMIN_CORE_HPP
    m.store = buf.store;
#else
    if (buf.u) {
        CV_XADD(&buf.u->refcount, 1);
        m.u = buf.u;
    }
#endif
    return m;
}

const size_t kPage = 4096;
const size_t kMaxPyramidSlots = 8;

// the page-aligned registered range inside a slot's storage (whole pages only: no page shared with another allocation)
uint8_t* slotBase(const cv::Mat& b) { return (uint8_t*)(((uintptr_t)b.data + kPage - 1) & ~(uintptr_t)(kPage - 1)); }

}  // namespace

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST), mpHandle(nullptr), mHandleW(0), mHandleH(0), mDevice(0), mHostPyramid(-1),
      mbPyramidStale(false) {
    const char* dev = getenv("ORBAMD_DEVICE");
    if (dev) mDevice = atoi(dev);
    const char* hp = getenv("ORBAMD_HOST_PYRAMID");
    if (hp) mHostPyramid = atoi(hp) != 0 ? 1 : 0;
    // the tables are computed by the library with the reference's float semantics
    // (ORBextractor.cc:415-431), host-only, so the getters answer even without a usable device; the
    // device handle is created on the first frame (at that frame's size)
    mvScaleFactor.assign(nlevels > 0 ? nlevels : 0, 1.f);
    mvInvScaleFactor.assign(mvScaleFactor.size(), 1.f);
    mvLevelSigma2.assign(mvScaleFactor.size(), 1.f);
    mvInvLevelSigma2.assign(mvScaleFactor.size(), 1.f);
    orbx_params p = params();
    amd::StatusOk(orbx_compute_scale_tables(&p, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                                            mvInvLevelSigma2.data()),
                  "orbx_compute_scale_tables");
    mvImagePyramid.resize(mvScaleFactor.size());
}

orbx_params ORBextractor::params() const {
    orbx_params p;
    p.nfeatures = nfeatures;
    p.scale_factor = (float)scaleFactor;
    p.nlevels = nlevels;
    p.ini_th_fast = iniThFAST;
    p.min_th_fast = minThFAST;
    return p;
}

ORBextractor::~ORBextractor() {
    dropPyramidSlots();  // held levels stay valid as ordinary memory
    if (mpHandle) orbx_destroy(mpHandle);
}

void ORBextractor::dropPyramidSlots() {
    if (mpHandle) orbx_set_host_pyramid_target(mpHandle, nullptr, 0);
    for (size_t i = 0; i < mPyrSlots.size(); i++) amd::StatusOk(orbx_host_unregister(slotBase(mPyrSlots[i])), "orbx_host_unregister");
    mPyrSlots.clear();
    mPyrSlotBytes = 0;
    mPyrCur = -1;
    mPyrW = mPyrH = 0;
}

int ORBextractor::selectPyramidSlot(int width, int height) {
    mPyrCur = -1;
    size_t need = mPyrSlotBytes;
    int rc = ORBX_OK;
    if (width != mPyrW || height != mPyrH || !need) {
        rc = orbx_host_pyramid_bytes(mpHandle, width, height, &need);
        if (rc != ORBX_OK) {
            orbx_set_host_pyramid_target(mpHandle, nullptr, 0);  // never the last call's buffer: a caller may hold it
            return rc;
        }
        need = (need + kPage - 1) & ~(kPage - 1);
    }
    if (need != mPyrSlotBytes) {
        dropPyramidSlots();
        mPyrSlotBytes = need;
    }
    mPyrW = width;
    mPyrH = height;
    // the member drops the last call's levels first (the reference reassigns it every call), so a slot referenced only
    // by the extractor is one no caller holds
    for (size_t l = 0; l < mvImagePyramid.size(); l++) mvImagePyramid[l].release();
    for (size_t i = 0; i < mPyrSlots.size() && mPyrCur < 0; i++)
        if (storageRefs(mPyrSlots[i]) == 1) mPyrCur = (int)i;
    if (mPyrCur < 0) {
        if (mPyrSlots.size() >= kMaxPyramidSlots) {  // every slot held: the oldest becomes its holders' ordinary memory
            amd::StatusOk(orbx_host_unregister(slotBase(mPyrSlots.front())), "orbx_host_unregister");
            mPyrSlots.erase(mPyrSlots.begin());
        }
        cv::Mat b(1, (int)(need + kPage), CV_8U);
        rc = orbx_host_register(slotBase(b), need);
        if (rc != ORBX_OK) {
            orbx_set_host_pyramid_target(mpHandle, nullptr, 0);
            return rc;
        }
        mPyrSlots.push_back(b);
        mPyrCur = (int)mPyrSlots.size() - 1;
    }
    rc = orbx_set_host_pyramid_target(mpHandle, slotBase(mPyrSlots[mPyrCur]), need);
    if (rc != ORBX_OK) {
        mPyrCur = -1;
        orbx_set_host_pyramid_target(mpHandle, nullptr, 0);
    }
    return rc;
}

int ORBextractor::ensureHandle(int width, int height) {
    if (mpHandle && width <= mHandleW && height <= mHandleH) return ORBX_OK;
    dropPyramidSlots();
    if (mpHandle) orbx_destroy(mpHandle);
    mpHandle = nullptr;
    mHandleW = mHandleH = 0;
    const orbx_params p = params();
    orbx_handle* h = nullptr;
    const int rc = orbx_create(&p, mDevice, width, height, 1, &h);
    if (rc != ORBX_OK) return rc;  // retried on the next frame
    mpHandle = h;
    mHandleW = width;
    mHandleH = height;
    // eager mvImagePyramid: every call also delivers the levels into the handle's pinned memory (copied beside the
    // octree on the device), so SyncImagePyramid only points the member's Mats at them
    if (HostPyramidEager()) amd::StatusOk(orbx_set_host_pyramid(h, 1), "orbx_set_host_pyramid");
    return ORBX_OK;
}

void ORBextractor::failed(int rc, const char* what, std::vector<cv::KeyPoint>& kps, cv::OutputArray desc) {
    amd::StatusOk(rc, what);
    mLastStatus = rc;
    // the reference's zero-keypoint result (ORBextractor.cc:1064-1065, 1075)
    kps.clear();
    desc.release();
    for (size_t l = 0; l < mvImagePyramid.size(); l++) mvImagePyramid[l].release();
    mbPyramidStale = false;
    // a device error may have left the handle unusable: start from a fresh one on the next frame
    if (rc == ORBX_EDEVICE && mpHandle) {
        orbx_destroy(mpHandle);
        mpHandle = nullptr;
        mHandleW = mHandleH = 0;
    }
}

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint>& _keypoints,
                              cv::OutputArray _descriptors) {
    (void)_mask;
    if (_image.empty()) return;  // ORBextractor.cc:1046-1047
    cv::Mat image = _image.getMat();
    assert(image.type() == CV_8UC1);  // ORBextractor.cc:1050
    int rc = ensureHandle(image.cols, image.rows);
    if (rc != ORBX_OK) return failed(rc, "orbx_create", _keypoints, _descriptors);
    const int cap = orbx_max_keypoints(mpHandle, image.cols, image.rows);
    if (cap < 0) return failed(cap, "orbx_max_keypoints", _keypoints, _descriptors);
    mKpBuf.resize(sizeof(orbx_kp) * (size_t)cap);
    mDescBuf.resize(32 * (size_t)cap);
    int n = 0;
    if (HostPyramidEager()) {
        // storage for this frame's levels that no caller holds; on failure the handle's own pinned memory
        // (valid until the next call) serves instead
        const int sr = selectPyramidSlot(image.cols, image.rows);
        if (sr != ORBX_OK) amd::StatusOk(sr, "host pyramid storage");
    }
    rc = orbx_extract(mpHandle, image.data, image.cols, image.rows, image.step, (orbx_kp*)mKpBuf.data(),
                      mDescBuf.data(), cap, &n);
    if (rc != ORBX_OK) return failed(rc, "orbx_extract", _keypoints, _descriptors);
    mLastStatus = ORBX_OK;
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
    if (HostPyramidEager()) SyncImagePyramid();
}

bool ORBextractor::HostPyramidEager() const {
    // default: eager unless the drop-in Frame::ComputeStereoMatches (the reference's one reader of the
    // member, which reads the device copy instead) is linked in; ORBAMD_HOST_PYRAMID=1 / 0 forces it
    return mHostPyramid >= 0 ? mHostPyramid == 1 : !amd::DevicePyramidReaderRegistered();
}

const std::vector<cv::Mat>& ORBextractor::SyncImagePyramid() {
    if (!mbPyramidStale) return mvImagePyramid;
    mbPyramidStale = false;
    // the levels the last call delivered to pinned host memory (orbx_set_host_pyramid): the member's Mats are headers
    // over them (no copy). Like the reference's member they hold this frame's levels until the next operator() call.
    bool mapped = mpHandle != nullptr;
    for (int l = 0; l < nlevels && mapped; l++) {
        const uint8_t* p = nullptr;
        size_t step = 0;
        int w = 0, h = 0;
        if (orbx_host_pyramid_level(mpHandle, l, &p, &step, &w, &h) != ORBX_OK) {
            mapped = false;
            break;
        }
        mvImagePyramid[l] = mPyrCur >= 0 ? storageView(mPyrSlots[mPyrCur], p, h, w, step) : cv::Mat(h, w, CV_8U, (void*)p, step);
    }
    if (mapped) return mvImagePyramid;
    for (int l = 0; l < nlevels; l++) {
        int w = 0, h = 0;
        int rc = mpHandle ? orbx_pyramid_level(mpHandle, 0, l, nullptr, 0, &w, &h) : ORBX_EDEVICE;
        if (rc == ORBX_OK) {
            // an earlier eager call left a header over the handle's pinned memory here: drop it, so create() allocates
            // storage this member owns instead of writing into (possibly freed) handle memory
            mvImagePyramid[l].release();
            mvImagePyramid[l].create(h, w, CV_8U);
            rc = orbx_pyramid_level(mpHandle, 0, l, mvImagePyramid[l].data, mvImagePyramid[l].step, &w, &h);
        }
        if (!amd::StatusOk(rc, "orbx_pyramid_level")) {  // no pyramid rather than a stale one
            mLastStatus = rc;
            for (int k = 0; k < nlevels; k++) mvImagePyramid[k].release();
            break;
        }
    }
    return mvImagePyramid;
}

}  // namespace ORB_SLAM2
