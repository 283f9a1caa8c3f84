/*
 * ORBextractor.h -- drop-in replacement of ORB_SLAM2/include/ORBextractor.h (public surface of
 * ORBextractor.h:45-85 kept verbatim in meaning: ctor, operator(), the six getters, public
 * mvImagePyramid). The work runs on an MI355X through include/orbslam_amd.h; protected state is
 * a device handle instead of the reference's tables (callers never touch it: Frame.cc:69-75,
 * 252-258; Tracking.cc:119-125).
 *
 * Error behaviour: like the reference, an empty image returns with outputs untouched and a
 * non-8UC1 image asserts (ORBextractor.cc:1046-1050). A device failure never throws into the
 * caller's thread (the reference has no failure mode there and no CPU fallback exists): the call
 * returns the reference's zero-keypoint result (keypoints cleared, descriptors released,
 * ORBextractor.cc:1064-1065), logs the status to stderr (orbamd_status.h) and keeps it in
 * LastStatus(); the next frame retries on a fresh device handle.
 *
 * mvImagePyramid: by default every operator() fills the public member with this frame's levels, as the
 * reference does (ORBextractor.cc:1107-1132), so stock readers (Frame::ComputeStereoMatches, A1
 * Frame.cc:474-581) see the current frame: the device writes the levels into the handle's pinned host
 * memory during the call (orbx_set_host_pyramid) and the member's Mats are views of refcounted storage
 * that this extractor registered for device writes. Like the reference, which assigns every level a
 * freshly allocated Mat in each call (ORBextractor.cc:1114-1115), a level a caller keeps (a shallow
 * copy of the Mat) keeps this frame's pixels after later calls: each call fills storage no caller
 * holds (the one buffer of the last call when nobody kept a level, so no copy and no allocation in the
 * steady state; up to 8 buffers are kept registered, beyond that a held one is handed over to its
 * holders as ordinary memory). When the drop-in Frame::ComputeStereoMatches
 * (host/Frame_stereo_amd.cc) is linked in, it registers itself as the reader of the device copy and the
 * extractor skips the PCIe copy; the member is then filled lazily by SyncImagePyramid() (once per call).
 * ORBAMD_HOST_PYRAMID=1 / 0 forces the eager / lazy form.
 */
#ifndef ORBEXTRACTOR_H
#define ORBEXTRACTOR_H

#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>
#include <vector>

#include "orbslam_amd.h"

namespace ORB_SLAM2 {

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
    ~ORBextractor();

    // Compute the ORB features and descriptors on an image (mask ignored, as in the reference).
    void operator()(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                    cv::OutputArray descriptors);

    int inline GetLevels() { return nlevels; }
    float inline GetScaleFactor() { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    std::vector<cv::Mat> mvImagePyramid;

    // materialise mvImagePyramid from the device for the last call (no-op if already done); returns it
    const std::vector<cv::Mat>& SyncImagePyramid();

    // the device handle holding this extractor's last pyramid (used by the drop-in
    // Frame::ComputeStereoMatches, host/Frame_stereo_amd.cc); addition to the reference surface
    orbx_handle* DeviceHandle() const { return mpHandle; }

    // status of the last operator() / SyncImagePyramid (ORBX_OK or a negative ORBX_E* code); addition
    int LastStatus() const { return mLastStatus; }

    // whether operator() fills mvImagePyramid itself (see above); addition
    bool HostPyramidEager() const;

protected:
    int ensureHandle(int width, int height);
    orbx_params params() const;
    void failed(int rc, const char* what, std::vector<cv::KeyPoint>& kps, cv::OutputArray desc);

    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    std::vector<float> mvScaleFactor;
    std::vector<float> mvInvScaleFactor;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;

    orbx_handle* mpHandle;
    int mHandleW, mHandleH;
    int mDevice;
    int mHostPyramid;     // ORBAMD_HOST_PYRAMID: 1 eager, 0 lazy, -1 (unset) eager unless a device reader is linked
    bool mbPyramidStale;  // mvImagePyramid does not hold the last call's levels yet
    int mLastStatus = 0;
    std::vector<unsigned char> mKpBuf, mDescBuf;
    // eager mvImagePyramid storage: refcounted buffers registered for device writes (orbx_host_register); a call
    // fills one no caller holds (selectPyramidSlot), the member's Mats are views sharing its reference count
    std::vector<cv::Mat> mPyrSlots;
    size_t mPyrSlotBytes = 0;
    int mPyrCur = -1;  // slot the last call filled
    int mPyrW = 0, mPyrH = 0;  // frame size mPyrSlotBytes was computed for
    int selectPyramidSlot(int width, int height);
    void dropPyramidSlots();
};

}  // namespace ORB_SLAM2

#endif
