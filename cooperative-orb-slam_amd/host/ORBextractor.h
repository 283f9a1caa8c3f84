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
 * mvImagePyramid: the pyramid stays on the device. Its one reader in the reference,
 * Frame::ComputeStereoMatches (A1 Frame.cc:474-581), is replaced by host/Frame_stereo_amd.cc, which
 * reads the device copy, so no PCIe copy is made by default. A caller that does read the public
 * member calls SyncImagePyramid() first (a lazy copy of the last call's levels, done once per call),
 * or sets ORBAMD_HOST_PYRAMID=1 to have every call materialise it as the reference does.
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
    bool mbHostPyramid;   // ORBAMD_HOST_PYRAMID=1: materialise after every call
    bool mbPyramidStale;  // mvImagePyramid does not hold the last call's levels yet
    int mLastStatus = 0;
    std::vector<unsigned char> mKpBuf, mDescBuf;
};

}  // namespace ORB_SLAM2

#endif
