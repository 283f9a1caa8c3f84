/*
 * KeyFrameSlot_amd.h -- the C++ side of the cross-agent keyframe slot (include/orbslam_amd.h,
 * "Cross-agent keyframe slot"), replacing the LCM message lcmKeyFrame::lcmKeyFrameInfo
 * (ORB_SLAM2.1/include/lcmKeyFrame/lcmKeyFrameInfo.hpp:24-150).
 *
 * ReceivedKeyFrame mirrors the receiving agent's receiveKeyframeInfo (ORB_SLAM2/Examples/ROS/
 * ORB_SLAM2/src/ros_mono.cc:79-166) field for field, so Tracking::CreateNewKeyFrame (:2108-2192)
 * builds its KeyFrame / MapPoints from it unchanged. DecodeKeyFrameSlot replaces the LCM handler's
 * message-to-struct copy (:230-544) and validates the slot first (orbx_slot_parse);
 * EncodeKeyFrameSlot replaces the sender's struct-to-message copy (ORB_SLAM2.1/Examples/ROS/
 * ORB_SLAM2/src/ros_mono.cc:1907-2410) for host-resident keyframes (device-resident ones are packed
 * on the GPU by orbx_pack_keyframe_device). Differences from the LCM message, by design: keypoint
 * coordinates and sizes stay float (LCM: int16), descriptors stay bytes (LCM: float rows).
 */
#ifndef KEYFRAME_SLOT_AMD_H
#define KEYFRAME_SLOT_AMD_H

#include <cstddef>
#include <cstdint>
#include <vector>

#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>

#include "KeyFrame.h"  // DBoW2::BowVector / FeatureVector
#include "orbslam_amd.h"

namespace ORB_SLAM2 {
namespace amd {

/* receivePoints (ros_mono.cc:79-86): one per keypoint, as the sender emits them (:2353-2382) */
struct receivePoints {
    bool ifMapPoints;
    int x;  // keypoint index
    float poseX, poseY, poseZ;
};

/* receiveKeyframeInfo (ros_mono.cc:88-166) */
struct ReceivedKeyFrame {
    long unsigned int nNextId = 0, mnId = 0, mnFrameId = 0;
    double mTimeStamp = 0;
    int mnGridCols = 0, mnGridRows = 0;
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    long unsigned int mnTrackReferenceForFrame = 0, mnFuseTargetForKF = 0;
    long unsigned int mnBALocalForKF = 0, mnBAFixedForKF = 0;
    long unsigned int mnLoopQuery = 0;
    int mnLoopWords = 0;
    float mLoopScore = 0;
    long unsigned int mnRelocQuery = 0;
    int mnRelocWords = 0;
    float mRelocScore = 0;
    cv::Mat mTcwGBA, mTcwBefGBA;
    long unsigned int mnBAGlobalForKF = 0;
    float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, mbf = 0, mb = 0, mThDepth = 0;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    std::vector<float> mvuRight, mvDepth;
    cv::Mat mDescriptors;  // N x 32, CV_8U
    DBoW2::BowVector mBowVec;
    DBoW2::FeatureVector mFeatVec;
    cv::Mat mTcp;
    int mnScaleLevels = 0;
    float mfScaleFactor = 0, mfLogScaleFactor = 0;
    std::vector<float> mvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
    int mnMinX = 0, mnMinY = 0, mnMaxX = 0, mnMaxY = 0;
    cv::Mat mK, mTcw;
    std::vector<receivePoints> receiveMapPoints;
    int agent = 0;  // sending agent (not in the LCM message)
    uint32_t flags = 0;  // ORBX_SLOT_F_*: which optional fields the sender filled
};

/* Validate and decode one received slot (host memory, e.g. a row of the all-gather receive buffer
 * copied to the host). Returns false (and leaves `out` untouched) if orbx_slot_parse rejects it. */
bool DecodeKeyFrameSlot(const uint8_t* slot, size_t slot_bytes, ReceivedKeyFrame& out);

/* Encode a keyframe held in host containers into a slot of capacity cap (slot resized to
 * orbx_slot_bytes(cap)). receiveMapPoints entries with ifMapPoints set mark keypoint x as having a
 * MapPoint at pose. Returns the orbx status (ORBX_ECAPACITY if N > cap). */
int EncodeKeyFrameSlot(const ReceivedKeyFrame& kf, int cap, std::vector<uint8_t>& slot);

}  // namespace amd
}  // namespace ORB_SLAM2

#endif
