/* TEST-ONLY mock of the Frame members ORBmatcher and Frame::ComputeStereoMatches read. */
#ifndef FRAME_H
#define FRAME_H
#include "KeyFrame.h"
namespace ORB_SLAM2 {
class ORBextractor;
class Frame {
public:
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn, mvKeysRight;
    cv::Mat mDescriptors, mDescriptorsRight;
    DBoW2::FeatureVector mFeatVec;
    DBoW2::BowVector mBowVec;
    ORBVocabulary* mpORBvocabulary = nullptr;
    void ComputeBoW();
    std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2;
    std::vector<float> mvuRight, mvDepth;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    cv::Mat mTcw;
    float fx = 0, fy = 0, cx = 0, cy = 0, mbf = 0, mb = 0;  // static in the reference
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;    // static in the reference
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    int mnScaleLevels = 0;
    float mfLogScaleFactor = 0;
    ORBextractor* mpORBextractorLeft = nullptr;
    ORBextractor* mpORBextractorRight = nullptr;
    void ComputeStereoMatches();
};
}  // namespace ORB_SLAM2
#endif
