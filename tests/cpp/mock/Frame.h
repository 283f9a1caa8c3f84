/* TEST-ONLY mock of the Frame members ORBmatcher::SearchByBoW reads. */
#ifndef FRAME_H
#define FRAME_H
#include "KeyFrame.h"
namespace ORB_SLAM2 {
class Frame {
public:
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    std::vector<float> mvScaleFactors, mvLevelSigma2;
};
}  // namespace ORB_SLAM2
#endif
