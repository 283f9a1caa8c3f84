/* TEST-ONLY mock of the KeyFrame members ORBmatcher reads (names as in ORB_SLAM2/include/KeyFrame.h). */
#ifndef KEYFRAME_H
#define KEYFRAME_H
#include <map>
#include <set>
#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>
#include <vector>
#include "MapPoint.h"
#include "ORBVocabulary.h"
namespace DBoW2 {
typedef std::map<unsigned int, std::vector<unsigned int> > FeatureVector;
typedef std::map<unsigned int, double> BowVector;
}
namespace ORB_SLAM2 {
class KeyFrame {
public:
    long unsigned int mnId = 0;
    int N = 0;
    float fx = 0, fy = 0, cx = 0, cy = 0;
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    int mnScaleLevels = 0;
    float mfLogScaleFactor = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    std::vector<float> mvuRight;
    cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    DBoW2::BowVector mBowVec;
    ORBVocabulary* mpORBvocabulary = nullptr;
    bool mbBad = false;
    bool isBad() { return mbBad; }
    void ComputeBoW();
    std::vector<float> mvScaleFactors, mvLevelSigma2;
    std::vector<MapPoint*> mvpMapPoints;
    cv::Mat Rcw, tcw, Ow;
    std::vector<MapPoint*> GetMapPointMatches() { return mvpMapPoints; }
    MapPoint* GetMapPoint(const size_t& i) { return mvpMapPoints[i]; }
    cv::Mat GetRotation() { return Rcw.clone(); }
    cv::Mat GetTranslation() { return tcw.clone(); }
    cv::Mat GetCameraCenter() { return Ow.clone(); }
    float mbf = 0;
    std::vector<float> mvInvLevelSigma2;
    void AddMapPoint(MapPoint* pMP, const size_t& idx) { mvpMapPoints[idx] = pMP; }
    std::set<MapPoint*> GetMapPoints() {  // KeyFrame.cc:173-186
        std::set<MapPoint*> s;
        for (MapPoint* p : mvpMapPoints)
            if (p && !p->isBad()) s.insert(p);
        return s;
    }
};
inline void MapPoint::AddObservation(KeyFrame* pKF, size_t idx) {  // MapPoint.cc:63-74
    if (mObservations.count(pKF)) return;
    mObservations[pKF] = idx;
    nObs += pKF->mvuRight[idx] >= 0 ? 2 : 1;
}
inline void MapPoint::Replace(MapPoint* pMP) {  // MapPoint.cc:130-170 (map bookkeeping only)
    if (pMP == this) return;
    std::map<KeyFrame*, size_t> obs = mObservations;
    mObservations.clear();
    bad = true;
    for (auto& o : obs) {
        if (!pMP->IsInKeyFrame(o.first)) {
            o.first->mvpMapPoints[o.second] = pMP;  // ReplaceMapPointMatch
            pMP->AddObservation(o.first, o.second);
        } else {
            o.first->mvpMapPoints[o.second] = nullptr;  // EraseMapPointMatch
        }
    }
}
}  // namespace ORB_SLAM2
#endif
