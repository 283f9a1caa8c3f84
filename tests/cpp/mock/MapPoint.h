/* TEST-ONLY mock of the MapPoint members ORBmatcher reads (names as in ORB_SLAM2/include/MapPoint.h).
 * GetMinDistance/GetMaxDistance are the two getters INTEGRATION.md asks a maintainer to add
 * (mfMinDistance / mfMaxDistance are private in the reference). */
#ifndef MAPPOINT_H
#define MAPPOINT_H
#include <map>
#include <mutex>
#include <vector>
#include <opencv2/core/core.hpp>
namespace ORB_SLAM2 {
class KeyFrame;
class MapPoint {
public:
    bool bad = false;
    bool& mbBad = bad;  // the reference's flag behind isBad()
    std::map<KeyFrame*, size_t> mObservations;
    std::mutex mMutexFeatures;
    MapPoint() = default;
    MapPoint(const MapPoint& o)
        : bad(o.bad), mObservations(o.mObservations), nObs(o.nObs), mWorldPos(o.mWorldPos),
          mNormalVector(o.mNormalVector), mDescriptor(o.mDescriptor), mfMinDistance(o.mfMinDistance),
          mfMaxDistance(o.mfMaxDistance), mbTrackInView(o.mbTrackInView), mTrackProjX(o.mTrackProjX),
          mTrackProjY(o.mTrackProjY), mTrackProjXR(o.mTrackProjXR), mTrackViewCos(o.mTrackViewCos),
          mnTrackScaleLevel(o.mnTrackScaleLevel) {}
    void ComputeDistinctiveDescriptors();
    static void ComputeDistinctiveDescriptorsBatch(const std::vector<MapPoint*>& vpMPs);
    int nObs = 1;
    cv::Mat mWorldPos, mNormalVector, mDescriptor;
    float mfMinDistance = 0, mfMaxDistance = 0;
    bool mbTrackInView = false;
    float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = 0, mTrackViewCos = 0;
    int mnTrackScaleLevel = 0;
    bool isBad() { return bad; }
    /* MapPoint.cc:63-120, 130-170 (Fuse's updates): observations, replacement */
    bool IsInKeyFrame(KeyFrame* pKF) { return mObservations.count(pKF) > 0; }
    int GetIndexInKeyFrame(KeyFrame* pKF) {  // MapPoint.cc:315-322
        std::map<KeyFrame*, size_t>::iterator it = mObservations.find(pKF);
        return it == mObservations.end() ? -1 : (int)it->second;
    }
    void AddObservation(KeyFrame* pKF, size_t idx);
    void Replace(MapPoint* pMP);
    int Observations() { return nObs; }
    cv::Mat GetWorldPos() { return mWorldPos.clone(); }
    cv::Mat GetNormal() { return mNormalVector.clone(); }
    cv::Mat GetDescriptor() { return mDescriptor.clone(); }
    float GetMinDistance() { return mfMinDistance; }
    float GetMaxDistance() { return mfMaxDistance; }
};
}  // namespace ORB_SLAM2
#endif
