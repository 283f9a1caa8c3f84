/*
 * MapPoint_distinctive_amd.cc -- MI355X definition of MapPoint::ComputeDistinctiveDescriptors
 * (replaces ORB_SLAM2/src/MapPoint.cc:242-307), plus the batch form
 * MapPoint::ComputeDistinctiveDescriptorsBatch for the call sites that loop over MapPoints
 * (LocalMapping::CreateNewMapPoints and SearchInNeighbors, the cooperative receive path
 * ros_mono.cc:2140): one launch for the whole list instead of one per point.
 *
 * Per MapPoint the observations are copied under mMutexFeatures and the descriptor rows of the
 * non-bad observing KeyFrames gathered in mObservations order, exactly as the reference does; the
 * N x N Hamming matrix, the per-row medians (vDists[0.5*(N-1)] of the sorted row) and the first
 * strict minimum run in k_distinctive (orbm_compute_distinctive_descriptors); mDescriptor is set
 * under the lock. A bad point or one without usable observations is left untouched. A device
 * failure does not throw (orbamd_status.h): every mDescriptor is left unchanged and the status
 * logged. MapPoint.h gains one declaration:
 *     static void ComputeDistinctiveDescriptorsBatch(const std::vector<MapPoint*>& vpMPs);
 */
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "KeyFrame.h"
#include "MapPoint.h"
#include "orbamd_status.h"
#include "orbslam_amd.h"

namespace ORB_SLAM2 {

void MapPoint::ComputeDistinctiveDescriptors() {
    ComputeDistinctiveDescriptorsBatch(std::vector<MapPoint*>(1, this));
}

void MapPoint::ComputeDistinctiveDescriptorsBatch(const std::vector<MapPoint*>& vpMPs) {
    std::vector<MapPoint*> pts;
    std::vector<int32_t> off(1, 0);
    std::vector<uint8_t> desc;
    for (MapPoint* pMP : vpMPs) {
        if (!pMP) continue;
        std::map<KeyFrame*, size_t> observations;
        {
            std::unique_lock<std::mutex> lock1(pMP->mMutexFeatures);
            if (pMP->mbBad) continue;
            observations = pMP->mObservations;
        }
        if (observations.empty()) continue;
        const size_t before = desc.size();
        for (std::map<KeyFrame*, size_t>::iterator mit = observations.begin(); mit != observations.end(); mit++) {
            KeyFrame* pKF = mit->first;
            if (!pKF->isBad()) {
                const unsigned char* r = pKF->mDescriptors.ptr<unsigned char>((int)mit->second);
                desc.insert(desc.end(), r, r + 32);
            }
        }
        if (desc.size() == before) continue;  // vDescriptors.empty(): return
        pts.push_back(pMP);
        off.push_back((int32_t)(desc.size() / 32));
    }
    if (pts.empty()) return;
    std::vector<int32_t> best(pts.size());
    std::vector<uint8_t> out(32 * pts.size());
    orbm_ctx* c = amd::ThreadMatcher();
    if (!c || !amd::StatusOk(orbm_compute_distinctive_descriptors(c, (int)pts.size(), off.data(), desc.data(),
                                                                  best.data(), out.data()),
                             "orbm_compute_distinctive_descriptors"))
        return;
    for (size_t i = 0; i < pts.size(); i++) {
        std::unique_lock<std::mutex> lock(pts[i]->mMutexFeatures);
        pts[i]->mDescriptor = cv::Mat(1, 32, CV_8U, out.data() + 32 * i).clone();
    }
}

}  // namespace ORB_SLAM2
