/*
 * Frame_stereo_amd.cc -- MI355X definition of Frame::ComputeStereoMatches (replaces
 * ORB_SLAM2.1/src/Frame.cc:470-641). The two extractors' pyramids of the
 * stereo pair are still on the device after ExtractORB(0/1) (drop-in ORBextractor), so only the
 * keypoints and descriptors travel; orbx_compute_stereo_matches writes mvuRight / mvDepth.
 * Where the reference would assert (a correlation window outside the level: cv::Mat::rowRange /
 * colRange CV_Assert, which throws cv::Exception) this throws std::runtime_error (ORBX_EARG); a device
 * failure does not throw (orbamd_status.h): every keypoint stays without a stereo match (-1).
 */
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "Frame.h"
#include "ORBextractor.h"
#include "orbamd_status.h"
#include "orbslam_amd.h"

namespace ORB_SLAM2 {

namespace {
// this definition reads the extractors' device pyramids, so they need not materialise mvImagePyramid
const bool kReaderRegistered = (amd::RegisterDevicePyramidReader(), true);

void gather_kps(const std::vector<cv::KeyPoint>& k, std::vector<orbx_kp>& out) {
    out.resize(k.size());
    for (size_t i = 0; i < k.size(); i++) {
        out[i].x = k[i].pt.x;
        out[i].y = k[i].pt.y;
        out[i].size = k[i].size;
        out[i].angle = k[i].angle;
        out[i].response = k[i].response;
        out[i].octave = k[i].octave;
    }
}
}  // namespace

void Frame::ComputeStereoMatches() {
    mvuRight = std::vector<float>(N, -1.0f);
    mvDepth = std::vector<float>(N, -1.0f);
    if (N == 0) return;
    std::vector<orbx_kp> kl, kr;
    gather_kps(mvKeys, kl);
    gather_kps(mvKeysRight, kr);
    cv::Mat dl = mDescriptors.isContinuous() ? mDescriptors : mDescriptors.clone();
    cv::Mat dr = mDescriptorsRight.isContinuous() ? mDescriptorsRight : mDescriptorsRight.clone();
    int nst = 0;
    orbx_handle* hl = mpORBextractorLeft->DeviceHandle();
    orbx_handle* hr = mpORBextractorRight->DeviceHandle();
    if (!hl || !hr) {  // an extractor without a device handle (its device failed): no stereo matches
        amd::StatusOk(ORBX_EDEVICE, "ComputeStereoMatches (no device pyramid)");
        return;
    }
    const int rc = orbx_compute_stereo_matches(hl, hr,
                                               kl.data(), dl.data, N, kr.data(), kr.empty() ? nullptr : dr.data,
                                               (int)kr.size(), mbf, mb, mvuRight.data(), mvDepth.data(), &nst);
    if (rc == ORBX_EARG) throw std::runtime_error("orbslam_amd: orbx_compute_stereo_matches: window outside the level");
    if (!amd::StatusOk(rc, "orbx_compute_stereo_matches")) {
        mvuRight.assign(N, -1.0f);
        mvDepth.assign(N, -1.0f);
    }
}

}  // namespace ORB_SLAM2
