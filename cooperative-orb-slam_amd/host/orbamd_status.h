/*
 * orbamd_status.h -- how the C++ drop-ins handle a non-OK status of the C ABI.
 *
 * The reference's ORBextractor / ORBmatcher never throw on their data paths
 * (ORBextractor.cc:1043-1105; ORBmatcher.cc), and Tracking, LocalMapping and LoopClosing run them
 * on threads without a handler (System.cc:86-101). The drop-ins therefore never throw on a device
 * failure: they log the status to stderr, leave the reference's "nothing found" result (no
 * keypoints and released descriptors, as ORBextractor.cc:1064-1065 does for zero keypoints; zero
 * matches and untouched / NULL-filled match containers for the matchers) and record the status for
 * the calling thread, which a caller may read with amd::LastStatus() (the device-side sticky flag
 * of batched work is orbx_check_error / orbm_check_error of the C ABI).
 */
#ifndef ORBAMD_STATUS_H
#define ORBAMD_STATUS_H

#include <stdint.h>

#include "orbslam_amd.h"

namespace ORB_SLAM2 {
namespace amd {

/* rc == ORBX_OK -> true. Otherwise logs "orbslam_amd: <what> failed (status rc)" to stderr
 * (the first failure of a kind per thread, then every 1000th), records rc as this thread's last
 * status and returns false. */
bool StatusOk(int rc, const char* what);
/* this thread's last non-OK status since the previous call (then reset to ORBX_OK) */
int LastStatus();
/* the calling thread's matcher context (one per thread, as the reference's matchers are stack
 * objects of the Tracking / LocalMapping / LoopClosing threads), created on first use on device
 * ORBAMD_DEVICE (default 0); nullptr (status recorded) when no device is usable. */
orbm_ctx* ThreadMatcher();
/* the process-wide keyframe cache of the drop-in matchers (orbm_kf_cache on ORBAMD_DEVICE, capacity
 * ORBAMD_KF_CACHE_MB MiB, default 1024; ORBAMD_KF_CACHE_MB=0 disables it: nullptr, the uncached calls) */
orbm_kf_cache* KeyFrameCache();
/* cache key of a KeyFrame: its address mixed with mnId (ORB-SLAM2 never frees a KeyFrame, and the id
 * guards against an address reused after one is freed) */
inline uint64_t KeyFrameKey(const void* pKF, unsigned long mnId) {
    return (uint64_t)(uintptr_t)pKF ^ ((uint64_t)mnId * 0x9E3779B97F4A7C15ull);
}
/* the drop-in readers of the device pyramid (host/Frame_stereo_amd.cc, the replacement of the reference's
 * only reader of ORBextractor::mvImagePyramid, Frame::ComputeStereoMatches) register themselves at static
 * initialisation. Without one linked in, every ORBextractor::operator() materialises mvImagePyramid on the
 * host as the reference does (ORBextractor.cc:1107-1132), so a stock reader sees the current frame's levels. */
void RegisterDevicePyramidReader();
bool DevicePyramidReaderRegistered();
/* drop a KeyFrame's cached device arrays (a no-op without the cache): the hook for KeyFrame::SetBadFlag
 * (KeyFrame.cc, after mbBad = true), so culled keyframes stop holding cache capacity until LRU evicts them */
void ForgetKeyFrame(const void* pKF, unsigned long mnId);

}  // namespace amd
}  // namespace ORB_SLAM2
#endif
