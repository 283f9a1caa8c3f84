/*
 * orbamd_status.cc -- status reporting and the per-thread matcher context of the C++ drop-ins
 * (orbamd_status.h).
 */
#include "orbamd_status.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>

namespace ORB_SLAM2 {
namespace amd {

namespace {
thread_local int t_last = ORBX_OK;
thread_local unsigned long t_failures = 0;
}  // namespace

bool StatusOk(int rc, const char* what) {
    if (rc == ORBX_OK) return true;
    t_last = rc;
    if (t_failures++ % 1000 == 0)
        fprintf(stderr, "orbslam_amd: %s failed (status %d%s); returning no features / matches\n", what, rc,
                rc == ORBX_EDEVICE ? ", device" : rc == ORBX_ECAPACITY ? ", capacity" : rc == ORBX_EARG ? ", argument" : "");
    return false;
}

int LastStatus() {
    const int s = t_last;
    t_last = ORBX_OK;
    return s;
}

orbm_ctx* ThreadMatcher() {
    struct Holder {
        orbm_ctx* c = nullptr;
        ~Holder() { if (c) orbm_destroy(c); }
    };
    static thread_local Holder h;
    if (!h.c) {
        const char* dev = getenv("ORBAMD_DEVICE");
        orbm_ctx* c = nullptr;
        if (!StatusOk(orbm_create(dev ? atoi(dev) : 0, &c), "orbm_create")) return nullptr;
        h.c = c;
    }
    return h.c;
}

orbm_kf_cache* KeyFrameCache() {
    static orbm_kf_cache* cache = [] {
        const char* mb = getenv("ORBAMD_KF_CACHE_MB");
        const long long cap = mb ? atoll(mb) : 1024;
        if (cap <= 0) return (orbm_kf_cache*)nullptr;
        const char* dev = getenv("ORBAMD_DEVICE");
        orbm_kf_cache* c = nullptr;
        if (!StatusOk(orbm_kf_cache_create(dev ? atoi(dev) : 0, (size_t)cap << 20, &c), "orbm_kf_cache_create"))
            return (orbm_kf_cache*)nullptr;
        return c;
    }();
    return cache;
}

namespace {
std::atomic<bool>& pyramid_reader() {
    static std::atomic<bool> registered{false};  // function-local: safe from any static initialiser
    return registered;
}
}  // namespace

void RegisterDevicePyramidReader() { pyramid_reader().store(true); }
bool DevicePyramidReaderRegistered() { return pyramid_reader().load(); }

void ForgetKeyFrame(const void* pKF, unsigned long mnId) {
    if (orbm_kf_cache* c = KeyFrameCache()) StatusOk(orbm_kf_cache_erase(c, KeyFrameKey(pKF, mnId)), "orbm_kf_cache_erase");
}

}  // namespace amd
}  // namespace ORB_SLAM2
