/* test_kf_cache_tsan.cpp -- the concurrent host code of the drop-ins under ThreadSanitizer (CPU, no device).
 *
 * 1. The keyframe cache's books (csrc/kf_cache.h, the KfLru that orbm_kf_cache uses) driven by the three ORB-SLAM2
 *    threads that call the matchers (Tracking.cc:767, LocalMapping.cc:268, LoopClosing.cc:267): each looks keyframes
 *    up, builds a missing entry outside the lock and inserts it (so two threads can race on one key), reads the
 *    entry's buffer while the others evict and replace entries (the capacity holds a quarter of the keys), changes a
 *    keyframe's shape now and then (a stale entry is dropped), and forgets keyframes (KeyFrame::SetBadFlag ->
 *    amd::ForgetKeyFrame). Every entry read must hold its own key's bytes, and the books must balance at the end.
 * 2. The C++ drop-in classes on their device-less path (run with ORBAMD_DEVICE=99: every C ABI call returns
 *    ORBX_EDEVICE): 2 extractor threads (the stereo Frame's left / right, Frame.cc:80-81) and 3 matcher threads call
 *    operator() and SearchForTriangulation / SearchByBoW / SearchByProjection / Fuse at once, exercising the drop-ins'
 *    shared state (the per-thread matcher context, the process-wide keyframe cache's static initialisation, the
 *    status counters, ForgetKeyFrame).
 * Prints "ALL PASS" on success; ThreadSanitizer reports any data race on stderr (and fails the exit status). */
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "kf_cache.h"

#ifdef WITH_DROPINS
#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "orbamd_status.h"
using namespace ORB_SLAM2;
#endif

static std::atomic<int> failures{0};
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            printf("FAIL %s:%d ", __FILE__, __LINE__);     \
            printf(__VA_ARGS__);                           \
            printf("\n");                                  \
            failures++;                                    \
        }                                                  \
    } while (0)

struct HostEntry {
    uint64_t key = 0;
    int n = 0;  // the keyframe's N (shape)
    std::vector<uint8_t> data;
    size_t bytes() const { return data.size(); }
};

static uint32_t rng(uint32_t& s) {
    s = s * 1664525u + 1013904223u;
    return s >> 8;
}

static void cache_thread(orbamd::KfLru<HostEntry>* lru, std::atomic<int>* shape, int tid, int iters) {
    uint32_t s = 12345u + 977u * (uint32_t)tid;
    for (int it = 0; it < iters; it++) {
        const uint64_t key = rng(s) % 48;
        const int kind = (int)(key & 1);
        const int n = 200 + 10 * (int)key + shape[key].load(std::memory_order_relaxed);
        auto matches = [&](const HostEntry& e) { return e.n == n; };
        std::shared_ptr<HostEntry> e = lru->find(kind, key, matches);
        if (!e) {  // miss: build outside the lock, then insert (another thread may have won meanwhile)
            auto b = std::make_shared<HostEntry>();
            b->key = key;
            b->n = n;
            b->data.assign((size_t)n * 64, (uint8_t)(key * 7 + 1));
            e = lru->insert(kind, key, b, matches);
        }
        // read the whole buffer while the other threads evict / replace: the shared_ptr keeps it alive
        size_t bad = 0;
        for (uint8_t v : e->data) bad += v != (uint8_t)(key * 7 + 1);
        CHECK(e->key == key && bad == 0 && e->data.size() == (size_t)e->n * 64, "entry of key %llu corrupt",
              (unsigned long long)key);
        const uint32_t r = rng(s) % 64;
        if (r == 0) lru->erase(key);                                                   // ForgetKeyFrame
        if (r == 1) shape[key].fetch_add(1, std::memory_order_relaxed);              // the keyframe changed shape
    }
}

static void test_cache() {
    std::atomic<int> shape[48];
    for (auto& a : shape) a = 0;
    // capacity for about a quarter of the keys' entries: constant eviction
    orbamd::KfLru<HostEntry> lru((size_t)12 * 500 * 64);
    std::vector<std::thread> th;
    for (int t = 0; t < 3; t++) th.emplace_back(cache_thread, &lru, shape, t, 20000);
    for (auto& t : th) t.join();
    int entries = 0;
    size_t bytes = 0;
    long long hits = 0, misses = 0;
    lru.stats(&entries, &bytes, &hits, &misses);
    CHECK(lru.consistent(), "books do not balance: %d entries, %zu bytes", entries, bytes);
    CHECK(hits > 0 && misses > 0 && hits + misses == 60000, "hits %lld misses %lld", hits, misses);
    CHECK(entries > 0 && bytes <= (size_t)12 * 500 * 64, "%d entries, %zu bytes over capacity", entries, bytes);
    lru.clear();
    CHECK(lru.consistent(), "clear");
    printf("cache: %lld hits, %lld misses, %d entries left\n", hits, misses, entries);
}

#ifdef WITH_DROPINS
static void make_kf(KeyFrame& kf, int n, int salt) {
    kf.N = n;
    kf.mnId = (unsigned long)salt;
    kf.mvKeys.clear();
    for (int i = 0; i < n; i++)
        kf.mvKeys.push_back(cv::KeyPoint(20.f + 3 * i, 30.f + 2 * i, 31.f, 10.f * i, 20.f, 0, -1));
    kf.mvKeysUn = kf.mvKeys;
    kf.mDescriptors = cv::Mat(n, 32, CV_8U);
    for (int i = 0; i < n; i++)
        for (int b = 0; b < 32; b++) kf.mDescriptors.at<unsigned char>(i, b) = (unsigned char)(i * 7 + b + salt);
    kf.mvScaleFactors.assign(8, 1.f);
    kf.mvLevelSigma2.assign(8, 1.f);
    kf.mvInvLevelSigma2.assign(8, 1.f);
    kf.mvuRight.assign(n, -1.f);
    kf.fx = kf.fy = 500.f;
    kf.cx = 320.f;
    kf.cy = 240.f;
    kf.mnMaxX = 640.f;
    kf.mnMaxY = 480.f;
    kf.mfGridElementWidthInv = 0.1f;
    kf.mfGridElementHeightInv = 0.1f;
    for (int i = 0; i < n; i++) kf.mFeatVec[5].push_back(i);
    kf.mvpMapPoints.assign(n, nullptr);
    kf.Rcw = cv::Mat(3, 3, CV_32F);
    kf.tcw = cv::Mat(3, 1, CV_32F);
    kf.Ow = cv::Mat(3, 1, CV_32F);
    for (int i = 0; i < 9; i++) kf.Rcw.at<float>(i / 3, i % 3) = (i % 4 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; i++) kf.tcw.at<float>(i) = kf.Ow.at<float>(i) = 0.f;
}

static void extractor_thread(int tid) {
    ORBextractor ext(1000, 1.2f, 8, 20, 7);
    cv::Mat img(480, 640, CV_8U);
    for (int i = 0; i < 640 * 480; i++) img.data[i] = (unsigned char)(i * 31 + tid);
    for (int it = 0; it < 200; it++) {
        std::vector<cv::KeyPoint> kps(3);
        cv::Mat desc(1, 32, CV_8U);
        ext(img, cv::Mat(), kps, desc);
        CHECK(kps.empty() && desc.empty(), "extractor %d: features without a device", tid);
        CHECK(ext.GetLevels() == 8 && ext.GetScaleFactors().size() == 8, "getters");
    }
}

static void matcher_thread(int tid) {
    KeyFrame k1, k2;
    make_kf(k1, 40, tid);
    make_kf(k2, 40, tid + 100);
    std::vector<MapPoint> pool(40);
    std::vector<MapPoint*> local;
    for (int i = 0; i < 40; i += 2) {
        pool[i].mWorldPos = cv::Mat(3, 1, CV_32F);
        pool[i].mNormalVector = cv::Mat(3, 1, CV_32F);
        pool[i].mDescriptor = cv::Mat(1, 32, CV_8U);
        for (int k = 0; k < 3; k++) {
            pool[i].mWorldPos.at<float>(k, 0) = k == 2 ? 2.f : 0.f;
            pool[i].mNormalVector.at<float>(k, 0) = k == 2 ? 1.f : 0.f;
        }
        pool[i].mbTrackInView = true;
        local.push_back(&pool[i]);
    }
    Frame F;
    F.N = k2.N; F.mvKeys = k2.mvKeys; F.mvKeysUn = k2.mvKeysUn; F.mDescriptors = k2.mDescriptors;
    F.mFeatVec = k2.mFeatVec; F.mvScaleFactors = k2.mvScaleFactors; F.mvLevelSigma2 = k2.mvLevelSigma2;
    F.mvuRight = k2.mvuRight; F.mvpMapPoints.assign(F.N, nullptr); F.mvbOutlier.assign(F.N, false);
    F.fx = F.fy = 500.f; F.cx = 320.f; F.cy = 240.f; F.mnMaxX = 640.f; F.mnMaxY = 480.f;
    F.mfGridElementWidthInv = F.mfGridElementHeightInv = 0.1f;
    F.mTcw = cv::Mat(4, 4, CV_32F);
    for (int i = 0; i < 16; i++) F.mTcw.at<float>(i / 4, i % 4) = (i % 5 == 0) ? 1.f : 0.f;
    cv::Mat F12(3, 3, CV_32F);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) F12.at<float>(r, c) = r == c ? 1.f : 0.f;
    for (int it = 0; it < 300; it++) {
        ORBmatcher m(0.75f, true);
        std::vector<std::pair<size_t, size_t>> vm;
        const int a = m.SearchForTriangulation(&k1, &k2, F12, vm, false);
        CHECK(a == 0 && vm.empty(), "thread %d: triangulation without a device", tid);
        std::vector<MapPoint*> v12;
        const int b = m.SearchByBoW(&k1, &k2, v12);
        CHECK(b == 0, "thread %d: SearchByBoW without a device", tid);
        std::vector<MapPoint*> vf;
        CHECK(m.SearchByBoW(&k1, F, vf) == 0, "thread %d: SearchByBoW(KF,F)", tid);       // Tracking
        CHECK(m.SearchByProjection(F, local, 3.f) == 0, "thread %d: SearchByProjection", tid);
        CHECK(m.Fuse(&k2, local, 3.f) == 0, "thread %d: Fuse", tid);                          // LocalMapping
        if (it % 50 == 0) amd::ForgetKeyFrame(&k1, k1.mnId);
        amd::LastStatus();
    }
}

static void test_dropins() {
    std::vector<std::thread> th;
    for (int t = 0; t < 2; t++) th.emplace_back(extractor_thread, t);
    for (int t = 0; t < 3; t++) th.emplace_back(matcher_thread, t);
    for (auto& t : th) t.join();
    printf("drop-ins: 2 extractor + 3 matcher threads done\n");
}
#endif

#ifdef TSAN_CANARY
/* the sanitizer is live: an unsynchronised counter must be reported (tests/test_sanitizers.py builds this form too) */
static int canary_counter = 0;
static void canary_thread() {
    for (int i = 0; i < 100000; i++) canary_counter++;
}
#endif

int main() {
#ifdef TSAN_CANARY
    std::thread a(canary_thread), b(canary_thread);
    a.join();
    b.join();
    printf("canary %d\n", canary_counter);
    return 0;
#endif
    test_cache();
#ifdef WITH_DROPINS
    test_dropins();
#endif
    if (failures) {
        printf("%d FAILURES\n", failures.load());
        return 1;
    }
    printf("ALL PASS\n");
    return 0;
}
