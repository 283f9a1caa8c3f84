/* test_pyramid_reader.cpp -- a stock reader of ORBextractor::mvImagePyramid (the reference's
 * Frame::ComputeStereoMatches reads it straight after ExtractORB, A1 Frame.cc:474-581) against the drop-in
 * extractor built WITHOUT the drop-in stereo (host/Frame_stereo_amd.cc, the device pyramid's reader), and
 * with no ORBAMD_HOST_PYRAMID: every operator() must leave this frame's levels in the public member
 * (ORBextractor.cc:1107-1132), bit-exact against the oracle's pyramid, with no SyncImagePyramid() call.
 * Needs a GPU; prints "ALL PASS". Build: tests/cpp/build.sh */
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ORBextractor.h"
#include "orb_oracle.h"

using namespace ORB_SLAM2;

static int failures = 0;
#define CHECK(cond, ...)                               \
    do {                                               \
        if (!(cond)) {                                 \
            printf("FAIL %s:%d ", __FILE__, __LINE__); \
            printf(__VA_ARGS__);                       \
            printf("\n");                              \
            failures++;                                \
        }                                              \
    } while (0)

int main() {
    const int W = 640, H = 480;
    ORBextractor ext(1000, 1.2f, 8, 20, 7);
    orbx_params prm;
    prm.nfeatures = 1000;
    prm.scale_factor = 1.2f;
    prm.nlevels = 8;
    prm.ini_th_fast = 20;
    prm.min_th_fast = 7;
    oc_extractor* orc = oc_create(&prm);
    CHECK(ext.HostPyramidEager(), "no device pyramid reader linked: operator() must fill mvImagePyramid");
    std::vector<orbx_kp> okp(64 * 1024);
    std::vector<uint8_t> odesc(32 * 64 * 1024), img((size_t)W * H);
    for (int t = 0; t < 3; t++) {  // distinct frames: a stale member would show the previous frame's levels
        orbx_synth_frame(1, t, W, H, img.data());
        cv::Mat im(H, W, CV_8U, img.data(), W);
        std::vector<cv::KeyPoint> kps;
        cv::Mat desc;
        ext(im, cv::Mat(), kps, desc);
        int n = 0;
        oc_extract(orc, img.data(), W, H, W, okp.data(), odesc.data(), 64 * 1024, &n);
        CHECK((int)kps.size() == n && n > 0, "frame %d: %zu keypoints vs oracle %d", t, kps.size(), n);
        // the stock reader: straight after the call, no SyncImagePyramid()
        CHECK((int)ext.mvImagePyramid.size() == ext.GetLevels(), "pyramid levels");
        for (int l = 0; l < ext.GetLevels(); l++) {
            int w, h;
            oc_level_size(orc, l, &w, &h);
            const uint8_t* p = oc_pyramid(orc, l);
            const cv::Mat& m = ext.mvImagePyramid[l];
            CHECK(m.rows == h && m.cols == w, "frame %d level %d size %dx%d vs %dx%d", t, l, m.cols, m.rows, w, h);
            int diff = 0;
            for (int y = 0; y < h && m.rows == h && m.cols == w; y++)
                diff += memcmp(m.ptr<unsigned char>(y), p + (size_t)y * w, w) != 0;
            CHECK(diff == 0, "frame %d: pyramid level %d differs in %d rows", t, l, diff);
        }
    }
    // A level kept past later calls keeps its frame: the reference assigns every level a new Mat per call
    // (ORBextractor.cc:1114-1115), so a reader's shallow copy is never overwritten by the next ExtractORB.
    auto run = [&](int t, std::vector<std::vector<uint8_t> >* lv) {
        orbx_synth_frame(1, t, W, H, img.data());
        cv::Mat im(H, W, CV_8U, img.data(), W);
        std::vector<cv::KeyPoint> kps;
        cv::Mat desc;
        ext(im, cv::Mat(), kps, desc);
        int n = 0;
        oc_extract(orc, img.data(), W, H, W, okp.data(), odesc.data(), 64 * 1024, &n);
        lv->assign(ext.GetLevels(), std::vector<uint8_t>());
        for (int l = 0; l < ext.GetLevels(); l++) {
            int w, h;
            oc_level_size(orc, l, &w, &h);
            (*lv)[l].assign(oc_pyramid(orc, l), oc_pyramid(orc, l) + (size_t)w * h);
        }
    };
    auto same = [&](const cv::Mat& m, const std::vector<uint8_t>& ref) {
        if (m.empty() || (size_t)m.rows * m.cols != ref.size()) return false;
        for (int y = 0; y < m.rows; y++)
            if (memcmp(m.ptr<unsigned char>(y), ref.data() + (size_t)y * m.cols, m.cols)) return false;
        return true;
    };
    std::vector<std::vector<uint8_t> > la, lb;
    run(10, &la);
    std::vector<cv::Mat> kept(ext.mvImagePyramid);  // shallow copies, as a reader that stores the Mats holds them
    run(11, &lb);
    for (int l = 0; l < ext.GetLevels(); l++) {
        CHECK(same(ext.mvImagePyramid[l], lb[l]), "member level %d is not the current frame's", l);
        CHECK(same(kept[l], la[l]), "a kept level %d was overwritten by the next call", l);
        CHECK(kept[l].data != ext.mvImagePyramid[l].data, "kept level %d shares the current frame's storage", l);
    }
    kept.clear();
    // nobody holds a level: consecutive calls reuse one buffer (no allocation, no copy in the steady state)
    run(12, &la);
    const unsigned char* p12 = ext.mvImagePyramid[1].data;
    run(13, &lb);
    CHECK(ext.mvImagePyramid[1].data == p12, "steady state: the level storage was not reused");
    for (int l = 0; l < ext.GetLevels(); l++) CHECK(same(ext.mvImagePyramid[l], lb[l]), "frame 13 level %d", l);
    // more frames held than the extractor keeps registered (8): every held level keeps its frame
    std::vector<cv::Mat> held;
    std::vector<std::vector<uint8_t> > want;
    for (int t = 20; t < 32; t++) {
        std::vector<std::vector<uint8_t> > lt;
        run(t, &lt);
        held.push_back(ext.mvImagePyramid[t % ext.GetLevels()]);
        want.push_back(lt[t % ext.GetLevels()]);
    }
    for (size_t i = 0; i < held.size(); i++) CHECK(same(held[i], want[i]), "held level of frame %d changed", 20 + (int)i);
    oc_destroy(orc);
    printf(failures ? "FAILURES %d\n" : "ALL PASS\n", failures);
    return failures ? 1 : 0;
}
