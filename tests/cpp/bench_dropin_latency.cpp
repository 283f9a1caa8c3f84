// bench_dropin_latency.cpp -- per-call latency of the drop-in C++ class ORB_SLAM2::ORBextractor (host/ORBextractor.cc)
// as a stock ORB-SLAM2 build calls it, in its default form: no drop-in Frame::ComputeStereoMatches linked, so every
// operator() leaves this frame's levels in the public mvImagePyramid (ORBextractor.cc:1107-1132), as the
// reference does. Rows (one JSON line each, medians over the repetitions, every output checked against the oracle):
//
//   extract_capi          orbx_extract on the same frame (the C ABI the class calls), for a same-box comparison
//   dropin_extract_eager  ORBextractor::operator() + mvImagePyramid filled (Frame::ExtractORB, Frame.cc:252-258)
//   dropin_stereo_pair    two extractors on two std::threads, left and right image, joined: the stereo Frame
//                         constructor's ExtractORB(0) / ExtractORB(1) (Frame.cc:78-81), both pyramids filled
//
// Test infrastructure: the oracle is the checker, never the thing measured. Needs a GPU.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "ORBextractor.h"
#include "orb_oracle.h"

using namespace ORB_SLAM2;

namespace {

struct Stat {
    double median, mean;
};
Stat time_us(int reps, const std::function<void()>& f) {
    for (int i = 0; i < std::max(3, reps / 20); i++) f();
    std::vector<double> t(reps);
    double sum = 0;
    for (int i = 0; i < reps; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        sum += t[i];
    }
    std::nth_element(t.begin(), t.begin() + reps / 2, t.end());
    return {t[reps / 2], sum / reps};
}

struct Ref {
    std::vector<orbx_kp> kp;
    std::vector<uint8_t> desc;
    std::vector<std::vector<uint8_t>> pyr;
    std::vector<int> w, h;
};

Ref oracle_frame(oc_extractor* oc, const std::vector<uint8_t>& img, int W, int H) {
    Ref r;
    r.kp.resize(64 * 1024);
    r.desc.resize(32 * 64 * 1024);
    int n = 0;
    oc_extract(oc, img.data(), W, H, W, r.kp.data(), r.desc.data(), 64 * 1024, &n);
    r.kp.resize(n);
    r.desc.resize(32 * (size_t)n);
    for (int l = 0; l < 8; l++) {
        int w, h;
        oc_level_size(oc, l, &w, &h);
        const uint8_t* p = oc_pyramid(oc, l);
        r.pyr.emplace_back(p, p + (size_t)w * h);
        r.w.push_back(w);
        r.h.push_back(h);
    }
    return r;
}

// keypoints (every cv::KeyPoint field as the C ABI's raw floats), descriptors and every pyramid level
bool same(const ORBextractor& ext, const std::vector<cv::KeyPoint>& kps, const cv::Mat& desc, const Ref& r) {
    if (kps.size() != r.kp.size() || (int)ext.mvImagePyramid.size() != 8) return false;
    for (size_t i = 0; i < kps.size(); i++) {
        const orbx_kp& o = r.kp[i];
        const cv::KeyPoint& k = kps[i];
        if (memcmp(&k.pt.x, &o.x, 4) || memcmp(&k.pt.y, &o.y, 4) || memcmp(&k.size, &o.size, 4) ||
            memcmp(&k.angle, &o.angle, 4) || memcmp(&k.response, &o.response, 4) || k.octave != o.octave)
            return false;
        if (memcmp(desc.ptr<unsigned char>((int)i), r.desc.data() + 32 * i, 32)) return false;
    }
    for (int l = 0; l < 8; l++) {
        const cv::Mat& m = ext.mvImagePyramid[l];
        if (m.rows != r.h[l] || m.cols != r.w[l]) return false;
        for (int y = 0; y < m.rows; y++)
            if (memcmp(m.ptr<unsigned char>(y), r.pyr[l].data() + (size_t)y * r.w[l], r.w[l])) return false;
    }
    return true;
}

void row(const char* name, const char* what, Stat s, bool ok, int n) {
    printf("{\"row\": \"%s\", \"workload\": \"%s\", \"us_per_call\": %.1f, \"mean_us\": %.1f, \"stat\": \"median\", "
           "\"identical\": %s, \"n\": %d, \"harness\": \"C++ drop-in\"}\n",
           name, what, s.median, s.mean, ok ? "true" : "false", n);
    fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 2000;
    const int W = 640, H = 480;
    orbx_params prm = {1000, 1.2f, 8, 20, 7};
    oc_extractor* oc = oc_create(&prm);
    std::vector<uint8_t> imL((size_t)W * H), imR((size_t)W * H);
    orbx_synth_frame(1, 5, W, H, imL.data());
    orbx_synth_frames_shifted(1, 5, 1, W, H, 9, imR.data());  // the right image: disparity 9 px
    const Ref rL = oracle_frame(oc, imL, W, H), rR = oracle_frame(oc, imR, W, H);
    int failures = 0;
    {
        orbx_handle* h = nullptr;
        if (orbx_create(&prm, 0, W, H, 1, &h)) {
            printf("orbx_create failed\n");
            return 1;
        }
        const int cap = orbx_max_keypoints(h, W, H);
        std::vector<orbx_kp> kp(cap);
        std::vector<uint8_t> d(32 * (size_t)cap);
        int n = 0;
        const Stat s = time_us(reps, [&] { orbx_extract(h, imL.data(), W, H, W, kp.data(), d.data(), cap, &n); });
        const bool ok = n == (int)rL.kp.size() && !memcmp(kp.data(), rL.kp.data(), sizeof(orbx_kp) * n) &&
                        !memcmp(d.data(), rL.desc.data(), 32 * (size_t)n);
        failures += !ok;
        row("extract_capi", "orbx_extract, one 640x480 frame, 1000 features (no pyramid to the host)", s, ok, n);
        orbx_destroy(h);
    }
    {
        ORBextractor ext(1000, 1.2f, 8, 20, 7);
        if (!ext.HostPyramidEager()) printf("warning: the extractor is not in its eager default\n");
        cv::Mat im(H, W, CV_8U, imL.data(), W);
        std::vector<cv::KeyPoint> kps;
        cv::Mat desc;
        const Stat s = time_us(reps, [&] { ext(im, cv::Mat(), kps, desc); });
        const bool ok = same(ext, kps, desc, rL);
        failures += !ok;
        row("dropin_extract_eager",
            "ORB_SLAM2::ORBextractor::operator() default (mvImagePyramid filled), one 640x480 frame, 1000 features", s,
            ok, (int)kps.size());
    }
    {
        ORBextractor left(1000, 1.2f, 8, 20, 7), right(1000, 1.2f, 8, 20, 7);
        cv::Mat iml(H, W, CV_8U, imL.data(), W), imr(H, W, CV_8U, imR.data(), W);
        std::vector<cv::KeyPoint> kl, kr;
        cv::Mat dl, dr;
        const Stat s = time_us(reps / 2, [&] {
            std::thread tl([&] { left(iml, cv::Mat(), kl, dl); });
            std::thread tr([&] { right(imr, cv::Mat(), kr, dr); });
            tl.join();
            tr.join();
        });
        const bool ok = same(left, kl, dl, rL) && same(right, kr, dr, rR);
        failures += !ok;
        row("dropin_stereo_pair",
            "two ORBextractor::operator() on two std::threads (Frame.cc:78-81), left + right 640x480, both "
            "mvImagePyramid filled",
            s, ok, (int)(kl.size() + kr.size()));
    }
    oc_destroy(oc);
    return failures ? 1 : 0;
}
