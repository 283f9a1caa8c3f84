// bench_latency.cpp -- per-call latency of the host C ABI entry points the C++ drop-ins call, measured
// from C++ (no Python in the loop), next to the CPU oracle's same call on the same inputs (1 thread).
// Each row also checks the two outputs are identical. One JSON line per row.
//
//   extract            ORBextractor::operator() on one 640x480 frame (ORBextractor.cc:1043-1105;
//                      Tracking per frame)
//   tri_bf             SearchForTriangulation, one FeatureVector node holding every feature
//   tri_nodes          SearchForTriangulation over ~90 common BoW nodes (LocalMapping.cc:268)
//   bow_kf_f           SearchByBoW(KF, F), 80% MapPoints, ratio 0.7, rotation check (Tracking.cc:767)
//   bow_kf_kf          SearchByBoW(KF, KF), ratio 0.75, rotation check (LoopClosing.cc:267)
//
// Test infrastructure (tests/): the oracle is the baseline and the checker, never the thing measured.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <random>
#include <vector>

#include "orb_oracle.h"
#include "orbslam_amd.h"

namespace {

// a textured synthetic scene: rectangles of random grey over a gradient, plus noise; frame 2 is
// the same scene shifted by (dx, dy) with fresh noise
std::vector<uint8_t> scene(int W, int H, int dx, int dy, unsigned seed) {
    std::mt19937 rs(1234), rn(seed);
    std::vector<int> img((size_t)W * H);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) img[(size_t)y * W + x] = 40 + (x + y) / 16;
    for (int r = 0; r < 700; r++) {
        const int w = 6 + rs() % 40, h = 6 + rs() % 40, x0 = rs() % W + dx, y0 = rs() % H + dy, v = rs() % 200;
        for (int y = std::max(0, y0); y < std::min(H, y0 + h); y++)
            for (int x = std::max(0, x0); x < std::min(W, x0 + w); x++) img[(size_t)y * W + x] = v + 30;
    }
    std::vector<uint8_t> out(img.size());
    for (size_t i = 0; i < img.size(); i++) out[i] = (uint8_t)std::min(255, std::max(0, img[i] + (int)(rn() % 7) - 3));
    return out;
}

struct KF {
    std::vector<orbx_kp> kp;
    std::vector<uint8_t> desc;
    std::vector<float> x, y, ang;
    std::vector<int32_t> oct;
    std::vector<uint8_t> mp;
    std::vector<uint32_t> node_id;
    std::vector<int32_t> node_off, node_feat;
    orbm_kf_view v;
};

void make_view(KF& k, const float* scale, const float* sigma2, int nodes, const std::vector<uint32_t>& ids,
               std::mt19937& rng, double mp_frac) {
    const int n = (int)k.kp.size();
    for (const orbx_kp& p : k.kp) {
        k.x.push_back(p.x);
        k.y.push_back(p.y);
        k.ang.push_back(p.angle);
        k.oct.push_back(p.octave);
    }
    k.mp.resize(n);
    for (int i = 0; i < n; i++) k.mp[i] = (rng() % 1000) < mp_frac * 1000;
    std::map<uint32_t, std::vector<int>> fv;
    for (int i = 0; i < n; i++) fv[nodes == 1 ? 7u : ids[rng() % ids.size()]].push_back(i);
    k.node_off.push_back(0);
    for (auto& e : fv) {
        k.node_id.push_back(e.first);
        for (int i : e.second) k.node_feat.push_back(i);
        k.node_off.push_back((int32_t)k.node_feat.size());
    }
    memset(&k.v, 0, sizeof(k.v));
    k.v.n = n;
    k.v.desc = k.desc.data();
    k.v.x = k.x.data();
    k.v.y = k.y.data();
    k.v.angle = k.ang.data();
    k.v.octave = k.oct.data();
    k.v.has_mp = mp_frac > 0 ? k.mp.data() : nullptr;
    k.v.n_nodes = (int32_t)k.node_id.size();
    k.v.node_id = k.node_id.data();
    k.v.node_off = k.node_off.data();
    k.v.node_feat = k.node_feat.data();
    k.v.nlevels = 8;
    k.v.scale_factors = scale;
    k.v.level_sigma2 = sigma2;
}

/* per-call wall time: the median over reps (robust to preemption of the host thread on a shared box), and
 * the mean beside it */
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

int failures = 0;
void row(const char* name, const char* what, Stat gpu, Stat cpu, bool same, int nmatch) {
    failures += !same;
    printf("{\"row\": \"%s\", \"workload\": \"%s\", \"gpu_host_api_us_per_call\": %.1f, "
           "\"cpu_oracle_us_per_call\": %.1f, \"gpu_mean_us\": %.1f, \"cpu_mean_us\": %.1f, \"stat\": \"median\", "
           "\"cpu_threads\": 1, \"identical\": %s, \"n\": %d, \"harness\": \"C++\"}\n",
           name, what, gpu.median, cpu.median, gpu.mean, cpu.mean, same ? "true" : "false", nmatch);
    fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 2000;
    const int W = 640, H = 480;
    orbx_params prm = {1000, 1.2f, 8, 20, 7};
    orbx_handle* h = nullptr;
    if (orbx_create(&prm, 0, W, H, 1, &h)) {
        printf("orbx_create failed\n");
        return 1;
    }
    oc_extractor* oc = oc_create(&prm);
    const int cap = orbx_max_keypoints(h, W, H);
    std::vector<uint8_t> img1 = scene(W, H, 0, 0, 1), img2 = scene(W, H, 3, 2, 2);
    KF k1, k2;
    {
        std::vector<orbx_kp> kp(cap), kq(cap);
        std::vector<uint8_t> d(32 * (size_t)cap), e(32 * (size_t)cap);
        int n = 0, m = 0;
        bool same = true;
        const Stat g = time_us(reps / 4, [&] { orbx_extract(h, img1.data(), W, H, W, kp.data(), d.data(), cap, &n); });
        const Stat c = time_us(std::max(20, reps / 100),
                                 [&] { oc_extract(oc, img1.data(), W, H, W, kq.data(), e.data(), cap, &m); });
        same = n == m && memcmp(kp.data(), kq.data(), sizeof(orbx_kp) * n) == 0 && memcmp(d.data(), e.data(), 32 * (size_t)n) == 0;
        row("extract", "ORBextractor::operator(), one 640x480 frame, 1000 features", g, c, same, n);
        k1.kp.assign(kq.begin(), kq.begin() + m);
        k1.desc.assign(e.begin(), e.begin() + 32 * (size_t)m);
        oc_extract(oc, img2.data(), W, H, W, kq.data(), e.data(), cap, &m);
        k2.kp.assign(kq.begin(), kq.begin() + m);
        k2.desc.assign(e.begin(), e.begin() + 32 * (size_t)m);
    }
    float scale[8], inv_scale[8], sigma2[8], inv_sigma2[8];
    orbx_get_scale_tables(h, scale, inv_scale, sigma2, inv_sigma2);
    orbm_ctx* ctx = nullptr;
    if (orbm_create(0, &ctx)) {
        printf("orbm_create failed\n");
        return 1;
    }
    // a pure-translation pair's fundamental matrix (any F works for timing; the check is identity)
    const float F12[9] = {0, -1e-3f, 2e-3f * 2, 1e-3f, 0, -3e-3f * 2, -2e-3f * 2, 3e-3f * 2, 0};
    const float ex = 1e4f, ey = 1e4f;
    std::mt19937 rng(7);
    std::vector<uint32_t> ids;
    while (ids.size() < 90) ids.push_back(rng() % 100000);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    for (int variant = 0; variant < 2; variant++) {
        KF a = k1, b = k2;
        a.x.clear(); a.y.clear(); a.ang.clear(); a.oct.clear(); a.node_id.clear(); a.node_off.clear(); a.node_feat.clear();
        b.x.clear(); b.y.clear(); b.ang.clear(); b.oct.clear(); b.node_id.clear(); b.node_off.clear(); b.node_feat.clear();
        const int nodes = variant == 0 ? 1 : 90;
        make_view(a, scale, sigma2, nodes, ids, rng, variant == 0 ? 0.0 : 0.8);
        make_view(b, scale, sigma2, nodes, ids, rng, variant == 0 ? 0.0 : 0.8);
        std::vector<int32_t> mg(a.v.n), mc(a.v.n);
        int ng = 0, nc = 0;
        orbm_kf_view av = a.v, bv = b.v;
        av.has_mp = bv.has_mp = nullptr;  // triangulation: new points only where no MapPoint (none here)
        Stat g = time_us(reps, [&] { orbm_search_for_triangulation(ctx, &av, &bv, F12, ex, ey, 0, 0, mg.data(), &ng); });
        Stat c = time_us(std::max(20, reps / (variant == 0 ? 50 : 2)),
                           [&] { nc = oc_search_for_triangulation(&av, &bv, F12, ex, ey, 0, 0, mc.data()); });
        row(variant == 0 ? "tri_bf" : "tri_nodes",
            variant == 0 ? "SearchForTriangulation, one node (BF), 640x480, ~1000 features"
                         : "SearchForTriangulation over ~90 common BoW nodes (LocalMapping.cc:268)",
            g, c, ng == nc && mg == mc, ng);
        if (variant == 0) continue;
        std::vector<int32_t> fg(b.v.n), fc(b.v.n);
        g = time_us(reps, [&] { orbm_search_by_bow_kf_f(ctx, &a.v, &b.v, 0.7f, 1, fg.data(), &ng); });
        c = time_us(reps / 2, [&] { nc = oc_search_by_bow_kf_f(&a.v, &b.v, 0.7f, 1, fc.data()); });
        row("bow_kf_f", "SearchByBoW(KF, F), ~90 nodes, 80% MapPoints, ratio 0.7, rotation check (Tracking.cc:767)", g, c,
            ng == nc && fg == fc, ng);
        g = time_us(reps, [&] { orbm_search_by_bow_kf_kf(ctx, &a.v, &b.v, 0.75f, 1, mg.data(), &ng); });
        c = time_us(reps / 2, [&] { nc = oc_search_by_bow_kf_kf(&a.v, &b.v, 0.75f, 1, mc.data()); });
        row("bow_kf_kf", "SearchByBoW(KF, KF), ~90 nodes, 80% MapPoints, ratio 0.75 (LoopClosing.cc:267)", g, c,
            ng == nc && mg == mc, ng);
        // the same three calls with both keyframes held in the device keyframe cache (orbm_kf_cache): the
        // drop-ins' default (LocalMapping reuses one keyframe for ~20 calls, LocalMapping.cc:207-268)
        orbm_kf_cache* kc = nullptr;
        if (orbm_kf_cache_create(0, 0, &kc)) {
            printf("orbm_kf_cache_create failed\n");
            return 1;
        }
        g = time_us(reps, [&] {
            orbm_search_for_triangulation_cached(ctx, kc, 1, &av, 2, &bv, F12, ex, ey, 0, 0, mg.data(), &ng);
        });
        c = time_us(reps / 2, [&] { nc = oc_search_for_triangulation(&av, &bv, F12, ex, ey, 0, 0, mc.data()); });
        row("tri_nodes_cached", "SearchForTriangulation over ~90 common BoW nodes, both keyframes in the device cache", g,
            c, ng == nc && mg == mc, ng);
        g = time_us(reps, [&] { orbm_search_by_bow_kf_f_cached(ctx, kc, 1, &a.v, &b.v, 0.7f, 1, fg.data(), &ng); });
        c = time_us(reps / 2, [&] { nc = oc_search_by_bow_kf_f(&a.v, &b.v, 0.7f, 1, fc.data()); });
        row("bow_kf_f_cached", "SearchByBoW(KF, F), ~90 nodes, the keyframe in the device cache", g, c,
            ng == nc && fg == fc, ng);
        g = time_us(reps, [&] { orbm_search_by_bow_kf_kf_cached(ctx, kc, 1, &a.v, 2, &b.v, 0.75f, 1, mg.data(), &ng); });
        c = time_us(reps / 2, [&] { nc = oc_search_by_bow_kf_kf(&a.v, &b.v, 0.75f, 1, mc.data()); });
        row("bow_kf_kf_cached", "SearchByBoW(KF, KF), ~90 nodes, both keyframes in the device cache", g, c,
            ng == nc && mg == mc, ng);
        orbm_kf_cache_destroy(kc);
    }
    orbm_destroy(ctx);
    oc_destroy(oc);
    orbx_destroy(h);
    return failures ? 1 : 0;
}
