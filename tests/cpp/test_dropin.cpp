/* test_dropin.cpp -- the C++ drop-in classes (cooperative-orb-slam_amd/host/) used the way
 * ORB-SLAM2's callers use them (Frame::ExtractORB, the stereo Frame's ComputeStereoMatches,
 * LocalMapping/LoopClosing/Tracking matcher calls incl. SearchByProjection), checked bit-exactly
 * against the CPU oracle. Needs a GPU to run; prints
 * "ALL PASS" on success. Build: tests/cpp/build.sh */
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <thread>
#include <string>
#include <set>
#include <vector>

#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "orb_oracle.h"
#include "orbslam_amd.h"
#include "orbamd_status.h"
#include "ORBVocabulary_amd.h"

using namespace ORB_SLAM2;

static int failures = 0;
#define CHECK(cond, ...)                          \
    do {                                          \
        if (!(cond)) {                            \
            printf("FAIL %s:%d ", __FILE__, __LINE__); \
            printf(__VA_ARGS__);                  \
            printf("\n");                         \
            failures++;                           \
        }                                         \
    } while (0)

static uint32_t lcg(uint32_t& s) { s = s * 1664525u + 1013904223u; return s >> 8; }

struct OracleFrame {
    std::vector<orbx_kp> kps;
    std::vector<uint8_t> desc;
};

static bool same_bits(float a, float b) { return memcmp(&a, &b, 4) == 0; }

static void check_extract(ORBextractor& ext, oc_extractor* orc, const uint8_t* img, int W, int H, OracleFrame& of,
                          std::vector<cv::KeyPoint>& kps, cv::Mat& desc) {
    cv::Mat im(H, W, CV_8U, (void*)img, W);
    ext(im, cv::Mat(), kps, desc);
    of.kps.resize(64 * 1024);
    of.desc.resize(32 * 64 * 1024);
    int n = 0;
    oc_extract(orc, img, W, H, W, of.kps.data(), of.desc.data(), 64 * 1024, &n);
    of.kps.resize(n);
    of.desc.resize(32 * (size_t)n);
    CHECK((int)kps.size() == n, "keypoint count %zu vs oracle %d", kps.size(), n);
    if ((int)kps.size() != n) return;
    int bad = 0;
    for (int i = 0; i < n; i++) {
        const cv::KeyPoint& k = kps[i];
        const orbx_kp& o = of.kps[i];
        bad += !(same_bits(k.pt.x, o.x) && same_bits(k.pt.y, o.y) && same_bits(k.size, o.size) &&
                 same_bits(k.angle, o.angle) && same_bits(k.response, o.response) && k.octave == o.octave &&
                 k.class_id == -1);
        bad += memcmp(desc.ptr<unsigned char>(i), of.desc.data() + 32 * (size_t)i, 32) != 0;
    }
    CHECK(bad == 0, "%d keypoint/descriptor rows differ", bad);
    // this binary links the drop-in Frame::ComputeStereoMatches (the device pyramid's reader), so the host
    // pyramid is lazy: no PCIe copy unless a caller asks for it (tests/cpp/test_pyramid_reader.cpp: eager
    // without it)
    if (!getenv("ORBAMD_HOST_PYRAMID")) CHECK(!ext.HostPyramidEager(), "host pyramid eager with the drop-in stereo linked");
    ext.SyncImagePyramid();
    for (int l = 0; l < ext.GetLevels(); l++) {
        int w, h;
        oc_level_size(orc, l, &w, &h);
        const uint8_t* p = oc_pyramid(orc, l);
        const cv::Mat& m = ext.mvImagePyramid[l];
        CHECK(m.rows == h && m.cols == w, "pyramid %d size", l);
        int diff = 0;
        for (int y = 0; y < h && m.rows == h; y++) diff += memcmp(m.ptr<unsigned char>(y), p + (size_t)y * w, w) != 0;
        CHECK(diff == 0, "pyramid level %d differs in %d rows", l, diff);
    }
}

/* KeyFrame built the way KeyFrame(Frame&) fills it (KeyFrame.cc:31), with a synthetic
 * FeatureVector and MapPoint pattern */
static void make_kf(KeyFrame& kf, const std::vector<cv::KeyPoint>& kps, const cv::Mat& desc, ORBextractor& ext,
                    int nodes, uint32_t seed, std::vector<MapPoint>& pool, float mp_frac, float stereo_frac) {
    kf.mnId = 1000 + seed;
    kf.N = (int)kps.size();
    kf.mvKeys = kps;
    kf.mvKeysUn = kps;
    kf.mDescriptors = desc;
    kf.mvScaleFactors = ext.GetScaleFactors();
    kf.mvLevelSigma2 = ext.GetScaleSigmaSquares();
    kf.fx = 715.092024f; kf.fy = 719.025258f; kf.cx = 334.298489f; kf.cy = 256.326097f;
    uint32_t s = seed;
    kf.mFeatVec.clear();
    for (int i = 0; i < kf.N; i++) kf.mFeatVec[100 + 7 * (lcg(s) % nodes)].push_back(i);
    kf.mvuRight.assign(kf.N, -1.f);
    kf.mvpMapPoints.assign(kf.N, nullptr);
    pool.resize(kf.N);
    for (int i = 0; i < kf.N; i++) {
        if ((lcg(s) % 1000) < stereo_frac * 1000) kf.mvuRight[i] = (float)(lcg(s) % 600);
        if ((lcg(s) % 1000) < mp_frac * 1000) {
            pool[i].bad = (lcg(s) % 10) == 0;
            kf.mvpMapPoints[i] = &pool[i];
        }
    }
    kf.Rcw = cv::Mat(3, 3, CV_32F);
    kf.tcw = cv::Mat(3, 1, CV_32F);
    kf.Ow = cv::Mat(3, 1, CV_32F);
    for (int i = 0; i < 9; i++) kf.Rcw.at<float>(i / 3, i % 3) = (i % 4 == 0) ? 1.f : 0.f;
}

struct OView {
    std::vector<float> x, y, a, ur;
    std::vector<int32_t> o, off, feat;
    std::vector<uint32_t> id;
    std::vector<uint8_t> mp, bad;
    orbm_kf_view v;
};
static void oview(KeyFrame& kf, OView& w, bool with_mp, bool with_ur) {
    for (const cv::KeyPoint& k : kf.mvKeysUn) {
        w.x.push_back(k.pt.x); w.y.push_back(k.pt.y); w.a.push_back(k.angle); w.o.push_back(k.octave);
    }
    w.off.push_back(0);
    for (auto& it : kf.mFeatVec) {
        w.id.push_back(it.first);
        for (unsigned f : it.second) w.feat.push_back((int32_t)f);
        w.off.push_back((int32_t)w.feat.size());
    }
    for (MapPoint* p : kf.mvpMapPoints) { w.mp.push_back(p != nullptr); w.bad.push_back(p ? p->bad : 0); }
    w.ur = kf.mvuRight;
    memset(&w.v, 0, sizeof(w.v));
    w.v.n = kf.N; w.v.desc = kf.mDescriptors.data; w.v.x = w.x.data(); w.v.y = w.y.data(); w.v.angle = w.a.data();
    w.v.octave = w.o.data(); w.v.uright = with_ur ? w.ur.data() : nullptr;
    w.v.has_mp = with_mp ? w.mp.data() : nullptr; w.v.mp_bad = with_mp ? w.bad.data() : nullptr;
    w.v.n_nodes = (int32_t)w.id.size(); w.v.node_id = w.id.data(); w.v.node_off = w.off.data();
    w.v.node_feat = w.feat.data(); w.v.nlevels = (int32_t)kf.mvScaleFactors.size();
    w.v.scale_factors = kf.mvScaleFactors.data(); w.v.level_sigma2 = kf.mvLevelSigma2.data();
}

/* ---- Fuse x2 (ORBmatcher.cc:825-975, 977-1100): the drop-in (device search + in-order updates) vs a
 * literal restatement of the reference loop that searches each MapPoint from the map state of its own
 * iteration (oracle oc_fuse* on that one MapPoint), compared on the final map state. */
struct FuseWorld {
    KeyFrame kf;
    std::vector<MapPoint> pre, mps;
    std::vector<MapPoint*> vp;
};
static void build_fuse_world(FuseWorld& w, const std::vector<cv::KeyPoint>& kps, const cv::Mat& desc,
                             ORBextractor& ext, int W, int H, uint32_t seed) {
    KeyFrame& kf = w.kf;
    kf.mnId = seed;  // the drop-ins' keyframe-cache key mixes the address with mnId
    uint32_t s = seed;
    auto urand = [&](float a, float b) { return a + (b - a) * (float)(lcg(s) % 100000) / 100000.f; };
    kf.N = (int)kps.size(); kf.mvKeys = kps; kf.mvKeysUn = kps; kf.mDescriptors = desc;
    kf.mvScaleFactors = ext.GetScaleFactors(); kf.mvLevelSigma2 = ext.GetScaleSigmaSquares();
    kf.mvInvLevelSigma2 = ext.GetInverseScaleSigmaSquares();
    kf.mnScaleLevels = 8; kf.mfLogScaleFactor = logf(1.2f);
    kf.fx = 715.092024f; kf.fy = 719.025258f; kf.cx = 334.298489f; kf.cy = 256.326097f; kf.mbf = 47.9f;
    kf.mnMinX = 0.f; kf.mnMaxX = (float)W; kf.mnMinY = 0.f; kf.mnMaxY = (float)H;
    kf.mfGridElementWidthInv = 64.f / (kf.mnMaxX - kf.mnMinX);
    kf.mfGridElementHeightInv = 48.f / (kf.mnMaxY - kf.mnMinY);
    kf.mvuRight.assign(kf.N, -1.f);
    for (int i = 0; i < kf.N; i++) if (lcg(s) % 2) kf.mvuRight[i] = kps[i].pt.x - urand(1.f, 30.f);
    kf.Rcw = cv::Mat(3, 3, CV_32F);
    for (int i = 0; i < 9; i++) kf.Rcw.at<float>(i / 3, i % 3) = (i % 4 == 0) ? 1.f : 0.f;
    kf.tcw = cv::Mat(3, 1, CV_32F);
    kf.tcw.at<float>(0) = 0.02f; kf.tcw.at<float>(1) = -0.01f; kf.tcw.at<float>(2) = 0.03f;
    kf.Ow = cv::Mat(3, 1, CV_32F);
    for (int k = 0; k < 3; k++) kf.Ow.at<float>(k) = -kf.tcw.at<float>(k);  // -R^T t, R = I
    w.pre.resize(kf.N);
    kf.mvpMapPoints.assign(kf.N, nullptr);
    for (int i = 0; i < kf.N; i++) {
        if (lcg(s) % 5) continue;
        MapPoint& p = w.pre[i];
        p.bad = lcg(s) % 10 == 0;
        p.nObs = 0;
        p.mObservations[&kf] = i;
        p.nObs = (int)(lcg(s) % 6) + 1;
        kf.mvpMapPoints[i] = &p;
    }
    const int M = 700;
    w.mps.resize(M);
    w.vp.resize(M);
    for (int j = 0; j < M; j++) {
        MapPoint& p = w.mps[j];
        w.vp[j] = &p;
        const int src = (int)(lcg(s) % (uint32_t)(j < 100 ? 40 : kf.N));  // the first 100 crowd 40 features
        const float z = urand(1.f, 10.f), nz = lcg(s) % 3 ? 0.002f : 0.02f;
        const float Xc[3] = {(kps[src].pt.x - kf.cx) / kf.fx * z + urand(-nz, nz),
                             (kps[src].pt.y - kf.cy) / kf.fy * z + urand(-nz, nz), z + urand(-nz, nz)};
        p.mWorldPos = cv::Mat(3, 1, CV_32F);
        float d2 = 0;
        for (int k = 0; k < 3; k++) {
            p.mWorldPos.at<float>(k) = Xc[k] - kf.tcw.at<float>(k);  // R = I
            const float o = p.mWorldPos.at<float>(k) - kf.Ow.at<float>(k);
            d2 += o * o;
        }
        const float dist = sqrtf(d2);
        p.mNormalVector = cv::Mat(3, 1, CV_32F);
        const float sg = lcg(s) % 20 == 0 ? -1.f : 1.f;
        for (int k = 0; k < 3; k++)
            p.mNormalVector.at<float>(k) = sg * (p.mWorldPos.at<float>(k) - kf.Ow.at<float>(k)) / dist;
        p.mfMaxDistance = dist * powf(1.2f, (float)kps[src].octave + urand(-0.9f, 0.1f));
        p.mfMinDistance = p.mfMaxDistance / powf(1.2f, 7.f);
        p.mDescriptor = cv::Mat(1, 32, CV_8U);
        memcpy(p.mDescriptor.data, desc.ptr<unsigned char>(src), 32);
        const int nb = (int)(lcg(s) % 31);
        for (int b = 0; b < nb; b++) { const uint32_t r = lcg(s) % 256; p.mDescriptor.data[r >> 3] ^= (uint8_t)(1u << (r & 7)); }
        p.bad = lcg(s) % 20 == 0;
        p.nObs = (int)(lcg(s) % 6) + 1;
        if (lcg(s) % 20 == 0) p.mObservations[&kf] = (size_t)(lcg(s) % kf.N);  // already in the keyframe
    }
}
static orbm_frame_view fuse_kf_view(KeyFrame& kf, std::vector<float>& x, std::vector<float>& y, std::vector<int32_t>& o) {
    x.clear(); y.clear(); o.clear();
    for (const cv::KeyPoint& k : kf.mvKeysUn) { x.push_back(k.pt.x); y.push_back(k.pt.y); o.push_back(k.octave); }
    orbm_frame_view v;
    memset(&v, 0, sizeof(v));
    v.n = kf.N; v.desc = kf.mDescriptors.data; v.x = x.data(); v.y = y.data(); v.octave = o.data();
    v.uright = kf.mvuRight.data();
    v.min_x = kf.mnMinX; v.min_y = kf.mnMinY; v.max_x = kf.mnMaxX; v.max_y = kf.mnMaxY;
    v.grid_w_inv = kf.mfGridElementWidthInv; v.grid_h_inv = kf.mfGridElementHeightInv;
    v.fx = kf.fx; v.fy = kf.fy; v.cx = kf.cx; v.cy = kf.cy; v.bf = kf.mbf;
    v.nlevels = 8; v.scale_factors = kf.mvScaleFactors.data(); v.log_scale_factor = kf.mfLogScaleFactor;
    return v;
}
/* one MapPoint's current state as a 1-entry orbm_mappoints */
struct OneMP {
    float pos[3], nrm[3], mind, maxd;
    orbm_mappoints m;
    explicit OneMP(MapPoint* p) {
        for (int k = 0; k < 3; k++) { pos[k] = p->mWorldPos.at<float>(k); nrm[k] = p->mNormalVector.at<float>(k); }
        mind = p->mfMinDistance; maxd = p->mfMaxDistance;
        memset(&m, 0, sizeof(m));
        m.n = 1; m.desc = p->mDescriptor.data; m.pos = pos; m.normal = nrm; m.min_dist = &mind; m.max_dist = &maxd;
    }
};
/* the reference loops, literally (ORBmatcher.cc:843-972 / 1000-1097) */
static int ref_fuse(FuseWorld& w, float th) {
    KeyFrame* pKF = &w.kf;
    std::vector<float> x, y;
    std::vector<int32_t> o;
    const orbm_frame_view v = fuse_kf_view(*pKF, x, y, o);
    float T[16] = {0};
    for (int r = 0; r < 3; r++) { for (int c = 0; c < 3; c++) T[4 * r + c] = pKF->Rcw.at<float>(r, c); T[4 * r + 3] = pKF->tcw.at<float>(r); }
    int nFused = 0;
    for (MapPoint* pMP : w.vp) {
        if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
        OneMP one(pMP);
        int32_t best = -1;
        oc_fuse(&v, T, pKF->Ow.ptr<float>(), &one.m, th, pKF->mvInvLevelSigma2.data(), &best);
        if (best < 0) continue;
        MapPoint* pMPinKF = pKF->GetMapPoint((size_t)best);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations()) pMP->Replace(pMPinKF);
                else pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, (size_t)best);
            pKF->AddMapPoint(pMP, (size_t)best);
        }
        nFused++;
    }
    return nFused;
}
static int ref_fuse_sim3(FuseWorld& w, const cv::Mat& Scw, float th, std::vector<MapPoint*>& repl) {
    KeyFrame* pKF = &w.kf;
    std::vector<float> x, y;
    std::vector<int32_t> o;
    const orbm_frame_view v = fuse_kf_view(*pKF, x, y, o);
    const std::set<MapPoint*> already = pKF->GetMapPoints();
    int nFused = 0;
    for (size_t i = 0; i < w.vp.size(); i++) {
        MapPoint* pMP = w.vp[i];
        if (pMP->isBad() || already.count(pMP)) continue;
        OneMP one(pMP);
        int32_t best = -1;
        oc_fuse_sim3(&v, Scw.ptr<float>(), &one.m, th, &best);
        if (best < 0) continue;
        MapPoint* pMPinKF = pKF->GetMapPoint((size_t)best);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) repl[i] = pMPinKF;
        } else {
            pMP->AddObservation(pKF, (size_t)best);
            pKF->AddMapPoint(pMP, (size_t)best);
        }
        nFused++;
    }
    return nFused;
}
/* map state as labels: keyframe slot -> "p<k>" / "m<j>"; per MapPoint: bad, index observed in kf */
static std::string label(FuseWorld& w, const MapPoint* p) {
    if (!p) return "-";
    if (p >= w.pre.data() && p < w.pre.data() + w.pre.size()) return "p" + std::to_string(p - w.pre.data());
    return "m" + std::to_string(p - w.mps.data());
}
static int fuse_state_diff(FuseWorld& a, FuseWorld& b) {
    int d = 0;
    for (int i = 0; i < a.kf.N; i++) d += label(a, a.kf.mvpMapPoints[i]) != label(b, b.kf.mvpMapPoints[i]);
    for (size_t j = 0; j < a.mps.size(); j++) {
        MapPoint &p = a.mps[j], &q = b.mps[j];
        const long ia = p.mObservations.count(&a.kf) ? (long)p.mObservations[&a.kf] : -1;
        const long ib = q.mObservations.count(&b.kf) ? (long)q.mObservations[&b.kf] : -1;
        d += p.bad != q.bad || ia != ib || p.nObs != q.nObs;
    }
    for (size_t k = 0; k < a.pre.size(); k++) d += a.pre[k].bad != b.pre[k].bad || a.pre[k].nObs != b.pre[k].nObs;
    return d;
}
static void test_fuse(const std::vector<cv::KeyPoint>& kps, const cv::Mat& desc, ORBextractor& ext, int W, int H) {
    for (float th : {3.0f, 5.0f}) {
        FuseWorld a, b;
        build_fuse_world(a, kps, desc, ext, W, H, 91);
        build_fuse_world(b, kps, desc, ext, W, H, 91);
        const int na = ref_fuse(a, th);
        ORBmatcher m(0.6f, true);
        const int nb = m.Fuse(&b.kf, b.vp, th);
        const int d = fuse_state_diff(a, b);
        CHECK(na == nb && na > 100 && d == 0, "Fuse(pKF, vpMapPoints) th=%.0f: %d vs reference loop %d, %d state diffs",
              th, nb, na, d);
    }
    {
        FuseWorld a, b;
        build_fuse_world(a, kps, desc, ext, W, H, 92);
        build_fuse_world(b, kps, desc, ext, W, H, 92);
        cv::Mat Scw(4, 4, CV_32F);
        for (int i = 0; i < 16; i++) Scw.at<float>(i / 4, i % 4) = (i % 5 == 0) ? 1.f : 0.f;
        const float sc = 1.1f;
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) Scw.at<float>(r, c) = sc * a.kf.Rcw.at<float>(r, c);
            Scw.at<float>(r, 3) = sc * a.kf.tcw.at<float>(r);
        }
        std::vector<MapPoint*> ra(a.vp.size(), nullptr), rb(b.vp.size(), nullptr);
        const int na = ref_fuse_sim3(a, Scw, 4.0f, ra);
        ORBmatcher m(0.75f, true);
        const int nb = m.Fuse(&b.kf, Scw, b.vp, 4.0f, rb);
        int d = fuse_state_diff(a, b);
        for (size_t i = 0; i < ra.size(); i++) d += label(a, ra[i]) != label(b, rb[i]);
        CHECK(na == nb && na > 100 && d == 0, "Fuse(pKF, Scw, vpPoints) : %d vs reference loop %d, %d state diffs", nb, na, d);
    }
}

/* ---- SearchForInitialization (ORBmatcher.cc:405-520) and SearchBySim3 (ORBmatcher.cc:1102-1326) through the
 * drop-in class, vs the oracle on independently gathered views */
static void grid_frame(Frame& F, const std::vector<cv::KeyPoint>& k, const cv::Mat& d, ORBextractor& ext, int W, int H) {
    F.N = (int)k.size(); F.mvKeys = k; F.mvKeysUn = k; F.mDescriptors = d;
    F.mvScaleFactors = ext.GetScaleFactors(); F.mvLevelSigma2 = ext.GetScaleSigmaSquares();
    F.mnScaleLevels = 8; F.mfLogScaleFactor = logf(1.2f);
    F.fx = 715.092024f; F.fy = 719.025258f; F.cx = 334.298489f; F.cy = 256.326097f;
    F.mnMinX = 0.f; F.mnMaxX = (float)W; F.mnMinY = 0.f; F.mnMaxY = (float)H;
    F.mfGridElementWidthInv = 64.f / (F.mnMaxX - F.mnMinX);
    F.mfGridElementHeightInv = 48.f / (F.mnMaxY - F.mnMinY);
}
struct OFrame {
    std::vector<float> x, y, a;
    std::vector<int32_t> o;
    orbm_frame_view v;
};
template <class FK>
static void oframe(FK& F, OFrame& w) {
    for (const cv::KeyPoint& k : F.mvKeysUn) { w.x.push_back(k.pt.x); w.y.push_back(k.pt.y); w.a.push_back(k.angle); w.o.push_back(k.octave); }
    memset(&w.v, 0, sizeof(w.v));
    w.v.n = (int)F.mvKeysUn.size(); w.v.desc = F.mDescriptors.data; w.v.x = w.x.data(); w.v.y = w.y.data();
    w.v.octave = w.o.data(); w.v.angle = w.a.data();
    w.v.min_x = F.mnMinX; w.v.min_y = F.mnMinY; w.v.max_x = F.mnMaxX; w.v.max_y = F.mnMaxY;
    w.v.grid_w_inv = F.mfGridElementWidthInv; w.v.grid_h_inv = F.mfGridElementHeightInv;
    w.v.fx = F.fx; w.v.fy = F.fy; w.v.cx = F.cx; w.v.cy = F.cy;
    w.v.nlevels = (int)F.mvScaleFactors.size(); w.v.scale_factors = F.mvScaleFactors.data();
    w.v.log_scale_factor = F.mfLogScaleFactor;
}

static void test_init_sim3(const std::vector<cv::KeyPoint>& k1, const cv::Mat& d1, const std::vector<cv::KeyPoint>& k2,
                           const cv::Mat& d2, ORBextractor& ext, int W, int H) {
    Frame F1, F2;
    grid_frame(F1, k1, d1, ext, W, H);
    grid_frame(F2, k2, d2, ext, W, H);
    OFrame o1, o2;
    oframe(F1, o1);
    oframe(F2, o2);
    for (int ori = 0; ori < 2; ori++) {
        ORBmatcher m(0.9f, ori != 0);
        std::vector<cv::Point2f> prev;
        for (const cv::KeyPoint& k : F1.mvKeysUn) prev.push_back(k.pt);
        std::vector<float> oprev;
        for (const cv::Point2f& p : prev) { oprev.push_back(p.x); oprev.push_back(p.y); }
        std::vector<int> v12;
        const int n = m.SearchForInitialization(F1, F2, prev, v12, 100);
        std::vector<int32_t> om(F1.N);
        const int on = oc_search_for_initialization(&o1.v, &o2.v, oprev.data(), 100, 0.9f, ori, om.data());
        int diff = 0;
        for (int i = 0; i < F1.N; i++)
            diff += v12[i] != om[i] || !same_bits(prev[i].x, oprev[2 * i]) || !same_bits(prev[i].y, oprev[2 * i + 1]);
        CHECK(n == on && n > 50 && diff == 0, "SearchForInitialization ori=%d: %d vs oracle %d, %d diffs", ori, n, on, diff);
    }
    // SearchBySim3: KF2 = the same features seen through (s12, R12 = I, t12 = 0): Xc2 = Xc1 / s12
    KeyFrame kf1, kf2;
    std::vector<MapPoint> pool1(F1.N), pool2(F1.N);
    for (KeyFrame* kf : {&kf1, &kf2}) {
        kf->N = F1.N; kf->mvKeys = F1.mvKeys; kf->mvKeysUn = F1.mvKeysUn; kf->mDescriptors = F1.mDescriptors;
        kf->mvScaleFactors = F1.mvScaleFactors; kf->mvLevelSigma2 = F1.mvLevelSigma2; kf->mnScaleLevels = 8;
        kf->mfLogScaleFactor = F1.mfLogScaleFactor; kf->fx = F1.fx; kf->fy = F1.fy; kf->cx = F1.cx; kf->cy = F1.cy;
        kf->mnMinX = F1.mnMinX; kf->mnMaxX = F1.mnMaxX; kf->mnMinY = F1.mnMinY; kf->mnMaxY = F1.mnMaxY;
        kf->mfGridElementWidthInv = F1.mfGridElementWidthInv; kf->mfGridElementHeightInv = F1.mfGridElementHeightInv;
        kf->Rcw = cv::Mat(3, 3, CV_32F); kf->tcw = cv::Mat(3, 1, CV_32F); kf->Ow = cv::Mat(3, 1, CV_32F);
        for (int i = 0; i < 9; i++) kf->Rcw.at<float>(i / 3, i % 3) = (i % 4 == 0) ? 1.f : 0.f;
        kf->mvpMapPoints.assign(F1.N, nullptr);
        kf->mvuRight.assign(F1.N, -1.f);
    }
    for (int i = 0; i < 3; i++) { kf1.tcw.at<float>(i, 0) = 0.f; kf2.tcw.at<float>(i, 0) = i == 0 ? 0.1f : 0.f; }
    const float s12 = 1.1f;
    uint32_t s = 4242;
    for (int i = 0; i < F1.N; i++) {
        const float z = 1.f + (float)(lcg(s) % 1000) * 0.01f;
        const float X = (F1.mvKeysUn[i].pt.x - F1.cx) / F1.fx * z, Y = (F1.mvKeysUn[i].pt.y - F1.cy) / F1.fy * z;
        const float sc = powf(1.2f, (float)F1.mvKeysUn[i].octave);
        for (int side = 0; side < 2; side++) {
            if (lcg(s) % 10 < 3) continue;  // no MapPoint
            MapPoint& p = side ? pool2[i] : pool1[i];
            const float f = side ? 1.f / s12 : 1.f;  // camera coordinates of this side
            p.mWorldPos = cv::Mat(3, 1, CV_32F);
            p.mWorldPos.at<float>(0, 0) = X * f - (side ? 0.1f : 0.f);  // Xw = Xc - t (R = I)
            p.mWorldPos.at<float>(1, 0) = Y * f;
            p.mWorldPos.at<float>(2, 0) = z * f;
            p.mDescriptor = cv::Mat(1, 32, CV_8U);
            memcpy(p.mDescriptor.data, F1.mDescriptors.ptr<unsigned char>(i), 32);
            for (int b = 0; b < 6; b++) { const uint32_t r = lcg(s) % 256; p.mDescriptor.data[r >> 3] ^= (uint8_t)(1u << (r & 7)); }
            const float dother = sqrtf(X * X + Y * Y + z * z) * (side ? 1.f : 1.f / s12);
            p.mfMaxDistance = dother * sc * 1.1f;
            p.mfMinDistance = p.mfMaxDistance / 3.6f;
            p.bad = lcg(s) % 20 == 0;
            (side ? kf2 : kf1).mvpMapPoints[i] = &p;
        }
    }
    // a few pairs already matched (vbAlreadyMatched1/2 through GetIndexInKeyFrame)
    std::vector<MapPoint*> v12(F1.N, nullptr);
    for (int i = 0; i < F1.N; i += 37)
        if (kf1.mvpMapPoints[i] && kf2.mvpMapPoints[i]) {
            v12[i] = kf2.mvpMapPoints[i];
            kf2.mvpMapPoints[i]->mObservations[&kf2] = (size_t)i;
        }
    const std::vector<MapPoint*> v12_in = v12;
    cv::Mat R12(3, 3, CV_32F), t12(3, 1, CV_32F);
    for (int i = 0; i < 9; i++) R12.at<float>(i / 3, i % 3) = (i % 4 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; i++) t12.at<float>(i, 0) = 0.f;
    ORBmatcher m(0.75f, true);
    const int n = m.SearchBySim3(&kf1, &kf2, v12, s12, R12, t12, 7.5f);
    // oracle on independently built inputs
    auto omp = [&](KeyFrame& kf, std::vector<uint8_t>& skip, std::vector<uint8_t>& bad, std::vector<uint8_t>& desc,
                   std::vector<float>& pos, std::vector<float>& mind, std::vector<float>& maxd, orbm_mappoints& mp) {
        const int N = kf.N;
        bad.assign(N, 0); desc.assign(32 * (size_t)N, 0); pos.assign(3 * (size_t)N, 0.f); mind.assign(N, 0.f); maxd.assign(N, 0.f);
        for (int i = 0; i < N; i++) {
            MapPoint* p = kf.mvpMapPoints[i];
            if (!p) { skip[i] = 1; continue; }
            bad[i] = p->bad;
            memcpy(&desc[32 * (size_t)i], p->mDescriptor.data, 32);
            for (int k = 0; k < 3; k++) pos[3 * i + k] = p->mWorldPos.at<float>(k, 0);
            mind[i] = p->mfMinDistance; maxd[i] = p->mfMaxDistance;
        }
        memset(&mp, 0, sizeof(mp));
        mp.n = N; mp.desc = desc.data(); mp.pos = pos.data(); mp.min_dist = mind.data(); mp.max_dist = maxd.data();
        mp.bad = bad.data(); mp.skip = skip.data();
    };
    std::vector<uint8_t> sk1(F1.N, 0), sk2(F1.N, 0), b1, b2, de1, de2;
    std::vector<float> p1, p2, mi1, mi2, ma1, ma2;
    for (int i = 0; i < F1.N; i++)
        if (v12_in[i]) { sk1[i] = 1; sk2[i] = 1; }  // GetIndexInKeyFrame(pKF2) == i
    orbm_mappoints m1, m2;
    omp(kf1, sk1, b1, de1, p1, mi1, ma1, m1);
    omp(kf2, sk2, b2, de2, p2, mi2, ma2, m2);
    OFrame ok1, ok2;
    oframe(kf1, ok1);
    oframe(kf2, ok2);
    float T1[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}, T2[16] = {1, 0, 0, 0.1f, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0, 0, 0};
    std::vector<int32_t> om(F1.N);
    const int on = oc_search_by_sim3(&ok1.v, T1, &m1, &ok2.v, T2, &m2, s12, R, t, 7.5f, om.data());
    int diff = 0;
    for (int i = 0; i < F1.N; i++)
        diff += v12[i] != (om[i] >= 0 ? kf2.mvpMapPoints[om[i]] : v12_in[i]);
    CHECK(n == on && n > 50 && diff == 0, "SearchBySim3: %d vs oracle %d, %d diffs", n, on, diff);
}

int main() {
    const int W = 640, H = 480;
    std::vector<uint8_t> frames((size_t)W * H * 3);
    orbx_synth_frames(0, 0, 3, W, H, frames.data());
    ORBextractor ext(1000, 1.2f, 8, 20, 7);
    orbx_params p = {1000, 1.2f, 8, 20, 7};
    oc_extractor* orc = oc_create(&p);
    // getters (ORBextractor.h:63-81) vs the oracle's constructor tables
    std::vector<float> sc(8), isc(8), s2(8), is2(8);
    oc_get_tables(orc, sc.data(), isc.data(), s2.data(), is2.data(), nullptr, nullptr);
    CHECK(ext.GetLevels() == 8 && ext.GetScaleFactor() == 1.2f, "levels/scale");
    CHECK(ext.GetScaleFactors() == sc && ext.GetInverseScaleFactors() == isc && ext.GetScaleSigmaSquares() == s2 &&
              ext.GetInverseScaleSigmaSquares() == is2, "scale tables");
    std::vector<std::vector<cv::KeyPoint> > K(3);
    std::vector<cv::Mat> D(3);
    std::vector<OracleFrame> OF(3);
    for (int f = 0; f < 3; f++) check_extract(ext, orc, frames.data() + (size_t)f * W * H, W, H, OF[f], K[f], D[f]);
    // empty image: outputs untouched (ORBextractor.cc:1046-1047)
    {
        std::vector<cv::KeyPoint> k0 = K[0];
        cv::Mat d0 = D[0];
        ext(cv::Mat(), cv::Mat(), k0, d0);
        CHECK(k0.size() == K[0].size() && d0.data == D[0].data, "empty image must leave outputs untouched");
    }
    // flat image: no keypoints -> descriptors released (ORBextractor.cc:1064-1065)
    {
        std::vector<uint8_t> flat((size_t)W * H, 128);
        std::vector<cv::KeyPoint> k0;
        cv::Mat d0(5, 32, CV_8U);
        ext(cv::Mat(H, W, CV_8U, flat.data(), W), cv::Mat(), k0, d0);
        CHECK(k0.empty() && d0.empty(), "flat image");
    }
    // matcher
    std::vector<MapPoint> pool1, pool2;
    KeyFrame kf1, kf2;
    make_kf(kf1, K[1], D[1], ext, 30, 1, pool1, 0.3f, 0.2f);
    make_kf(kf2, K[0], D[0], ext, 30, 2, pool2, 0.3f, 0.2f);
    kf2.tcw.at<float>(0) = 0.05f; kf2.tcw.at<float>(1) = 0.f; kf2.tcw.at<float>(2) = 0.01f;
    for (int i = 0; i < 3; i++) { kf1.tcw.at<float>(i) = 0.f; kf1.Ow.at<float>(i) = 0.f; kf2.Ow.at<float>(i) = 0.f; }
    // F12 for R12 = I, t12 = -(0.05,0,0.01): K^-T [t]x K^-1 (the matcher only consumes the floats)
    cv::Mat F12(3, 3, CV_32F);
    {
        double fx = kf1.fx, fy = kf1.fy, cx = kf1.cx, cy = kf1.cy, t[3] = {-0.05, 0, -0.01};
        double Kinv[3][3] = {{1 / fx, 0, -cx / fx}, {0, 1 / fy, -cy / fy}, {0, 0, 1}};
        double tx[3][3] = {{0, -t[2], t[1]}, {t[2], 0, -t[0]}, {-t[1], t[0], 0}};
        double A[3][3], F[3][3];
        for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) { A[i][j] = 0; for (int k = 0; k < 3; k++) A[i][j] += Kinv[k][i] * tx[k][j]; }
        for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) { F[i][j] = 0; for (int k = 0; k < 3; k++) F[i][j] += A[i][k] * Kinv[k][j]; F12.at<float>(i, j) = (float)F[i][j]; }
    }
    float ex, ey;
    orbm_epipole(kf2.Rcw.ptr<float>(), kf2.tcw.ptr<float>(), kf1.Ow.ptr<float>(), kf2.fx, kf2.fy, kf2.cx, kf2.cy, &ex, &ey);
    OView o1, o2;
    oview(kf1, o1, true, true);
    oview(kf2, o2, true, true);
    for (int ori = 0; ori < 2; ori++) {
        for (int stereo = 0; stereo < 2; stereo++) {
            ORBmatcher m(0.6f, ori != 0);
            std::vector<std::pair<size_t, size_t> > pairs;
            int n = m.SearchForTriangulation(&kf1, &kf2, F12, pairs, stereo != 0);
            std::vector<int32_t> om(kf1.N);
            int on = oc_search_for_triangulation(&o1.v, &o2.v, F12.ptr<float>(), ex, ey, stereo, ori, om.data());
            std::vector<std::pair<size_t, size_t> > op;
            for (int i = 0; i < kf1.N; i++) if (om[i] >= 0) op.push_back(std::make_pair((size_t)i, (size_t)om[i]));
            CHECK(n == on && pairs == op, "SearchForTriangulation ori=%d stereo=%d: %d vs oracle %d", ori, stereo, n, on);
        }
    }
    for (float ratio : {0.6f, 0.75f}) {
        for (int ori = 0; ori < 2; ori++) {
            ORBmatcher m(ratio, ori != 0);
            std::vector<MapPoint*> v12;
            int n = m.SearchByBoW(&kf1, &kf2, v12);
            std::vector<int32_t> om(kf1.N);
            int on = oc_search_by_bow_kf_kf(&o1.v, &o2.v, ratio, ori, om.data());
            int diff = 0;
            for (int i = 0; i < kf1.N; i++) diff += v12[i] != (om[i] >= 0 ? kf2.mvpMapPoints[om[i]] : nullptr);
            CHECK(n == on && diff == 0, "SearchByBoW(KF,KF) ratio=%.2f ori=%d: %d vs %d, %d diffs", ratio, ori, n, on, diff);
            Frame F;
            F.N = kf2.N; F.mvKeys = kf2.mvKeys; F.mvKeysUn = kf2.mvKeysUn; F.mDescriptors = kf2.mDescriptors;
            F.mFeatVec = kf2.mFeatVec; F.mvScaleFactors = kf2.mvScaleFactors; F.mvLevelSigma2 = kf2.mvLevelSigma2;
            std::vector<MapPoint*> vf;
            n = m.SearchByBoW(&kf1, F, vf);
            OView ofv;
            oview(kf2, ofv, false, false);
            std::vector<int32_t> omf(F.N);
            on = oc_search_by_bow_kf_f(&o1.v, &ofv.v, ratio, ori, omf.data());
            diff = 0;
            for (int i = 0; i < F.N; i++) diff += vf[i] != (omf[i] >= 0 ? kf1.mvpMapPoints[omf[i]] : nullptr);
            CHECK(n == on && diff == 0, "SearchByBoW(KF,F) ratio=%.2f ori=%d: %d vs %d, %d diffs", ratio, ori, n, on, diff);
        }
    }
    // ---- SearchByProjection(Frame&, vector<MapPoint*>, th) and (Frame&, const Frame&, th, bMono)
    {
        Frame F;
        F.N = (int)K[0].size(); F.mvKeys = K[0]; F.mvKeysUn = K[0]; F.mDescriptors = D[0];
        F.mvScaleFactors = ext.GetScaleFactors(); F.mvLevelSigma2 = ext.GetScaleSigmaSquares();
        F.mnScaleLevels = 8; F.mfLogScaleFactor = logf(1.2f);
        F.fx = 715.092024f; F.fy = 719.025258f; F.cx = 334.298489f; F.cy = 256.326097f; F.mbf = 47.9f; F.mb = F.mbf / F.fx;
        F.mnMinX = 0.f; F.mnMaxX = (float)W; F.mnMinY = 0.f; F.mnMaxY = (float)H;
        F.mfGridElementWidthInv = 64.f / (F.mnMaxX - F.mnMinX);
        F.mfGridElementHeightInv = 48.f / (F.mnMaxY - F.mnMinY);
        uint32_t s = 77;
        F.mvuRight.assign(F.N, -1.f);
        for (int i = 0; i < F.N; i++) if (lcg(s) % 2) F.mvuRight[i] = F.mvKeys[i].pt.x - (float)(lcg(s) % 30);
        std::vector<MapPoint> pre(F.N);
        F.mvpMapPoints.assign(F.N, nullptr);
        for (int i = 0; i < F.N; i++)
            if (lcg(s) % 20 == 0) { pre[i].nObs = (int)(lcg(s) % 2); F.mvpMapPoints[i] = &pre[i]; }
        const std::vector<MapPoint*> F0 = F.mvpMapPoints;
        // local-map points near the frame's features (isInFrustum fields), with duplicates
        const int M = 900;
        std::vector<MapPoint> mp(M);
        std::vector<MapPoint*> vp(M);
        for (int j = 0; j < M; j++) {
            const int src = (int)(lcg(s) % F.N);
            MapPoint& p = mp[j];
            vp[j] = &p;
            p.mDescriptor = cv::Mat(1, 32, CV_8U);
            memcpy(p.mDescriptor.data, F.mDescriptors.ptr<unsigned char>(src), 32);
            for (int b = 0; b < 8; b++) { const uint32_t r = lcg(s) % 256; p.mDescriptor.data[r >> 3] ^= (uint8_t)(1u << (r & 7)); }
            p.bad = lcg(s) % 25 == 0;
            p.nObs = lcg(s) % 6 ? 2 : 0;
            p.mbTrackInView = lcg(s) % 10 != 0;
            p.mTrackProjX = F.mvKeys[src].pt.x + (float)((int)(lcg(s) % 7) - 3) * 0.5f;
            p.mTrackProjY = F.mvKeys[src].pt.y + (float)((int)(lcg(s) % 7) - 3) * 0.5f;
            p.mTrackProjXR = p.mTrackProjX - (float)(lcg(s) % 30);
            p.mnTrackScaleLevel = F.mvKeys[src].octave;
            p.mTrackViewCos = lcg(s) % 2 ? 0.9995f : 0.99f;
        }
        // oracle inputs built independently of the drop-in's gathering
        std::vector<float> fx_(F.N), fy_(F.N), fa_(F.N);
        std::vector<int32_t> fo_(F.N);
        std::vector<uint8_t> occ(F.N);
        for (int i = 0; i < F.N; i++) {
            fx_[i] = F.mvKeysUn[i].pt.x; fy_[i] = F.mvKeysUn[i].pt.y; fa_[i] = F.mvKeysUn[i].angle;
            fo_[i] = F.mvKeysUn[i].octave; occ[i] = F0[i] && F0[i]->nObs > 0;
        }
        orbm_frame_view fv;
        memset(&fv, 0, sizeof(fv));
        fv.n = F.N; fv.desc = F.mDescriptors.data; fv.x = fx_.data(); fv.y = fy_.data(); fv.octave = fo_.data();
        fv.angle = fa_.data(); fv.uright = F.mvuRight.data(); fv.occupied = occ.data();
        fv.min_x = F.mnMinX; fv.min_y = F.mnMinY; fv.max_x = F.mnMaxX; fv.max_y = F.mnMaxY;
        fv.grid_w_inv = F.mfGridElementWidthInv; fv.grid_h_inv = F.mfGridElementHeightInv;
        fv.fx = F.fx; fv.fy = F.fy; fv.cx = F.cx; fv.cy = F.cy; fv.bf = F.mbf; fv.b = F.mb;
        fv.nlevels = 8; fv.scale_factors = F.mvScaleFactors.data(); fv.log_scale_factor = F.mfLogScaleFactor;
        std::vector<uint8_t> md(32 * M), mbad(M), mobs(M), miv(M);
        std::vector<float> mpx(M), mpy(M), mpxr(M), mcos(M);
        std::vector<int32_t> mlv(M);
        for (int j = 0; j < M; j++) {
            memcpy(&md[32 * j], mp[j].mDescriptor.data, 32);
            mbad[j] = mp[j].bad; mobs[j] = mp[j].nObs > 0; miv[j] = mp[j].mbTrackInView;
            mpx[j] = mp[j].mTrackProjX; mpy[j] = mp[j].mTrackProjY; mpxr[j] = mp[j].mTrackProjXR;
            mlv[j] = mp[j].mnTrackScaleLevel; mcos[j] = mp[j].mTrackViewCos;
        }
        orbm_mappoints om;
        memset(&om, 0, sizeof(om));
        om.n = M; om.desc = md.data(); om.bad = mbad.data(); om.has_obs = mobs.data(); om.track_in_view = miv.data();
        om.track_proj_x = mpx.data(); om.track_proj_y = mpy.data(); om.track_proj_xr = mpxr.data();
        om.track_level = mlv.data(); om.track_view_cos = mcos.data();
        for (float th : {1.0f, 3.0f}) {
            F.mvpMapPoints = F0;
            ORBmatcher m(0.8f, false);
            const int n = m.SearchByProjection(F, vp, th);
            std::vector<int32_t> ref(F.N);
            const int on = oc_search_by_projection_local(&fv, &om, th, 0.8f, ref.data());
            int diff = 0;
            for (int i = 0; i < F.N; i++) diff += F.mvpMapPoints[i] != (ref[i] >= 0 ? vp[ref[i]] : F0[i]);
            CHECK(n == on && diff == 0, "SearchByProjection(F, local) th=%.0f: %d vs oracle %d, %d diffs", th, n, on, diff);
        }
        // motion model: LastFrame's MapPoints back-projected from the current keypoints (identity current pose)
        Frame L;
        L.N = F.N; L.mvKeys = F.mvKeys; L.mvKeysUn = F.mvKeysUn;
        L.mvpMapPoints.assign(L.N, nullptr);
        L.mvbOutlier.assign(L.N, false);
        std::vector<MapPoint> lp(L.N);
        for (int i = 0; i < L.N; i++) {
            if (lcg(s) % 8 == 0) continue;
            MapPoint& p = lp[i];
            const float z = 1.f + (float)(lcg(s) % 1000) * 0.01f;
            p.mWorldPos = cv::Mat(3, 1, CV_32F);
            p.mWorldPos.at<float>(0, 0) = (F.mvKeys[i].pt.x - F.cx) / F.fx * z;
            p.mWorldPos.at<float>(1, 0) = (F.mvKeys[i].pt.y - F.cy) / F.fy * z;
            p.mWorldPos.at<float>(2, 0) = z;
            p.mDescriptor = cv::Mat(1, 32, CV_8U);
            memcpy(p.mDescriptor.data, F.mDescriptors.ptr<unsigned char>(i), 32);
            p.mDescriptor.data[lcg(s) % 32] ^= 0x11;
            p.nObs = lcg(s) % 5 ? 1 : 0;
            L.mvpMapPoints[i] = &p;
            L.mvbOutlier[i] = lcg(s) % 15 == 0;
        }
        F.mTcw = cv::Mat(4, 4, CV_32F);
        L.mTcw = cv::Mat(4, 4, CV_32F);
        for (int i = 0; i < 16; i++) F.mTcw.at<float>(i / 4, i % 4) = L.mTcw.at<float>(i / 4, i % 4) = (i % 5 == 0) ? 1.f : 0.f;
        L.mTcw.at<float>(2, 3) = -0.02f;
        std::vector<uint8_t> lsk(L.N), lobs(L.N), lmd(32 * L.N);
        std::vector<float> lpos(3 * L.N), lang(L.N);
        std::vector<int32_t> loct(L.N);
        for (int i = 0; i < L.N; i++) {
            lsk[i] = !L.mvpMapPoints[i] || L.mvbOutlier[i];
            loct[i] = L.mvKeys[i].octave; lang[i] = L.mvKeysUn[i].angle;
            if (!L.mvpMapPoints[i]) continue;
            lobs[i] = L.mvpMapPoints[i]->nObs > 0;
            memcpy(&lmd[32 * i], L.mvpMapPoints[i]->mDescriptor.data, 32);
            for (int k = 0; k < 3; k++) lpos[3 * i + k] = L.mvpMapPoints[i]->mWorldPos.at<float>(k, 0);
        }
        orbm_mappoints ol;
        memset(&ol, 0, sizeof(ol));
        ol.n = L.N; ol.desc = lmd.data(); ol.pos = lpos.data(); ol.has_obs = lobs.data(); ol.skip = lsk.data();
        ol.octave = loct.data(); ol.angle = lang.data();
        for (int mono = 0; mono < 2; mono++) {
            F.mvpMapPoints = F0;
            ORBmatcher m(0.9f, true);
            const int n = m.SearchByProjection(F, L, 7.0f, mono != 0);
            std::vector<int32_t> ref(F.N);
            const int on = oc_search_by_projection_last_frame(&fv, F.mTcw.ptr<float>(), &ol, L.mTcw.ptr<float>(), 7.0f,
                                                              mono, 1, ref.data());
            int diff = 0;
            for (int i = 0; i < F.N; i++)
                diff += F.mvpMapPoints[i] != (ref[i] >= 0 ? L.mvpMapPoints[ref[i]] : (ref[i] == -2 ? nullptr : F0[i]));
            CHECK(n == on && n > F.N / 4 && diff == 0, "SearchByProjection(F, LastFrame) mono=%d: %d vs oracle %d, %d diffs",
                  mono, n, on, diff);
        }
    }
    // ---- Frame::ComputeStereoMatches with two extractors (the stereo Frame ctor, Frame.cc:80-98)
    {
        std::vector<uint8_t> right((size_t)W * H);
        orbx_synth_frames_shifted(0, 0, 1, W, H, 9, right.data());
        ORBextractor el(1000, 1.2f, 8, 20, 7), er(1000, 1.2f, 8, 20, 7);
        Frame F;
        cv::Mat iml(H, W, CV_8U, frames.data(), W), imr(H, W, CV_8U, right.data(), W);
        el(iml, cv::Mat(), F.mvKeys, F.mDescriptors);
        er(imr, cv::Mat(), F.mvKeysRight, F.mDescriptorsRight);
        F.N = (int)F.mvKeys.size();
        F.mpORBextractorLeft = &el; F.mpORBextractorRight = &er;
        F.mbf = 47.90639384423901f; F.mb = 0.11f;
        F.ComputeStereoMatches();
        oc_extractor* ol = oc_create(&p);
        oc_extractor* orr = oc_create(&p);
        std::vector<orbx_kp> kl(64 * 1024), kr(64 * 1024);
        std::vector<uint8_t> dl(32 * 64 * 1024), dr(32 * 64 * 1024);
        int nl = 0, nr = 0;
        oc_extract(ol, frames.data(), W, H, W, kl.data(), dl.data(), 64 * 1024, &nl);
        oc_extract(orr, right.data(), W, H, W, kr.data(), dr.data(), 64 * 1024, &nr);
        std::vector<float> ur(nl), dp(nl);
        const int ok = oc_compute_stereo_matches(ol, orr, kl.data(), dl.data(), nl, kr.data(), dr.data(), nr, F.mbf, F.mb,
                                                 ur.data(), dp.data());
        int diff = 0, kept = 0;
        for (int i = 0; i < nl && nl == F.N; i++) {
            diff += !same_bits(F.mvuRight[i], ur[i]) || !same_bits(F.mvDepth[i], dp[i]);
            kept += F.mvuRight[i] >= 0;
        }
        CHECK(nl == F.N && diff == 0 && ok == kept && kept > F.N / 4, "ComputeStereoMatches: %d diffs, kept %d vs %d", diff,
              kept, ok);
        oc_destroy(ol);
        oc_destroy(orr);
    }
    // ---- MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307): single and batched
    {
        const int NKF = 12, NP = 300;
        std::vector<KeyFrame> kfs(NKF);
        uint32_t s = 4242;
        for (int k = 0; k < NKF; k++) {
            kfs[k].mDescriptors = cv::Mat(64, 32, CV_8U);
            for (int i = 0; i < 64 * 32; i++) kfs[k].mDescriptors.data[i] = (uint8_t)(lcg(s) & 0xFF);
            kfs[k].mbBad = k == 5;  // its rows are skipped
        }
        std::vector<MapPoint> mps(NP);
        std::vector<MapPoint*> vp(NP);
        std::vector<int32_t> off(1, 0);
        std::vector<uint8_t> od;
        std::vector<int> has(NP, 0);
        for (int p = 0; p < NP; p++) {
            MapPoint& m = mps[p];
            vp[p] = &m;
            m.mDescriptor = cv::Mat(1, 32, CV_8U);
            memset(m.mDescriptor.data, 0xEE, 32);
            m.bad = p % 37 == 0;
            const int nobs = (int)(lcg(s) % 14);  // 0 .. 13 observations
            for (int o = 0; o < nobs; o++) m.mObservations[&kfs[lcg(s) % NKF]] = lcg(s) % 64;
            // oracle input: the same gathering, done independently
            const size_t before = od.size();
            if (!m.bad)
                for (auto& ob : m.mObservations)
                    if (!ob.first->mbBad) {
                        const unsigned char* r = ob.first->mDescriptors.ptr<unsigned char>((int)ob.second);
                        od.insert(od.end(), r, r + 32);
                    }
            if (od.size() > before) { has[p] = (int)off.size(); off.push_back((int32_t)(od.size() / 32)); }
        }
        std::vector<int32_t> ob(off.size() - 1);
        oc_compute_distinctive_descriptors((int)ob.size(), off.data(), od.data(), ob.data());
        mps[1].ComputeDistinctiveDescriptors();
        MapPoint::ComputeDistinctiveDescriptorsBatch(vp);
        int diff = 0, untouched = 0;
        for (int p = 0; p < NP; p++) {
            if (!has[p]) {
                for (int b = 0; b < 32; b++) diff += mps[p].mDescriptor.data[b] != 0xEE;
                untouched++;
                continue;
            }
            const int q = has[p] - 1;
            diff += memcmp(mps[p].mDescriptor.data, od.data() + 32 * (off[q] + ob[q]), 32) != 0;
        }
        CHECK(diff == 0 && untouched > 0 && untouched < NP, "ComputeDistinctiveDescriptors: %d diffs (%d untouched)", diff,
              untouched);
    }
    // ---- Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame.cc:396-403, KeyFrame.cc:60-69) on a synthetic
    // vocabulary (k = 6, L = 4, breadth-first node lines) registered for a stand-in ORBVocabulary
    {
        const int k = 6, L = 4;
        std::vector<int32_t> parent;
        std::vector<uint8_t> leaf, vdesc;
        std::vector<double> weight;
        uint32_t s = 99;
        std::vector<std::pair<int, int> > frontier(1, std::make_pair(0, 0));  // (node id, depth)
        std::vector<std::vector<uint8_t> > nd(1, std::vector<uint8_t>(32));
        for (auto& b : nd[0]) b = (uint8_t)(lcg(s) & 0xFF);
        int nid = 0;
        while (!frontier.empty()) {
            std::vector<std::pair<int, int> > nxt;
            for (auto& fr : frontier) {
                if (fr.second >= L) continue;
                for (int c = 0; c < k; c++) {
                    std::vector<uint8_t> d = nd[fr.first];
                    for (int b = 0; b < (fr.second ? 40 : 256); b++) {
                        const uint32_t r = lcg(s) % 256;
                        d[r >> 3] ^= (uint8_t)(1u << (r & 7));
                    }
                    nd.push_back(d);
                    nid++;
                    parent.push_back(fr.first);
                    leaf.push_back(fr.second + 1 == L ? 1 : 0);
                    vdesc.insert(vdesc.end(), d.begin(), d.end());
                    weight.push_back(0.1 + (double)(lcg(s) % 1000) / 125.0);
                    nxt.push_back(std::make_pair(nid, fr.second + 1));
                }
            }
            frontier = nxt;
        }
        const int nlines = (int)parent.size();
        for (int scoring = 0; scoring < 2; scoring++) {  // L1_NORM (ORB-SLAM2's) and L2_NORM
            orbv_handle* h = nullptr;
            CHECK(orbv_create(k, L, scoring, 0, nlines, parent.data(), leaf.data(), vdesc.data(), weight.data(), 0, &h) ==
                      ORBX_OK, "orbv_create");
            oc_vocab* ov = oc_vocab_create(k, L, scoring, 0, nlines, parent.data(), leaf.data(), vdesc.data(), weight.data());
            ORBVocabulary voc;
            amd::RegisterVocabulary(&voc, h);
            Frame F;
            F.mDescriptors = D[2];
            F.mpORBvocabulary = &voc;
            F.ComputeBoW();
            KeyFrame KF;
            KF.mDescriptors = D[1];
            KF.mpORBvocabulary = &voc;
            KF.ComputeBoW();
            int bad = 0;
            for (int which = 0; which < 2; which++) {
                const cv::Mat& Dm = which ? D[1] : D[2];
                const DBoW2::BowVector& bv = which ? KF.mBowVec : F.mBowVec;
                const DBoW2::FeatureVector& fv = which ? KF.mFeatVec : F.mFeatVec;
                const int n = Dm.rows;
                std::vector<uint32_t> w(n), nodes(n);
                std::vector<double> val(n);
                std::vector<int32_t> fo(n + 1), ff(n);
                int nb = 0, nf = 0;
                oc_vocab_transform(ov, Dm.ptr<unsigned char>(0), n, 4, w.data(), val.data(), &nb, nodes.data(), fo.data(),
                                   ff.data(), &nf);
                bad += (int)bv.size() != nb || (int)fv.size() != nf;
                int i = 0;
                for (auto& e : bv) { bad += i >= nb || e.first != w[i] || memcmp(&e.second, &val[i], 8) != 0; i++; }
                int j = 0;
                for (auto& e : fv) {
                    bad += j >= nf || e.first != nodes[j] ||
                           e.second != std::vector<unsigned int>(ff.begin() + fo[j], ff.begin() + fo[j + 1]);
                    j++;
                }
                bad += nb == 0 || nf == 0;
            }
            // guards: a Frame with a BowVector is not recomputed
            F.mDescriptors = D[0];
            const DBoW2::BowVector keep = F.mBowVec;
            F.ComputeBoW();
            bad += F.mBowVec != keep;
            CHECK(bad == 0, "ComputeBoW scoring=%d: %d mismatches", scoring, bad);
            oc_vocab_destroy(ov);
        }
    }
    // ---- concurrency (SURVEY.md 8(b) "Threading"): two extractors on two std::threads, as the stereo Frame
    // constructor runs them (Frame.cc:80-81), while matchers run on a Tracking-like (SearchByBoW(KF,F),
    // Tracking.cc:767), a LocalMapping-like (SearchForTriangulation, LocalMapping.cc:268) and a
    // LoopClosing-like thread (SearchByBoW(KF,KF), LoopClosing.cc:267); every call must equal the
    // single-threaded result
    {
        Frame F2;
        F2.N = kf2.N; F2.mvKeys = kf2.mvKeys; F2.mvKeysUn = kf2.mvKeysUn; F2.mDescriptors = kf2.mDescriptors;
        F2.mFeatVec = kf2.mFeatVec; F2.mvScaleFactors = kf2.mvScaleFactors; F2.mvLevelSigma2 = kf2.mvLevelSigma2;
        std::vector<std::pair<size_t, size_t> > e_tri;
        std::vector<MapPoint*> e_kk, e_kf;
        int e_ntri, e_nkk, e_nkf;
        {
            ORBmatcher a(0.6f, false), b(0.75f, true), c(0.7f, true);
            e_ntri = a.SearchForTriangulation(&kf1, &kf2, F12, e_tri, false);
            e_nkk = b.SearchByBoW(&kf1, &kf2, e_kk);
            e_nkf = c.SearchByBoW(&kf1, F2, e_kf);
        }
        std::atomic<int> bad(0), calls(0);
        const int iters = 30;
        auto extractor = [&](int f) {
            ORBextractor e(1000, 1.2f, 8, 20, 7);
            for (int it = 0; it < iters; it++) {
                std::vector<cv::KeyPoint> k;
                cv::Mat d;
                e(cv::Mat(H, W, CV_8U, frames.data() + (size_t)f * W * H, W), cv::Mat(), k, d);
                bool ok = k.size() == K[f].size() && d.rows == D[f].rows;
                for (size_t i = 0; ok && i < k.size(); i++)
                    ok = same_bits(k[i].pt.x, K[f][i].pt.x) && same_bits(k[i].pt.y, K[f][i].pt.y) &&
                         same_bits(k[i].angle, K[f][i].angle) && k[i].octave == K[f][i].octave &&
                         memcmp(d.ptr<unsigned char>((int)i), D[f].ptr<unsigned char>((int)i), 32) == 0;
                bad += !ok;
                calls++;
            }
        };
        auto tri = [&]() {
            ORBmatcher m(0.6f, false);
            for (int it = 0; it < iters; it++) {
                std::vector<std::pair<size_t, size_t> > pr;
                bad += m.SearchForTriangulation(&kf1, &kf2, F12, pr, false) != e_ntri || pr != e_tri;
                calls++;
            }
        };
        auto kk = [&]() {
            ORBmatcher m(0.75f, true);
            for (int it = 0; it < iters; it++) {
                std::vector<MapPoint*> v;
                bad += m.SearchByBoW(&kf1, &kf2, v) != e_nkk || v != e_kk;
                calls++;
            }
        };
        auto kf = [&]() {
            ORBmatcher m(0.7f, true);
            for (int it = 0; it < iters; it++) {
                std::vector<MapPoint*> v;
                bad += m.SearchByBoW(&kf1, F2, v) != e_nkf || v != e_kf;
                calls++;
            }
        };
        std::vector<std::thread> th;
        th.emplace_back(extractor, 0);
        th.emplace_back(extractor, 1);
        th.emplace_back(tri);
        th.emplace_back(kk);
        th.emplace_back(kf);
        for (std::thread& t : th) t.join();
        CHECK(bad == 0 && calls == 5 * iters, "concurrent drop-ins: %d of %d calls differ", (int)bad, (int)calls);
        // with the keyframe cache on (the default), the three matcher threads shared kf1's (and kf2's)
        // device-resident entries: every call after the first of each kind was a hit
        if (ORB_SLAM2::amd::KeyFrameCache()) {
            int entries = 0;
            size_t bytes = 0;
            long long hits = 0, misses = 0;
            orbm_kf_cache_stats(ORB_SLAM2::amd::KeyFrameCache(), &entries, &bytes, &hits, &misses);
            printf("keyframe cache: %d entries, %zu bytes, %lld hits, %lld misses\n", entries, bytes, hits, misses);
            CHECK(entries >= 2 && hits >= 3 * iters - 3, "keyframe cache not shared: %lld hits", hits);
            // KeyFrame::SetBadFlag's hook drops the keyframe's entry; the next call uploads it again (a miss)
            ORB_SLAM2::amd::ForgetKeyFrame(&kf1, kf1.mnId);
            int entries2 = 0;
            orbm_kf_cache_stats(ORB_SLAM2::amd::KeyFrameCache(), &entries2, nullptr, nullptr, nullptr);
            CHECK(entries2 == entries - 1, "ForgetKeyFrame: %d entries after, %d before", entries2, entries);
            {
                ORBmatcher m(0.75f, true);
                std::vector<MapPoint*> v;
                CHECK(m.SearchByBoW(&kf1, &kf2, v) == e_nkk && v == e_kk, "SearchByBoW after ForgetKeyFrame");
            }
            long long misses2 = 0;
            orbm_kf_cache_stats(ORB_SLAM2::amd::KeyFrameCache(), &entries2, nullptr, nullptr, &misses2);
            CHECK(entries2 == entries && misses2 == misses + 1, "re-upload after ForgetKeyFrame: %d entries, %lld misses",
                  entries2, misses2);
        } else {
            printf("keyframe cache off (ORBAMD_KF_CACHE_MB=0)\n");
        }
    }
    test_fuse(K[2], D[2], ext, W, H);
    test_init_sim3(K[0], D[0], K[1], D[1], ext, W, H);
    // DescriptorDistance (ORBmatcher.cc:1647-1663)
    int dd = 0;
    for (int i = 0; i + 1 < kf1.N; i += 17)
        dd += ORBmatcher::DescriptorDistance(kf1.mDescriptors.row(i), kf1.mDescriptors.row(i + 1)) !=
              oc_descriptor_distance(kf1.mDescriptors.ptr<unsigned char>(i), kf1.mDescriptors.ptr<unsigned char>(i + 1));
    CHECK(dd == 0, "DescriptorDistance");
    oc_destroy(orc);
    printf(failures ? "FAILURES %d\n" : "ALL PASS\n", failures);
    return failures ? 1 : 0;
}
