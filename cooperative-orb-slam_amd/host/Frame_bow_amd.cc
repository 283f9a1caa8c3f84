/*
 * Frame_bow_amd.cc -- MI355X definitions of Frame::ComputeBoW (Frame.cc:396-403) and
 * KeyFrame::ComputeBoW (KeyFrame.cc:60-69), replacing the two reference definitions
 * (INTEGRATION.md §5), and the device-vocabulary registry of ORBVocabulary_amd.h.
 *
 * Both keep the reference's guards (Frame: only if mBowVec is empty; KeyFrame: if mBowVec or
 * mFeatVec is empty) and levelsup 4. ORBVocabulary::transform(features, BowVector&,
 * FeatureVector&, 4) becomes orbv_transform on the registered device copy of mpORBvocabulary:
 * descent of every descriptor through the k-ary tree (k_voc_descend) and the BowVector /
 * FeatureVector assembly with DBoW2's weighting, normalisation and ordering (k_voc_bow). The
 * outputs are cleared first, as TemplatedVocabulary::transform does. DBoW2 is not vendored in
 * the reference: its ORB-SLAM2 fork is restated (parity unpinned).
 */
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "Frame.h"
#include "KeyFrame.h"
#include "ORBVocabulary_amd.h"
#include "orbamd_status.h"

namespace ORB_SLAM2 {
namespace amd {

namespace {
std::mutex& reg_mutex() {
    static std::mutex m;
    return m;
}
std::map<const ORBVocabulary*, orbv_handle*>& registry() {
    static std::map<const ORBVocabulary*, orbv_handle*> r;
    return r;
}
}  // namespace

void RegisterVocabulary(const ORBVocabulary* pVoc, orbv_handle* h) {
    std::unique_lock<std::mutex> lock(reg_mutex());
    orbv_handle*& slot = registry()[pVoc];
    if (slot && slot != h) orbv_destroy(slot);
    slot = h;
}

void RegisterVocabulary(const ORBVocabulary* pVoc, const std::string& strVocFile) {
    const char* dev = getenv("ORBAMD_DEVICE");
    orbv_handle* h = nullptr;
    const int rc = orbv_load_text(strVocFile.c_str(), dev ? atoi(dev) : 0, &h);
    if (rc != ORBX_OK)
        throw std::runtime_error("orbslam_amd: orbv_load_text(" + strVocFile + ") failed rc=" + std::to_string(rc));
    RegisterVocabulary(pVoc, h);
}

orbv_handle* DeviceVocabulary(const ORBVocabulary* pVoc) {
    std::unique_lock<std::mutex> lock(reg_mutex());
    std::map<const ORBVocabulary*, orbv_handle*>::iterator it = registry().find(pVoc);
    return it == registry().end() ? nullptr : it->second;
}

}  // namespace amd

namespace {

/* ORBVocabulary::transform(toDescriptorVector(D), bv, fv, levelsup) on the device copy */
void bow_transform(const ORBVocabulary* pVoc, const cv::Mat& D, DBoW2::BowVector& bv, DBoW2::FeatureVector& fv,
                   int levelsup) {
    orbv_handle* h = amd::DeviceVocabulary(pVoc);
    if (!h) throw std::runtime_error("orbslam_amd: ComputeBoW with an unregistered vocabulary (ORBVocabulary_amd.h)");
    bv.clear();
    fv.clear();  // a device failure below leaves both empty (no BoW matches), logged, not thrown
    const int n = D.rows;
    if (n == 0) return;
    std::vector<uint8_t> desc((size_t)n * 32);
    for (int i = 0; i < n; i++) {
        const unsigned char* r = D.ptr<unsigned char>(i);
        std::copy(r, r + 32, desc.begin() + (size_t)i * 32);
    }
    std::vector<uint32_t> word(n), node(n);
    std::vector<double> value(n);
    std::vector<int32_t> off(n + 1), feat(n);
    int nb = 0, nf = 0;
    const int rc = orbv_transform(h, desc.data(), n, levelsup, word.data(), value.data(), &nb, node.data(), off.data(),
                                  feat.data(), &nf);
    if (!amd::StatusOk(rc, "orbv_transform")) return;
    for (int i = 0; i < nb; i++) bv.insert(std::make_pair(word[i], value[i]));  // ascending word id
    for (int j = 0; j < nf; j++)
        fv.insert(std::make_pair(node[j], std::vector<unsigned int>(feat.begin() + off[j], feat.begin() + off[j + 1])));
}

}  // namespace

void Frame::ComputeBoW() {
    if (mBowVec.empty()) bow_transform(mpORBvocabulary, mDescriptors, mBowVec, mFeatVec, 4);
}

void KeyFrame::ComputeBoW() {
    // We assume the vocabulary tree has 6 levels, change the 4 otherwise (KeyFrame.cc:65-66)
    if (mBowVec.empty() || mFeatVec.empty()) bow_transform(mpORBvocabulary, mDescriptors, mBowVec, mFeatVec, 4);
}

}  // namespace ORB_SLAM2
