/*
 * ORBVocabulary_amd.h -- the device copy of a loaded ORBVocabulary, used by the MI355X
 * Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame_bow_amd.cc). System.cc:64-65 loads the
 * vocabulary with mpVocabulary->loadFromTextFile(strVocFile); the maintainer adds, right after:
 *     ORB_SLAM2::amd::RegisterVocabulary(mpVocabulary, strVocFile);
 * which parses the same ORBvoc.txt into HBM (orbv_load_text). Frames and KeyFrames look their
 * mpORBvocabulary up here; a vocabulary that was never registered is an error (no CPU fallback).
 */
#ifndef ORBVOCABULARY_AMD_H
#define ORBVOCABULARY_AMD_H
#include <string>

#include "ORBVocabulary.h"
#include "orbslam_amd.h"

namespace ORB_SLAM2 {
namespace amd {

/* device copy of the text vocabulary at strVocFile for pVoc (device from ORBAMD_DEVICE, default 0);
 * throws std::runtime_error if the file cannot be loaded */
void RegisterVocabulary(const ORBVocabulary* pVoc, const std::string& strVocFile);
/* an already built device vocabulary (orbv_create / orbv_load_text); ownership passes here */
void RegisterVocabulary(const ORBVocabulary* pVoc, orbv_handle* h);
/* the registered device vocabulary of pVoc, or nullptr */
orbv_handle* DeviceVocabulary(const ORBVocabulary* pVoc);

}  // namespace amd
}  // namespace ORB_SLAM2
#endif
