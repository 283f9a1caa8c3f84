/*
 * ORBmatcher_base_amd.cc -- the ORBmatcher constants and constructor (ORBmatcher.cc:37-45).
 * Only for builds that do NOT compile the reference's ORB_SLAM2/src/ORBmatcher.cc (the
 * standalone drop-in test, tests/cpp/build.sh). An ORB-SLAM2 build keeps the reference file
 * for the non-hot-path members and takes these definitions from it.
 */
#include "ORBmatcher.h"

namespace ORB_SLAM2 {

const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

}  // namespace ORB_SLAM2
