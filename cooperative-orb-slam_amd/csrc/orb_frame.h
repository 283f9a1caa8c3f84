/*
 * orb_frame.h -- arguments of the Frame-level kernels (frame_kernels.hip): the consumers of
 * the extractor output that ORB-SLAM2's Frame runs next on the Tracking thread.
 */
#pragma once
#include <stdint.h>

#include "orb_device.h"

namespace orbamd {

/* one side (left or right extractor) of a stereo batch: the pyramid of its last extraction.
 * level 0 = the caller's frames (read in place), levels >= 1 = the handle's pyramid buffer */
struct PyrSide {
    const uint8_t* l0;
    long long l0_fstride;
    const uint8_t* pyr;
    long long pyr_fstride;
    int l0_pitch;
    int nframes;  // frames of that extraction (bounds of the frame-index arrays)
};

/* Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641) constants and the level
 * geometry of both pyramids (identical: same size and ORB parameters) */
struct StereoArgs {
    PyrSide left, right;
    int L;
    int nrows;      // mvImagePyramid[0].rows: size of vRowIndices (Frame.cc:477-483)
    int rspan;      // >= max over octaves of maxr - minr (Frame.cc:491-494)
    float maxD;     // mbf / minZ with minZ = mb (Frame.cc:501-503)
    float bf;       // mbf
    float thc;      // 1.5f*1.4f (Frame.cc:639), folded in float
    float scale[kMaxLevels], inv_scale[kMaxLevels];
    int lw[kMaxLevels], lh[kMaxLevels], lpitch[kMaxLevels];
    long long pyr_off[kMaxLevels];
};

}  // namespace orbamd
