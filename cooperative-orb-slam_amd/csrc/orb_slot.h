/*
 * orb_slot.h -- layout of the cross-agent keyframe slot (include/orbslam_amd.h, "Cross-agent
 * keyframe slot"), shared by the host C ABI (capi.cpp) and the device pack / match kernels
 * (exchange_kernels.hip) so both compute the same section offsets from the capacity.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbslam_amd.h"

namespace orbamd {

constexpr uint32_t kSlotMetaOff = 128;
constexpr uint32_t kSlotBodyOff = 1024;
constexpr int kSlotMaxCap = 1 << 20;  // keeps every offset in u32

static_assert(sizeof(orbx_slot_header) == 128, "slot header is 128 bytes");
static_assert(sizeof(orbx_kf_meta) == 704, "kf meta is 704 bytes");
static_assert(kSlotMetaOff + sizeof(orbx_kf_meta) <= kSlotBodyOff, "meta fits before the body");

/* bytes of section s for capacity cap */
__host__ __device__ inline uint64_t slot_section_bytes(int s, int cap) {
    const uint64_t c = (uint64_t)cap;
    switch (s) {
        case ORBX_SLOT_KPS: return c * sizeof(orbx_kp);
        case ORBX_SLOT_KUN: return c * 8;
        case ORBX_SLOT_URIGHT: return c * 4;
        case ORBX_SLOT_DEPTH: return c * 4;
        case ORBX_SLOT_DESC: return c * 32;
        case ORBX_SLOT_MPFLAGS: return c;
        case ORBX_SLOT_MPPOS: return c * 12;
        case ORBX_SLOT_BOWWORD: return c * 4;
        case ORBX_SLOT_BOWVALUE: return c * 8;
        case ORBX_SLOT_FVNODE: return c * 4;
        case ORBX_SLOT_FVOFF: return (c + 1) * 4;
        case ORBX_SLOT_FVFEAT: return c * 4;
        default: return 0;
    }
}

/* section offsets (256-byte aligned) and the total size; false if cap is out of range */
__host__ __device__ inline bool slot_offsets(int cap, uint32_t off[ORBX_SLOT_NSECTIONS], uint32_t* total) {
    if (cap < 0 || cap > kSlotMaxCap) return false;
    uint64_t o = kSlotBodyOff;
    for (int s = 0; s < ORBX_SLOT_NSECTIONS; s++) {
        off[s] = (uint32_t)o;
        o += (slot_section_bytes(s, cap) + 255) & ~(uint64_t)255;
    }
    *total = (uint32_t)o;
    return true;
}

/* Section offsets handed to the device kernels by value. */
struct SlotLayout {
    uint32_t off[ORBX_SLOT_NSECTIONS];
    uint32_t bytes;
    int cap;
};

/* the query keyframe (this agent's), device arrays */
struct QueryKF {
    const orbx_kp* kps;
    const float2* kun;      // NULL: mvKeysUn = mvKeys
    const float* uright;    // NULL: monocular
    const uint8_t* mpf;     // NULL: no MapPoints
    const uint8_t* desc;
    const int32_t* count;
    const uint32_t* fv_node;
    const int32_t* fv_off;
    const int32_t* fv_feat;
    const int32_t* nfv;
    int cap;
};

}  // namespace orbamd
