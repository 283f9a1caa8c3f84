/*
 * orb_wave.h -- wave64 reductions on gfx950 by DPP (no LDS crossbar round trips).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbamd {

/* minimum over the 64 lanes of a wave, uniform result. Every lane must be active (EXEC all ones): quad
 * butterfly and row rotations by DPP leave every lane holding its row's minimum, then the four rows'
 * minima by readlane. 4 DPP min + 4 readlane + 3 scalar min, against 6 ds_bpermute round trips of an
 * __shfl_xor butterfly. */
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}

}  // namespace orbamd
