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

/* sum over each row of 16 lanes, every lane of the row holds it (quad butterfly + row rotations by DPP, 4 VALU
 * ops against 4 ds_bpermute round trips and their lane-index arithmetic for a width-16 __shfl_xor butterfly).
 * Every lane of the row must be active. */
__device__ __forceinline__ int row16_sum_i32(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return v;
}

/* inclusive prefix sum over the 64 lanes of a wave by DPP: Hillis-Steele within each row of 16 (row_shr 1, 2, 4, 8;
 * lanes shifted in from outside the row read 0), then row 0's total into row 1 and row 2's into row 3
 * (row_bcast:15 on rows 1, 3) and row 1's total into rows 2, 3 (row_bcast:31). 6 VALU ops against 6 ds_bpermute
 * round trips of a __shfl_up scan. Every lane must be active. */
__device__ __forceinline__ int wave_scan_incl_i32(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

}  // namespace orbamd
