/* fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
 * pipeline's kernels use (MI355X_MICROARCH.md "HBM": only 16-B-per-lane streaming reads are calibrated, at 1/2):
 * one read of a 1 GiB buffer (past the 256 MiB Infinity Cache) per kernel, coalesced, with
 *   k_ld_u8      1 B per lane            (global_load_ubyte)
 *   k_ld_b32     4 B per lane            (global_load_dword: FAST's ROI staging, the blur)
 *   k_ld_lds32   4 B per lane into LDS   (global_load_lds_dword: describe's patch staging)
 *   k_ld_b64     8 B per lane            (global_load_dwordx2: describe's IC rows)
 *   k_ld_b128    16 B per lane           (global_load_dwordx4: the guide's calibrated case)
 *   k_st_b32     4 B per lane store      (global_store_dword)
 *   k_gather48   48-B row segments at random 4-aligned offsets, 12 dword lanes each (describe's patch-row gather and
 *                the octree's scattered reads are partial-line accesses, not the streams above: ADVICE r05)
 *   k_gather48_lds  the same segments by 4-B LDS-DMA (k_describe_blur's staging form)
 * The gather kernels read kGatherSegs segments of 48 B (kGatherSegs * 48 bytes); their tally factor is FETCH_SIZE
 * (KiB) * 1024 / (kGatherSegs * 48).
 * Each kernel writes one word per workgroup so its loads are live. FETCH_SIZE (KiB) per dispatch / 2^20 =
 * the tally factor of that width. usage: rocprofv3 --pmc FETCH_SIZE -- tools/bin/fetch_calib
 *                                     rocprofv3 --pmc WRITE_SIZE -- tools/bin/fetch_calib */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr size_t kBytes = (size_t)1 << 30;
constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void k_ld_u8(const uint8_t* __restrict__ p, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < kBytes; i += (size_t)gridDim.x * kThreads)
        acc += p[i];
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void k_ld_b32(const uint32_t* __restrict__ p, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < kBytes / 4; i += (size_t)gridDim.x * kThreads)
        acc += p[i];
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void k_ld_b64(const uint2* __restrict__ p, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < kBytes / 8; i += (size_t)gridDim.x * kThreads)
        acc += p[i].x ^ p[i].y;
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void k_ld_b128(const uint4* __restrict__ p, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < kBytes / 16; i += (size_t)gridDim.x * kThreads) {
        const uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void k_ld_lds32(const uint32_t* __restrict__ p, uint32_t* __restrict__ out) {
    __shared__ uint32_t s[kThreads];
    const int w = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (size_t b = (size_t)blockIdx.x * kThreads; b < kBytes / 4; b += (size_t)gridDim.x * kThreads) {
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(p + b + threadIdx.x),
                                         (__attribute__((address_space(3))) void*)(s + 64 * w), 4, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc += s[threadIdx.x];
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

constexpr size_t kGatherSegs = (size_t)1 << 22;  // 4 Mi segments x 48 B = 192 MiB requested, over the 1 GiB buffer

__device__ __forceinline__ size_t seg_offset(size_t seg) {  // a pseudo-random 4-aligned offset in the buffer
    uint64_t h = (uint64_t)seg * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    return (size_t)(h % ((kBytes - 64) / 4)) * 4;
}

// 16 segments per 256-thread block iteration: lanes 16j .. 16j+11 read segment j's 12 dwords (4 idle lanes per 16)
__global__ __launch_bounds__(kThreads) void k_gather48(const uint8_t* __restrict__ p, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const int j = threadIdx.x >> 4, d = threadIdx.x & 15;
    for (size_t sg = (size_t)blockIdx.x * 16 + j; sg < kGatherSegs; sg += (size_t)gridDim.x * 16)
        if (d < 12) acc += *(const uint32_t*)(p + seg_offset(sg) + 4 * d);
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void k_gather48_lds(const uint8_t* __restrict__ p, uint32_t* __restrict__ out) {
    __shared__ uint32_t s[kThreads];
    const int j = threadIdx.x >> 4, d = threadIdx.x & 15, w = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (size_t sb = (size_t)blockIdx.x * 16; sb < kGatherSegs; sb += (size_t)gridDim.x * 16) {
        const size_t sg = sb + j;
        // every lane issues (LDS-DMA writes 64 consecutive dwords per wave); lanes 12..15 of a segment re-read its head
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(p + seg_offset(sg) + 4 * (d < 12 ? d : 0)),
                                         (__attribute__((address_space(3))) void*)(s + 64 * w), 4, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc += s[threadIdx.x];
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void k_st_b32(uint32_t* __restrict__ p) {
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < kBytes / 4; i += (size_t)gridDim.x * kThreads)
        p[i] = (uint32_t)i;
}

int main() {
    void *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) {
        printf("hipMalloc failed\n");
        return 1;
    }
    (void)hipMemset(buf, 1, kBytes);
    const dim3 grid(8192), blk(kThreads);
    hipLaunchKernelGGL(k_ld_u8, grid, blk, 0, 0, (const uint8_t*)buf, (uint32_t*)out);
    hipLaunchKernelGGL(k_ld_b32, grid, blk, 0, 0, (const uint32_t*)buf, (uint32_t*)out);
    hipLaunchKernelGGL(k_ld_lds32, grid, blk, 0, 0, (const uint32_t*)buf, (uint32_t*)out);
    hipLaunchKernelGGL(k_ld_b64, grid, blk, 0, 0, (const uint2*)buf, (uint32_t*)out);
    hipLaunchKernelGGL(k_ld_b128, grid, blk, 0, 0, (const uint4*)buf, (uint32_t*)out);
    hipLaunchKernelGGL(k_gather48, grid, blk, 0, 0, (const uint8_t*)buf, (uint32_t*)out);
    hipLaunchKernelGGL(k_gather48_lds, grid, blk, 0, 0, (const uint8_t*)buf, (uint32_t*)out);
    hipLaunchKernelGGL(k_st_b32, grid, blk, 0, 0, (uint32_t*)buf);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    printf("fetch_calib done: 6 kernels over %zu bytes each, 2 gathers of %zu x 48-B segments (%zu bytes)\n", kBytes,
           kGatherSegs, kGatherSegs * 48);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
