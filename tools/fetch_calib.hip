/* fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
 * pipeline's kernels use (MI355X_MICROARCH.md "HBM": only 16-B-per-lane streaming reads are calibrated, at 1/2):
 * one read of a 1 GiB buffer (past the 256 MiB Infinity Cache) per kernel, coalesced, with
 *   k_ld_u8      1 B per lane            (global_load_ubyte)
 *   k_ld_b32     4 B per lane            (global_load_dword: FAST's ROI staging, the blur)
 *   k_ld_lds32   4 B per lane into LDS   (global_load_lds_dword: describe's patch staging)
 *   k_ld_b64     8 B per lane            (global_load_dwordx2: describe's IC rows)
 *   k_ld_b128    16 B per lane           (global_load_dwordx4: the guide's calibrated case)
 *   k_st_b32     4 B per lane store      (global_store_dword)
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
    hipLaunchKernelGGL(k_st_b32, grid, blk, 0, 0, (uint32_t*)buf);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    printf("fetch_calib done: 6 kernels over %zu bytes each\n", kBytes);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
