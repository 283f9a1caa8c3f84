// One-off check of v_cvt_pk_u8_f32 rounding/saturation against the integer forms used by
// k_blur_strips (run on the GPU box: hipcc --offload-arch=gfx950 -O2 tools/check_cvtpk.hip).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned n, unsigned* bad) {
    unsigned s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    float sf = (float)s * (1.0f / 65536.0f);
    unsigned a = __builtin_amdgcn_cvt_pk_u8_f32(sf, 0u, 0u) & 0xFFu;
    unsigned ra = (s + 0x7FFFu + ((s >> 16) & 1u)) >> 16; ra = ra > 255u ? 255u : ra;
    if (a != ra) atomicAdd(&bad[0], 1u);
    float h = floorf(sf + 0.5f);
    unsigned b = __builtin_amdgcn_cvt_pk_u8_f32(h, 0u, 0u) & 0xFFu;
    unsigned rb = (s + (1u << 15)) >> 16; rb = rb > 255u ? 255u : rb;
    if (b != rb) atomicAdd(&bad[1], 1u);
}
int main() {
    unsigned n = 66049u * 255u + 1u, *d, h[2];
    hipMalloc(&d, 8); hipMemset(d, 0, 8);
    k<<<(n + 255) / 256, 256>>>(n, d);
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("cvt_pk_u8 RNE mismatches %u, half-up mismatches %u over %u values\n", h[0], h[1], n);
    return (h[0] || h[1]) ? 1 : 0;
}
