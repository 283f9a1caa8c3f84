// latency_floor.hip -- per-call latency floor of a host-API matcher call on one stream: what an
// H2D upload, N dependent kernel launches, an async memset, a D2H download and the final
// hipStreamSynchronize cost with no work in the kernels. Sizes are those of one SearchByBoW call
// (two 1000-keypoint views, ~100 KB in, 4 KB out). Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void k_empty(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}
__global__ void k_write_host(int* __restrict__ out, const int* __restrict__ in, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = in[i];
}

// the completion word of a call: the kernel stores it last, with release at system scope, into fine-grained
// pinned memory, and the host polls it instead of hipStreamSynchronize
__global__ void k_signal(int* __restrict__ done, int v) {
    if (threadIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_read_host_signal(int* __restrict__ out, const int* __restrict__ in, int n, int* __restrict__ done,
                                   int v) {
    int s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += in[i];
    out[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// per-call inputs passed by value in the kernel arguments instead of an H2D copy
template <int WORDS>
struct ArgBlock {
    int w[WORDS];
};
template <int WORDS>
__global__ void k_args_signal(ArgBlock<WORDS> a, int* __restrict__ out, int* __restrict__ done, int v) {
    int s = 0;
    for (int i = threadIdx.x; i < WORDS; i += blockDim.x) s += a.w[i];
    out[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CK(x)                                                   \
    do {                                                        \
        hipError_t e = (x);                                     \
        if (e != hipSuccess) {                                  \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                           \
        }                                                       \
    } while (0)

int main(int argc, char** argv) {
    // argv[1] == "spin": the runtime spins in hipStreamSynchronize instead of yielding / blocking
    if (argc > 1 && !strcmp(argv[1], "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const size_t in_b = 100 << 10, out_b = 4 << 10;
    char *hp, *dp;
    CK(hipHostMalloc((void**)&hp, in_b + out_b, 0));
    CK(hipMalloc((void**)&dp, in_b + out_b));
    memset(hp, 0, in_b + out_b);
    const int iters = 2000;
    int* done;
    CK(hipHostMalloc((void**)&done, 64, hipHostMallocCoherent));
    *done = 0;
    int seq = 0;
    const char* mode = argc > 1 ? argv[1] : "default";
    // sync = false: the body waits for its own completion word
    auto run_w = [&](const char* name, bool sync, auto&& body) -> int {
        for (int i = 0; i < 200; i++) {
            if (body()) return 1;
            if (sync && hipStreamSynchronize(st) != hipSuccess) return 1;
        }
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; i++) {
            if (body()) return 1;
            if (sync && hipStreamSynchronize(st) != hipSuccess) return 1;
        }
        const double us =
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
        printf("{\"case\": \"%s\", \"sched\": \"%s\", \"us_per_call\": %.2f}\n", name, mode, us);
        return 0;
    };
    auto run = [&](const char* name, auto&& body) -> int { return run_w(name, true, body); };
    auto wait_done = [&](int v) -> int {
        for (long spins = 0; __atomic_load_n((volatile int*)done, __ATOMIC_ACQUIRE) != v; spins++)
            if ((spins & 4095) == 4095 && hipStreamQuery(st) == hipSuccess &&
                __atomic_load_n((volatile int*)done, __ATOMIC_ACQUIRE) != v)
                return 1;  // the stream drained without the word: a failed launch
        return 0;
    };
    int* di = (int*)dp;
    int rc = 0;
    rc |= run("sync_only", [&] { return 0; });
    rc |= run("1_kernel", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, di); return (int)hipGetLastError(); });
    rc |= run("2_kernels", [&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, di);
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, di);
        return (int)hipGetLastError();
    });
    rc |= run("h2d_100k", [&] { return (int)hipMemcpyAsync(dp, hp, in_b, hipMemcpyHostToDevice, st); });
    rc |= run("d2h_4k", [&] { return (int)hipMemcpyAsync(hp + in_b, dp + in_b, out_b, hipMemcpyDeviceToHost, st); });
    rc |= run("memset_4k", [&] { return (int)hipMemsetAsync(dp + in_b, 0xFF, out_b, st); });
    rc |= run("h2d+kernel+d2h", [&] {
        if (hipMemcpyAsync(dp, hp, in_b, hipMemcpyHostToDevice, st)) return 1;
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, di);
        return (int)hipMemcpyAsync(hp + in_b, dp + in_b, out_b, hipMemcpyDeviceToHost, st);
    });
    rc |= run("h2d+memset+2kernels+d2h", [&] {
        if (hipMemcpyAsync(dp, hp, in_b, hipMemcpyHostToDevice, st)) return 1;
        if (hipMemsetAsync(dp + in_b, 0xFF, out_b, st)) return 1;
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, di);
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, di);
        return (int)hipMemcpyAsync(hp + in_b, dp + in_b, out_b, hipMemcpyDeviceToHost, st);
    });
    rc |= run("h2d+kernel_writes_host", [&] {
        if (hipMemcpyAsync(dp, hp, in_b, hipMemcpyHostToDevice, st)) return 1;
        hipLaunchKernelGGL(k_write_host, dim3(1), dim3(256), 0, st, (int*)(hp + in_b), di, (int)(out_b / 4));
        return (int)hipGetLastError();
    });
    rc |= run("h2d+kernel+d2h_small_h2d_4k", [&] {
        if (hipMemcpyAsync(dp, hp, 4096, hipMemcpyHostToDevice, st)) return 1;
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, di);
        return (int)hipMemcpyAsync(hp + in_b, dp + in_b, out_b, hipMemcpyDeviceToHost, st);
    });
    rc |= run("kernel_reads_host_writes_host", [&] {
        hipLaunchKernelGGL(k_write_host, dim3(1), dim3(256), 0, st, (int*)(hp + in_b), (const int*)hp, (int)(out_b / 4));
        return (int)hipGetLastError();
    });
    rc |= run_w("1_kernel_poll_word", false, [&] {
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, st, done, ++seq);
        if (hipGetLastError()) return 1;
        return wait_done(seq);
    });
    rc |= run_w("h2d_4k+kernel_poll_word", false, [&] {
        if (hipMemcpyAsync(dp, hp, 4096, hipMemcpyHostToDevice, st)) return 1;
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, st, done, ++seq);
        if (hipGetLastError()) return 1;
        return wait_done(seq);
    });
    rc |= run_w("kernel_reads_host_4k_poll_word", false, [&] {
        hipLaunchKernelGGL(k_read_host_signal, dim3(1), dim3(256), 0, st, di, (const int*)hp, 1024, done, ++seq);
        if (hipGetLastError()) return 1;
        return wait_done(seq);
    });
    rc |= run_w("h2d_100k+kernel_poll_word", false, [&] {
        if (hipMemcpyAsync(dp, hp, in_b, hipMemcpyHostToDevice, st)) return 1;
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, st, done, ++seq);
        if (hipGetLastError()) return 1;
        return wait_done(seq);
    });
    static ArgBlock<256> a1;
    static ArgBlock<768> a3;
    static ArgBlock<1000> a4;
    for (int i = 0; i < 1000; i++) a4.w[i] = i;
    rc |= run_w("kernel_args_1k_poll_word", false, [&] {
        a1.w[seq & 255]++;
        hipLaunchKernelGGL(k_args_signal<256>, dim3(1), dim3(256), 0, st, a1, di, done, ++seq);
        if (hipGetLastError()) return 1;
        return wait_done(seq);
    });
    rc |= run_w("kernel_args_3k_poll_word", false, [&] {
        a3.w[seq % 768]++;
        hipLaunchKernelGGL(k_args_signal<768>, dim3(1), dim3(256), 0, st, a3, di, done, ++seq);
        if (hipGetLastError()) return 1;
        return wait_done(seq);
    });
    rc |= run_w("kernel_args_4000B_poll_word", false, [&] {
        a4.w[seq % 1000]++;
        hipLaunchKernelGGL(k_args_signal<1000>, dim3(90), dim3(256), 0, st, a4, di, done, ++seq);
        if (hipGetLastError()) return 1;
        return wait_done(seq);
    });
    {   // the 4000-byte block arrives intact
        int* chk;
        CK(hipHostMalloc((void**)&chk, 4096, hipHostMallocCoherent));
        memset(chk, 0, 4096);
        for (int i = 0; i < 1000; i++) a4.w[i] = 3 * i + 1;
        hipLaunchKernelGGL(k_args_signal<1000>, dim3(1), dim3(256), 0, st, a4, chk, done, ++seq);
        CK(hipStreamSynchronize(st));
        long want = 0, got = 0;
        for (int t = 0; t < 256; t++) {
            for (int i = t; i < 1000; i += 256) want += 3 * i + 1;
            got += chk[t];
        }
        printf("{\"case\": \"kernel_args_4000B_intact\", \"ok\": %s}\n", want == got ? "true" : "false");
        (void)hipHostFree(chk);
    }
    CK(hipStreamSynchronize(st));
    (void)hipHostFree(done);
    (void)hipFree(dp);
    (void)hipHostFree(hp);
    (void)hipStreamDestroy(st);
    return rc;
}
