/*
 * bow_kernels.hip -- gfx950 kernels of the DBoW2 vocabulary transform behind Frame::ComputeBoW
 * (ORB_SLAM2/src/Frame.cc:400-407, KeyFrame::ComputeBoW): TemplatedVocabulary<FORB>::transform(
 * features, BowVector&, FeatureVector&, levelsup) of the ORB-SLAM2 DBoW2 fork (not vendored in
 * the reference; restated from the published algorithm, parity unpinned -- DESIGN.md).
 *
 *   k_voc_descend  16 lanes per descriptor: at every level the node's children (file order) are
 *                  scored with the 256-bit Hamming distance (FORB::distance), the group minimum of
 *                  (dist, child position) is DBoW2's first strict minimum; the descent stops at a
 *                  node without children (Node::isLeaf) and records the word id, its weight and
 *                  the node at level L - levelsup (the FeatureVector key). The children's descriptors
 *                  and records sit in child-slot order, so a level is one round of independent loads.
 *   k_voc_bow      one workgroup per frame: stable bitonic sorts (registers + LDS) of (node, feature) and (word,
 *                  feature) keys build FeatureVector::addFeature's map (ascending node id, ascending
 *                  feature per node) and BowVector's map; a word's weights are added in feature
 *                  order (addWeight) or the first kept (addIfNotExist), the TF division by the word
 *                  count or BowVector::normalize (L1 / L2) sum in ascending word order -- the same
 *                  double operations in the same order as the std::map code.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_bow.h"

namespace orbamd {

__global__ __launch_bounds__(256) void k_voc_descend(VocDev v, int levelsup, const uint8_t* __restrict__ desc,
                                                     const int32_t* __restrict__ counts, int stride,
                                                     int32_t* __restrict__ word, double* __restrict__ weight,
                                                     uint32_t* __restrict__ nid_out) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * 16 + (threadIdx.x >> 4), gl = threadIdx.x & 15, gbase = threadIdx.x & ~15;
    const int n = counts[f];
    if (blockIdx.x * 16 >= n) return;  // block-uniform
    const bool in = i < n;
    const long long fi = (long long)f * stride + (in ? i : 0);
    const uint4* q = (const uint4*)(desc + fi * 32);
    const uint4 q0 = q[0], q1 = q[1];
    const int nid_level = v.L - levelsup;
    uint32_t nid = 0;  // root (also what a branch shallower than nid_level reports)
    int final_id = 0, w_id = 0, level = 0;
    double w = 0.0;
    int c0 = v.root_c0, nc = v.root_nc;
    for (int step = 0; step < v.n && nc > 0; step++) {  // nc == 0: Node::isLeaf; node ids strictly increase
        ++level;
        uint32_t best = 0xffffffffu;
        VocChild br{};
        for (int j = gl; j < nc; j += 16) {
            const uint4* d = (const uint4*)(v.cdesc + (long long)(c0 + j) * 32);
            const uint4 d0 = d[0], d1 = d[1];
            const VocChild r = v.crec[c0 + j];
            const int dist = __popc(q0.x ^ d0.x) + __popc(q0.y ^ d0.y) + __popc(q0.z ^ d0.z) + __popc(q0.w ^ d0.w) +
                             __popc(q1.x ^ d1.x) + __popc(q1.y ^ d1.y) + __popc(q1.z ^ d1.z) + __popc(q1.w ^ d1.w);
            const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)j;  // first strict minimum: lowest j on ties
            if (key < best) {
                best = key;
                br = r;
            }
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o));
        const int src = gbase + (int)(best & 15u);  // child j was scored by lane j mod 16
        final_id = __shfl(br.id, src);
        c0 = __shfl(br.c0, src);
        nc = __shfl(br.nc, src);
        w_id = __shfl(br.word, src);
        w = __shfl(br.weight, src);
        if (level == nid_level) nid = (uint32_t)final_id;
    }
    if (in && gl == 0) {
        word[fi] = w_id;
        weight[fi] = w;
        nid_out[fi] = nid;
    }
}

constexpr int kVocThreads = 1024;  // k_voc_bow: one compare-exchange per thread per bitonic stage at 2048 keys
constexpr int kVocWaves = kVocThreads / 64;

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long x, int m) {
    const int lo = __shfl_xor((int)(uint32_t)x, m), hi = __shfl_xor((int)(uint32_t)(x >> 32), m);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}

/* the bitonic stages of strides 64 .. 1 of sorting size `size` over a 128-key block held in registers: key g0 =
 * base + lane in x0, g0 + 64 in x1 (stride 64 pairs a lane's own two keys, the smaller strides the lanes lane ^ s) */
__device__ __forceinline__ void reg_bitonic_tail(unsigned long long& x0, unsigned long long& x1, int base, int size,
                                                 int top) {
    const int lane = threadIdx.x & 63, g0 = base + lane, g1 = g0 + 64;
    if (top >= 64) {
        const bool up = (g0 & size) == 0;  // g0 and g1 share the bit for size >= 128
        const unsigned long long lo = x0 < x1 ? x0 : x1, hi = x0 < x1 ? x1 : x0;
        x0 = up ? lo : hi;
        x1 = up ? hi : lo;
    }
    for (int st = (top < 32 ? top : 32); st > 0; st >>= 1) {
        const bool lower = (lane & st) == 0;
        const unsigned long long y0 = shfl_xor_u64(x0, st), y1 = shfl_xor_u64(x1, st);
        const bool up0 = (g0 & size) == 0, up1 = (g1 & size) == 0;
        const unsigned long long mn0 = x0 < y0 ? x0 : y0, mx0 = x0 < y0 ? y0 : x0;
        const unsigned long long mn1 = x1 < y1 ? x1 : y1, mx1 = x1 < y1 ? y1 : x1;
        x0 = (lower == up0) ? mn0 : mx0;
        x1 = (lower == up1) ? mn1 : mx1;
    }
}

/* ascending bitonic sort of n2 (power of two, >= 128) u64 keys in LDS by kVocThreads threads. Every stage of stride
 * <= 64 stays inside a 128-key block, which one wave holds in registers (two keys per lane): sizes 2..128 run there
 * from one load, and after the LDS stages of stride >= 128 of every larger size, its strides 64..1 run there too
 * (log2(n2/128) + 1 register passes and (log2(n2/128)) (log2(n2/128) + 1) / 2 LDS stages, the only workgroup
 * barriers; 55 LDS stages at 1024 keys before) */
__device__ void lds_bitonic_u64(unsigned long long* a, int n2) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nb = n2 >> 7;
    __syncthreads();  // the keys written by every thread
    for (int b = wv; b < nb; b += kVocWaves) {
        unsigned long long x0 = a[b * 128 + lane], x1 = a[b * 128 + 64 + lane];
        for (int size = 2; size <= 128; size <<= 1) reg_bitonic_tail(x0, x1, b * 128, size, size >> 1);
        a[b * 128 + lane] = x0;
        a[b * 128 + 64 + lane] = x1;
    }
    for (int size = 256; size <= n2; size <<= 1) {
        for (int stride = size >> 1; stride >= 128; stride >>= 1) {
            __syncthreads();
            for (int t = threadIdx.x; t < n2 / 2; t += kVocThreads) {
                const int lo = 2 * t - (t & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long x = a[lo], y = a[hi];
                if ((x > y) == up) {
                    a[lo] = y;
                    a[hi] = x;
                }
            }
        }
        __syncthreads();
        for (int b = wv; b < nb; b += kVocWaves) {
            unsigned long long x0 = a[b * 128 + lane], x1 = a[b * 128 + 64 + lane];
            reg_bitonic_tail(x0, x1, b * 128, size, 64);
            a[b * 128 + lane] = x0;
            a[b * 128 + 64 + lane] = x1;
        }
    }
    __syncthreads();
}

/* segments of equal key-high-words in a sorted array (block scan of the segment heads): returns the
 * segment count; s_start[s] = first element of segment s */
__device__ int lds_segments(const unsigned long long* a, int n, int* s_start, int* s_tmp) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int carry = 0;
    for (int base = 0; base < n; base += kVocThreads) {
        const int i = base + tid;
        const int head = i < n && (i == 0 || (a[i] >> 32) != (a[i - 1] >> 32));
        int incl = head;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        if (lane == 63) s_tmp[wv] = incl;
        __syncthreads();
        int off = carry;
        for (int w = 0; w < wv; w++) off += s_tmp[w];
        int tot = 0;
#pragma unroll
        for (int w = 0; w < kVocWaves; w++) tot += s_tmp[w];
        if (i < n && head) s_start[off + incl - 1] = i;
        carry += tot;
        __syncthreads();
    }
    return carry;
}

/* BowVector::normalize's sum over n values in LDS, in order, one f64 add after another (uncontracted, as the oracle's
 * -ffp-contract=off build): L2 the squares, L1 the magnitudes. One lane; the next 8 values are loaded while the
 * current 8 are added, so the chain waits on the adds alone (16 in flight measured slower in the schedule: the
 * kernel's 84 VGPRs against 54 make its 1024-thread workgroup harder to place beside the other graphs' kernels) */
template <bool L2>
__device__ double norm_chain(const double* __restrict__ s_val, int n) {
    constexpr int kQ = 8;
    double norm = 0.0;
    const int nfull = n & ~(kQ - 1);
    double t[kQ];
    if (nfull) {
#pragma unroll
        for (int k = 0; k < kQ; k++) t[k] = s_val[k];
    }
    for (int s = 0; s < nfull; s += kQ) {
        const int nx = s + kQ < nfull ? s + kQ : s;  // the last chunk re-reads itself
        double u[kQ];
#pragma unroll
        for (int k = 0; k < kQ; k++) u[k] = s_val[nx + k];
#pragma unroll
        for (int k = 0; k < kQ; k++) norm = __dadd_rn(norm, L2 ? __dmul_rn(t[k], t[k]) : fabs(t[k]));
#pragma unroll
        for (int k = 0; k < kQ; k++) t[k] = u[k];
    }
    for (int s = nfull; s < n; s++) norm = __dadd_rn(norm, L2 ? __dmul_rn(s_val[s], s_val[s]) : fabs(s_val[s]));
    return norm;
}

#ifdef ORBX_BOW_TRACE
__device__ unsigned long long g_bow_trace[16];
#define BOW_T(k) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_bow_trace[(k)] = wall_clock64(); } while (0)
#else
#define BOW_T(k) do { } while (0)
#endif

__global__ __launch_bounds__(kVocThreads) void k_voc_bow(VocDev v, const int32_t* __restrict__ counts, int stride,
                                                 const int32_t* __restrict__ word, const double* __restrict__ weight,
                                                 const uint32_t* __restrict__ nid, uint32_t* __restrict__ bow_word,
                                                 double* __restrict__ bow_value, int32_t* __restrict__ nbow,
                                                 uint32_t* __restrict__ fv_node, int32_t* __restrict__ fv_off,
                                                 int32_t* __restrict__ fv_feat, int32_t* __restrict__ nfv) {
    __shared__ unsigned long long s_key[kVocMaxFeatures];
    __shared__ int s_start[kVocMaxFeatures + 1];
    __shared__ int s_tmp[2 * kVocWaves];
    __shared__ double s_norm;
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = counts[f];
    const long long fb = (long long)f * stride;
    int n2 = 128;  // the sort's block: 128 keys (padding sorts last)
    while (n2 < n) n2 <<= 1;
    BOW_T(0);
    // ---- FeatureVector: stable by (node id, feature index); stopped features (weight <= 0) sort last
    for (int i = tid; i < n2; i += kVocThreads)
        s_key[i] = i < n && weight[fb + i] > 0 ? ((unsigned long long)nid[fb + i] << 32) | (unsigned)i : ~0ull;
    BOW_T(1);
    lds_bitonic_u64(s_key, n2);
    BOW_T(2);
    int kept = 0;
    for (int i = tid; i < n; i += kVocThreads) kept += s_key[i] != ~0ull;
    for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o);
    if ((tid & 63) == 0) s_tmp[kVocWaves + (tid >> 6)] = kept;
    __syncthreads();
    int m = 0;
#pragma unroll
    for (int w = 0; w < kVocWaves; w++) m += s_tmp[kVocWaves + w];
    __syncthreads();
    const int nseg = lds_segments(s_key, m, s_start, s_tmp);
    for (int i = tid; i < m; i += kVocThreads) fv_feat[fb + i] = (int32_t)(s_key[i] & 0xffffffffu);
    for (int s = tid; s < nseg; s += kVocThreads) {
        fv_node[fb + s] = (uint32_t)(s_key[s_start[s]] >> 32);
        fv_off[(long long)f * (stride + 1) + s] = s_start[s];
    }
    if (tid == 0) {
        fv_off[(long long)f * (stride + 1) + nseg] = m;
        nfv[f] = nseg;
    }
    __syncthreads();
    BOW_T(3);
    // ---- BowVector: stable by (word id, feature index)
    for (int i = tid; i < n2; i += kVocThreads)
        s_key[i] = i < n && weight[fb + i] > 0 ? ((unsigned long long)(uint32_t)word[fb + i] << 32) | (unsigned)i : ~0ull;
    BOW_T(4);
    lds_bitonic_u64(s_key, n2);
    BOW_T(5);
    const int nw = lds_segments(s_key, m, s_start, s_tmp);
    if (tid == 0) s_start[nw] = m;
    __syncthreads();
    const bool add = v.weighting == 0 || v.weighting == 1;  // TF_IDF / TF: addWeight; IDF / BINARY: addIfNotExist
    const bool must = v.scoring != 5;                       // every scoring but DOT_PRODUCT normalises
    constexpr int kPer = kVocMaxFeatures / kVocThreads;  // words per thread (word s = tid + k kVocThreads)
    double vals[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int s = tid + k * kVocThreads;
        vals[k] = 0.0;
        if (s < nw) {
            const int b = s_start[s], e = s_start[s + 1];
            double val = weight[fb + (int)(s_key[b] & 0xffffffffu)];
            if (add)
                for (int i = b + 1; i < e; i++) val += weight[fb + (int)(s_key[i] & 0xffffffffu)];
            if (add && !must) val /= (double)nw;
            bow_word[fb + s] = (uint32_t)(s_key[b] >> 32);
            vals[k] = val;
            if (!must) bow_value[fb + s] = val;
        }
    }
    BOW_T(6);
    if (must) {
        // BowVector::normalize: the sum in ascending word order, as the map iteration, by one lane over the values
        // staged in LDS (the sorted keys' space, read above)
        __syncthreads();
        double* s_val = (double*)s_key;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int s = tid + k * kVocThreads;
            if (s < nw) s_val[s] = vals[k];
        }
        __syncthreads();
        if (tid == 0) s_norm = v.scoring == 1 ? sqrt(norm_chain<true>(s_val, nw)) : norm_chain<false>(s_val, nw);
        __syncthreads();
        const double norm = s_norm;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int s = tid + k * kVocThreads;
            if (s < nw) bow_value[fb + s] = norm > 0.0 ? vals[k] / norm : vals[k];
        }
    }
    if (tid == 0) nbow[f] = nw;
    BOW_T(7);
}

hipError_t launch_voc_transform(const VocDev& v, int levelsup, int nframes, const uint8_t* desc, const int32_t* counts,
                                int stride, int max_n, int32_t* word, double* weight, uint32_t* nid, uint32_t* bow_word,
                                double* bow_value, int32_t* nbow, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat,
                                int32_t* nfv, hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    if (max_n > 0)
        hipLaunchKernelGGL(k_voc_descend, dim3((max_n + 15) / 16, nframes), dim3(256), 0, st, v, levelsup, desc, counts,
                           stride, word, weight, nid);
    hipLaunchKernelGGL(k_voc_bow, dim3(nframes), dim3(kVocThreads), 0, st, v, counts, stride, word, weight, nid, bow_word,
                       bow_value, nbow, fv_node, fv_off, fv_feat, nfv);
    return hipGetLastError();
}

}  // namespace orbamd

#ifdef ORBX_BOW_TRACE
extern "C" int orbx_debug_bow_trace(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbamd::g_bow_trace), sizeof(orbamd::g_bow_trace)) == hipSuccess ? 0 : -1;
}
#endif
