/*
 * orb_bow.h -- device view of a DBoW2 vocabulary (bow_kernels.hip, capi.cpp).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbamd {

constexpr int kVocMaxFeatures = 4096;  // descriptors per frame of one transform (LDS sort capacity)

struct VocDev {
    const uint8_t* desc;       // [n][32] node descriptors (node 0 = root)
    const double* weight;      // [n]
    const int32_t* word_id;    // [n] (Node() default 0 for nodes not flagged as words)
    const int32_t* child_off;  // [n+1] children of node i: child[child_off[i] .. child_off[i+1]) in file order
    const int32_t* child;      // [n]
    int n, L, scoring, weighting;
};

hipError_t launch_voc_transform(const VocDev& v, int levelsup, int nframes, const uint8_t* desc, const int32_t* counts,
                                int stride, int max_n, int32_t* word, double* weight, uint32_t* nid, uint32_t* bow_word,
                                double* bow_value, int32_t* nbow, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat,
                                int32_t* nfv, hipStream_t st);

}  // namespace orbamd
