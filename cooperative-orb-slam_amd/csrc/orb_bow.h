/*
 * orb_bow.h -- device view of a DBoW2 vocabulary (bow_kernels.hip, capi.cpp).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbamd {

constexpr int kVocMaxFeatures = 4096;  // descriptors per frame of one transform (LDS sort capacity)

/* a node as its parent's child: the descent reads, for every child of the current node, the child's
 * descriptor and this record in one round of independent loads, and takes the next node's children from the
 * winning lane's record -- one dependent round per level instead of three (child_off -> child -> desc) */
struct VocChild {
    int32_t id;      // node id (file order)
    int32_t c0, nc;  // its children: child slots c0 .. c0 + nc - 1 (file order)
    int32_t word;    // word id (Node() default 0 for nodes not flagged as words)
    double weight;
    int32_t pad[2];
};
static_assert(sizeof(VocChild) == 32, "one 32-byte record per child slot");

struct VocDev {
    const uint8_t* cdesc;      // [child slot][32] descriptor of the node in that slot (root's children first)
    const VocChild* crec;      // [child slot]
    int root_c0, root_nc;      // the root's children
    int n, L, scoring, weighting;
};

hipError_t launch_voc_transform(const VocDev& v, int levelsup, int nframes, const uint8_t* desc, const int32_t* counts,
                                int stride, int max_n, int32_t* word, double* weight, uint32_t* nid, uint32_t* bow_word,
                                double* bow_value, int32_t* nbow, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat,
                                int32_t* nfv, hipStream_t st);

}  // namespace orbamd
