/*
 * orb_oracle_voc.c -- CPU restatement of the DBoW2 vocabulary transform that produces the
 * BowVector / FeatureVector of every Frame and KeyFrame (Frame::ComputeBoW, ORB_SLAM2/src/
 * Frame.cc:400-407: mpORBvocabulary->transform(vCurrentDesc, mBowVec, mFeatVec, 4)).
 * TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * DBoW2 (ORB-SLAM2's fork: TemplatedVocabulary<FORB::TDescriptor, FORB>) is NOT vendored in
 * /root/reference (Thirdparty/ is absent) and ORBvoc.txt is absent: this restates the published
 * algorithm -- TemplatedVocabulary::loadFromTextFile, transform(features, BowVector&,
 * FeatureVector&, levelsup), transform(feature, word, weight, nid, levelsup), BowVector::
 * addWeight / addIfNotExist / normalize, FeatureVector::addFeature, FORB::distance -- so parity
 * of this row is UNPINNED (no reference output exists to check it against).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

struct oc_vocab {
    int k, L, scoring, weighting;
    int n;           /* nodes (0 = root) */
    int* parent;
    uint8_t* desc;   /* n x 32 */
    double* weight;
    int* word_id;    /* Node() default 0 for nodes not flagged leaf */
    int* child_off;  /* children of node i: child[child_off[i] .. child_off[i+1]) in file order */
    int* child;
    int nwords;
};

/* TemplatedVocabulary::loadFromTextFile (the ORB-SLAM2 fork) from arrays of the node lines in
 * file order: node i (1-based) has parent[i-1], is_leaf[i-1], desc[(i-1)*32], weight[i-1]. */
oc_vocab* oc_vocab_create(int k, int L, int scoring, int weighting, int nlines, const int32_t* parent,
                          const uint8_t* is_leaf, const uint8_t* desc, const double* weight) {
    if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3 ||
        nlines < 0)
        return NULL;
    oc_vocab* v = (oc_vocab*)calloc(1, sizeof(oc_vocab));
    v->k = k, v->L = L, v->scoring = scoring, v->weighting = weighting;
    v->n = nlines + 1;
    v->parent = (int*)calloc((size_t)v->n, sizeof(int));
    v->desc = (uint8_t*)calloc((size_t)v->n, 32);
    v->weight = (double*)calloc((size_t)v->n, sizeof(double));
    v->word_id = (int*)calloc((size_t)v->n, sizeof(int));
    v->child_off = (int*)calloc((size_t)v->n + 1, sizeof(int));
    v->child = (int*)calloc((size_t)v->n, sizeof(int));
    for (int i = 1; i < v->n; i++) {
        const int pid = parent[i - 1];
        if (pid < 0 || pid >= i) { /* a parent must precede its children */
            oc_vocab_destroy(v);
            return NULL;
        }
        v->parent[i] = pid;
        memcpy(v->desc + 32 * (size_t)i, desc + 32 * (size_t)(i - 1), 32);
        v->weight[i] = weight[i - 1];
        if (is_leaf[i - 1] > 0) v->word_id[i] = v->nwords++;
        v->child_off[pid + 1]++;
    }
    for (int i = 0; i < v->n; i++) v->child_off[i + 1] += v->child_off[i];
    int* fill = (int*)calloc((size_t)v->n, sizeof(int));
    for (int i = 1; i < v->n; i++) { /* children.push_back in file order */
        const int pid = v->parent[i];
        v->child[v->child_off[pid] + fill[pid]++] = i;
    }
    free(fill);
    return v;
}

void oc_vocab_destroy(oc_vocab* v) {
    if (!v) return;
    free(v->parent), free(v->desc), free(v->weight), free(v->word_id), free(v->child_off), free(v->child);
    free(v);
}

/* TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup) */
static void transform_one(const oc_vocab* v, const uint8_t* f, int* word_id, double* weight, int* nid, int levelsup) {
    const int nid_level = v->L - levelsup;
    if (nid_level <= 0) *nid = 0;
    int final_id = 0;
    int current_level = 0;
    do {
        ++current_level;
        const int* nodes = v->child + v->child_off[final_id];
        const int nn = v->child_off[final_id + 1] - v->child_off[final_id];
        final_id = nodes[0];
        double best_d = oc_descriptor_distance(f, v->desc + 32 * (size_t)final_id); /* FORB::distance */
        for (int c = 1; c < nn; c++) {
            const int id = nodes[c];
            const double d = oc_descriptor_distance(f, v->desc + 32 * (size_t)id);
            if (d < best_d) {
                best_d = d;
                final_id = id;
            }
        }
        if (current_level == nid_level) *nid = final_id;
    } while (v->child_off[final_id + 1] > v->child_off[final_id]); /* !isLeaf() = children not empty */
    *word_id = v->word_id[final_id];
    *weight = v->weight[final_id];
}

/* std::map emulations: sorted arrays with insertion */
static int find_u32(const uint32_t* keys, int n, uint32_t k, int* pos) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if (keys[mid] < k) lo = mid + 1; else hi = mid;
    }
    *pos = lo;
    return lo < n && keys[lo] == k;
}

/* TemplatedVocabulary::transform(features, BowVector& v, FeatureVector& fv, levelsup).
 * Outputs: bow_word/bow_value (ascending word id, *nbow entries), fv_node ascending (*nfv),
 * fv_off[*nfv+1], fv_feat. Caps: n entries each (fv_off n+1). */
int oc_vocab_transform(const oc_vocab* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_word,
                       double* bow_value, int* nbow, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat, int* nfv) {
    *nbow = 0;
    *nfv = 0;
    if (v->n <= 1 || v->child_off[1] == v->child_off[0]) return 0; /* empty() */
    /* mustNormalize: L1_NORM -> L1, L2_NORM -> L2, CHI_SQUARE/KL/BHATTACHARYYA -> L1, DOT_PRODUCT: no */
    const int must = v->scoring != 5;
    const int l2 = v->scoring == 1;
    int nb = 0, nf = 0;
    int* fcount = (int*)calloc((size_t)n + 1, sizeof(int));
    int* fnode_feat_n = fcount; /* per fv node entry count */
    int32_t* tmp_feat = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int* tmp_node_of = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    for (int i_feature = 0; i_feature < n; i_feature++) {
        int id, nid = 0;
        double w;
        transform_one(v, desc + 32 * (size_t)i_feature, &id, &w, &nid, levelsup);
        if (w > 0) { /* not stopped */
            int pos;
            const int found = find_u32(bow_word, nb, (uint32_t)id, &pos);
            if (v->weighting == 0 || v->weighting == 1) { /* TF_IDF / TF: BowVector::addWeight */
                if (found) {
                    bow_value[pos] += w;
                } else {
                    memmove(bow_word + pos + 1, bow_word + pos, sizeof(uint32_t) * (size_t)(nb - pos));
                    memmove(bow_value + pos + 1, bow_value + pos, sizeof(double) * (size_t)(nb - pos));
                    bow_word[pos] = (uint32_t)id;
                    bow_value[pos] = w;
                    nb++;
                }
            } else if (!found) { /* IDF / BINARY: BowVector::addIfNotExist */
                memmove(bow_word + pos + 1, bow_word + pos, sizeof(uint32_t) * (size_t)(nb - pos));
                memmove(bow_value + pos + 1, bow_value + pos, sizeof(double) * (size_t)(nb - pos));
                bow_word[pos] = (uint32_t)id;
                bow_value[pos] = w;
                nb++;
            }
            /* FeatureVector::addFeature(nid, i_feature) */
            int fpos;
            if (!find_u32(fv_node, nf, (uint32_t)nid, &fpos)) {
                memmove(fv_node + fpos + 1, fv_node + fpos, sizeof(uint32_t) * (size_t)(nf - fpos));
                memmove(fnode_feat_n + fpos + 1, fnode_feat_n + fpos, sizeof(int) * (size_t)(nf - fpos));
                fv_node[fpos] = (uint32_t)nid;
                fnode_feat_n[fpos] = 0;
                nf++;
            }
            fnode_feat_n[fpos]++;
            tmp_feat[i_feature] = i_feature;
            tmp_node_of[i_feature] = nid;
        } else {
            tmp_node_of[i_feature] = -1;
        }
    }
    if ((v->weighting == 0 || v->weighting == 1) && nb > 0 && !must) {
        const double nd = nb; /* unnecessary when normalizing */
        for (int i = 0; i < nb; i++) bow_value[i] /= nd;
    }
    if (must) { /* BowVector::normalize */
        double norm = 0.0;
        if (!l2) {
            for (int i = 0; i < nb; i++) norm += fabs(bow_value[i]);
        } else {
            for (int i = 0; i < nb; i++) norm += bow_value[i] * bow_value[i];
            norm = sqrt(norm);
        }
        if (norm > 0.0)
            for (int i = 0; i < nb; i++) bow_value[i] /= norm;
    }
    /* CSR of the FeatureVector: features of a node in insertion (= ascending) order */
    fv_off[0] = 0;
    for (int i = 0; i < nf; i++) fv_off[i + 1] = fv_off[i] + fnode_feat_n[i];
    int* fill = (int*)calloc((size_t)nf + 1, sizeof(int));
    for (int i_feature = 0; i_feature < n; i_feature++) {
        const int nid = tmp_node_of[i_feature];
        if (nid < 0) continue;
        int fpos;
        find_u32(fv_node, nf, (uint32_t)nid, &fpos);
        fv_feat[fv_off[fpos] + fill[fpos]++] = tmp_feat[i_feature];
    }
    free(fill);
    free(fcount);
    free(tmp_feat);
    free(tmp_node_of);
    *nbow = nb;
    *nfv = nf;
    return 0;
}

/* per-feature descent outputs (for stage-isolated tests) */
void oc_vocab_descend(const oc_vocab* v, const uint8_t* desc, int n, int levelsup, int32_t* word, double* weight,
                      int32_t* nid) {
    for (int i = 0; i < n; i++) {
        int w_id, nd = 0;
        double w;
        transform_one(v, desc + 32 * (size_t)i, &w_id, &w, &nd, levelsup);
        word[i] = w_id;
        weight[i] = w;
        nid[i] = nd;
    }
}
