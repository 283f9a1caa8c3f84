/* test_oracle_asan.c -- the CPU oracle (oracle/orb_oracle*.c) and the synthetic frame generator
 * (csrc/synth.c) built with AddressSanitizer + UndefinedBehaviorSanitizer: extraction at
 * the BASELINE geometries and edge cases (flat, tiny, noise-free), the matchers with MapPoint /
 * stereo / FeatureVector variants, stereo matching, ComputeDistinctiveDescriptors and a vocabulary
 * transform. Any sanitizer report aborts the run (-fno-sanitize-recover). Prints "ALL PASS".
 * Build + run: tests/test_sanitizers.py (host only; GPU sanitizers are not available on the pool). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

static uint32_t lcg(uint32_t* s) { *s = *s * 1664525u + 1013904223u; return *s >> 8; }

static int extract(oc_extractor* e, const uint8_t* img, int W, int H, orbx_kp** k, uint8_t** d) {
    const int cap = 64 * 1024;
    *k = (orbx_kp*)malloc(sizeof(orbx_kp) * cap);
    *d = (uint8_t*)malloc(32 * (size_t)cap);
    int n = 0;
    oc_extract(e, img, W, H, W, *k, *d, cap, &n);
    return n;
}

static void view(orbm_kf_view* v, const orbx_kp* k, const uint8_t* d, int n, float* x, float* y, float* a, int32_t* o,
                 const float* sc, const float* s2, uint32_t* ids, int32_t* off, int32_t* feat, int nodes, uint32_t* seed,
                 float* ur, uint8_t* mp, uint8_t* bad) {
    memset(v, 0, sizeof(*v));
    for (int i = 0; i < n; i++) { x[i] = k[i].x; y[i] = k[i].y; a[i] = k[i].angle; o[i] = k[i].octave; }
    /* FeatureVector: node of feature i = i % nodes, features ascending within a node */
    int pos = 0;
    for (int j = 0; j < nodes; j++) {
        ids[j] = 100u + 13u * (uint32_t)j;
        off[j] = pos;
        for (int i = j; i < n; i += nodes) feat[pos++] = i;
    }
    off[nodes] = pos;
    for (int i = 0; i < n; i++) {
        ur[i] = (lcg(seed) % 4 == 0) ? x[i] - (float)(lcg(seed) % 40) : -1.f;
        mp[i] = lcg(seed) % 3 != 0;
        bad[i] = lcg(seed) % 10 == 0;
    }
    v->n = n; v->desc = d; v->x = x; v->y = y; v->angle = a; v->octave = o; v->uright = ur; v->has_mp = mp;
    v->mp_bad = bad; v->n_nodes = nodes; v->node_id = ids; v->node_off = off; v->node_feat = feat; v->nlevels = 8;
    v->scale_factors = sc; v->level_sigma2 = s2;
}

int main(void) {
    const int geo[][3] = {{640, 480, 1000}, {752, 480, 1200}, {1241, 376, 2000}, {200, 150, 500}};
    int total = 0;
    for (int g = 0; g < 4; g++) {
        const int W = geo[g][0], H = geo[g][1];
        orbx_params p = {geo[g][2], 1.2f, 8, 20, 7};
        if (g == 3) p.nlevels = 4; /* a small frame: fewer levels so every level keeps a cell grid */
        oc_extractor *e = oc_create(&p), *er = oc_create(&p);
        uint8_t* fr = (uint8_t*)malloc((size_t)W * H * 2);
        uint8_t* right = (uint8_t*)malloc((size_t)W * H);
        orbx_synth_frames(g, 0, 2, W, H, fr);
        orbx_synth_frames_shifted(g, 0, 1, W, H, 9, right);
        orbx_kp *k1, *k2, *kr;
        uint8_t *d1, *d2, *dr;
        const int n1 = extract(e, fr, W, H, &k1, &d1);
        const int nr = extract(er, right, W, H, &kr, &dr);
        const int n2 = extract(e, fr + (size_t)W * H, W, H, &k2, &d2);
        total += n1 + n2;
        /* stereo (Frame::ComputeStereoMatches) needs the left extractor's pyramid of the left frame */
        oc_extractor* el = oc_create(&p);
        orbx_kp* kl;
        uint8_t* dl;
        const int nl = extract(el, fr, W, H, &kl, &dl);
        float *url = malloc(4 * (size_t)(nl + 1)), *dpl = malloc(4 * (size_t)(nl + 1));
        oc_compute_stereo_matches(el, er, kl, dl, nl, kr, dr, nr, 47.9f, 0.11f, url, dpl);
        float sc[16], isc[16], s2[16], is2[16];
        oc_get_tables(e, sc, isc, s2, is2, NULL, NULL);
        uint32_t seed = 7u + (uint32_t)g;
        const int nodes = 1 + g * 20;
        float *x1 = malloc(4 * (size_t)n1 + 4), *y1 = malloc(4 * (size_t)n1 + 4), *a1 = malloc(4 * (size_t)n1 + 4),
              *u1 = malloc(4 * (size_t)n1 + 4);
        float *x2 = malloc(4 * (size_t)n2 + 4), *y2 = malloc(4 * (size_t)n2 + 4), *a2 = malloc(4 * (size_t)n2 + 4),
              *u2 = malloc(4 * (size_t)n2 + 4);
        int32_t *o1 = malloc(4 * (size_t)n1 + 4), *o2 = malloc(4 * (size_t)n2 + 4);
        uint32_t *id1 = malloc(4 * (size_t)nodes), *id2 = malloc(4 * (size_t)nodes);
        int32_t *of1 = malloc(4 * (size_t)nodes + 4), *of2 = malloc(4 * (size_t)nodes + 4);
        int32_t *f1 = malloc(4 * (size_t)n1 + 4), *f2 = malloc(4 * (size_t)n2 + 4);
        uint8_t *m1 = malloc((size_t)n1 + 1), *b1 = malloc((size_t)n1 + 1), *m2 = malloc((size_t)n2 + 1),
                *b2 = malloc((size_t)n2 + 1);
        orbm_kf_view v1, v2;
        view(&v1, k1, d1, n1, x1, y1, a1, o1, sc, s2, id1, of1, f1, nodes, &seed, u1, m1, b1);
        view(&v2, k2, d2, n2, x2, y2, a2, o2, sc, s2, id2, of2, f2, nodes, &seed, u2, m2, b2);
        int32_t* out = malloc(4 * (size_t)(n1 > n2 ? n1 : n2) + 4);
        const float F[9] = {0, -1.4e-5f, 3.6e-3f, 1.4e-5f, 0, -1.7e-2f, -3.6e-3f, 1.7e-2f, 0.1f};
        for (int st = 0; st < 2; st++)
            for (int ori = 0; ori < 2; ori++) oc_search_for_triangulation(&v1, &v2, F, 3900.f, 256.f, st, ori, out);
        oc_search_by_bow_kf_kf(&v1, &v2, 0.75f, 1, out);
        oc_search_by_bow_kf_f(&v1, &v2, 0.7f, 1, out);
        /* distinctive descriptors over ragged observation lists built from d1 */
        const int P = 50;
        int32_t offs[51];
        offs[0] = 0;
        for (int i = 0; i < P; i++) offs[i + 1] = offs[i] + (int)(lcg(&seed) % 9);
        if (offs[P] > n1) offs[P] = n1;
        for (int i = 0; i < P; i++) if (offs[i + 1] > offs[P]) offs[i + 1] = offs[P];
        int32_t best[50];
        oc_compute_distinctive_descriptors(P, offs, d1, best);
        free(x1); free(y1); free(a1); free(u1); free(x2); free(y2); free(a2); free(u2); free(o1); free(o2);
        free(id1); free(id2); free(of1); free(of2); free(f1); free(f2); free(m1); free(b1); free(m2); free(b2);
        free(out); free(url); free(dpl); free(kl); free(dl);
        free(k1); free(d1); free(k2); free(d2); free(kr); free(dr); free(fr); free(right);
        oc_destroy(e); oc_destroy(er); oc_destroy(el);
    }
    /* edge cases: a flat image (no corners) and a 1-level extractor */
    {
        const int W = 320, H = 240;
        uint8_t* flat = malloc((size_t)W * H);
        memset(flat, 77, (size_t)W * H);
        orbx_params p = {300, 1.2f, 1, 20, 7};
        oc_extractor* e = oc_create(&p);
        orbx_kp* k;
        uint8_t* d;
        const int n = extract(e, flat, W, H, &k, &d);
        if (n != 0) { printf("flat image gave %d keypoints\n", n); return 1; }
        free(k); free(d); free(flat);
        oc_destroy(e);
    }
    /* a tiny vocabulary transform */
    {
        const int kk = 4, L = 3;
        int nlines = kk + kk * kk + kk * kk * kk;
        int32_t* parent = malloc(4 * (size_t)nlines);
        uint8_t *leaf = malloc((size_t)nlines), *vd = malloc(32 * (size_t)nlines);
        double* w = malloc(8 * (size_t)nlines);
        uint32_t seed = 5;
        for (int i = 0; i < nlines; i++) {
            parent[i] = i < kk ? 0 : (i < kk + kk * kk ? 1 + (i - kk) / kk : 1 + kk + (i - kk - kk * kk) / kk);
            leaf[i] = i >= kk + kk * kk;
            for (int b = 0; b < 32; b++) vd[32 * i + b] = (uint8_t)lcg(&seed);
            w[i] = 0.5 + (double)(lcg(&seed) % 100) / 50.0;
        }
        oc_vocab* v = oc_vocab_create(kk, L, 0, 0, nlines, parent, leaf, vd, w);
        uint8_t desc[32 * 64];
        for (int i = 0; i < 32 * 64; i++) desc[i] = (uint8_t)lcg(&seed);
        uint32_t bw[64], fn[64];
        double bv[64];
        int32_t fo[65], ff[64];
        int nb, nf;
        oc_vocab_transform(v, desc, 64, 1, bw, bv, &nb, fn, fo, ff, &nf);
        oc_vocab_destroy(v);
        free(parent); free(leaf); free(vd); free(w);
    }
    printf("ALL PASS (%d keypoints extracted under ASan/UBSan)\n", total);
    return 0;
}
