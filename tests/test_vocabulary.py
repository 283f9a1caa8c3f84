"""DBoW2 vocabulary transform (Frame::ComputeBoW, Frame.cc:400-407). CPU: the oracle restatement
(oracle/orb_oracle_voc.c) against a pure-Python restatement of TemplatedVocabulary::transform;
GPU: the device transform (k_voc_descend + k_voc_bow) against the oracle, bit-exact on word ids,
BowVector values (float64 bits) and the FeatureVector. DBoW2 and ORBvoc.txt are absent (not
vendored): the vocabularies are synthetic, parity with DBoW2 itself is unpinned."""
import numpy as np
import pytest

import oracle_py
import orbamd
import proj_scenes as ps
from orbamd.vocabulary import synth_vocabulary, to_text, L1_NORM, L2_NORM, DOT_PRODUCT, TF_IDF, TF, IDF, BINARY

VOCABS = [  # (k, L, seed, ragged, scoring, weighting, levelsup)
    (10, 4, 1, False, L1_NORM, TF_IDF, 2),
    (6, 6, 2, False, L1_NORM, TF_IDF, 4),
    (10, 4, 3, True, L2_NORM, TF, 1),
    (8, 5, 4, True, DOT_PRODUCT, TF_IDF, 3),
    (9, 4, 5, False, L1_NORM, IDF, 2),
    (7, 4, 6, True, DOT_PRODUCT, BINARY, 6),
]


def transform_py(k, L, scoring, weighting, parent, is_leaf, desc, weight, feats, levelsup):
    """Pure-Python TemplatedVocabulary::transform (features, BowVector, FeatureVector, levelsup)."""
    n = len(parent) + 1
    children = [[] for _ in range(n)]
    word = [0] * n
    nw = 0
    for i in range(1, n):
        children[parent[i - 1]].append(i)
        if is_leaf[i - 1] > 0:
            word[i] = nw
            nw += 1
    D = np.concatenate([np.zeros((1, 32), np.uint8), desc])
    W = np.concatenate([[0.0], weight])
    bits_nodes = np.unpackbits(D, axis=1)
    bow, fv = {}, {}
    must = scoring != DOT_PRODUCT
    for i, f in enumerate(feats):
        fb = np.unpackbits(f)
        nid_level = L - levelsup
        nid = 0
        node, level = 0, 0
        while children[node]:
            level += 1
            ch = children[node]
            d = [int(np.count_nonzero(bits_nodes[c] != fb)) for c in ch]
            node = ch[int(np.argmin(d))]  # first minimum = `d < best_d` scan
            if level == nid_level:
                nid = node
        w = float(W[node])
        if w > 0:
            wid = word[node]
            if weighting in (TF_IDF, TF):
                bow[wid] = bow[wid] + w if wid in bow else w
            else:
                bow.setdefault(wid, w)
            fv.setdefault(nid, []).append(i)
    keys = sorted(bow)
    vals = [bow[kk] for kk in keys]
    if weighting in (TF_IDF, TF) and vals and not must:
        vals = [v / float(len(vals)) for v in vals]
    if must:
        if scoring == L2_NORM:
            norm = 0.0
            for v in vals:
                norm += v * v
            norm = np.sqrt(norm)
        else:
            norm = 0.0
            for v in vals:
                norm += abs(v)
        if norm > 0:
            vals = [v / norm for v in vals]
    return (np.array(keys, np.uint32), np.array(vals, np.float64)), fv


@pytest.mark.parametrize("cfg", VOCABS[:4])
def test_vocab_oracle_matches_restatement(cfg):
    k, L, seed, ragged, scoring, weighting, levelsup = cfg
    v = synth_vocabulary(k, L, seed, ragged=ragged)
    ov = oracle_py.OracleVocabulary(k, L, scoring, weighting, *v[2:])
    _, d, _ = ps.frame_features(seed % 3, seed)
    d = d[:300]
    (bw, bv), fv = ov.transform(d, levelsup)
    (bw2, bv2), fv2 = transform_py(k, L, scoring, weighting, *v[2:], d, levelsup)
    np.testing.assert_array_equal(bw, bw2)
    np.testing.assert_array_equal(bv.view(np.uint64), bv2.view(np.uint64))
    assert fv == fv2


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", VOCABS)
def test_vocab_transform_gpu_bit_exact(cfg, tmp_path):
    k, L, seed, ragged, scoring, weighting, levelsup = cfg
    v = synth_vocabulary(k, L, seed, ragged=ragged)
    ov = oracle_py.OracleVocabulary(k, L, scoring, weighting, *v[2:])
    path = tmp_path / "voc.txt"
    to_text(path, *v, scoring=scoring, weighting=weighting)  # loadFromTextFile path
    gv = orbamd.ORBVocabulary(path)
    assert gv.info()["nodes"] == len(v[2]) + 1
    for agent, t in ((0, 0), (seed % 5, 17)):
        _, d, _ = ps.frame_features(agent, t)
        (bw, bv), fv = gv.transform(d, levelsup)
        (bw2, bv2), fv2 = ov.transform(d, levelsup)
        np.testing.assert_array_equal(bw, bw2)
        np.testing.assert_array_equal(bv.view(np.uint64), bv2.view(np.uint64))
        assert fv == fv2
    (bw, bv), fv = gv.transform(np.zeros((0, 32), np.uint8), levelsup)
    assert len(bw) == 0 and fv == {}


@pytest.mark.gpu
def test_vocab_batch_device_matches_host():
    torch = pytest.importorskip("torch")
    k, L = 10, 4
    v = synth_vocabulary(k, L, 11)
    gv = orbamd.ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, *v[2:])
    ov = oracle_py.OracleVocabulary(k, L, L1_NORM, TF_IDF, *v[2:])
    B, S = 4, 1200
    dev = torch.device("cuda", 0)
    descs = [ps.frame_features(a, 3 * a)[1] for a in range(B)]
    host = np.zeros((B, S, 32), np.uint8)
    cnt = np.zeros(B, np.int32)
    for b, d in enumerate(descs):
        host[b, :len(d)] = d
        cnt[b] = len(d)
    dd = torch.from_numpy(host).to(dev)
    dc = torch.from_numpy(cnt).to(dev)
    z = lambda *s, dt=torch.int32: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
    word, wt, nid = z(B, S), z(B, S, dt=torch.float64), z(B, S)
    bw, bv, nb = z(B, S), z(B, S, dt=torch.float64), z(B)
    fn, fo, ff, nf = z(B, S), z(B, S + 1), z(B, S), z(B)
    lib = orbamd.load()
    st = torch.cuda.current_stream(dev).cuda_stream
    rc = lib.orbv_transform_batch_device(gv._h, B, dd.data_ptr(), dc.data_ptr(), S, 2, word.data_ptr(), wt.data_ptr(),
                                         nid.data_ptr(), bw.data_ptr(), bv.data_ptr(), nb.data_ptr(), fn.data_ptr(),
                                         fo.data_ptr(), ff.data_ptr(), nf.data_ptr(), st)
    assert rc == 0
    torch.cuda.synchronize()
    for b in range(B):
        (ow, ov_), ofv = ov.transform(descs[b], 2)
        n = int(nb[b])
        assert np.array_equal(bw[b, :n].cpu().numpy().astype(np.uint32), ow)
        assert np.array_equal(bv[b, :n].cpu().numpy().view(np.uint64), ov_.view(np.uint64))
        m = int(nf[b])
        offs = fo[b, :m + 1].cpu().numpy()
        feats = ff[b].cpu().numpy()
        nodes = fn[b, :m].cpu().numpy().astype(np.uint32)
        assert {int(nodes[i]): feats[offs[i]:offs[i + 1]].tolist() for i in range(m)} == ofv
        w2, wt2, nid2 = ov.descend(descs[b], 2)
        assert np.array_equal(word[b, :cnt[b]].cpu().numpy(), w2)
        assert np.array_equal(nid[b, :cnt[b]].cpu().numpy(), nid2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [VOCABS[0], VOCABS[2]])
def test_vocab_transform_gpu_sort_sizes(cfg):
    """k_voc_bow's sort blocks (128 keys in registers, LDS stages above): descriptor counts either side of every
    block and register boundary up to the 4096 capacity, with repeated descriptors (equal words and nodes)"""
    k, L, seed, ragged, scoring, weighting, levelsup = cfg
    v = synth_vocabulary(k, L, seed, ragged=ragged)
    ov = oracle_py.OracleVocabulary(k, L, scoring, weighting, *v[2:])
    gv = orbamd.ORBVocabulary.from_arrays(k, L, scoring, weighting, *v[2:])
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 256, (5000, 32), dtype=np.uint8)
    for n in (1, 2, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 1024, 1025, 2048, 2049, 4095, 4096):
        d = pool[:n].copy() if n % 2 else pool[rng.integers(0, max(n // 3, 1), n)]
        (bw, bv), fv = gv.transform(d, levelsup)
        (bw2, bv2), fv2 = ov.transform(d, levelsup)
        np.testing.assert_array_equal(bw, bw2, err_msg="n=%d" % n)
        np.testing.assert_array_equal(bv.view(np.uint64), bv2.view(np.uint64), err_msg="n=%d" % n)
        assert fv == fv2, n
