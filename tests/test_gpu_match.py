"""GPU parity: ORBmatcher on the HIP path vs the CPU oracle (exact index equality)."""
import numpy as np
import pytest

import oracle_py
import orbamd
from orbamd.matcher import KeyFrameView

pytestmark = pytest.mark.gpu


def _frames_kf(agent, t, n=2, W=640, H=480, nf=1000):
    orc = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    tabs = orc.tables()
    out = []
    for img in orbamd.synth_frames(agent, t, n, W, H):
        k, d = orc(img)
        out.append((k, d))
    return out, tabs


def _view(k, d, tabs, **kw):
    return KeyFrameView(k, d, tabs["scale"], tabs["sigma2"], **kw)


def _random_featvec(rng, n, nodes):
    ids = rng.choice(10000, size=nodes, replace=False)
    assign = rng.integers(0, nodes, n)
    return {int(ids[a]): [] for a in range(nodes)} | {int(ids[a]): list(np.nonzero(assign == a)[0])
                                                    for a in range(nodes)}


# the BASELINE geometries: C2 640x480/1000, C3 752x480/1200, C4 1241x376/2000, and the monocular
# initialisation extractor (2000 features at 640x480, Tracking.cc:119-125); every n2 spans many
# 64-candidate MFMA chunks and 512-candidate SIMT tiles
CONFIGS = [(640, 480, 1000), (752, 480, 1200), (1241, 376, 2000), (640, 480, 2000)]


@pytest.mark.parametrize("W,H,nf", CONFIGS)
@pytest.mark.parametrize("check_ori", [False, True])
def test_triangulation_bf(check_ori, W, H, nf):
    (k1, d1), (k2, d2) = _frames_kf(0, 0, W=W, H=H, nf=nf)[0]
    tabs = _frames_kf(0, 0, 1, W=W, H=H, nf=nf)[1]
    assert len(k1) > 0.9 * nf and len(k2) > 0.9 * nf
    F12, ex, ey = orbamd.device.default_geometry()
    v1, v2 = _view(k1, d1, tabs), _view(k2, d2, tabs)
    m = orbamd.ORBmatcher(0.6, check_ori)
    ng, mg = m.SearchForTriangulation(v1, v2, F12, ex, ey)
    no, mo = oracle_py.search_for_triangulation(v1, v2, F12, ex, ey, False, check_ori)
    assert ng == no and no > 0
    np.testing.assert_array_equal(mg, mo)


@pytest.mark.parametrize("nodes,stereo2", [(40, True), (8, True), (40, False), (3, True)])
def test_triangulation_nodes_mappoints_stereo(nodes, stereo2):
    """40 nodes (~25-50 candidates: the small-call kernel, one candidate chunk), 8 (~125: two chunks), 3 (~330:
    over the small path's 256-candidate bound, the staged kernel); stereo2 = False: KF2 is monocular"""
    rng = np.random.default_rng(3 + nodes)
    (k1, d1), (k2, d2) = _frames_kf(1, 4)[0]
    tabs = _frames_kf(1, 4, 1)[1]
    F12, ex, ey = orbamd.device.default_geometry()
    ids = np.sort(rng.choice(5000, nodes, replace=False))
    fv1 = {int(i): [] for i in ids}
    fv2 = {int(i): [] for i in ids[::2]} | {int(i) + 5000: [] for i in ids[1::2]}  # partial overlap
    for i in range(len(k1)):
        fv1[int(ids[rng.integers(0, nodes)])].append(i)
    keys2 = sorted(fv2)
    for i in range(len(k2)):
        fv2[keys2[rng.integers(0, len(keys2))]].append(i)
    ur1 = np.where(rng.random(len(k1)) < 0.3, rng.random(len(k1)) * 600, -1).astype(np.float32)
    ur2 = np.where(rng.random(len(k2)) < 0.3, rng.random(len(k2)) * 600, -1).astype(np.float32)
    mp1 = rng.random(len(k1)) < 0.2
    mp2 = rng.random(len(k2)) < 0.2
    v1 = _view(k1, d1, tabs, feat_vec=fv1, uright=ur1, has_mp=mp1)
    v2 = _view(k2, d2, tabs, feat_vec=fv2, uright=ur2 if stereo2 else None, has_mp=mp2)
    for only_stereo in (False, True):
        for check_ori in (False, True):
            m = orbamd.ORBmatcher(0.6, check_ori)
            ng, mg = m.SearchForTriangulation(v1, v2, F12, ex, ey, only_stereo)
            no, mo = oracle_py.search_for_triangulation(v1, v2, F12, ex, ey, only_stereo, check_ori)
            assert ng == no
            np.testing.assert_array_equal(mg, mo)


@pytest.mark.parametrize("kfkf", [False, True])
@pytest.mark.parametrize("nodes", [1, 8, 60])
def test_search_by_bow(kfkf, nodes):
    rng = np.random.default_rng(11 + nodes)
    (k1, d1), (k2, d2) = _frames_kf(2, 9)[0]
    tabs = _frames_kf(2, 9, 1)[1]
    ids = np.sort(rng.choice(100000, nodes, replace=False))
    fv1 = {int(i): [] for i in ids}
    fv2 = {int(i): [] for i in ids}
    for i in range(len(k1)):
        fv1[int(ids[rng.integers(0, nodes)])].append(i)
    for i in range(len(k2)):
        fv2[int(ids[rng.integers(0, nodes)])].append(i)
    mp1 = rng.random(len(k1)) < 0.8
    bad1 = rng.random(len(k1)) < 0.1
    mp2 = rng.random(len(k2)) < 0.8
    bad2 = rng.random(len(k2)) < 0.1
    v1 = _view(k1, d1, tabs, feat_vec=fv1, has_mp=mp1, mp_bad=bad1)
    v2 = _view(k2, d2, tabs, feat_vec=fv2, has_mp=mp2, mp_bad=bad2)
    for ratio, ori in ((0.75, True), (0.7, True), (0.9, False), (0.6, True)):
        m = orbamd.ORBmatcher(ratio, ori)
        ng, mg = m.SearchByBoW(v1, v2, other_is_keyframe=kfkf)
        no, mo = oracle_py.search_by_bow(v1, v2, ratio, ori, other_is_keyframe=kfkf)
        assert ng == no
        np.testing.assert_array_equal(mg, mo)


@pytest.mark.parametrize("W,H,nf", CONFIGS)
@pytest.mark.parametrize("check_ori", [False, True])
def test_batch_pairs_match_oracle(W, H, nf, check_ori):
    """the MFMA batch kernel (k_tri_mfma) at every BASELINE geometry, rotation filter on and off"""
    torch = pytest.importorskip("torch")
    B = 4
    frames = orbamd.synth_frames(0, 0, B, W, H)
    pipe = orbamd.device.BatchPipeline(torch, W, H, B, nfeatures=nf, check_ori=check_ori)
    pipe.step(torch.from_numpy(frames).cuda())
    torch.cuda.synchronize()
    pipe.check_error()
    orc = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    tabs = orc.tables()
    res = [orc(frames[b]) for b in range(B)]
    for b in range(B):
        kg, dg, mg = pipe.host_results(b)
        pb = (b + B - 1) % B
        v1 = _view(res[b][0], res[b][1], tabs)
        v2 = _view(res[pb][0], res[pb][1], tabs)
        assert kg.tobytes() == res[b][0].tobytes() and np.array_equal(dg, res[b][1])
        no, mo = oracle_py.search_for_triangulation(v1, v2, pipe.F12, pipe.ex, pipe.ey, False, check_ori)
        np.testing.assert_array_equal(mg, mo)
        assert int(pipe.nmatch[b].item()) == no and no > 0
    pipe.close()


@pytest.mark.parametrize("levelsup,check_ori", [(2, False), (1, True)])
def test_batch_pairs_over_bow_nodes(levelsup, check_ori):
    """Device chain extract -> ComputeBoW (orbv_transform_batch_device) -> SearchForTriangulation over
    the common FeatureVector nodes (orbm_triangulation_nodes_batch_device) vs the oracle's
    SearchForTriangulation with the oracle vocabulary's FeatureVectors."""
    torch = pytest.importorskip("torch")
    from orbamd.vocabulary import synth_vocabulary, L1_NORM, TF_IDF
    k, L = 10, 3
    v = synth_vocabulary(k, L, 5, flip_bits=24)
    gv = orbamd.ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, *v[2:])
    ov = oracle_py.OracleVocabulary(k, L, L1_NORM, TF_IDF, *v[2:])
    W, H, B = 640, 480, 4
    frames = orbamd.synth_frames(1, 7, B, W, H)
    pipe = orbamd.device.BatchPipeline(torch, W, H, B, check_ori=check_ori)
    pipe.extract(torch.from_numpy(frames).cuda())
    pipe.bow(gv, levelsup)
    pipe.match_pairs_nodes()
    torch.cuda.synchronize()
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    tabs = orc.tables()
    res = [orc(frames[b]) for b in range(B)]
    fvs = [ov.transform(res[b][1], levelsup)[1] for b in range(B)]
    total = 0
    for b in range(B):
        pb = (b + B - 1) % B
        v1 = _view(res[b][0], res[b][1], tabs, feat_vec=fvs[b])
        v2 = _view(res[pb][0], res[pb][1], tabs, feat_vec=fvs[pb])
        no, mo = oracle_py.search_for_triangulation(v1, v2, pipe.F12, pipe.ex, pipe.ey, False, check_ori)
        n = len(res[b][0])
        mg = pipe.match[b, :n].cpu().numpy()
        np.testing.assert_array_equal(mg, mo)
        assert int(pipe.nmatch[b].item()) == no
        total += no
    assert total > 0
    pipe.close()


@pytest.mark.parametrize("mode", [1, 0])
def test_search_by_bow_pairs_device(mode):
    """SearchByBoW (KF,KF) / (KF,F) for frame pairs over the device FeatureVectors
    (orbm_search_by_bow_batch_device) vs the oracle with the oracle vocabulary's FeatureVectors."""
    torch = pytest.importorskip("torch")
    from orbamd.vocabulary import synth_vocabulary, L1_NORM, TF_IDF
    k, L, levelsup = 10, 3, 1
    v = synth_vocabulary(k, L, 9, flip_bits=24)
    gv = orbamd.ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, *v[2:])
    ov = oracle_py.OracleVocabulary(k, L, L1_NORM, TF_IDF, *v[2:])
    W, H, B = 640, 480, 4
    frames = orbamd.synth_frames(2, 4, B, W, H)
    pipe = orbamd.device.BatchPipeline(torch, W, H, B)
    pipe.extract(torch.from_numpy(frames).cuda())
    pipe.bow(gv, levelsup)
    rng = np.random.default_rng(5 + mode)
    S = pipe.stride
    has_mp = rng.random((B, S)) < 0.8
    bad = rng.random((B, S)) < 0.1
    flags = torch.from_numpy((has_mp.astype(np.uint8) | (bad.astype(np.uint8) << 1))).cuda()
    qf = torch.arange(B, dtype=torch.int32).cuda()
    cf = ((qf + 1) % B).to(torch.int32)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    tabs = orc.tables()
    res = [orc(frames[b]) for b in range(B)]
    fvs = [ov.transform(res[b][1], levelsup)[1] for b in range(B)]
    total = 0
    for ratio, ori in ((0.75, True), (0.6, False)):
        out = torch.empty((B, S), dtype=torch.int32).cuda()
        nm = torch.zeros(B, dtype=torch.int32).cuda()
        pipe.search_by_bow_pairs(mode, qf, cf, flags, ratio, ori, out, nm)
        torch.cuda.synchronize()
        for p in range(B):
            a, b = p, (p + 1) % B
            na, nb = len(res[a][0]), len(res[b][0])
            va = _view(res[a][0], res[a][1], tabs, feat_vec=fvs[a], has_mp=has_mp[a, :na], mp_bad=bad[a, :na])
            vb = _view(res[b][0], res[b][1], tabs, feat_vec=fvs[b], has_mp=has_mp[b, :nb], mp_bad=bad[b, :nb])
            no, mo = oracle_py.search_by_bow(va, vb, ratio, ori, other_is_keyframe=mode == 1)
            rows = na if mode == 1 else nb
            np.testing.assert_array_equal(out[p, :rows].cpu().numpy(), mo)
            assert int(nm[p].item()) == no
            total += no
    assert total > 0
    pipe.close()


def _crafted_descriptors(rng, n1, n2):
    """KF1 / KF2 descriptor rows that stress the MFMA selection: exact duplicates among the candidates
    (distance ties: the later candidate wins, ORBmatcher.cc:719 `dist > bestDist` skips only larger
    ones), candidates at Hamming distance exactly TH_LOW = 50 and 51 from a query (ORBmatcher.cc:715),
    all-zero / all-one rows (D = 0 and 256: the extremes of the fp4 dot product), random rows."""
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    d2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    pat = rng.integers(0, 256, 32, dtype=np.uint8)
    d2[::7] = pat                     # ties at D = 0 for the queries equal to pat, every 7th candidate
    d1[::5] = pat
    d1[1::11] = 0
    d1[2::11] = 255
    d2[3::13] = 0
    d2[4::13] = 255
    bits = np.unpackbits(pat)
    for i, flips in ((3, 50), (8, 51)):   # a query pat^50 bits and one pat^51 bits, next to pat rows
        b = bits.copy()
        b[rng.choice(256, flips, replace=False)] ^= 1
        d1[i] = np.packbits(b)
    for j, flips in ((10, 50), (17, 49), (24, 51)):
        b = bits.copy()
        b[rng.choice(256, flips, replace=False)] ^= 1
        d2[j] = np.packbits(b)
    return d1, d2


@pytest.mark.parametrize("W,H,nf", [(640, 480, 1000), (1241, 376, 2000)])
@pytest.mark.parametrize("check_ori", [False, True])
def test_batch_pairs_crafted_descriptors(W, H, nf, check_ori):
    """k_tri_mfma on real keypoint geometry with crafted descriptors (ties, the TH_LOW boundary,
    D = 0 / 256 extremes) vs the oracle's SearchForTriangulation, both pair directions."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(nf + check_ori)
    (k1, _), (k2, _) = _frames_kf(3, 2, W=W, H=H, nf=nf)[0]
    tabs = _frames_kf(3, 2, 1, W=W, H=H, nf=nf)[1]
    d1, d2 = _crafted_descriptors(rng, len(k1), len(k2))
    pipe = orbamd.device.BatchPipeline(torch, W, H, 2, nfeatures=nf, check_ori=check_ori)
    assert k1.dtype.itemsize == 24 and max(len(k1), len(k2)) <= pipe.stride
    kps = np.zeros((2, pipe.stride, 24), np.uint8)
    desc = np.zeros((2, pipe.stride, 32), np.uint8)
    for b, (k, d) in enumerate(((k1, d1), (k2, d2))):
        kps[b, :len(k)] = np.frombuffer(k.tobytes(), np.uint8).reshape(len(k), 24)
        desc[b, :len(k)] = d
    pipe.kps.copy_(torch.from_numpy(kps.view(np.float32).reshape(2, pipe.stride, 6)))
    pipe.desc.copy_(torch.from_numpy(desc))
    pipe.counts.copy_(torch.tensor([len(k1), len(k2)], dtype=torch.int32))
    pipe.match_pairs()
    torch.cuda.synchronize()
    mg = pipe.match.cpu().numpy()
    v = (_view(k1, d1, tabs), _view(k2, d2, tabs))
    for p, (a, b) in enumerate(((0, 1), (1, 0))):   # pair p = (frame p, frame p - 1 mod 2)
        no, mo = oracle_py.search_for_triangulation(v[a], v[b], pipe.F12, pipe.ex, pipe.ey, False, check_ori)
        np.testing.assert_array_equal(mg[p, :v[a].n], mo)
        assert int(pipe.nmatch[p].item()) == no
    pipe.close()


def _desc_nodes(d, shift=4):
    """a FeatureVector keyed like a vocabulary (similar descriptors share a node): node = 100 + the top
    (8 - shift) bits of descriptor byte 0"""
    fv = {}
    for i in range(len(d)):
        fv.setdefault(100 + int(d[i, 0] >> shift), []).append(i)
    return fv


@pytest.mark.parametrize("W,H,nf,shift", [(1241, 376, 2000, 2), (752, 480, 1200, 3), (1241, 376, 3000, 2)])
def test_per_call_matchers_large_frames(W, H, nf, shift):
    """the host-API SearchByBoW ×2 and SearchForTriangulation over nodes at C3 / C4 sizes: 2000 features
    (the small-call kernels' side limit is 2048 FeatureVector entries) and 3000 (over it: the staged
    kernels), nodes of ~30-60 features; MapPoints, bad flags, stereo, both rotation settings"""
    rng = np.random.default_rng(nf + shift)
    (k1, d1), (k2, d2) = _frames_kf(3, 2, W=W, H=H, nf=nf)[0]
    tabs = _frames_kf(3, 2, 1, W=W, H=H, nf=nf)[1]
    F12, ex, ey = orbamd.device.default_geometry()
    fv1, fv2 = _desc_nodes(d1, shift), _desc_nodes(d2, shift)
    ur1 = np.where(rng.random(len(k1)) < 0.4, k1["x"] - rng.random(len(k1)) * 40, -1).astype(np.float32)
    ur2 = np.where(rng.random(len(k2)) < 0.4, k2["x"] - rng.random(len(k2)) * 40, -1).astype(np.float32)
    for mp_frac in (0.2, 0.8):
        mp1, mp2 = rng.random(len(k1)) < mp_frac, rng.random(len(k2)) < mp_frac
        bad1, bad2 = rng.random(len(k1)) < 0.05, rng.random(len(k2)) < 0.05
        v1 = _view(k1, d1, tabs, feat_vec=fv1, uright=ur1, has_mp=mp1, mp_bad=bad1)
        v2 = _view(k2, d2, tabs, feat_vec=fv2, uright=ur2, has_mp=mp2, mp_bad=bad2)
        for ori in (False, True):
            m = orbamd.ORBmatcher(0.75, ori)
            for only_stereo in (False, True):
                ng, mg = m.SearchForTriangulation(v1, v2, F12, ex, ey, only_stereo)
                no, mo = oracle_py.search_for_triangulation(v1, v2, F12, ex, ey, only_stereo, ori)
                assert ng == no
                np.testing.assert_array_equal(mg, mo)
            for kfkf in (False, True):
                ng, mg = m.SearchByBoW(v1, v2, other_is_keyframe=kfkf)
                no, mo = oracle_py.search_by_bow(v1, v2, 0.75, ori, other_is_keyframe=kfkf)
                assert ng == no and (mp_frac < 0.5 or no > 0)
                np.testing.assert_array_equal(mg, mo)
            m.close()


@pytest.mark.parametrize("W,H,nf", CONFIGS[:3])
@pytest.mark.parametrize("only_stereo,check_ori", [(0, False), (1, False), (0, True)])
def test_triangulation_bf_stereo_batch(W, H, nf, only_stereo, check_ori):
    """orbm_triangulation_bf_stereo_batch_device (k_tri_mfma<true>): SearchForTriangulation's stereo branch
    (ORBmatcher.cc:703-749) over a device batch of frame pairs whose keypoints are a mix of stereo (mvuRight >= 0) and
    monocular ones: the epipole test only between two monocular keypoints, bOnlyStereo skipping monocular ones on
    either side, with and without the rotation filter; every pair's row against the oracle"""
    import ctypes as C
    torch = pytest.importorskip("torch")
    B = 4
    frames = orbamd.synth_frames(3, 5, B, W, H)
    pipe = orbamd.device.BatchPipeline(torch, W, H, B, nfeatures=nf, check_ori=check_ori)
    pipe.extract(torch.from_numpy(frames).cuda())
    S = pipe.stride
    rng = np.random.default_rng(W + nf + only_stereo)
    # mvuRight: about 60 % stereo (a plausible disparity), the rest -1; near-epipole keypoints included by the geometry
    ur = np.full((B, S), -1.0, np.float32)
    counts = pipe.counts.cpu().numpy()
    kps = [pipe.host_keypoints(b)[0] for b in range(B)]
    for b in range(B):
        n = int(counts[b])
        st = rng.random(n) < 0.6
        ur[b, :n] = np.where(st, kps[b]["x"] - rng.uniform(1, 40, n).astype(np.float32), -1.0).astype(np.float32)
    d_ur = torch.from_numpy(ur).cuda()
    lib = orbamd.load()
    F = np.ascontiguousarray(pipe.F12.reshape(9))
    rc = lib.orbm_triangulation_bf_stereo_batch_device(
        pipe.mh, B, pipe.q1.data_ptr(), pipe.q2.data_ptr(), pipe.kps.data_ptr(), pipe.desc.data_ptr(),
        pipe.counts.data_ptr(), d_ur.data_ptr(), S, F.ctypes.data, pipe.ex, pipe.ey, len(pipe.scale),
        pipe.scale.ctypes.data, pipe.sigma2.ctypes.data, only_stereo, int(check_ori), pipe.match.data_ptr(),
        pipe.nmatch.data_ptr(), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    tabs = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7).tables()
    for b in range(B):
        b2 = (b - 1) % B
        n1 = int(counts[b])
        k1, d1 = pipe.host_keypoints(b)
        k2, d2 = pipe.host_keypoints(b2)
        v1 = _view(k1, d1, tabs, uright=ur[b, :n1])
        v2 = _view(k2, d2, tabs, uright=ur[b2, :len(k2)])
        no, mo = oracle_py.search_for_triangulation(v1, v2, pipe.F12, pipe.ex, pipe.ey, bool(only_stereo), check_ori)
        mg = pipe.match[b, :n1].cpu().numpy()
        np.testing.assert_array_equal(mg, mo, err_msg="pair %d" % b)
        assert int(pipe.nmatch[b].item()) == no and no > 0
    pipe.close()
