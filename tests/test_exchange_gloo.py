"""Multi-agent exchange on CPU: world_size-2 gloo all-gather of keyframe slots (packed by the
library's host packer, orbx_pack_keyframe_host, with the keyframe's FeatureVector and MapPoint records
as the bench's exchange packs them; decoded by its validating parser, orbx_slot_parse) and the
cross-agent SearchForTriangulation and loop-candidate SearchByBoW(KF,KF) (oracle as the matcher) equal
a single-process run that matches the concatenated buffers."""
import os
import socket

import numpy as np
import pytest

pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _agent_keyframe(agent):
    import oracle_py
    import orbamd
    img = orbamd.synth_frames(agent, 0, 1, 640, 480, scene=0)[0]  # the agents' views of one scene
    orc = oracle_py.OracleExtractor()
    k, d = orc(img)
    return k, d, orc.tables()


_VOC = []


def _vocabulary():
    """a small synthetic vocabulary (k = 10, L = 4) on the oracle, built once per process"""
    if not _VOC:
        import oracle_py
        from orbamd.vocabulary import L1_NORM, TF_IDF, synth_vocabulary
        k, L, par, leaf, desc, w = synth_vocabulary(k=10, L=4, seed=3)
        _VOC.append(oracle_py.OracleVocabulary(k, L, L1_NORM, TF_IDF, par, leaf, desc, w))
    return _VOC[0]


def _fv_csr(fv):
    ids = sorted(fv)
    off = np.concatenate([[0], np.cumsum([len(fv[i]) for i in ids])]).astype(np.int32)
    feat = np.concatenate([np.asarray(fv[i], np.int32) for i in ids]) if ids else np.zeros(0, np.int32)
    return np.asarray(ids, np.uint32), off, feat


def _pack(agent, k, d, tabs, cap):
    from orbamd import exchange
    from orbamd.agent import kf_mp_flags
    meta = exchange.make_meta(agent=agent, mnId=agent, scale=tabs["scale"], sigma2=tabs["sigma2"])
    bow, fv = _vocabulary().transform(d, 2)
    return exchange.pack_host(meta, k, d, cap, mp_flags=kf_mp_flags(len(k)), bow=bow, fv=_fv_csr(fv))


def _cross_match(kq, dq, tabs, slots):
    """per slot: SearchForTriangulation (features with a MapPoint skipped on both sides) and SearchByBoW(KF,KF)
    (ORBmatcher(0.75, true), LoopClosing's loop-candidate match) of the querying keyframe, from the decoded slot"""
    import oracle_py
    import orbamd
    from orbamd import exchange
    from orbamd.agent import kf_mp_flags
    F12, ex, ey = orbamd.device.default_geometry()
    out = []
    fq = kf_mp_flags(len(kq))
    fvq = _vocabulary().transform(dq, 2)[1]
    vq = orbamd.KeyFrameView(kq, dq, tabs["scale"], tabs["sigma2"], has_mp=(fq & 1).astype(bool),
                             mp_bad=((fq >> 1) & 1).astype(bool))
    vqb = orbamd.KeyFrameView(kq, dq, tabs["scale"], tabs["sigma2"], feat_vec=fvq, has_mp=(fq & 1).astype(bool),
                              mp_bad=((fq >> 1) & 1).astype(bool))
    for buf in slots:
        got = exchange.parse(buf)
        k2, d2, f2 = got["kps"], got["desc"], got["mp_flags"]
        sc, sg = got["meta"].mvScaleFactors[:8], got["meta"].mvLevelSigma2[:8]
        mp2, bad2 = (f2 & 1).astype(bool), ((f2 >> 1) & 1).astype(bool)
        fv2 = {int(got["fv_node"][i]): list(got["fv_feat"][got["fv_off"][i]:got["fv_off"][i + 1]])
               for i in range(len(got["fv_node"]))}
        v2 = orbamd.KeyFrameView(k2, d2, sc, sg, has_mp=mp2, mp_bad=bad2)
        v2b = orbamd.KeyFrameView(k2, d2, sc, sg, feat_vec=fv2, has_mp=mp2, mp_bad=bad2)
        out.append(oracle_py.search_for_triangulation(vq, v2, F12, ex, ey, False, False)[1])
        out.append(oracle_py.search_by_bow(vqb, v2b, 0.75, True, other_is_keyframe=True)[1])
    return out


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "cooperative-orb-slam_amd"), os.path.join(root, "oracle")]
    import torch
    import torch.distributed as dist
    from orbamd import exchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k, d, tabs = _agent_keyframe(rank)
    cap = 1031
    mine = torch.from_numpy(_pack(rank, k, d, tabs, cap))
    allb = torch.empty(world * mine.numel(), dtype=torch.uint8)
    dist.all_gather_into_tensor(allb, mine)
    slots = allb.numpy().reshape(world, -1)
    res = _cross_match(k, d, tabs, slots)
    q.put((rank, [r.tolist() for r in res]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_allgather_cross_agent_match():
    import torch.multiprocessing as mp
    from orbamd import exchange
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    kfs = [_agent_keyframe(a) for a in range(world)]
    slots = [_pack(a, k, d, t, 1031) for a, (k, d, t) in enumerate(kfs)]
    for r in range(world):
        exp = _cross_match(kfs[r][0], kfs[r][1], kfs[r][2], slots)
        assert [e.tolist() for e in exp] == got[r]
        # self-match sanity: the features without a MapPoint triangulate against themselves, those with a good one
        # are found by the loop-candidate SearchByBoW
        assert sum(x >= 0 for x in got[r][2 * r]) > 0.3 * len(kfs[r][0])
        assert sum(x >= 0 for x in got[r][2 * r + 1]) > 0.3 * len(kfs[r][0])
        # and the other agent's view of the scene gives both cross-agent matchers real work
        o = 1 - r
        assert sum(x >= 0 for x in got[r][2 * o]) > 0.1 * len(kfs[r][0]), sum(x >= 0 for x in got[r][2 * o])
        assert sum(x >= 0 for x in got[r][2 * o + 1]) > 0.1 * len(kfs[r][0]), sum(x >= 0 for x in got[r][2 * o + 1])
