"""Checker of the bench schedule's outputs against the CPU oracle (test infrastructure).

Used by tests/test_gpu_schedule.py and by bench.py after its timed region (the oracle is the
checker here, never the measured path): recomputes, for sampled frames of an
orbamd.agent.AgentSchedule step, ORBextractor::operator() (oracle/orb_oracle.c) and the BF
SearchForTriangulation against the previous frame of the same graph, and the cross-agent
SearchForTriangulation and SearchByBoW(KF,KF) of this agent's keyframe against every agent's keyframe
(their FeatureVectors from the oracle vocabulary transform, their MapPoint records from
orbamd.agent.kf_mp_flags), and compares
every keypoint field (raw float bits), descriptor byte and match index with the device results.
A stereo schedule (sched.stereo = (mbf, mb)) also recomputes each sampled frame's right image and
Frame::ComputeStereoMatches (oracle/orb_oracle_frame.c) and compares the right keypoints, mvuRight /
mvDepth (raw float bits) and the kept count; the matchers then see both keyframes' mvuRight.
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import oracle_py  # noqa: E402


def host_threads():
    """CPU threads this process may use: the affinity set, capped by the cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except Exception:
        pass
    return max(1, n)


def check_schedule(sched, frames_np, samples=None, agent_frames=None, threads=None, nfeatures=None):
    """Checks the LAST step's batch (sched.last_batch of its frame pool). samples: list of (graph p,
    frame b) to check (default: first, middle and last frame of each graph, plus each one's
    predecessor so the match row can be recomputed); agent_frames(r, t) -> the keyframe image of
    agent r, t = the host frame index of this agent's keyframe (default: frames_np[t] for every
    agent, i.e. world 1).
    Returns dict(bit_exact, checked_frames, checked_pairs, checked_slots, mismatches[...])."""
    import orbamd
    sub = sched.sub
    nfeat = nfeatures or getattr(sched, "nfeatures", 1000)
    if samples is None:
        samples = sorted({(p, b) for p in range(sched.P) for b in (0, sub // 2, sub - 1)})
    F12, ex, ey = orbamd.device.default_geometry()
    tabs = oracle_py.OracleExtractor(nfeat, 1.2, 8, 20, 7).tables()
    need = set()
    for p, b in samples:
        need.add((p, b))
        need.add((p, (b - 1) % sub))
    need = sorted(need)
    local = {}

    stereo = getattr(sched, "stereo", None)

    def extract(img):
        """(keypoints, descriptors, stereo) of one frame; stereo (img = [2, H, W]): (right keypoints, right
        descriptors, mvuRight, mvDepth, kept) from two extractors as the stereo Frame holds them (Frame.cc:80-92)"""
        orc = oracle_py.OracleExtractor(nfeat, 1.2, 8, 20, 7)
        if not stereo:
            k, d = orc(img)
            return k, d, None
        k, d = orc(img[0])
        orr = oracle_py.OracleExtractor(nfeat, 1.2, 8, 20, 7)
        kr, dr = orr(img[1])
        ur, dp, ns = oracle_py.compute_stereo_matches(orc, orr, k, d, kr, dr, stereo[0], stereo[1])
        return k, d, (kr, dr, ur, dp, ns)

    threads = threads or host_threads()
    with ThreadPoolExecutor(max_workers=threads) as ex_pool:
        outs = list(ex_pool.map(lambda pb: extract(frames_np[sched.frame_index(*pb)]), need))
    for pb, o in zip(need, outs):
        local[pb] = o
    mism = []

    def bits_differ(a, b):
        a, b = np.ascontiguousarray(a, np.float32), np.ascontiguousarray(b, np.float32)
        return a.shape != b.shape or not np.array_equal(a.view(np.uint32), b.view(np.uint32))

    for p, b in samples:
        kg, dg, mg = sched.frame_results(p, b)
        ko, do, so = local[(p, b)]
        if len(kg) != len(ko) or kg.tobytes() != ko.tobytes() or not np.array_equal(dg, do):
            mism.append("frame p=%d b=%d: %d vs %d keypoints or differing fields" % (p, b, len(kg), len(ko)))
            continue
        if stereo:
            (krg, drg), (urg, dpg, nsg) = sched.stereo_results(p, b)
            kro, dro, uro, dpo, nso = so
            if len(krg) != len(kro) or krg.tobytes() != kro.tobytes() or not np.array_equal(drg, dro):
                mism.append("right image p=%d b=%d: %d vs %d keypoints or differing fields" % (p, b, len(krg), len(kro)))
                continue
            if bits_differ(urg, uro) or bits_differ(dpg, dpo) or nsg != nso:
                mism.append("stereo p=%d b=%d: mvuRight / mvDepth / kept (%d vs %d) differ" % (p, b, nsg, nso))
                continue
        kp, dp, sp = local[(p, (b - 1) % sub)]
        v1 = orbamd.KeyFrameView(ko, do, tabs["scale"], tabs["sigma2"], uright=so[2] if stereo else None)
        v2 = orbamd.KeyFrameView(kp, dp, tabs["scale"], tabs["sigma2"], uright=sp[2] if stereo else None)
        _, mo = oracle_py.search_for_triangulation(v1, v2, F12, ex, ey, False, False)
        if not np.array_equal(mg, mo):
            mism.append("match p=%d b=%d vs b-1: %s" % (p, b, "%d entries differ" % int((mg != mo).sum())
                                                        if mg.shape == mo.shape else "length %d vs %d" % (len(mg), len(mo))))
    nslots = 0
    bow_counts = []
    if sched.exchange_on:
        from orbamd.agent import KF_LEVELSUP, LOOP_NNRATIO, kf_mp_flags
        xm, xn, xb, xbn = sched.exchange_results()
        t_kf = sched.frame_index(0, 0)
        kq, dq, sq = local.get((0, 0)) or extract(frames_np[t_kf])
        voc = _oracle_vocabulary(sched)

        def kf_view(k, d, s, with_fv):
            """the keyframe as the slot carries it: MapPoint records (kf_mp_flags), mvuRight when stereo and, for
            SearchByBoW, the FeatureVector of the vocabulary transform (KeyFrame::ComputeBoW, levelsup 4)"""
            f = kf_mp_flags(len(k))
            fv = voc.transform(d, KF_LEVELSUP)[1] if with_fv else None
            return orbamd.KeyFrameView(k, d, tabs["scale"], tabs["sigma2"], feat_vec=fv, has_mp=(f & 1).astype(bool),
                                       mp_bad=((f >> 1) & 1).astype(bool), uright=s[2] if s is not None else None)
        vq, vq_bow = kf_view(kq, dq, sq, False), kf_view(kq, dq, sq, True)
        for r in range(sched.world):
            img = frames_np[t_kf] if agent_frames is None else agent_frames(r, t_kf)
            kr, dr, sr = extract(img) if agent_frames is not None else (kq, dq, sq)
            vr, vr_bow = ((vq, vq_bow) if agent_frames is None else
                          (kf_view(kr, dr, sr, False), kf_view(kr, dr, sr, True)))
            # LocalMapping's SearchForTriangulation (features with a MapPoint skipped on both sides, :699-726)
            n_o, mo = oracle_py.search_for_triangulation(vq, vr, F12, ex, ey, False, False)
            if not np.array_equal(xm[r], mo) or int(xn[r]) != int(n_o):
                ndiff = int((xm[r] != mo).sum()) if xm[r].shape == mo.shape else -1
                mism.append("cross-agent triangulation vs agent %d: %s, count %d vs %d"
                            % (r, "%d entries differ" % ndiff if ndiff >= 0 else
                               "%d vs %d query keypoints" % (len(xm[r]), len(mo)), int(xn[r]), int(n_o)))
            # LoopClosing's SearchByBoW(KF,KF) (ORBmatcher(0.75, true))
            nb_o, mb = oracle_py.search_by_bow(vq_bow, vr_bow, LOOP_NNRATIO, True, other_is_keyframe=True)
            if not np.array_equal(xb[r], mb) or int(xbn[r]) != int(nb_o):
                ndiff = int((xb[r] != mb).sum()) if xb[r].shape == mb.shape else -1
                mism.append("cross-agent SearchByBoW vs agent %d: %s, count %d vs %d"
                            % (r, "%d entries differ" % ndiff if ndiff >= 0 else
                               "%d vs %d query keypoints" % (len(xb[r]), len(mb)), int(xbn[r]), int(nb_o)))
            bow_counts.append(int(nb_o))
            nslots += 1
    return {"bit_exact": not mism, "checked_frames": len(samples), "checked_pairs": len(samples),
            "checked_slots": nslots, "slot_bow_matches": bow_counts, "mismatches": mism[:8]}


_VOC = {}


def _oracle_vocabulary(sched):
    """the oracle restatement of the schedule's (synthetic) vocabulary, built once per process"""
    from orbamd.vocabulary import L1_NORM, TF_IDF
    key = id(sched.voc_arrays)
    if key not in _VOC:
        k, L, par, leaf, desc, w = sched.voc_arrays
        _VOC.clear()
        _VOC[key] = oracle_py.OracleVocabulary(k, L, L1_NORM, TF_IDF, par, leaf, desc, w)
    return _VOC[key]
