#!/usr/bin/env python3
"""Measurements of the SURVEY.md 8(f) rows built beside the headline path (one JSON line each).

  stereo       Frame::ComputeStereoMatches on C3 (752x480 stereo, 1200 features): B pairs resident in
               HBM, one step = extract 2B frames + k_stereo over the B pairs (device batch API);
               reported as stereo pairs/s, k_stereo's share from HIP events, and the CPU oracle's
               ComputeStereoMatches alone on the same pairs.
  projection   SearchByProjection(Frame&, vector<MapPoint*>, th) host API (H2D + grid + scan + resolve
               + D2H) per call on a 640x480 frame with ~900 candidate MapPoints vs the CPU oracle.
  distinctive  MapPoint::ComputeDistinctiveDescriptors for 20k MapPoints x ~25 observations (device
               batch) vs the CPU oracle.
  bow          Frame::ComputeBoW (DBoW2 transform, levelsup 4) of 256 extracted 640x480 frames with a synthetic
               vocabulary of ORBvoc.txt's shape (k=10, L=6, 1.1M nodes) resident in HBM, vs the CPU oracle.
  tri_nodes    SearchForTriangulation over common BoW nodes (levelsup 4, ORBvoc.txt-shaped synthetic
               vocabulary) for 256 frame pairs, FeatureVectors from the device BoW transform, vs the
               BF batch (one node) on the same pairs and vs the oracle per pair.
  extract_host ORBextractor::operator() through the host-buffer C ABI on one 640x480 frame per call
               (H2D + whole pipeline + D2H): the Tracking thread's per-frame latency, vs the oracle.
  matcher_host SearchForTriangulation (BF and over BoW nodes), SearchByBoW(KF,F), SearchByBoW(KF,KF)
               through the host C ABI, one keyframe pair per call (how the C++ drop-ins call them).
The CPU figures are the oracle (a plain-C restatement, 1 thread), not the reference build.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cooperative-orb-slam_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def bench_stereo(torch, steps, B=128):
    import orbamd
    import oracle_py
    W, H, nf = 752, 480, 1200
    MBF, MB = 47.90639384423901, 0.11
    dev = torch.device("cuda", 0)
    left = orbamd.synth_frames(0, 0, B, W, H)
    right = orbamd.synth_frames(0, 0, B, W, H, dx=9)
    ext = orbamd.ORBextractor(nf, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=2 * B)
    stride = ext.max_keypoints(W, H)
    frames = torch.from_numpy(np.concatenate([left, right])).to(dev)
    kps = torch.empty((2 * B, stride, 6), dtype=torch.float32, device=dev)
    desc = torch.empty((2 * B, stride, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    fl = torch.arange(B, dtype=torch.int32, device=dev)
    fr = fl + B
    ur = torch.empty((B, stride), dtype=torch.float32, device=dev)
    dp = torch.empty((B, stride), dtype=torch.float32, device=dev)
    ns = torch.zeros(B, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    def step(ev=None):
        ext.extract_batch_device(frames, kps, desc, cnt, st)
        if ev:
            ev[0].record()
        orbamd.frame.stereo_matches_batch_device(ext, ext, fl, fr, kps, desc, cnt, kps, desc, cnt, MBF, MB, ur, dp,
                                                 ns, st)
        if ev:
            ev[1].record()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        step(evs[i])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k_ms = sum(a.elapsed_time(b) for a, b in evs) / steps
    # CPU oracle: ComputeStereoMatches alone (extraction excluded) on a sample of the pairs
    ol = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    orr = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    tc, nc = 0.0, 0
    for p in range(8):
        ko, do_ = ol(left[p])
        kro, dro = orr(right[p])
        t = time.perf_counter()
        oracle_py.compute_stereo_matches(ol, orr, ko, do_, kro, dro, MBF, MB)
        tc += time.perf_counter() - t
        nc += 1
    return {"row": "stereo", "workload": "C3 752x480 stereo, 1200 feat, B=%d pairs/step" % B,
            "pairs_per_s_extract_plus_stereo": round(B * steps / el, 1),
            "k_stereo_ms_per_step": round(k_ms, 4), "k_stereo_us_per_pair": round(k_ms * 1e3 / B, 3),
            "stereo_kept_per_pair": round(float(ns.float().mean().item()), 1),
            "cpu_oracle_ms_per_pair": round(tc / nc * 1e3, 3), "cpu_threads": 1}


def bench_tri_nodes(torch, reps):
    import orbamd
    import oracle_py
    from orbamd.matcher import KeyFrameView
    from orbamd.vocabulary import synth_vocabulary_full, L1_NORM, TF_IDF
    k, L, parent, leaf, desc, weight = synth_vocabulary_full(10, 6, 7)
    gv = orbamd.ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, parent, leaf, desc, weight)
    B = 256
    pipe = orbamd.device.BatchPipeline(torch, 640, 480, B)
    frames = orbamd.synth_frames(0, 0, B, 640, 480)
    pipe.extract(torch.from_numpy(frames).cuda())
    pipe.bow(gv, 4)
    torch.cuda.synchronize()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    t_nodes = timed(pipe.match_pairs_nodes)
    n_nodes = float(pipe.nmatch.float().mean().item())
    t_bow = timed(lambda: pipe.bow(gv, 4))
    t_bf = timed(pipe.match_pairs)
    n_bf = float(pipe.nmatch.float().mean().item())
    ov = oracle_py.OracleVocabulary(k, L, L1_NORM, TF_IDF, parent, leaf, desc, weight)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    tabs = orc.tables()
    r0, r1 = orc(frames[1]), orc(frames[0])
    v1 = KeyFrameView(r0[0], r0[1], tabs["scale"], tabs["sigma2"], feat_vec=ov.transform(r0[1], 4)[1])
    v2 = KeyFrameView(r1[0], r1[1], tabs["scale"], tabs["sigma2"], feat_vec=ov.transform(r1[1], 4)[1])
    t = time.perf_counter()
    for _ in range(5):
        oracle_py.search_for_triangulation(v1, v2, pipe.F12, pipe.ex, pipe.ey, False, False)
    c = (time.perf_counter() - t) / 5
    pipe.close()
    return {"row": "search_for_triangulation_bow_nodes", "workload": "256 pairs of 640x480 frames, levelsup 4, "
            "vocabulary k=10 L=6", "gpu_ms_per_256_pairs_nodes": round(t_nodes, 4),
            "gpu_ms_per_256_frames_bow": round(t_bow, 4), "gpu_ms_per_256_pairs_bf": round(t_bf, 4),
            "matches_per_pair_nodes": round(n_nodes, 1), "matches_per_pair_bf": round(n_bf, 1),
            "cpu_oracle_ms_per_pair_nodes": round(c * 1e3, 3), "cpu_threads": 1}


def bench_extract_host(reps):
    import orbamd
    import oracle_py
    img = orbamd.synth_frames(0, 5, 1, 640, 480)[0]
    ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7)
    for _ in range(5):
        ext(img)
    t = time.perf_counter()
    for _ in range(reps):
        k, d = ext(img)
    g = (time.perf_counter() - t) / reps
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    t = time.perf_counter()
    for _ in range(5):
        ko, do = orc(img)
    c = (time.perf_counter() - t) / 5
    assert len(k) == len(ko) and np.array_equal(d, do)
    return {"row": "extract_single_frame_host_api", "workload": "640x480, 1000 features, one frame per call",
            "gpu_ms_per_call": round(g * 1e3, 4), "cpu_oracle_ms_per_call": round(c * 1e3, 3), "cpu_threads": 1}


def bench_matcher_host(reps):
    """per-call latency of the drop-in matcher entry points through the host C ABI (one keyframe pair
    per call, as LocalMapping.cc:268 / Tracking.cc:767 / LoopClosing.cc:267 call them) vs the oracle"""
    import orbamd
    import oracle_py
    from orbamd.matcher import KeyFrameView
    rng = np.random.default_rng(7)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    tabs = orc.tables()
    (k1, d1), (k2, d2) = [orc(img) for img in orbamd.synth_frames(0, 10, 2, 640, 480)]
    F12, ex, ey = orbamd.device.default_geometry()
    ids = np.sort(rng.choice(100000, 90, replace=False))  # ~ the node count at levelsup 4 of ORBvoc.txt

    def fv(n):
        a = rng.integers(0, len(ids), n)
        return {int(ids[i]): list(np.nonzero(a == i)[0]) for i in range(len(ids)) if (a == i).any()}
    fv1, fv2 = fv(len(k1)), fv(len(k2))
    mp1, mp2 = rng.random(len(k1)) < 0.8, rng.random(len(k2)) < 0.8
    rows = []
    cases = [
        ("search_for_triangulation_bf", "SearchForTriangulation, one node (BF), mono, no MapPoints",
         lambda m, a, b: m.SearchForTriangulation(a, b, F12, ex, ey),
         lambda a, b: oracle_py.search_for_triangulation(a, b, F12, ex, ey, False, False),
         KeyFrameView(k1, d1, tabs["scale"], tabs["sigma2"]), KeyFrameView(k2, d2, tabs["scale"], tabs["sigma2"]),
         (0.6, False)),
        ("search_for_triangulation_nodes", "SearchForTriangulation over ~90 common BoW nodes (LocalMapping.cc:268)",
         lambda m, a, b: m.SearchForTriangulation(a, b, F12, ex, ey),
         lambda a, b: oracle_py.search_for_triangulation(a, b, F12, ex, ey, False, False),
         KeyFrameView(k1, d1, tabs["scale"], tabs["sigma2"], feat_vec=fv1),
         KeyFrameView(k2, d2, tabs["scale"], tabs["sigma2"], feat_vec=fv2), (0.6, False)),
        ("search_by_bow_kf_f", "SearchByBoW(KF, F), ~90 nodes, 80% MapPoints, ratio 0.7, rotation check (Tracking.cc:767)",
         lambda m, a, b: m.SearchByBoW(a, b, other_is_keyframe=False),
         lambda a, b: oracle_py.search_by_bow(a, b, 0.7, True, other_is_keyframe=False),
         KeyFrameView(k1, d1, tabs["scale"], tabs["sigma2"], feat_vec=fv1, has_mp=mp1),
         KeyFrameView(k2, d2, tabs["scale"], tabs["sigma2"], feat_vec=fv2), (0.7, True)),
        ("search_by_bow_kf_kf", "SearchByBoW(KF, KF), ~90 nodes, 80% MapPoints, ratio 0.75 (LoopClosing.cc:267)",
         lambda m, a, b: m.SearchByBoW(a, b, other_is_keyframe=True),
         lambda a, b: oracle_py.search_by_bow(a, b, 0.75, True, other_is_keyframe=True),
         KeyFrameView(k1, d1, tabs["scale"], tabs["sigma2"], feat_vec=fv1, has_mp=mp1),
         KeyFrameView(k2, d2, tabs["scale"], tabs["sigma2"], feat_vec=fv2, has_mp=mp2), (0.75, True)),
    ]
    for name, what, g_call, o_call, a, b, (ratio, ori) in cases:
        m = orbamd.ORBmatcher(ratio, ori)
        for _ in range(5):
            ng, mg = g_call(m, a, b)
        t = time.perf_counter()
        for _ in range(reps):
            g_call(m, a, b)
        g = (time.perf_counter() - t) / reps
        t = time.perf_counter()
        for _ in range(max(reps // 5, 3)):
            no, mo = o_call(a, b)
        c = (time.perf_counter() - t) / max(reps // 5, 3)
        assert ng == no and np.array_equal(mg, mo), name
        rows.append({"row": name, "workload": what + "; 640x480 frames, %d / %d features" % (len(k1), len(k2)),
                     "gpu_host_api_ms_per_call": round(g * 1e3, 4), "cpu_oracle_ms_per_call": round(c * 1e3, 4),
                     "nmatches": int(ng), "cpu_threads": 1})
        m.close()
    return rows


def bench_projection(reps):
    import orbamd
    import oracle_py
    import proj_scenes as ps
    F, mps = ps.local_scene(1, True)
    mt = orbamd.ORBmatcher(0.8, False)
    for _ in range(3):
        mt.SearchByProjectionLocal(F, mps, 3.0)
    t = time.perf_counter()
    for _ in range(reps):
        n, _m = mt.SearchByProjectionLocal(F, mps, 3.0)
    g = (time.perf_counter() - t) / reps
    t = time.perf_counter()
    for _ in range(reps):
        oracle_py.search_by_projection_local(F, mps, 3.0, 0.8)
    c = (time.perf_counter() - t) / reps
    return {"row": "search_by_projection_local", "workload": "640x480 frame, %d features, %d MapPoints" % (F.n, mps.n),
            "gpu_host_api_ms_per_call": round(g * 1e3, 4), "cpu_oracle_ms_per_call": round(c * 1e3, 4),
            "nmatches": int(n), "cpu_threads": 1}


def bench_fuse(reps):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th) (ORBmatcher.cc:825-975) per call: the device search
    (host prologue + one H2D, three kernels, one D2H) vs the oracle's search loop (the map updates that
    follow are host bookkeeping in both)."""
    import orbamd
    import oracle_py
    import proj_scenes as ps
    F, Tcw, Ow, mps, inv = ps.fuse_scene(3, True)
    mt = orbamd.ORBmatcher(0.6, True)
    for _ in range(3):
        mt.Fuse(F, Tcw, Ow, mps, 3.0, inv)
    t = time.perf_counter()
    for _ in range(reps):
        n, _b = mt.Fuse(F, Tcw, Ow, mps, 3.0, inv)
    g = (time.perf_counter() - t) / reps
    # the keyframe (arrays + feature grid) held in the keyframe cache: only the MapPoint queries travel
    cache = orbamd.KeyFrameCache()
    for _ in range(3):
        mt.FuseCached(cache, 7, F, Tcw, Ow, mps, 3.0, inv)
    t = time.perf_counter()
    for _ in range(reps):
        n2, b2 = mt.FuseCached(cache, 7, F, Tcw, Ow, mps, 3.0, inv)
    gc = (time.perf_counter() - t) / reps
    t = time.perf_counter()
    for _ in range(reps):
        no, bo = oracle_py.fuse(F, Tcw, Ow, mps, 3.0, inv)
    c = (time.perf_counter() - t) / reps
    same = no == n == n2 and (bo == _b).all() and (bo == b2).all()
    return {"row": "fuse", "workload": "Fuse(pKF, vpMapPoints, 3) (LocalMapping::SearchInNeighbors), 640x480 keyframe, "
            "%d features, %d MapPoints" % (F.n, mps.n),
            "gpu_host_api_ms_per_call": round(g * 1e3, 4), "gpu_cached_kf_ms_per_call": round(gc * 1e3, 4),
            "cpu_oracle_ms_per_call": round(c * 1e3, 4), "identical": bool(same), "nfused": int(n), "cpu_threads": 1}


def bench_distinctive(torch, reps):
    import orbamd
    import oracle_py
    rng = np.random.default_rng(3)
    P = 20000
    sizes = rng.integers(2, 50, P)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    desc = rng.integers(0, 256, (int(off[-1]), 32), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    d_off = torch.from_numpy(off).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_best = torch.empty(P, dtype=torch.int32, device=dev)
    d_out = torch.empty((P, 32), dtype=torch.uint8, device=dev)
    mt = orbamd.ORBmatcher()
    lib = orbamd.load()
    st = torch.cuda.current_stream(dev).cuda_stream

    def run():
        lib.orbm_compute_distinctive_descriptors_device(mt._h, P, d_off.data_ptr(), d_desc.data_ptr(),
                                                        d_best.data_ptr(), d_out.data_ptr(), st)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    g = e0.elapsed_time(e1) / reps
    ref = None
    t = time.perf_counter()
    ref = oracle_py.compute_distinctive_descriptors(off[:2001], desc)
    c = (time.perf_counter() - t) / 2000 * P
    assert (d_best[:2000].cpu().numpy() == ref).all()
    return {"row": "compute_distinctive_descriptors", "workload": "%d MapPoints, %d observations" % (P, int(off[-1])),
            "gpu_ms_per_batch": round(g, 4), "cpu_oracle_ms_per_batch": round(c * 1e3, 2), "cpu_threads": 1}


def bench_bow(torch, reps):
    import orbamd
    import oracle_py
    from orbamd.vocabulary import synth_vocabulary_full, L1_NORM, TF_IDF
    k, L, parent, leaf, desc, weight = synth_vocabulary_full(10, 6, 7)
    gv = orbamd.ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, parent, leaf, desc, weight)
    B = 256
    pipe = orbamd.device.BatchPipeline(torch, 640, 480, B)
    dev = torch.device("cuda", 0)
    frames = torch.from_numpy(orbamd.synth_frames(0, 0, B, 640, 480)).to(dev)
    pipe.extract(frames)
    S = pipe.stride
    z = lambda *s, dt=torch.int32: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
    word, wt, nid = z(B, S), z(B, S, dt=torch.float64), z(B, S)
    bw, bv, nb = z(B, S), z(B, S, dt=torch.float64), z(B)
    fn, fo, ff, nf = z(B, S), z(B, S + 1), z(B, S), z(B)
    lib = orbamd.load()
    st = torch.cuda.current_stream(dev).cuda_stream

    def run():
        lib.orbv_transform_batch_device(gv._h, B, pipe.desc.data_ptr(), pipe.counts.data_ptr(), S, 4, word.data_ptr(),
                                        wt.data_ptr(), nid.data_ptr(), bw.data_ptr(), bv.data_ptr(), nb.data_ptr(),
                                        fn.data_ptr(), fo.data_ptr(), ff.data_ptr(), nf.data_ptr(), st)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    g = e0.elapsed_time(e1) / reps
    ov = oracle_py.OracleVocabulary(k, L, L1_NORM, TF_IDF, parent, leaf, desc, weight)
    k0, d0, _m = pipe.host_results(0)
    t = time.perf_counter()
    (ow, oval), ofv = ov.transform(d0, 4)
    c = time.perf_counter() - t
    assert int(nb[0]) == len(ow) and np.array_equal(bw[0, :len(ow)].cpu().numpy().astype(np.uint32), ow)
    mean_n = float(pipe.counts.float().mean().item())
    return {"row": "dbow2_transform", "workload": "256 frames x %.0f descriptors, vocabulary k=10 L=6 (%d nodes)" % (
            mean_n, len(parent) + 1),
            "gpu_ms_per_256_frames": round(g, 4), "gpu_us_per_frame": round(g * 1e3 / B, 3),
            "cpu_oracle_ms_per_frame": round(c * 1e3, 3), "cpu_threads": 1}
    # (pipe's buffers are torch tensors; its handles close with the process)


def main():
    import torch
    steps = int(os.environ.get("BENCH_ROWS_STEPS", "10"))
    only = os.environ.get("BENCH_ROWS_ONLY")
    rows = {"extract_host": lambda: bench_extract_host(100), "matcher_host": lambda: bench_matcher_host(100),
            "stereo": lambda: bench_stereo(torch, steps), "projection": lambda: bench_projection(50), "fuse": lambda: bench_fuse(50),
            "distinctive": lambda: bench_distinctive(torch, 10), "bow": lambda: bench_bow(torch, 10),
            "tri_nodes": lambda: bench_tri_nodes(torch, 10)}
    for name, fn in rows.items():
        if only and name not in only.split(","):
            continue
        r = fn()
        for line in (r if isinstance(r, list) else [r]):
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
