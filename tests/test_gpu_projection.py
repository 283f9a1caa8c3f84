"""GPU parity: ORBmatcher::SearchByProjection x4 (ORBmatcher.cc:45-129, 1328-1470, 1472-1599,
290-403) on the HIP path (k_grid + k_proj_scan + k_proj_resolve) vs the CPU oracle: the
per-feature assignment (which MapPoint, last writer wins, -2 = reset by the rotation filter)
and the returned count must be identical."""
import numpy as np
import pytest

import oracle_py
import orbamd
import proj_scenes as ps

pytestmark = pytest.mark.gpu


def _same(g, o):
    (ng, mg), (no, mo) = g, o
    bad = np.nonzero(mg != mo)[0]
    assert bad.size == 0, "assignment differs at %s: gpu %s oracle %s" % (bad[:8], mg[bad[:8]], mo[bad[:8]])
    assert ng == no, "nmatches %d vs oracle %d" % (ng, no)
    return ng


@pytest.mark.parametrize("seed,stereo,th,nnratio", [(1, True, 3.0, 0.8), (2, False, 1.0, 0.8),
                                                    (3, True, 5.0, 0.6), (8, True, 10.0, 0.9)])
def test_projection_local(seed, stereo, th, nnratio):
    F, mps = ps.local_scene(seed, stereo)
    g = orbamd.ORBmatcher(nnratio, False).SearchByProjectionLocal(F, mps, th)
    o = oracle_py.search_by_projection_local(F, mps, th, nnratio)
    assert _same(g, o) > F.n // 4


@pytest.mark.parametrize("seed,bmono,forward,check_ori,th", [(4, False, 0, True, 7.0), (5, True, 0, True, 15.0),
                                                             (6, False, 1, False, 7.0), (7, False, -1, True, 7.0)])
def test_projection_last_frame(seed, bmono, forward, check_ori, th):
    F, Tcw, mps, Tl = ps.last_frame_scene(seed, bmono, not bmono, forward)
    g = orbamd.ORBmatcher(0.9, check_ori).SearchByProjectionLastFrame(F, Tcw, mps, Tl, th, bmono)
    o = oracle_py.search_by_projection_last_frame(F, Tcw, mps, Tl, th, bmono, check_ori)
    assert _same(g, o) > F.n // 4


@pytest.mark.parametrize("seed,th,orb_dist,check_ori", [(5, 10.0, 100, True), (9, 3.0, 64, False),
                                                        (10, 10.0, 100, False)])
def test_projection_keyframe(seed, th, orb_dist, check_ori):
    F, Tcw, mps = ps.keyframe_scene(seed)
    g = orbamd.ORBmatcher(0.9, check_ori).SearchByProjectionKeyFrame(F, Tcw, mps, th, orb_dist)
    o = oracle_py.search_by_projection_keyframe(F, Tcw, mps, th, orb_dist, check_ori)
    assert _same(g, o) > F.n // 8


@pytest.mark.parametrize("seed,th", [(6, 10), (11, 3)])
def test_projection_sim3(seed, th):
    F, Scw, mps = ps.sim3_scene(seed)
    g = orbamd.ORBmatcher(0.75, True).SearchByProjectionSim3(F, Scw, mps, th)
    o = oracle_py.search_by_projection_sim3(F, Scw, mps, th)
    assert _same(g, o) > F.n // 8


def test_projection_edge_cases():
    """no MapPoints; every feature occupied; all MapPoints on one feature (a chain of claims)."""
    F, mps = ps.local_scene(12, True)
    mt = orbamd.ORBmatcher(0.8, False)
    empty = orbamd.MapPoints(0, desc=np.zeros((0, 32), np.uint8), track_in_view=[], track_proj_x=[],
                             track_proj_y=[], track_proj_xr=[], track_level=[], track_view_cos=[])
    n, m = mt.SearchByProjectionLocal(F, empty, 3.0)
    assert n == 0 and (m == -1).all()
    F.occupied = np.ones(F.n, np.uint8)
    assert _same(mt.SearchByProjectionLocal(F, mps, 3.0), oracle_py.search_by_projection_local(F, mps, 3.0, 0.8)) == 0
    F.occupied = np.zeros(F.n, np.uint8)
    k = 300
    same = orbamd.MapPoints(k, desc=np.repeat(F.desc[7:8], k, 0), bad=np.zeros(k), has_obs=np.arange(k) % 3 != 0,
                            track_in_view=np.ones(k), track_proj_x=np.full(k, F.x[7]), track_proj_y=np.full(k, F.y[7]),
                            track_proj_xr=np.full(k, F.x[7]), track_level=np.full(k, F.octave[7]),
                            track_view_cos=np.ones(k))
    _same(mt.SearchByProjectionLocal(F, same, 4.0), oracle_py.search_by_projection_local(F, same, 4.0, 0.8))


def test_distinctive_descriptors_batch():
    from test_oracle_frame import distinctive_scene
    off, desc = distinctive_scene(2, big=True)
    best, chosen = orbamd.matcher.compute_distinctive_descriptors(off, desc)
    ref = oracle_py.compute_distinctive_descriptors(off, desc)
    np.testing.assert_array_equal(best, ref)
    for p in np.nonzero(ref >= 0)[0]:
        assert (chosen[p] == desc[off[p] + ref[p]]).all()


def _same_fuse(g, o):
    (ng, bg), (no, bo) = g, o
    bad = np.nonzero(bg != bo)[0]
    assert bad.size == 0, "best_idx differs at %s: gpu %s oracle %s" % (bad[:8], bg[bad[:8]], bo[bad[:8]])
    assert ng == no, "nfused %d vs oracle %d" % (ng, no)
    return ng


@pytest.mark.parametrize("seed,stereo,th", [(3, True, 3.0), (4, False, 3.0), (5, True, 5.0), (13, False, 1.5)])
def test_fuse(seed, stereo, th):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th) (ORBmatcher.cc:825-975): per-MapPoint fused keypoint."""
    F, Tcw, Ow, mps, inv = ps.fuse_scene(seed, stereo)
    g = orbamd.ORBmatcher(0.6, True).Fuse(F, Tcw, Ow, mps, th, inv)
    o = oracle_py.fuse(F, Tcw, Ow, mps, th, inv)
    assert _same_fuse(g, o) > mps.n // 4


@pytest.mark.parametrize("seed,th", [(6, 4.0), (11, 10.0)])
def test_fuse_sim3(seed, th):
    """ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (ORBmatcher.cc:977-1100)."""
    F, Scw, mps = ps.fuse_sim3_scene(seed)
    g = orbamd.ORBmatcher(0.75, True).FuseSim3(F, Scw, mps, th)
    o = oracle_py.fuse_sim3(F, Scw, mps, th)
    assert _same_fuse(g, o) > mps.n // 4


def test_fuse_edge_cases():
    """no MapPoints; every MapPoint skipped; many MapPoints on one feature (no claims: all may fuse to it)."""
    F, Tcw, Ow, mps, inv = ps.fuse_scene(7, True)
    mt = orbamd.ORBmatcher(0.6, True)
    empty = orbamd.MapPoints(0, desc=np.zeros((0, 32), np.uint8), pos=np.zeros((0, 3), np.float32),
                             normal=np.zeros((0, 3), np.float32), min_dist=[], max_dist=[])
    n, b = mt.Fuse(F, Tcw, Ow, empty, 3.0, inv)
    assert n == 0 and b.size == 0
    mps.skip = np.ones(mps.n, np.uint8)
    n, b = mt.Fuse(F, Tcw, Ow, mps, 3.0, inv)
    assert n == 0 and (b == -1).all()
    mps.skip = np.zeros(mps.n, np.uint8)
    k = 200
    rep = orbamd.MapPoints(k, desc=np.repeat(mps.desc[:1], k, 0), pos=np.repeat(mps.pos[:1], k, 0),
                           normal=np.repeat(mps.normal[:1], k, 0), min_dist=np.repeat(mps.min_dist[:1], k),
                           max_dist=np.repeat(mps.max_dist[:1], k))
    _same_fuse(mt.Fuse(F, Tcw, Ow, rep, 3.0, inv), oracle_py.fuse(F, Tcw, Ow, rep, 3.0, inv))


@pytest.mark.parametrize("seed,noise,check_ori,ratio,window", [(1, 0.0, True, 0.9, 100), (2, 3.0, True, 0.9, 100),
                                                               (3, 0.0, False, 0.7, 100), (4, 8.0, True, 0.9, 30)])
def test_search_for_initialization(seed, noise, check_ori, ratio, window):
    """ORBmatcher::SearchForInitialization (ORBmatcher.cc:405-520) at 640x480 with the 2000-feature
    initialisation extractor, windowSize 100 as Tracking::MonocularInitialization calls it (Tracking.cc:600):
    vnMatches12, the count and the updated vbPrevMatched must equal the oracle's (k_init_resolve: in-order
    resolution with vMatchedDistance stealing)."""
    F1, F2, prev = ps.init_scene(seed, prev_noise=noise)
    ng, mg, pg = orbamd.ORBmatcher(ratio, check_ori).SearchForInitialization(F1, F2, prev, window)
    no, mo, po = oracle_py.search_for_initialization(F1, F2, prev, window, ratio, check_ori)
    bad = np.nonzero(mg != mo)[0]
    assert bad.size == 0, "vnMatches12 differs at %s: gpu %s oracle %s" % (bad[:8], mg[bad[:8]], mo[bad[:8]])
    assert ng == no and ng > 50
    assert pg.tobytes() == po.tobytes()


def test_search_for_initialization_stealing():
    """many F1 keypoints whose windows hold the same F2 features: a later, closer query takes an F2 feature
    from an earlier one (ORBmatcher.cc:463-467), repeatedly, inside one 64-query chunk and across chunks"""
    F1, F2, prev = ps.init_scene(5)
    rng = np.random.default_rng(5)
    lvl0 = np.nonzero(F1.octave == 0)[0]
    tgt = np.nonzero(F2.octave == 0)[0][:20]
    # every level-0 query looks at one of 20 F2 features with a descriptor 0..40 bits away from it
    pick = tgt[rng.integers(0, len(tgt), len(lvl0))]
    F1.desc = F1.desc.copy()  # (the frame cache of proj_scenes is shared)
    F1.desc[lvl0] = ps.flip_bits(rng, F2.desc[pick], 40)
    prev[lvl0, 0], prev[lvl0, 1] = F2.x[pick], F2.y[pick]
    ng, mg, pg = orbamd.ORBmatcher(0.9, True).SearchForInitialization(F1, F2, prev, 100)
    no, mo, po = oracle_py.search_for_initialization(F1, F2, prev, 100, 0.9, True)
    np.testing.assert_array_equal(mg, mo)
    assert ng == no and pg.tobytes() == po.tobytes()


@pytest.mark.parametrize("seed,th", [(2, 7.5), (5, 7.5), (8, 3.0)])
def test_search_by_sim3(seed, th):
    """ORBmatcher::SearchBySim3 (ORBmatcher.cc:1102-1326): both projections through (s12, R12, t12), the
    windowed first-strict-minimum search on the device, the mutual-consistency check."""
    sc = list(ps.sim3_pair_scene(seed))
    sc[-1] = th
    ng, mg = orbamd.ORBmatcher(0.75, True).SearchBySim3(*sc)
    no, mo = oracle_py.search_by_sim3(*sc)
    bad = np.nonzero(mg != mo)[0]
    assert bad.size == 0, "match12 differs at %s: gpu %s oracle %s" % (bad[:8], mg[bad[:8]], mo[bad[:8]])
    assert ng == no and ng > 50


def test_search_by_sim3_edge_cases():
    """no MapPoints on one side; every MapPoint already matched"""
    KF1, T1w, mp1, KF2, T2w, mp2, s12, R12, t12, th = ps.sim3_pair_scene(3)
    mt = orbamd.ORBmatcher(0.75, True)
    empty = orbamd.MapPoints(0, desc=np.zeros((0, 32), np.uint8), pos=np.zeros((0, 3), np.float32), min_dist=[],
                             max_dist=[])
    n, m = mt.SearchBySim3(KF1, T1w, mp1, KF2, T2w, empty, s12, R12, t12, th)
    assert n == 0 and (m == -1).all()
    mp1.skip = np.ones(mp1.n, np.uint8)
    n, m = mt.SearchBySim3(KF1, T1w, mp1, KF2, T2w, mp2, s12, R12, t12, th)
    assert n == 0 and (m == -1).all()
