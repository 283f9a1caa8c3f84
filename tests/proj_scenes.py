"""Deterministic SearchByProjection scenarios (ORBmatcher.cc:45-129, 290-403, 1328-1470,
1472-1599) for the oracle/GPU parity tests.

A frame's keypoints and descriptors come from the CPU oracle extractor on a synthetic image;
MapPoints are back-projected from a subset of those keypoints at random depths (so projections
land near real features), with perturbed descriptors, duplicates (several MapPoints competing
for one feature: exercises the in-order claim resolution), outliers and every per-variant flag
drawn at random."""
import numpy as np

import oracle_py
import orbamd

FX, FY, CX, CY = 715.092024, 719.025258, 334.298489, 256.326097  # ORB_SLAM2/my.yaml:8-11
W, H = 640, 480

_cache = {}


def frame_features(agent=0, t=0, nfeatures=1000):
    key = (agent, t, nfeatures)
    if key not in _cache:
        img = orbamd.synth_frames(agent, t, 1, W, H)[0]
        orc = oracle_py.OracleExtractor(nfeatures, 1.2, 8, 20, 7)
        k, d = orc(img)
        _cache[key] = (k, d, orc.tables()["scale"])
    return _cache[key]


def rot(rng, deg):
    a = np.deg2rad(rng.uniform(-deg, deg, 3))
    cx, sx, cy, sy, cz, sz = np.cos(a[0]), np.sin(a[0]), np.cos(a[1]), np.sin(a[1]), np.cos(a[2]), np.sin(a[2])
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def pose(R, t, s=1.0):
    T = np.eye(4)
    T[:3, :3] = s * R
    T[:3, 3] = s * np.asarray(t)
    return T.astype(np.float32)


def flip_bits(rng, d, nmax):
    d = d.copy()
    for i in range(len(d)):
        nb = int(rng.integers(0, nmax + 1))
        if nb:
            pos = rng.choice(256, nb, replace=False)
            for p in pos:
                d[i, p >> 3] ^= np.uint8(1 << (p & 7))
    return d


def make_frame(rng, agent, t, stereo, occupied_frac=0.05, nfeatures=1000):
    k, d, scale = frame_features(agent, t, nfeatures)
    n = len(k)
    bf = 47.9 if stereo else 0.0
    ur = None
    if stereo:
        ur = np.full(n, -1, np.float32)
        has = rng.random(n) < 0.6
        ur[has] = (k["x"][has] - rng.uniform(1, 40, has.sum())).astype(np.float32)
    occ = (rng.random(n) < occupied_frac).astype(np.uint8)
    F = orbamd.FrameView(k, d, scale, W, H, FX, FY, CX, CY, bf=bf, uright=ur, occupied=occ)
    return F, k, d, scale


def pick_sources(rng, n, m, dup_frac=0.15):
    """m MapPoint source features out of n, with duplicates (competing MapPoints)."""
    base = rng.choice(n, size=min(n, m), replace=False)
    ndup = int(len(base) * dup_frac)
    dups = rng.choice(base, size=ndup, replace=True)
    src = np.concatenate([base, dups])
    rng.shuffle(src)
    return src


def local_scene(seed, stereo=True, th=3.0):
    """SearchByProjection(Frame&, vector<MapPoint*>, th): isInFrustum-style tracking fields."""
    rng = np.random.default_rng(seed)
    F, k, d, scale = make_frame(rng, seed % 5, 3 + seed, stereo)
    src = pick_sources(rng, F.n, int(F.n * 0.8))
    m = len(src)
    px = (k["x"][src] + rng.normal(0, 2.0, m)).astype(np.float32)
    py = (k["y"][src] + rng.normal(0, 2.0, m)).astype(np.float32)
    lvl = np.clip(k["octave"][src] + rng.integers(-1, 2, m), 0, 7).astype(np.int32)
    desc = flip_bits(rng, d[src], 40)
    rnd = rng.random(m) < 0.1
    desc[rnd] = rng.integers(0, 256, (rnd.sum(), 32), dtype=np.uint8)
    mps = orbamd.MapPoints(
        m, desc=desc, bad=(rng.random(m) < 0.05), has_obs=(rng.random(m) < 0.85),
        track_in_view=(rng.random(m) < 0.9), track_proj_x=px, track_proj_y=py,
        track_proj_xr=(px - rng.uniform(0, 40, m)).astype(np.float32), track_level=lvl,
        track_view_cos=rng.choice([0.9995, 0.999, 0.998, 0.99], m).astype(np.float32))
    return F, mps


def backproject(rng, k, src, Tcw):
    z = rng.uniform(1.0, 12.0, len(src))
    xc = np.stack([(k["x"][src] - CX) / FX * z, (k["y"][src] - CY) / FY * z, z], 1)
    R, t = Tcw[:3, :3].astype(np.float64), Tcw[:3, 3].astype(np.float64)
    return ((xc - t) @ R).astype(np.float32)  # Xw = R^T (Xc - t)


def last_frame_scene(seed, bmono=False, stereo=True, forward=0):
    """SearchByProjection(CurrentFrame, LastFrame, th, bMono). forward: +1 / -1 moves the last
    frame ahead / behind along the optical axis by more than mb (bForward / bBackward)."""
    rng = np.random.default_rng(seed)
    F, k, d, scale = make_frame(rng, seed % 5, 7 + seed, stereo)
    Tcw = pose(rot(rng, 2.0), rng.normal(0, 0.05, 3))
    src = pick_sources(rng, F.n, int(F.n * 0.9))
    m = len(src)
    Xw = backproject(rng, k, src, Tcw) + rng.normal(0, 0.003, (m, 3)).astype(np.float32)
    dz = 0.5 * forward if forward else rng.normal(0, 0.01)
    Tl = Tcw.copy()
    Tl[2, 3] += np.float32(-dz)  # tlc.z = dz (camera centre of Current in Last)
    mps = orbamd.MapPoints(
        m, desc=flip_bits(rng, d[src], 35), pos=Xw, has_obs=(rng.random(m) < 0.85),
        skip=(rng.random(m) < 0.1), octave=np.clip(k["octave"][src] + rng.integers(-1, 2, m), 0, 7),
        angle=((k["angle"][src] + rng.normal(0, 4.0, m)) % 360).astype(np.float32))
    return F, Tcw, mps, Tl


def dist_bounds(rng, Xw, Tcw, octs):
    Ow = -(Tcw[:3, :3].astype(np.float64).T @ Tcw[:3, 3].astype(np.float64))
    dist = np.linalg.norm(Xw - Ow, axis=1)
    maxd = dist * 1.2 ** (octs + rng.uniform(-0.9, 0.1, len(octs)))
    maxd[rng.random(len(octs)) < 0.05] *= 0.5  # out of the invariance region
    mind = maxd / 1.2 ** 7
    return mind.astype(np.float32), maxd.astype(np.float32)


def keyframe_scene(seed, th=10.0, orb_dist=100):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (relocalisation)."""
    rng = np.random.default_rng(seed)
    F, k, d, scale = make_frame(rng, seed % 5, 11 + seed, False, occupied_frac=0.1)
    Tcw = pose(rot(rng, 3.0), rng.normal(0, 0.05, 3))
    src = pick_sources(rng, F.n, int(F.n * 0.9))
    m = len(src)
    Xw = backproject(rng, k, src, Tcw) + rng.normal(0, 0.003, (m, 3)).astype(np.float32)
    mind, maxd = dist_bounds(rng, Xw, Tcw, k["octave"][src])
    mps = orbamd.MapPoints(
        m, desc=flip_bits(rng, d[src], 40), pos=Xw, min_dist=mind, max_dist=maxd, bad=(rng.random(m) < 0.05),
        skip=(rng.random(m) < 0.1), angle=((k["angle"][src] + rng.normal(0, 4.0, m)) % 360).astype(np.float32))
    return F, Tcw, mps


def sim3_scene(seed):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (loop closing)."""
    rng = np.random.default_rng(seed)
    F, k, d, scale = make_frame(rng, seed % 5, 13 + seed, False, occupied_frac=0.1)
    s = np.float32(rng.uniform(0.7, 1.4))
    R = rot(rng, 3.0)
    t = rng.normal(0, 0.05, 3)
    Scw = pose(R, t, s)
    Tcw = pose(R, t)
    src = pick_sources(rng, F.n, int(F.n * 0.9))
    m = len(src)
    Xw = backproject(rng, k, src, Tcw) + rng.normal(0, 0.003, (m, 3)).astype(np.float32)
    Ow = -(R.T @ t)
    nrm = (Xw - Ow)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    flip = rng.random(m) < 0.05
    nrm[flip] *= -1
    mind, maxd = dist_bounds(rng, Xw, Tcw, k["octave"][src])
    mps = orbamd.MapPoints(
        m, desc=flip_bits(rng, d[src], 25), pos=Xw, normal=nrm.astype(np.float32), min_dist=mind, max_dist=maxd,
        bad=(rng.random(m) < 0.05), skip=(rng.random(m) < 0.1))
    return F, Scw, mps


def inv_level_sigma2(scale):
    """mvInvLevelSigma2 = 1.0f / (mvScaleFactor^2) in float (ORBextractor.cc:416-424, Frame.cc)."""
    s = np.asarray(scale, np.float32)
    return (np.float32(1.0) / (s * s)).astype(np.float32)


def fuse_scene(seed, stereo=True):
    """Fuse(pKF, vpMapPoints, th) (LocalMapping::SearchInNeighbors): MapPoints of a neighbour keyframe
    projected into pKF, 3-D noise so that part of them fail the reprojection-error (chi2) test."""
    rng = np.random.default_rng(seed)
    F, k, d, scale = make_frame(rng, seed % 5, 17 + seed, stereo, occupied_frac=0.0)
    R, t = rot(rng, 3.0), rng.normal(0, 0.05, 3)
    Tcw = pose(R, t)
    Ow = (-(R.T @ t)).astype(np.float32)
    src = pick_sources(rng, F.n, int(F.n * 0.9))
    m = len(src)
    noise = np.where(rng.random(m)[:, None] < 0.3, 0.02, 0.002)
    Xw = (backproject(rng, k, src, Tcw) + rng.normal(0, 1, (m, 3)) * noise).astype(np.float32)
    nrm = Xw - Ow
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm[rng.random(m) < 0.05] *= -1
    mind, maxd = dist_bounds(rng, Xw, Tcw, k["octave"][src])
    mps = orbamd.MapPoints(
        m, desc=flip_bits(rng, d[src], 30), pos=Xw, normal=nrm.astype(np.float32), min_dist=mind, max_dist=maxd,
        bad=(rng.random(m) < 0.05), skip=(rng.random(m) < 0.1))
    return F, Tcw, Ow, mps, inv_level_sigma2(scale)


def fuse_sim3_scene(seed):
    """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (LoopClosing::SearchAndFuse)."""
    F, Scw, mps = sim3_scene(seed)
    return F, Scw, mps


def init_scene(seed, nfeatures=2000, dt=2, prev_noise=0.0):
    """SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (Tracking::
    MonocularInitialization, Tracking.cc:600): two frames of one synthetic stream, dt steps apart, from
    the 2000-feature initialisation extractor; vbPrevMatched starts at F1's keypoints (Tracking.cc:583-585),
    optionally perturbed."""
    rng = np.random.default_rng(seed)
    agent, t = seed % 5, 20 + seed
    k1, d1, scale = frame_features(agent, t, nfeatures)
    k2, d2, _ = frame_features(agent, t + dt, nfeatures)
    F1 = orbamd.FrameView(k1, d1, scale, W, H, FX, FY, CX, CY)
    F2 = orbamd.FrameView(k2, d2, scale, W, H, FX, FY, CX, CY)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    if prev_noise:
        prev = (prev + rng.normal(0, prev_noise, prev.shape)).astype(np.float32)
    return F1, F2, prev


def sim3_pair_scene(seed, th=7.5):
    """SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (LoopClosing::ComputeSim3): two keyframes
    of one image whose MapPoints are one scene seen through the similarity (s12, R12, t12), camera 1 from
    camera 2: Xc1 = s12 R12 Xc2 + t12. Each keyframe has its own pose, MapPoint subset, descriptor noise,
    bad flags and already-matched entries (vbAlreadyMatched1/2)."""
    rng = np.random.default_rng(seed)
    k, d, scale = frame_features(seed % 5, 30 + seed, 1000)
    n = len(k)
    KF1 = orbamd.FrameView(k, d, scale, W, H, FX, FY, CX, CY)
    KF2 = orbamd.FrameView(k, d, scale, W, H, FX, FY, CX, CY)
    T1w = pose(rot(rng, 3.0), rng.normal(0, 0.05, 3))
    T2w = pose(rot(rng, 3.0), rng.normal(0, 0.05, 3))
    s12 = np.float32(rng.uniform(0.8, 1.25))
    R12 = rot(rng, 0.3).astype(np.float32)
    t12 = rng.normal(0, 0.01, 3).astype(np.float32)
    z = rng.uniform(1.0, 12.0, n)
    Xc1 = np.stack([(k["x"] - CX) / FX * z, (k["y"] - CY) / FY * z, z], 1)
    Xc2 = ((Xc1 - t12) @ R12.astype(np.float64)) / float(s12)  # R12^T (Xc1 - t12) / s12

    def to_world(Xc, T):
        R, t = T[:3, :3].astype(np.float64), T[:3, 3].astype(np.float64)
        return ((Xc - t) @ R).astype(np.float32)

    def mappoints(Xc_self, Xc_other, T, frac):
        has = rng.random(n) < frac
        Xw = to_world(Xc_self + rng.normal(0, 0.002, Xc_self.shape), T)
        dother = np.linalg.norm(Xc_other, axis=1)
        maxd = dother * 1.2 ** (k["octave"] + rng.uniform(-0.9, 0.1, n))
        maxd[rng.random(n) < 0.05] *= 0.5
        return has, orbamd.MapPoints(n, desc=flip_bits(rng, d, 30), pos=Xw, min_dist=(maxd / 1.2 ** 7).astype(np.float32),
                                     max_dist=maxd.astype(np.float32), bad=(rng.random(n) < 0.05))

    has1, mp1 = mappoints(Xc1, Xc2, T1w, 0.7)
    has2, mp2 = mappoints(Xc2, Xc1, T2w, 0.7)
    # vpMatches12 already set for ~8 % of KF1's MapPoints; vbAlreadyMatched2 at their index in pKF2 (:1129-1142)
    pre = has1 & (rng.random(n) < 0.08)
    already2 = np.zeros(n, bool)
    already2[np.nonzero(pre)[0]] = True
    mp1.skip = (~has1 | pre).astype(np.uint8)
    mp2.skip = (~has2 | already2).astype(np.uint8)
    return KF1, T1w, mp1, KF2, T2w, mp2, s12, R12, t12, th
