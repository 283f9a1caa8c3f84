"""ORBmatcher -- Python mirror of ORB_SLAM2::ORBmatcher over the C ABI.

Reference surface: ORB_SLAM2/include/ORBmatcher.h:37-102. A :class:`KeyFrameView` stands
in for the KeyFrame/Frame accessors the matcher reads (mvKeysUn, mDescriptors, mvuRight,
GetMapPoint/isBad, mFeatVec, mvScaleFactors, mvLevelSigma2).
"""
import ctypes as C

import numpy as np

from ._lib import OrbmKfView, check, load

TH_HIGH = 100  # ORBmatcher.cc:37
TH_LOW = 50  # ORBmatcher.cc:38
HISTO_LENGTH = 30  # ORBmatcher.cc:39


class KeyFrameView:
    """What ORBmatcher reads from a KeyFrame / Frame.

    keypoints: structured array with fields x, y, angle, octave (mvKeysUn); descriptors: uint8
    [N,32]; feat_vec: dict node_id -> list of feature indices (DBoW2::FeatureVector; default
    one node holding every feature); has_mp / mp_bad: bool [N]; uright: float [N] or None.
    """

    def __init__(self, keypoints, descriptors, scale_factors, level_sigma2, feat_vec=None, uright=None,
                 has_mp=None, mp_bad=None):
        n = len(keypoints)
        self.n = n
        self.desc = np.ascontiguousarray(descriptors if descriptors is not None else np.zeros((0, 32), np.uint8),
                                         dtype=np.uint8).reshape(n, 32)
        self.x = np.ascontiguousarray(keypoints["x"], np.float32)
        self.y = np.ascontiguousarray(keypoints["y"], np.float32)
        self.angle = np.ascontiguousarray(keypoints["angle"], np.float32)
        self.octave = np.ascontiguousarray(keypoints["octave"], np.int32)
        self.uright = None if uright is None else np.ascontiguousarray(uright, np.float32)
        self.has_mp = None if has_mp is None else np.ascontiguousarray(has_mp, np.uint8)
        self.mp_bad = None if mp_bad is None else np.ascontiguousarray(mp_bad, np.uint8)
        if feat_vec is None:
            feat_vec = {0: list(range(n))} if n else {}
        ids = sorted(feat_vec)
        self.node_id = np.array(ids, np.uint32)
        offs = [0]
        feats = []
        for i in ids:
            f = sorted(int(v) for v in feat_vec[i])
            feats.extend(f)
            offs.append(len(feats))
        self.node_off = np.array(offs, np.int32)
        self.node_feat = np.array(feats if feats else [0], np.int32)
        self.scale_factors = np.ascontiguousarray(scale_factors, np.float32)
        self.level_sigma2 = np.ascontiguousarray(level_sigma2, np.float32)

    def cview(self):
        def p(a):
            return None if a is None else a.ctypes.data
        return OrbmKfView(self.n, p(self.desc), p(self.x), p(self.y), p(self.angle), p(self.octave), p(self.uright),
                          p(self.has_mp), p(self.mp_bad), len(self.node_id), p(self.node_id), p(self.node_off),
                          p(self.node_feat), len(self.scale_factors), p(self.scale_factors), p(self.level_sigma2))


def epipole(R2w, t2w, Cw, fx, fy, cx, cy):
    """(ex, ey) of KF1's centre in KF2 (ORBmatcher.cc:664-670) via orbm_epipole."""
    lib = load()
    R = np.ascontiguousarray(R2w, np.float32).reshape(9)
    t = np.ascontiguousarray(t2w, np.float32).reshape(3)
    c = np.ascontiguousarray(Cw, np.float32).reshape(3)
    ex = C.c_float()
    ey = C.c_float()
    lib.orbm_epipole(R.ctypes.data, t.ctypes.data, c.ctypes.data, fx, fy, cx, cy, C.byref(ex), C.byref(ey))
    return ex.value, ey.value


def compute_f12(R1w, t1w, R2w, t2w, K1, K2):
    """LocalMapping::ComputeF12 (LocalMapping.cc:536-553) in float64, rounded to float32.
    F12 is an input of the matcher; both the oracle and the device receive the same floats."""
    R1w, t1w, R2w, t2w, K1, K2 = [np.asarray(a, np.float64) for a in (R1w, t1w, R2w, t2w, K1, K2)]
    R12 = R1w @ R2w.T
    t12 = -R1w @ R2w.T @ t2w.reshape(3) + t1w.reshape(3)
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    return (np.linalg.inv(K1.T) @ tx @ R12 @ np.linalg.inv(K2)).astype(np.float32)


class KeyFrameCache:
    """orbm_kf_cache: keyframes' immutable per-feature arrays kept in HBM across matcher calls (the
    *Cached matcher methods take it with a 64-bit key per keyframe)."""

    def __init__(self, capacity_bytes=0, device=0):
        self._lib = load()
        h = C.c_void_p()
        check(self._lib.orbm_kf_cache_create(device, capacity_bytes, C.byref(h)), "orbm_kf_cache_create")
        self._h = h

    def erase(self, key):
        check(self._lib.orbm_kf_cache_erase(self._h, C.c_uint64(key)), "orbm_kf_cache_erase")

    def stats(self):
        e, b, hi, mi = C.c_int(), C.c_size_t(), C.c_longlong(), C.c_longlong()
        check(self._lib.orbm_kf_cache_stats(self._h, C.byref(e), C.byref(b), C.byref(hi), C.byref(mi)),
              "orbm_kf_cache_stats")
        return {"entries": e.value, "bytes": b.value, "hits": hi.value, "misses": mi.value}

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbm_kf_cache_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ORBmatcher:
    """ORB_SLAM2::ORBmatcher(nnratio=0.6, checkOri=true) -- device-backed."""
    TH_HIGH = TH_HIGH
    TH_LOW = TH_LOW
    HISTO_LENGTH = HISTO_LENGTH

    def __init__(self, nnratio=0.6, checkOri=True, device=0):
        self._lib = load()
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        h = C.c_void_p()
        check(self._lib.orbm_create(device, C.byref(h)), "orbm_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return int(load().orbm_descriptor_distance(a.ctypes.data, b.ctypes.data))

    def SearchForTriangulation(self, kf1, kf2, F12, ex, ey, bOnlyStereo=False):
        """Returns (nmatches, match12 int32 [kf1.n]) -- vMatchedPairs = [(i, match12[i]) | match12[i] >= 0]."""
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        out = np.empty(max(kf1.n, 1), np.int32)
        n = C.c_int()
        v1, v2 = kf1.cview(), kf2.cview()
        check(self._lib.orbm_search_for_triangulation(self._h, C.byref(v1), C.byref(v2), F.ctypes.data, ex, ey,
                                                      int(bOnlyStereo), int(self.mbCheckOrientation),
                                                      out.ctypes.data, C.byref(n)), "orbm_search_for_triangulation")
        return n.value, out[:kf1.n]

    def SearchByBoW(self, kf, other, other_is_keyframe=False):
        """SearchByBoW(KeyFrame*, Frame&) (default) or SearchByBoW(KeyFrame*, KeyFrame*).
        Returns (nmatches, matches): for (KF,F) matches[iF] = KF feature index (or -1);
        for (KF,KF) matches[i1] = idx2 (or -1)."""
        v1, v2 = kf.cview(), other.cview()
        n = C.c_int()
        if other_is_keyframe:
            out = np.empty(max(kf.n, 1), np.int32)
            check(self._lib.orbm_search_by_bow_kf_kf(self._h, C.byref(v1), C.byref(v2), self.mfNNratio,
                                                     int(self.mbCheckOrientation), out.ctypes.data, C.byref(n)),
                  "orbm_search_by_bow_kf_kf")
            return n.value, out[:kf.n]
        out = np.empty(max(other.n, 1), np.int32)
        check(self._lib.orbm_search_by_bow_kf_f(self._h, C.byref(v1), C.byref(v2), self.mfNNratio,
                                                int(self.mbCheckOrientation), out.ctypes.data, C.byref(n)),
              "orbm_search_by_bow_kf_f")
        return n.value, out[:other.n]

    # ---- the same matchers with keyframes held in a KeyFrameCache (identical results)
    def SearchForTriangulationCached(self, cache, key1, kf1, key2, kf2, F12, ex, ey, bOnlyStereo=False):
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        out = np.empty(max(kf1.n, 1), np.int32)
        n = C.c_int()
        v1, v2 = kf1.cview(), kf2.cview()
        check(self._lib.orbm_search_for_triangulation_cached(self._h, cache._h, key1, C.byref(v1), key2, C.byref(v2),
                                                             F.ctypes.data, ex, ey, int(bOnlyStereo),
                                                             int(self.mbCheckOrientation), out.ctypes.data,
                                                             C.byref(n)), "orbm_search_for_triangulation_cached")
        return n.value, out[:kf1.n]

    def SearchByBoWCached(self, cache, key, kf, other, other_is_keyframe=False, key2=None):
        v1, v2 = kf.cview(), other.cview()
        n = C.c_int()
        if other_is_keyframe:
            out = np.empty(max(kf.n, 1), np.int32)
            check(self._lib.orbm_search_by_bow_kf_kf_cached(self._h, cache._h, key, C.byref(v1), key2, C.byref(v2),
                                                            self.mfNNratio, int(self.mbCheckOrientation),
                                                            out.ctypes.data, C.byref(n)),
                  "orbm_search_by_bow_kf_kf_cached")
            return n.value, out[:kf.n]
        out = np.empty(max(other.n, 1), np.int32)
        check(self._lib.orbm_search_by_bow_kf_f_cached(self._h, cache._h, key, C.byref(v1), C.byref(v2),
                                                       self.mfNNratio, int(self.mbCheckOrientation), out.ctypes.data,
                                                       C.byref(n)), "orbm_search_by_bow_kf_f_cached")
        return n.value, out[:other.n]

    def FuseCached(self, cache, key, KF, Tcw, Ow, mps, th, inv_level_sigma2):
        m = mps.cstruct()
        fv = KF.cstruct()
        T = np.ascontiguousarray(Tcw, np.float32).reshape(16)
        O = np.ascontiguousarray(Ow, np.float32).reshape(3)
        inv = np.ascontiguousarray(inv_level_sigma2, np.float32)
        out = np.empty(max(mps.n, 1), np.int32)
        n = C.c_int()
        check(self._lib.orbm_fuse_cached(self._h, cache._h, key, C.byref(fv), T.ctypes.data, O.ctypes.data,
                                         C.byref(m), C.c_float(th), inv.ctypes.data, out.ctypes.data, C.byref(n)),
              "orbm_fuse_cached")
        return n.value, out[:mps.n]

    # ---- SearchByProjection x4 (ORBmatcher.cc:45-129, 1328-1470, 1472-1599, 290-403). Each returns
    # (nmatches, match[F.n]): index into the MapPoints of the assignment made to that feature
    # (last wins), -1 untouched, -2 reset to NULL by the rotation-consistency filter.
    def _proj(self, fn, F, *args):
        out = np.empty(max(F.n, 1), np.int32)
        n = C.c_int()
        fv = F.cstruct()
        check(getattr(self._lib, fn)(self._h, C.byref(fv), *args, out.ctypes.data, C.byref(n)), fn)
        return n.value, out[:F.n]

    def SearchByProjectionLocal(self, F, mps, th=3.0):
        """SearchByProjection(Frame&, const vector<MapPoint*>&, th): F.occupied = mvpMapPoints[i] with
        Observations() > 0; mps carry the isInFrustum tracking fields."""
        m = mps.cstruct()
        return self._proj("orbm_search_by_projection_local", F, C.byref(m), C.c_float(th), C.c_float(self.mfNNratio))

    def SearchByProjectionLastFrame(self, F, Tcw, last_mps, Tcw_last, th, bMono):
        m = last_mps.cstruct()
        T1 = np.ascontiguousarray(Tcw, np.float32).reshape(16)
        T2 = np.ascontiguousarray(Tcw_last, np.float32).reshape(16)
        return self._proj("orbm_search_by_projection_last_frame", F, T1.ctypes.data, C.byref(m), T2.ctypes.data,
                          C.c_float(th), int(bMono), int(self.mbCheckOrientation))

    def SearchByProjectionKeyFrame(self, F, Tcw, kf_mps, th, ORBdist):
        m = kf_mps.cstruct()
        T1 = np.ascontiguousarray(Tcw, np.float32).reshape(16)
        return self._proj("orbm_search_by_projection_keyframe", F, T1.ctypes.data, C.byref(m), C.c_float(th),
                          int(ORBdist), int(self.mbCheckOrientation))

    def SearchByProjectionSim3(self, KF, Scw, mps, th):
        m = mps.cstruct()
        S = np.ascontiguousarray(Scw, np.float32).reshape(16)
        return self._proj("orbm_search_by_projection_sim3", KF, S.ctypes.data, C.byref(m), int(th))

    # ---- Fuse x2 (ORBmatcher.cc:825-975, 977-1100): (nFused, best_idx[mps.n]) = the keypoint of KF each
    # MapPoint fuses with (-1: none); the map updates that follow stay with the caller, in order.
    def Fuse(self, KF, Tcw, Ow, mps, th, inv_level_sigma2):
        m = mps.cstruct()
        fv = KF.cstruct()
        T = np.ascontiguousarray(Tcw, np.float32).reshape(16)
        O = np.ascontiguousarray(Ow, np.float32).reshape(3)
        inv = np.ascontiguousarray(inv_level_sigma2, np.float32)
        out = np.empty(max(mps.n, 1), np.int32)
        n = C.c_int()
        check(self._lib.orbm_fuse(self._h, C.byref(fv), T.ctypes.data, O.ctypes.data, C.byref(m), C.c_float(th),
                                  inv.ctypes.data, out.ctypes.data, C.byref(n)), "orbm_fuse")
        return n.value, out[:mps.n]

    def FuseSim3(self, KF, Scw, mps, th):
        m = mps.cstruct()
        fv = KF.cstruct()
        S = np.ascontiguousarray(Scw, np.float32).reshape(16)
        out = np.empty(max(mps.n, 1), np.int32)
        n = C.c_int()
        check(self._lib.orbm_fuse_sim3(self._h, C.byref(fv), S.ctypes.data, C.byref(m), C.c_float(th),
                                       out.ctypes.data, C.byref(n)), "orbm_fuse_sim3")
        return n.value, out[:mps.n]

    # ---- SearchForInitialization (ORBmatcher.cc:405-520): (nmatches, vnMatches12[F1.n], updated vbPrevMatched)
    def SearchForInitialization(self, F1, F2, prev_xy, windowSize=10):
        f1, f2 = F1.cstruct(), F2.cstruct()
        prev = np.ascontiguousarray(prev_xy, np.float32).reshape(F1.n, 2).copy()
        out = np.empty(max(F1.n, 1), np.int32)
        n = C.c_int()
        check(self._lib.orbm_search_for_initialization(self._h, C.byref(f1), C.byref(f2), prev.ctypes.data,
                                                       int(windowSize), C.c_float(self.mfNNratio),
                                                       int(self.mbCheckOrientation), out.ctypes.data, C.byref(n)),
              "orbm_search_for_initialization")
        return n.value, out[:F1.n], prev

    # ---- SearchBySim3 (ORBmatcher.cc:1102-1326): (nFound, match12[mp1.n]) = agreeing idx2 or -1
    def SearchBySim3(self, KF1, T1w, mp1, KF2, T2w, mp2, s12, R12, t12, th):
        k1, k2 = KF1.cstruct(), KF2.cstruct()
        m1, m2 = mp1.cstruct(), mp2.cstruct()
        T1 = np.ascontiguousarray(T1w, np.float32).reshape(16)
        T2 = np.ascontiguousarray(T2w, np.float32).reshape(16)
        R = np.ascontiguousarray(R12, np.float32).reshape(9)
        t = np.ascontiguousarray(t12, np.float32).reshape(3)
        out = np.empty(max(mp1.n, 1), np.int32)
        n = C.c_int()
        check(self._lib.orbm_search_by_sim3(self._h, C.byref(k1), T1.ctypes.data, C.byref(m1), C.byref(k2),
                                            T2.ctypes.data, C.byref(m2), C.c_float(s12), R.ctypes.data, t.ctypes.data,
                                            C.c_float(th), out.ctypes.data, C.byref(n)), "orbm_search_by_sim3")
        return n.value, out[:mp1.n]


def compute_distinctive_descriptors(offsets, desc, device=0, matcher=None):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307) for a batch of MapPoints:
    MapPoint p's observed descriptors are desc[offsets[p]:offsets[p+1]]. Returns (best_idx int32 [P]
    (-1 = no descriptors), chosen descriptors uint8 [P, 32])."""
    lib = load()
    m = matcher or ORBmatcher(device=device)
    off = np.ascontiguousarray(offsets, np.int32)
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    P = len(off) - 1
    best = np.empty(max(P, 1), np.int32)
    out = np.zeros((max(P, 1), 32), np.uint8)
    check(lib.orbm_compute_distinctive_descriptors(m._h, P, off.ctypes.data, d.ctypes.data, best.ctypes.data,
                                                   out.ctypes.data), "orbm_compute_distinctive_descriptors")
    return best[:P], out[:P]
