"""ctypes binding of the CPU oracle (oracle/build/liborb_oracle.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module. Parity status: "parity unpinned" at the OpenCV boundary (see
orb_oracle.h and DESIGN.md).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborb_oracle.so")

KP_FIELDS = [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"), ("octave", "<i4")]
kp_dtype = np.dtype(KP_FIELDS)


class _Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class _View(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("x", C.c_void_p), ("y", C.c_void_p),
                ("angle", C.c_void_p), ("octave", C.c_void_p), ("uright", C.c_void_p),
                ("has_mp", C.c_void_p), ("mp_bad", C.c_void_p), ("n_nodes", C.c_int32),
                ("node_id", C.c_void_p), ("node_off", C.c_void_p), ("node_feat", C.c_void_p),
                ("nlevels", C.c_int32), ("scale_factors", C.c_void_p), ("level_sigma2", C.c_void_p)]


_P, _I, _F, _SZ = C.c_void_p, C.c_int, C.c_float, C.c_size_t
_SIG = {
    "oc_create": (_P, [C.POINTER(_Params)]),
    "oc_destroy": (None, [_P]),
    "oc_extract": (_I, [_P, _P, _I, _I, _SZ, _P, _P, _I, C.POINTER(_I)]),
    "oc_level_size": (_I, [_P, _I, C.POINTER(_I), C.POINTER(_I)]),
    "oc_pyramid": (C.POINTER(C.c_uint8), [_P, _I]),
    "oc_blurred": (C.POINTER(C.c_uint8), [_P, _I]),
    "oc_level_candidates": (_I, [_P, _I, _P, _I]),
    "oc_level_octree": (_I, [_P, _I, _P, _I]),
    "oc_get_tables": (None, [_P, _P, _P, _P, _P, _P, _P]),
    "oc_stage_times": (None, [_P, _P, _P]),
    "oc_fast_atan2": (_F, [_F, _F]),
    "oc_gauss_kernel_q8": (_I, [_P]),
    "oc_resize_linear": (None, [_P, _I, _I, _SZ, _P, _I, _I, _SZ]),
    "oc_gauss7": (None, [_P, _I, _I, _SZ, _P, _SZ]),
    "oc_fast": (_I, [_P, _I, _I, _SZ, _I, _P, _I]),
    "oc_set_fast_simd": (None, [_I]),
    "oc_descriptor_distance": (_I, [_P, _P]),
    "oc_sincosf_batch": (None, [_P, _P, _P, _I]),
    "oc_search_for_triangulation": (_I, [C.POINTER(_View), C.POINTER(_View), _P, _F, _F, _I, _I, _P]),
    "oc_search_by_bow_kf_f": (_I, [C.POINTER(_View), C.POINTER(_View), _F, _I, _P]),
    "oc_search_by_bow_kf_kf": (_I, [C.POINTER(_View), C.POINTER(_View), _F, _I, _P]),
    "oc_compute_stereo_matches": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _F, _F, _P, _P]),
    "oc_search_by_projection_local": (_I, [_P, _P, _F, _F, _P]),
    "oc_search_by_projection_last_frame": (_I, [_P, _P, _P, _P, _F, _I, _I, _P]),
    "oc_search_by_projection_keyframe": (_I, [_P, _P, _P, _F, _I, _I, _P]),
    "oc_search_by_projection_sim3": (_I, [_P, _P, _P, _I, _P]),
    "oc_fuse": (_I, [_P, _P, _P, _P, _F, _P, _P]),
    "oc_fuse_sim3": (_I, [_P, _P, _P, _F, _P]),
    "oc_search_for_initialization": (_I, [_P, _P, _P, _I, _F, _I, _P]),
    "oc_search_by_sim3": (_I, [_P, _P, _P, _P, _P, _P, _F, _P, _P, _F, _P]),
    "oc_compute_distinctive_descriptors": (None, [_I, _P, _P, _P]),
    "oc_vocab_create": (_P, [_I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "oc_vocab_destroy": (None, [_P]),
    "oc_vocab_transform": (_I, [_P, _P, _I, _I, _P, _P, C.POINTER(_I), _P, _P, _P, C.POINTER(_I)]),
    "oc_vocab_descend": (None, [_P, _P, _I, _I, _P, _P, _P]),
}

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        for k, (r, a) in _SIG.items():
            f = getattr(lib, k)
            f.restype = r
            f.argtypes = a
        _lib = lib
    return _lib


class OracleExtractor:
    """CPU restatement of ORBextractor (ORBextractor.cc:410-1132)."""

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7):
        self.lib = load()
        p = _Params(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        self.h = self.lib.oc_create(C.byref(p))
        if not self.h:
            raise ValueError("bad ORBextractor parameters")
        self.nlevels = nlevels

    def __del__(self):
        try:
            if self.h:
                self.lib.oc_destroy(self.h)
        except Exception:
            pass

    def __call__(self, img, cap=None):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        cap = cap or 64 * 1024
        kps = np.empty(cap, kp_dtype)
        desc = np.empty((cap, 32), np.uint8)
        n = C.c_int()
        rc = self.lib.oc_extract(self.h, img.ctypes.data, w, h, img.strides[0], kps.ctypes.data, desc.ctypes.data,
                                 cap, C.byref(n))
        if rc != 0:
            raise RuntimeError("oc_extract rc=%d" % rc)
        n = n.value
        return kps[:n].copy(), desc[:n].copy()

    def level_size(self, l):
        w, h = C.c_int(), C.c_int()
        self.lib.oc_level_size(self.h, l, C.byref(w), C.byref(h))
        return w.value, h.value

    def pyramid(self, l):
        w, h = self.level_size(l)
        p = self.lib.oc_pyramid(self.h, l)
        return np.ctypeslib.as_array(p, shape=(h * w,)).reshape(h, w).copy()

    def blurred(self, l):
        w, h = self.level_size(l)
        p = self.lib.oc_blurred(self.h, l)
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(h * w,)).reshape(h, w).copy()

    def _xyr(self, fn, l):
        n = fn(self.h, l, None, 0)
        out = np.empty((max(n, 1), 3), np.float32)
        fn(self.h, l, out.ctypes.data, n)
        return out[:n]

    def candidates(self, l):
        return self._xyr(self.lib.oc_level_candidates, l)

    def octree(self, l):
        return self._xyr(self.lib.oc_level_octree, l)

    STAGES = ("pyramid", "fast", "octree", "orientation", "blur", "descriptor")

    def stage_times(self):
        """accumulated seconds per stage over all calls, and the number of frames"""
        sec = (C.c_double * 6)()
        nf = C.c_int()
        self.lib.oc_stage_times(self.h, sec, C.byref(nf))
        return dict(zip(self.STAGES, list(sec))), nf.value

    def tables(self):
        L = self.nlevels
        a = [np.empty(L, np.float32) for _ in range(4)]
        nf = np.empty(L, np.int32)
        um = np.empty(16, np.int32)
        self.lib.oc_get_tables(self.h, *[x.ctypes.data for x in a], nf.ctypes.data, um.ctypes.data)
        return {"scale": a[0], "inv_scale": a[1], "sigma2": a[2], "inv_sigma2": a[3], "nfeat": nf, "umax": um}


def fast(img, threshold, cap=100000):
    lib = load()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.empty((cap, 3), np.float32)
    n = lib.oc_fast(img.ctypes.data, w, h, img.strides[0], threshold, out.ctypes.data, cap)
    return out[:n].copy()


def resize_linear(src, dw, dh):
    lib = load()
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.empty((dh, dw), np.uint8)
    lib.oc_resize_linear(src.ctypes.data, src.shape[1], src.shape[0], src.strides[0], dst.ctypes.data, dw, dh, dw)
    return dst


def gauss7(src):
    lib = load()
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.empty_like(src)
    lib.oc_gauss7(src.ctypes.data, src.shape[1], src.shape[0], src.strides[0], dst.ctypes.data, dst.strides[0])
    return dst


def gauss_kernel_q8():
    k = np.empty(7, np.int32)
    s = load().oc_gauss_kernel_q8(k.ctypes.data)
    return k, s


def set_fast_simd(on):
    """1: cv::FAST's vector form (AVX2 build), 0: scalar per pixel (same output)"""
    load().oc_set_fast_simd(1 if on else 0)


def fast_atan2(y, x):
    return load().oc_fast_atan2(y, x)


def sincosf(x):
    x = np.ascontiguousarray(x, np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    load().oc_sincosf_batch(x.ctypes.data, s.ctypes.data, c.ctypes.data, x.size)
    return s, c


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return load().oc_descriptor_distance(a.ctypes.data, b.ctypes.data)


def _cview(v):
    """v: an object with the KeyFrameView attributes (orbamd.matcher.KeyFrameView)."""
    def p(a):
        return None if a is None else a.ctypes.data
    return _View(v.n, p(v.desc), p(v.x), p(v.y), p(v.angle), p(v.octave), p(v.uright), p(v.has_mp), p(v.mp_bad),
                 len(v.node_id), p(v.node_id), p(v.node_off), p(v.node_feat), len(v.scale_factors),
                 p(v.scale_factors), p(v.level_sigma2))


def search_for_triangulation(kf1, kf2, F12, ex, ey, only_stereo=False, check_ori=False):
    lib = load()
    F = np.ascontiguousarray(F12, np.float32).reshape(9)
    out = np.empty(max(kf1.n, 1), np.int32)
    a, b = _cview(kf1), _cview(kf2)
    n = lib.oc_search_for_triangulation(C.byref(a), C.byref(b), F.ctypes.data, ex, ey, int(only_stereo),
                                        int(check_ori), out.ctypes.data)
    return n, out[:kf1.n]


def search_by_bow(kf, other, nnratio, check_ori, other_is_keyframe=False):
    lib = load()
    a, b = _cview(kf), _cview(other)
    if other_is_keyframe:
        out = np.empty(max(kf.n, 1), np.int32)
        n = lib.oc_search_by_bow_kf_kf(C.byref(a), C.byref(b), nnratio, int(check_ori), out.ctypes.data)
        return n, out[:kf.n]
    out = np.empty(max(other.n, 1), np.int32)
    n = lib.oc_search_by_bow_kf_f(C.byref(a), C.byref(b), nnratio, int(check_ori), out.ctypes.data)
    return n, out[:other.n]


def compute_stereo_matches(left, right, kpsL, descL, kpsR, descR, mbf, mb):
    """Frame::ComputeStereoMatches (Frame.cc:470-641) on the pyramids of the last call of the two
    OracleExtractor instances. Returns (mvuRight, mvDepth, number kept); raises where the reference throws."""
    lib = load()
    kpsL = np.ascontiguousarray(kpsL)
    kpsR = np.ascontiguousarray(kpsR)
    dL = np.ascontiguousarray(descL, np.uint8)
    dR = np.ascontiguousarray(descR, np.uint8)
    n = len(kpsL)
    ur = np.empty(max(n, 1), np.float32)
    dp = np.empty(max(n, 1), np.float32)
    rc = lib.oc_compute_stereo_matches(left.h, right.h, kpsL.ctypes.data, dL.ctypes.data, n, kpsR.ctypes.data,
                                       dR.ctypes.data, len(kpsR), float(mbf), float(mb), ur.ctypes.data,
                                       dp.ctypes.data)
    if rc < 0:
        raise RuntimeError("oc_compute_stereo_matches rc=%d" % rc)
    return ur[:n], dp[:n], rc


# ---- SearchByProjection x4 (ORBmatcher.cc:45-129, 1328-1470, 1472-1599, 290-403). F / mps: objects
# with the orbamd.projection FrameView / MapPoints attributes (their cstruct() builds the C structs).
def _proj(fn, F, *args):
    out = np.empty(max(F.n, 1), np.int32)
    fv = F.cstruct()
    n = getattr(load(), fn)(C.byref(fv), *args, out.ctypes.data)
    return n, out[:F.n]


def search_by_projection_local(F, mps, th, nnratio):
    m = mps.cstruct()
    return _proj("oc_search_by_projection_local", F, C.byref(m), C.c_float(th), C.c_float(nnratio))


def search_by_projection_last_frame(F, Tcw, last_mps, Tcw_last, th, bMono, check_ori):
    m = last_mps.cstruct()
    T1 = np.ascontiguousarray(Tcw, np.float32).reshape(16)
    T2 = np.ascontiguousarray(Tcw_last, np.float32).reshape(16)
    return _proj("oc_search_by_projection_last_frame", F, T1.ctypes.data, C.byref(m), T2.ctypes.data,
                 C.c_float(th), int(bMono), int(check_ori))


def search_by_projection_keyframe(F, Tcw, kf_mps, th, orb_dist, check_ori):
    m = kf_mps.cstruct()
    T1 = np.ascontiguousarray(Tcw, np.float32).reshape(16)
    return _proj("oc_search_by_projection_keyframe", F, T1.ctypes.data, C.byref(m), C.c_float(th), int(orb_dist),
                 int(check_ori))


def search_by_projection_sim3(KF, Scw, mps, th):
    m = mps.cstruct()
    S = np.ascontiguousarray(Scw, np.float32).reshape(16)
    return _proj("oc_search_by_projection_sim3", KF, S.ctypes.data, C.byref(m), int(th))


# ---- Fuse x2 (ORBmatcher.cc:825-975, 977-1100): (nFused, best_idx[mps.n]), -1 = no fuse.
def fuse(KF, Tcw, Ow, mps, th, inv_sigma2):
    m = mps.cstruct()
    fv = KF.cstruct()
    T = np.ascontiguousarray(Tcw, np.float32).reshape(16)
    O = np.ascontiguousarray(Ow, np.float32).reshape(3)
    inv = np.ascontiguousarray(inv_sigma2, np.float32)
    out = np.empty(max(mps.n, 1), np.int32)
    n = load().oc_fuse(C.byref(fv), T.ctypes.data, O.ctypes.data, C.byref(m), C.c_float(th), inv.ctypes.data,
                       out.ctypes.data)
    return n, out[:mps.n]


def fuse_sim3(KF, Scw, mps, th):
    m = mps.cstruct()
    fv = KF.cstruct()
    S = np.ascontiguousarray(Scw, np.float32).reshape(16)
    out = np.empty(max(mps.n, 1), np.int32)
    n = load().oc_fuse_sim3(C.byref(fv), S.ctypes.data, C.byref(m), C.c_float(th), out.ctypes.data)
    return n, out[:mps.n]


# ---- SearchForInitialization (ORBmatcher.cc:405-520): (nmatches, vnMatches12, updated vbPrevMatched)
def search_for_initialization(F1, F2, prev_xy, window, nnratio, check_ori):
    f1, f2 = F1.cstruct(), F2.cstruct()
    prev = np.ascontiguousarray(prev_xy, np.float32).reshape(F1.n, 2).copy()
    out = np.empty(max(F1.n, 1), np.int32)
    n = load().oc_search_for_initialization(C.byref(f1), C.byref(f2), prev.ctypes.data, int(window),
                                            C.c_float(nnratio), int(check_ori), out.ctypes.data)
    return n, out[:F1.n], prev


# ---- SearchBySim3 (ORBmatcher.cc:1102-1326): (nFound, match12[mp1.n])
def search_by_sim3(KF1, T1w, mp1, KF2, T2w, mp2, s12, R12, t12, th):
    k1, k2 = KF1.cstruct(), KF2.cstruct()
    m1, m2 = mp1.cstruct(), mp2.cstruct()
    T1 = np.ascontiguousarray(T1w, np.float32).reshape(16)
    T2 = np.ascontiguousarray(T2w, np.float32).reshape(16)
    R = np.ascontiguousarray(R12, np.float32).reshape(9)
    t = np.ascontiguousarray(t12, np.float32).reshape(3)
    out = np.empty(max(mp1.n, 1), np.int32)
    n = load().oc_search_by_sim3(C.byref(k1), T1.ctypes.data, C.byref(m1), C.byref(k2), T2.ctypes.data, C.byref(m2),
                                 C.c_float(s12), R.ctypes.data, t.ctypes.data, C.c_float(th), out.ctypes.data)
    return n, out[:mp1.n]


def compute_distinctive_descriptors(offsets, desc):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307) per CSR list; returns best_idx."""
    off = np.ascontiguousarray(offsets, np.int32)
    d = np.ascontiguousarray(desc, np.uint8)
    out = np.empty(max(len(off) - 1, 1), np.int32)
    load().oc_compute_distinctive_descriptors(len(off) - 1, off.ctypes.data, d.ctypes.data, out.ctypes.data)
    return out[:len(off) - 1]


class OracleVocabulary:
    """DBoW2 TemplatedVocabulary<FORB> restated in C (orb_oracle_voc.c; parity unpinned)."""

    def __init__(self, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        self.lib = load()
        self._keep = [np.ascontiguousarray(parent, np.int32), np.ascontiguousarray(is_leaf, np.uint8),
                      np.ascontiguousarray(desc, np.uint8), np.ascontiguousarray(weight, np.float64)]
        p, lf, d, w = self._keep
        self.h = self.lib.oc_vocab_create(k, L, scoring, weighting, len(p), p.ctypes.data, lf.ctypes.data,
                                          d.ctypes.data, w.ctypes.data)
        if not self.h:
            raise ValueError("bad vocabulary")

    def __del__(self):
        try:
            if self.h:
                self.lib.oc_vocab_destroy(self.h)
        except Exception:
            pass

    def transform(self, descriptors, levelsup=4):
        d = np.ascontiguousarray(descriptors, np.uint8)
        n = len(d)
        bw = np.empty(max(n, 1), np.uint32)
        bv = np.empty(max(n, 1), np.float64)
        fn = np.empty(max(n, 1), np.uint32)
        fo = np.empty(n + 1, np.int32)
        ff = np.empty(max(n, 1), np.int32)
        nb, nf = C.c_int(), C.c_int()
        self.lib.oc_vocab_transform(self.h, d.ctypes.data, n, levelsup, bw.ctypes.data, bv.ctypes.data, C.byref(nb),
                                    fn.ctypes.data, fo.ctypes.data, ff.ctypes.data, C.byref(nf))
        fv = {int(fn[i]): ff[fo[i]:fo[i + 1]].tolist() for i in range(nf.value)}
        return (bw[:nb.value].copy(), bv[:nb.value].copy()), fv

    def descend(self, descriptors, levelsup=4):
        d = np.ascontiguousarray(descriptors, np.uint8)
        n = len(d)
        w = np.empty(max(n, 1), np.int32)
        wt = np.empty(max(n, 1), np.float64)
        nid = np.empty(max(n, 1), np.int32)
        self.lib.oc_vocab_descend(self.h, d.ctypes.data, n, levelsup, w.ctypes.data, wt.ctypes.data, nid.ctypes.data)
        return w[:n], wt[:n], nid[:n]
