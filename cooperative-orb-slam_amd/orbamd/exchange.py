"""Cross-agent keyframe slot -- the replacement of the LCM message lcmKeyFrame::lcmKeyFrameInfo
(ORB_SLAM2.1/include/lcmKeyFrame/lcmKeyFrameInfo.hpp:24-150; published at ORB_SLAM2.1/Examples/
ROS/ORB_SLAM2/src/ros_mono.cc:1907-2410, decoded into receiveKeyframeInfo at ORB_SLAM2/Examples/
ROS/ORB_SLAM2/src/ros_mono.cc:88-166, 230-544).

Layout (include/orbslam_amd.h, "Cross-agent keyframe slot"): a 128-byte header, the 704-byte
orbx_kf_meta at 128, and from byte 1024 twelve 256-byte-aligned sections sized by the capacity.
This module holds
  * a numpy restatement of the layout and of the host packer / decoder (test infrastructure and
    the format's executable documentation: it never calls the library), and
  * thin wrappers of the C ABI: orbx_pack_keyframe_host / _device, orbx_slot_parse and the
    cross-agent SearchForTriangulation over slots (orbm_search_for_triangulation_slots_device).
"""
import ctypes as C

import numpy as np

from ._lib import (SLOT_F_BOW, SLOT_F_FV, SLOT_F_KUN, SLOT_F_MP, SLOT_F_STEREO, SLOT_MAGIC, SLOT_SECTIONS,
                   SLOT_VERSION, OrbmSlotGeom, OrbxKfMeta, OrbxKfSource, OrbxSlotView, check, load)

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])
META_OFF = 128
BODY_OFF = 1024
META_BYTES = C.sizeof(OrbxKfMeta)


def section_bytes(cap):
    c = int(cap)
    return [24 * c, 8 * c, 4 * c, 4 * c, 32 * c, c, 12 * c, 4 * c, 8 * c, 4 * c, 4 * (c + 1), 4 * c]


def layout(cap):
    """(offsets per section, total bytes) for capacity cap -- restates orb_slot.h:slot_offsets."""
    off, o = [], BODY_OFF
    for b in section_bytes(cap):
        off.append(o)
        o += (b + 255) // 256 * 256
    return off, o


def slot_bytes(cap):
    return layout(cap)[1]


def make_meta(agent=0, mnId=0, nlevels=8, scale=None, sigma2=None, inv_sigma2=None, scale_factor=1.2,
              K=None, Tcw=None, bf=0.0, b=0.0, th_depth=0.0, width=640, height=480, timestamp=0.0):
    """orbx_kf_meta for a keyframe (fields of lcmKeyFrameInfo; the defaults mirror a mono KeyFrame
    built by ORB-SLAM2's KeyFrame(Frame&) from a width x height camera without distortion)."""
    m = OrbxKfMeta()
    m.agent = int(agent)
    m.mnId = int(mnId)
    m.mnFrameId = int(mnId)
    m.nNextId = int(mnId) + 1
    m.mTimeStamp = float(timestamp)
    m.mnGridCols, m.mnGridRows = 64, 48  # FRAME_GRID_COLS / ROWS (Frame.h:34-35)
    m.mfGridElementWidthInv = np.float32(64) / np.float32(width)
    m.mfGridElementHeightInv = np.float32(48) / np.float32(height)
    m.mnMinX, m.mnMinY, m.mnMaxX, m.mnMaxY = 0, 0, int(width), int(height)
    m.mnScaleLevels = int(nlevels)
    m.mfScaleFactor = float(scale_factor)
    m.mfLogScaleFactor = float(np.log(np.float32(scale_factor)))
    for arr, src in ((m.mvScaleFactors, scale), (m.mvLevelSigma2, sigma2), (m.mvInvLevelSigma2, inv_sigma2)):
        if src is not None:
            for i, v in enumerate(np.asarray(src, np.float32)[:16]):
                arr[i] = float(v)
    K = np.eye(3, dtype=np.float32) if K is None else np.asarray(K, np.float32)
    for i, v in enumerate(K.reshape(9)):
        m.mK[i] = float(v)
    m.fx, m.fy, m.cx, m.cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    m.invfx = float(np.float32(1.0) / np.float32(K[0, 0]))
    m.invfy = float(np.float32(1.0) / np.float32(K[1, 1]))
    m.mbf, m.mb, m.mThDepth = float(bf), float(b), float(th_depth)
    T = np.eye(4, dtype=np.float32) if Tcw is None else np.asarray(Tcw, np.float32)
    for i, v in enumerate(T.reshape(16)):
        m.mTcw[i] = float(v)
        m.mTcwGBA[i] = float(v)
        m.mTcwBefGBA[i] = float(v)
    for i in range(4):
        m.mTcp[5 * i] = 1.0
    return m


def meta_bytes(meta):
    return np.frombuffer(C.string_at(C.addressof(meta), META_BYTES), np.uint8).copy()


# ------------------------------------------------------------------------------------------------
# numpy restatement (test infrastructure; the library's packer must produce the same bytes)
# ------------------------------------------------------------------------------------------------
def pack_slot_np(meta, kps, desc, cap, kun=None, uright=None, depth=None, mp_flags=None, mp_pos=None,
                 bow=None, fv=None):
    """bow = (word u32[nb], value f64[nb]); fv = (node u32[nf], off i32[nf+1], feat i32[...])."""
    n = len(kps)
    off, total = layout(cap)
    if n > cap:
        raise ValueError("slot capacity %d < %d keypoints" % (cap, n))
    buf = np.zeros(total, np.uint8)
    nbow = len(bow[0]) if bow is not None else 0
    nfv = len(fv[0]) if fv is not None else 0
    flags = ((SLOT_F_KUN if kun is not None else 0) | (SLOT_F_STEREO if uright is not None and depth is not None else 0)
             | (SLOT_F_MP if mp_flags is not None else 0) | (SLOT_F_BOW if bow is not None else 0)
             | (SLOT_F_FV if fv is not None else 0))
    hdr = np.array([SLOT_MAGIC, SLOT_VERSION, n, cap, nbow, nfv, flags, total] + off, np.uint32)
    buf[:4 * len(hdr)] = hdr.view(np.uint8)
    buf[META_OFF:META_OFF + META_BYTES] = meta_bytes(meta)

    def put(sec, arr):
        a = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        o = off[SLOT_SECTIONS.index(sec)]
        buf[o:o + a.size] = a

    k = np.ascontiguousarray(kps, KP_DTYPE)
    put("KPS", k)
    put("KUN", np.asarray(kun, np.float32).reshape(n, 2) if kun is not None else
        np.stack([k["x"], k["y"]], 1).astype(np.float32))
    st = uright is not None and depth is not None
    put("URIGHT", np.asarray(uright, np.float32) if st else np.full(n, -1, np.float32))
    put("DEPTH", np.asarray(depth, np.float32) if st else np.full(n, -1, np.float32))
    put("DESC", np.asarray(desc, np.uint8).reshape(n, 32))
    if mp_flags is not None:
        put("MPFLAGS", np.asarray(mp_flags, np.uint8))
        if mp_pos is not None:
            put("MPPOS", np.asarray(mp_pos, np.float32).reshape(n, 3))
    if bow is not None and nbow:
        put("BOWWORD", np.asarray(bow[0], np.uint32))
        put("BOWVALUE", np.asarray(bow[1], np.float64))
    if fv is not None and nfv:
        put("FVNODE", np.asarray(fv[0], np.uint32))
        put("FVOFF", np.asarray(fv[1][:nfv + 1], np.int32))
        put("FVFEAT", np.asarray(fv[2][:int(fv[1][nfv])], np.int32))
    return buf


def unpack_slot_np(buf):
    """dict of every field of a slot (numpy restatement of the decoder; no validation beyond the
    magic/version)."""
    buf = np.asarray(buf, np.uint8)
    h = buf[:80].view(np.uint32)
    if h[0] != SLOT_MAGIC or h[1] != SLOT_VERSION:
        raise ValueError("not a version-%d keyframe slot" % SLOT_VERSION)
    n, cap, nbow, nfv, flags = (int(h[2]), int(h[3]), int(h[4]), int(h[5]), int(h[6]))
    off = [int(x) for x in h[8:20]]

    def get(sec, dtype, count, shape=None):
        o = off[SLOT_SECTIONS.index(sec)]
        a = np.frombuffer(buf[o:o + np.dtype(dtype).itemsize * count].tobytes(), dtype).copy()
        return a.reshape(shape) if shape else a

    meta = OrbxKfMeta.from_buffer_copy(buf[META_OFF:META_OFF + META_BYTES].tobytes())
    fo = get("FVOFF", np.int32, nfv + 1)
    return {
        "n": n, "cap": cap, "flags": flags, "meta": meta,
        "kps": get("KPS", KP_DTYPE, n), "kun": get("KUN", np.float32, 2 * n, (n, 2)),
        "uright": get("URIGHT", np.float32, n), "depth": get("DEPTH", np.float32, n),
        "desc": get("DESC", np.uint8, 32 * n, (n, 32)), "mp_flags": get("MPFLAGS", np.uint8, n),
        "mp_pos": get("MPPOS", np.float32, 3 * n, (n, 3)),
        "bow_word": get("BOWWORD", np.uint32, nbow), "bow_value": get("BOWVALUE", np.float64, nbow),
        "fv_node": get("FVNODE", np.uint32, nfv), "fv_off": fo,
        "fv_feat": get("FVFEAT", np.int32, int(fo[nfv]) if nfv else 0),
    }


# ------------------------------------------------------------------------------------------------
# C ABI wrappers
# ------------------------------------------------------------------------------------------------
def _ptr(a):
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


def kf_source(kps, desc, count, kun=None, uright=None, depth=None, mp_flags=None, mp_pos=None, bow_word=None,
              bow_value=None, nbow=None, fv_node=None, fv_off=None, fv_feat=None, nfv=None):
    """orbx_kf_source from numpy arrays (host) or torch tensors (device); keeps the arrays alive."""
    s = OrbxKfSource()
    keep = []
    for name, a in (("kps", kps), ("desc", desc), ("count", count), ("kun", kun), ("uright", uright),
                    ("depth", depth), ("mp_flags", mp_flags), ("mp_pos", mp_pos), ("bow_word", bow_word),
                    ("bow_value", bow_value), ("nbow", nbow), ("fv_node", fv_node), ("fv_off", fv_off),
                    ("fv_feat", fv_feat), ("nfv", nfv)):
        if a is not None:
            keep.append(a)
            setattr(s, name, _ptr(a))
    s._keep = keep
    return s


def pack_host(meta, kps, desc, cap, kun=None, uright=None, depth=None, mp_flags=None, mp_pos=None, bow=None,
              fv=None):
    """orbx_pack_keyframe_host over numpy arrays -> slot bytes (numpy uint8)."""
    n = np.array([len(kps)], np.int32)
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    a = dict(kun=None if kun is None else np.ascontiguousarray(kun, np.float32),
             uright=None if uright is None else np.ascontiguousarray(uright, np.float32),
             depth=None if depth is None else np.ascontiguousarray(depth, np.float32),
             mp_flags=None if mp_flags is None else np.ascontiguousarray(mp_flags, np.uint8),
             mp_pos=None if mp_pos is None else np.ascontiguousarray(mp_pos, np.float32))
    if bow is not None:
        a.update(bow_word=np.ascontiguousarray(bow[0], np.uint32), bow_value=np.ascontiguousarray(bow[1], np.float64),
                 nbow=np.array([len(bow[0])], np.int32))
    if fv is not None:
        a.update(fv_node=np.ascontiguousarray(fv[0], np.uint32), fv_off=np.ascontiguousarray(fv[1], np.int32),
                 fv_feat=np.ascontiguousarray(fv[2], np.int32), nfv=np.array([len(fv[0])], np.int32))
    src = kf_source(kps, desc, n, **a)
    buf = np.zeros(slot_bytes(cap), np.uint8)
    check(load().orbx_pack_keyframe_host(C.byref(src), C.byref(meta), int(cap), buf.ctypes.data, buf.size),
          "orbx_pack_keyframe_host")
    return buf


def parse(buf):
    """orbx_slot_parse (validating decoder) -> dict of numpy copies of every field."""
    buf = np.ascontiguousarray(buf, np.uint8)
    v = OrbxSlotView()
    check(load().orbx_slot_parse(buf.ctypes.data, buf.size, C.byref(v)), "orbx_slot_parse")
    base = buf.ctypes.data
    h = buf[:80].view(np.uint32)
    n, nbow, nfv = int(h[2]), int(h[4]), int(h[5])

    def arr(p, dtype, count, shape=None):
        o = p - base
        a = np.frombuffer(buf[o:o + np.dtype(dtype).itemsize * count].tobytes(), dtype).copy()
        return a.reshape(shape) if shape else a

    fo = arr(v.fv_off, np.int32, nfv + 1)
    return {
        "n": n, "flags": int(h[6]), "meta": OrbxKfMeta.from_buffer_copy(
            buf[v.meta - base:v.meta - base + META_BYTES].tobytes()),
        "kps": arr(v.kps, KP_DTYPE, n), "kun": arr(v.kun, np.float32, 2 * n, (n, 2)),
        "uright": arr(v.uright, np.float32, n), "depth": arr(v.depth, np.float32, n),
        "desc": arr(v.desc, np.uint8, 32 * n, (n, 32)), "mp_flags": arr(v.mp_flags, np.uint8, n),
        "mp_pos": arr(v.mp_pos, np.float32, 3 * n, (n, 3)), "bow_word": arr(v.bow_word, np.uint32, nbow),
        "bow_value": arr(v.bow_value, np.float64, nbow), "fv_node": arr(v.fv_node, np.uint32, nfv),
        "fv_off": fo, "fv_feat": arr(v.fv_feat, np.int32, int(fo[nfv]) if nfv else 0),
    }


def pack_device(src, meta, cap, d_slot, d_err=None, stream=None):
    """orbx_pack_keyframe_device: src = kf_source over device tensors."""
    check(load().orbx_pack_keyframe_device(C.byref(src), C.byref(meta), int(cap), _ptr(d_slot), _ptr(d_err),
                                           stream), "orbx_pack_keyframe_device")


def slot_geoms(geoms):
    """[(F12 3x3, ex, ey), ...] -> ctypes array of orbm_slot_geom"""
    arr = (OrbmSlotGeom * max(len(geoms), 1))()
    for i, (F, ex, ey) in enumerate(geoms):
        for j, v in enumerate(np.asarray(F, np.float32).reshape(9)):
            arr[i].F12[j] = float(v)
        arr[i].ex = float(ex)
        arr[i].ey = float(ey)
    return arr


def match_slots_device(mh, query, cap1, nref, d_slots, slot_nbytes, geoms, d_match, d_nmatch, use_bow=False,
                       max_nodes=0, stream=None):
    """orbm_search_for_triangulation_slots_device (cross-agent SearchForTriangulation)."""
    g = geoms if not isinstance(geoms, list) else slot_geoms(geoms)
    check(load().orbm_search_for_triangulation_slots_device(mh, C.byref(query), int(cap1), int(nref), _ptr(d_slots),
                                                            int(slot_nbytes), g, int(bool(use_bow)), int(max_nodes),
                                                            _ptr(d_match), _ptr(d_nmatch), stream),
          "orbm_search_for_triangulation_slots_device")


def bow_slots_device(mh, query, cap1, nref, d_slots, slot_nbytes, d_match, d_nmatch, nnratio=0.75, check_ori=True,
                     max_nodes=0, stream=None):
    """orbm_search_by_bow_slots_device (cross-agent SearchByBoW(KF,KF), LoopClosing's loop-candidate match)."""
    check(load().orbm_search_by_bow_slots_device(mh, C.byref(query), int(cap1), int(nref), _ptr(d_slots),
                                                 int(slot_nbytes), float(nnratio), int(bool(check_ori)),
                                                 int(max_nodes), _ptr(d_match), _ptr(d_nmatch), stream),
          "orbm_search_by_bow_slots_device")
