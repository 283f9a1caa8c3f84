"""Inputs of the four ORBmatcher::SearchByProjection overloads (ORBmatcher.cc:45-129, 290-403,
1328-1470, 1472-1599) as numpy-backed views of the C ABI structs orbm_frame_view /
orbm_mappoints (include/orbslam_amd.h).
"""
import ctypes as C

import numpy as np

FRAME_GRID_COLS = 64  # Frame.h:38
FRAME_GRID_ROWS = 48  # Frame.h:37


class OrbmFrameView(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("x", C.c_void_p), ("y", C.c_void_p),
                ("octave", C.c_void_p), ("angle", C.c_void_p), ("uright", C.c_void_p), ("occupied", C.c_void_p),
                ("min_x", C.c_float), ("min_y", C.c_float), ("max_x", C.c_float), ("max_y", C.c_float),
                ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float), ("b", C.c_float),
                ("nlevels", C.c_int32), ("scale_factors", C.c_void_p), ("log_scale_factor", C.c_float)]


class OrbmMapPoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("pos", C.c_void_p), ("normal", C.c_void_p),
                ("min_dist", C.c_void_p), ("max_dist", C.c_void_p), ("bad", C.c_void_p), ("has_obs", C.c_void_p),
                ("skip", C.c_void_p), ("octave", C.c_void_p), ("angle", C.c_void_p), ("track_in_view", C.c_void_p),
                ("track_proj_x", C.c_void_p), ("track_proj_y", C.c_void_p), ("track_proj_xr", C.c_void_p),
                ("track_level", C.c_void_p), ("track_view_cos", C.c_void_p)]


def _p(a):
    return None if a is None else a.ctypes.data


def _arr(a, dt, shape=None):
    if a is None:
        return None
    a = np.ascontiguousarray(a, dt)
    return a if shape is None else a.reshape(shape)


class FrameView:
    """What SearchByProjection reads from a Frame / KeyFrame: mvKeysUn (x, y, octave, angle),
    mDescriptors, mvuRight, the variant's occupancy flags, image bounds and grid scale
    (ComputeImageBounds + Frame ctor, Frame.cc:155-160), camera, scale tables."""

    def __init__(self, keypoints, descriptors, scale_factors, width, height, fx, fy, cx, cy, bf=0.0, uright=None,
                 occupied=None, scale_factor=1.2):
        n = len(keypoints)
        self.n = n
        self.desc = _arr(descriptors if descriptors is not None else np.zeros((0, 32)), np.uint8, (n, 32))
        self.x = _arr(keypoints["x"], np.float32)
        self.y = _arr(keypoints["y"], np.float32)
        self.octave = _arr(keypoints["octave"], np.int32)
        self.angle = _arr(keypoints["angle"], np.float32)
        self.uright = _arr(uright, np.float32)
        self.occupied = _arr(occupied, np.uint8)
        f32 = np.float32
        self.min_x, self.min_y = f32(0.0), f32(0.0)  # no distortion (Frame.cc:461-467)
        self.max_x, self.max_y = f32(width), f32(height)
        # mfGridElementWidthInv = float(COLS)/float(mnMaxX-mnMinX) (Frame.cc:157-158)
        self.grid_w_inv = f32(FRAME_GRID_COLS) / f32(self.max_x - self.min_x)
        self.grid_h_inv = f32(FRAME_GRID_ROWS) / f32(self.max_y - self.min_y)
        self.fx, self.fy, self.cx, self.cy = f32(fx), f32(fy), f32(cx), f32(cy)
        self.bf = f32(bf)
        self.b = f32(f32(bf) / f32(fx)) if fx else f32(0)  # mb = mbf/fx (Frame.cc:97)
        self.scale_factors = _arr(scale_factors, np.float32)
        self.log_scale_factor = f32(np.log(f32(scale_factor)))  # mfLogScaleFactor = log(mfScaleFactor)

    def cstruct(self, cls=OrbmFrameView):
        return cls(self.n, _p(self.desc), _p(self.x), _p(self.y), _p(self.octave), _p(self.angle), _p(self.uright),
                   _p(self.occupied), self.min_x, self.min_y, self.max_x, self.max_y, self.grid_w_inv,
                   self.grid_h_inv, self.fx, self.fy, self.cx, self.cy, self.bf, self.b, len(self.scale_factors),
                   _p(self.scale_factors), self.log_scale_factor)


class MapPoints:
    """Candidate MapPoints of one SearchByProjection call (the reference's loop order).
    Fields follow orbm_mappoints; pass only what the overload reads."""

    FIELDS = [("desc", np.uint8, 32), ("pos", np.float32, 3), ("normal", np.float32, 3), ("min_dist", np.float32, 0),
              ("max_dist", np.float32, 0), ("bad", np.uint8, 0), ("has_obs", np.uint8, 0), ("skip", np.uint8, 0),
              ("octave", np.int32, 0), ("angle", np.float32, 0), ("track_in_view", np.uint8, 0),
              ("track_proj_x", np.float32, 0), ("track_proj_y", np.float32, 0), ("track_proj_xr", np.float32, 0),
              ("track_level", np.int32, 0), ("track_view_cos", np.float32, 0)]

    def __init__(self, n, **kw):
        self.n = int(n)
        for name, dt, w in self.FIELDS:
            v = kw.pop(name, None)
            setattr(self, name, None if v is None else _arr(v, dt, (self.n, w) if w else (self.n,)))
        if kw:
            raise TypeError("unknown MapPoints fields: %s" % sorted(kw))

    def cstruct(self, cls=OrbmMapPoints):
        return cls(self.n, *[_p(getattr(self, name)) for name, _, _ in self.FIELDS])
