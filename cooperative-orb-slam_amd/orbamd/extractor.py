"""ORBextractor -- Python mirror of ORB_SLAM2::ORBextractor over the C ABI.

Reference surface: ORB_SLAM2/include/ORBextractor.h:45-111 (ctor, operator(), six
getters, public mvImagePyramid). Outputs follow ORBextractor::operator()
(ORBextractor.cc:1043-1105): keypoints level by level in DistributeOctTree order,
descriptors an N x 32 uint8 matrix (None when N == 0, like ``_descriptors.release()``).
"""
import ctypes as C

import numpy as np

from ._lib import KP_FIELDS, OrbxParams, check, load

kp_dtype = np.dtype(KP_FIELDS)


def synth_frames(agent, t0, count, width, height, dx=0, scene=None):
    """Deterministic synthetic frames; returns uint8 [count, H, W]. dx > 0 gives the
    right image of a rectified stereo pair (the same crop shifted by dx px: disparity dx). scene=None: agent's
    own texture; scene=s: agent's view of the shared texture of scene s (orbx_synth_scene_frames: the agents'
    crops 12 px apart along the pan, overlapping views of one environment)."""
    lib = load()
    out = np.empty((count, height, width), np.uint8)
    if scene is None:
        check(lib.orbx_synth_frames_shifted(agent, t0, count, width, height, dx, out.ctypes.data),
              "orbx_synth_frames_shifted")
    else:
        check(lib.orbx_synth_scene_frames(scene, agent, t0, count, width, height, dx, out.ctypes.data),
              "orbx_synth_scene_frames")
    return out


class ORBextractor:
    """ORB_SLAM2::ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST).

    ``device``/``max_width``/``max_height``/``max_batch`` size the device buffers
    (the reference allocates per call; here buffers live on the GPU for the handle's life).
    """

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device=0, max_width=640,
                 max_height=480, max_batch=1):
        self._lib = load()
        self.nfeatures = int(nfeatures)
        self.scaleFactor = float(scaleFactor)
        self.nlevels = int(nlevels)
        self.iniThFAST = int(iniThFAST)
        self.minThFAST = int(minThFAST)
        p = OrbxParams(self.nfeatures, self.scaleFactor, self.nlevels, self.iniThFAST, self.minThFAST)
        h = C.c_void_p()
        check(self._lib.orbx_create(C.byref(p), device, max_width, max_height, max_batch, C.byref(h)),
              "orbx_create")
        self._h = h
        self.device = device
        self._last_shape = None

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- operator() (ORBextractor.cc:1043-1105)
    def __call__(self, image, mask=None):
        """Returns (keypoints: structured array of kp_dtype, descriptors: uint8 [N,32] or None)."""
        img = np.ascontiguousarray(image)
        if img.size == 0:
            return np.empty(0, kp_dtype), None
        if img.dtype != np.uint8 or img.ndim != 2:
            raise AssertionError("image.type() == CV_8UC1")  # ORBextractor.cc:1050
        h, w = img.shape
        cap = self.max_keypoints(w, h)
        kps = np.empty(cap, kp_dtype)
        desc = np.empty((cap, 32), np.uint8)
        n = C.c_int(0)
        check(self._lib.orbx_extract(self._h, img.ctypes.data, w, h, img.strides[0], kps.ctypes.data,
                                     desc.ctypes.data, cap, C.byref(n)), "orbx_extract")
        self._last_shape = (w, h)
        n = n.value
        return kps[:n].copy(), (desc[:n].copy() if n > 0 else None)

    def max_keypoints(self, width, height):
        return int(self._lib.orbx_max_keypoints(self._h, width, height))

    # ---- getters (ORBextractor.h:63-81)
    def _tables(self):
        L = self.nlevels
        arrs = [np.empty(L, np.float32) for _ in range(4)]
        check(self._lib.orbx_get_scale_tables(self._h, *[a.ctypes.data for a in arrs]), "orbx_get_scale_tables")
        return arrs

    def GetLevels(self):
        return int(self._lib.orbx_get_levels(self._h))

    def GetScaleFactor(self):
        return float(self._lib.orbx_get_scale_factor(self._h))

    def GetScaleFactors(self):
        return self._tables()[0]

    def GetInverseScaleFactors(self):
        return self._tables()[1]

    def GetScaleSigmaSquares(self):
        return self._tables()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._tables()[3]

    def feature_split(self):
        """(mnFeaturesPerLevel, umax) -- ORBextractor.cc:435-469."""
        per = np.empty(self.nlevels, np.int32)
        umax = np.empty(16, np.int32)
        check(self._lib.orbx_get_feature_split(self._h, per.ctypes.data, umax.ctypes.data), "orbx_get_feature_split")
        return per, umax

    # ---- public mvImagePyramid (ORBextractor.h:85), materialised lazily from the device
    def pyramid_level(self, level, frame=0):
        w = C.c_int()
        h = C.c_int()
        check(self._lib.orbx_pyramid_level(self._h, frame, level, None, 0, C.byref(w), C.byref(h)),
              "orbx_pyramid_level")
        out = np.empty((h.value, w.value), np.uint8)
        check(self._lib.orbx_pyramid_level(self._h, frame, level, out.ctypes.data, w.value, C.byref(w),
                                           C.byref(h)), "orbx_pyramid_level")
        return out

    @property
    def mvImagePyramid(self):
        return [self.pyramid_level(l) for l in range(self.nlevels)]

    # ---- batched device path (torch tensors; see orbamd.device)
    def extract_batch_device(self, frames, kps, desc, counts, stream=None):
        """frames: uint8 cuda tensor [B,H,W]; kps: uint8/any cuda buffer of B*stride*24 bytes viewed as
        [B, stride, 6] float32/int32; desc: uint8 [B, stride, 32]; counts: int32 [B]."""
        B, H, W = frames.shape
        stride = desc.shape[1]
        st = 0 if stream is None else stream
        check(self._lib.orbx_extract_batch_device(self._h, B, frames.data_ptr(), frames.stride(0), W, H,
                                                  frames.stride(1), kps.data_ptr(), desc.data_ptr(),
                                                  counts.data_ptr(), stride, st), "orbx_extract_batch_device")
