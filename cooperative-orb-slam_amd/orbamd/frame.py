"""Frame-level consumers of the extractor output over the C ABI.

* :func:`compute_stereo_matches` -- ``Frame::ComputeStereoMatches``
  (ORB_SLAM2.1/src/Frame.cc:470-641): mvuRight / mvDepth of the left keypoints, from the two
  extractors' device-resident pyramids.
"""
import ctypes as C

import numpy as np

from ._lib import check, load


def compute_stereo_matches(left, right, kpsL, descL, kpsR, descR, mbf, mb):
    """left/right: the two ORBextractor instances whose latest call produced (kpsL, descL) and
    (kpsR, descR). Returns (mvuRight float32 [N], mvDepth float32 [N], number of stereo matches)."""
    lib = load()
    nL, nR = len(kpsL), len(kpsR)
    kpsL = np.ascontiguousarray(kpsL)
    kpsR = np.ascontiguousarray(kpsR)
    dL = np.ascontiguousarray(descL if descL is not None else np.zeros((0, 32), np.uint8))
    dR = np.ascontiguousarray(descR if descR is not None else np.zeros((0, 32), np.uint8))
    ur = np.full(nL, -1.0, np.float32)
    dp = np.full(nL, -1.0, np.float32)
    ns = C.c_int(0)
    check(lib.orbx_compute_stereo_matches(left._h, right._h, kpsL.ctypes.data, dL.ctypes.data, nL, kpsR.ctypes.data,
                                          dR.ctypes.data, nR, float(mbf), float(mb), ur.ctypes.data, dp.ctypes.data,
                                          C.byref(ns)), "orbx_compute_stereo_matches")
    return ur, dp, ns.value


def stereo_matches_batch_device(left, right, fl, fr, kpsL, descL, cntL, kpsR, descR, cntR, mbf, mb, uright, depth,
                                nstereo, stream=0):
    """Device batch form (torch tensors): pair p = frame fl[p] of left's latest batch with frame fr[p] of
    right's. kps [B, stride, 6], desc [B, stride, 32], counts [B]; outputs uright/depth [P, stride], nstereo [P]."""
    lib = load()
    stride = descL.shape[1]
    check(lib.orbx_stereo_matches_batch_device(
        left._h, right._h, fl.shape[0], fl.data_ptr(), fr.data_ptr(), kpsL.data_ptr(), descL.data_ptr(),
        cntL.data_ptr(), kpsR.data_ptr(), descR.data_ptr(), cntR.data_ptr(), stride, float(mbf), float(mb),
        uright.data_ptr(), depth.data_ptr(), nstereo.data_ptr(), stream), "orbx_stereo_matches_batch_device")
