"""Cross-agent exchange slot (replaces LCM `KeyFrameexample`, ORB_SLAM2.1 ros_mono.cc:1907-2410).

Layout of one slot (orbx_slot_bytes(cap), written on the device by orbx_pack_keyframe_device):
  [0:4)    int32 n          keypoints in the slot
  [4:8)    int32 cap_even   slot capacity (cap rounded up to even)
  [8:64)   zero padding
  [64 : 64+24*cap_even)       n x orbx_kp {x, y, size, angle, response f32; octave i32}
  [64+24*cap_even : +32*cap_even)  n x 32-byte descriptors
Keypoint coordinates stay float (the LCM message truncated them to int16,
lcmKeyPoint.hpp:19-21). Host helpers below are the reference implementation of the
layout used by tests and by integrators who assemble slots on the CPU.
"""
import numpy as np

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])


def slot_bytes(cap):
    c = (cap + 1) & ~1
    return (64 + c * 24 + c * 32 + 255) // 256 * 256


def pack_slot_host(kps, desc, cap):
    n = len(kps)
    if n > cap:
        raise ValueError("slot capacity %d < %d keypoints" % (cap, n))
    c = (cap + 1) & ~1
    buf = np.zeros(slot_bytes(cap), np.uint8)
    buf[0:8] = np.array([n, c], np.int32).view(np.uint8)
    buf[64:64 + 24 * n] = np.ascontiguousarray(kps, KP_DTYPE).view(np.uint8).reshape(-1)
    off = 64 + 24 * c
    buf[off:off + 32 * n] = np.ascontiguousarray(desc, np.uint8).reshape(-1)
    return buf


def unpack_slot_host(buf):
    n, c = np.frombuffer(buf[0:8].tobytes(), np.int32)
    kps = np.frombuffer(buf[64:64 + 24 * n].tobytes(), KP_DTYPE).copy()
    off = 64 + 24 * c
    desc = np.frombuffer(buf[off:off + 32 * n].tobytes(), np.uint8).reshape(n, 32).copy()
    return kps, desc
