"""Cross-agent keyframe slot (include/orbslam_amd.h; replaces lcmKeyFrame::lcmKeyFrameInfo,
ORB_SLAM2.1/include/lcmKeyFrame/lcmKeyFrameInfo.hpp:24-150) on the CPU: the library's layout and
host packer agree byte for byte with the numpy restatement in orbamd.exchange, the validating
decoder (orbx_slot_parse) returns every field the receiving agent consumes (receiveKeyframeInfo,
ORB_SLAM2/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:88-166) and rejects malformed slots."""
import ctypes as C

import numpy as np
import pytest

import orbamd
from orbamd import exchange
from orbamd._lib import OrbxSlotHeader


def _keyframe(n, seed=0, full=True):
    rng = np.random.default_rng(seed)
    k = np.zeros(n, exchange.KP_DTYPE)
    for f in ("x", "y", "size", "angle", "response"):
        k[f] = rng.random(n, dtype=np.float32) * 500
    k["octave"] = rng.integers(0, 8, n)
    d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    extra = {}
    if full:
        ur = np.where(rng.random(n) < 0.5, rng.random(n, dtype=np.float32) * 600, np.float32(-1)).astype(np.float32)
        extra = dict(
            kun=(np.stack([k["x"], k["y"]], 1) + rng.random((n, 2), dtype=np.float32)).astype(np.float32),
            uright=ur, depth=np.where(ur >= 0, rng.random(n, dtype=np.float32) * 9, np.float32(-1)).astype(np.float32),
            mp_flags=rng.integers(0, 4, n).astype(np.uint8) & np.uint8(3),
            mp_pos=rng.standard_normal((n, 3)).astype(np.float32))
        nb = min(n, 300)
        words = np.sort(rng.choice(10 ** 6, nb, replace=False)).astype(np.uint32)
        extra["bow"] = (words, rng.random(nb))
        nodes = np.sort(rng.choice(10 ** 4, min(n, 60), replace=False)).astype(np.uint32)
        assign = np.sort(rng.integers(0, len(nodes), n))
        off = np.searchsorted(assign, np.arange(len(nodes) + 1)).astype(np.int32)
        feat = np.concatenate([np.sort(np.nonzero(assign == i)[0]) for i in range(len(nodes))] +
                              [np.zeros(0, np.int64)]).astype(np.int32)
        # features of a node ascending; nodes themselves ascending
        extra["fv"] = (nodes, off, feat)
    meta = exchange.make_meta(agent=3, mnId=42, scale=1.2 ** np.arange(8, dtype=np.float32),
                              sigma2=1.44 ** np.arange(8, dtype=np.float32),
                              inv_sigma2=1.0 / 1.44 ** np.arange(8, dtype=np.float32),
                              K=np.array([[715.0, 0, 334.3], [0, 719.0, 256.3], [0, 0, 1]], np.float32),
                              Tcw=np.arange(16, dtype=np.float32).reshape(4, 4), bf=40.0, b=0.11, th_depth=35.0)
    return meta, k, d, extra


@pytest.mark.parametrize("cap", [1, 2, 7, 1031, 1032, 2063, 4000])
def test_layout_matches_restatement(cap):
    lib = orbamd.load()
    h = OrbxSlotHeader()
    assert lib.orbx_slot_layout(cap, C.byref(h)) == 0
    off, total = exchange.layout(cap)
    assert list(h.off) == off and h.bytes == total == lib.orbx_slot_bytes(cap)
    assert total % 256 == 0 and all(o % 256 == 0 for o in off)
    assert lib.orbx_slot_layout(-1, C.byref(h)) == -1


@pytest.mark.parametrize("full", [True, False])
@pytest.mark.parametrize("n", [0, 1, 700, 1031])
def test_host_pack_equals_restatement_and_decodes(n, full):
    meta, k, d, extra = _keyframe(n, seed=n, full=full)
    cap = 1031
    buf_c = exchange.pack_host(meta, k, d, cap, **extra)
    buf_np = exchange.pack_slot_np(meta, k, d, cap, **extra)
    assert buf_c.tobytes() == buf_np.tobytes()
    got = exchange.parse(buf_c)
    ref = exchange.unpack_slot_np(buf_np)
    assert got["n"] == n and got["kps"].tobytes() == k.tobytes() and np.array_equal(got["desc"], d)
    assert exchange.meta_bytes(got["meta"]).tobytes() == exchange.meta_bytes(meta).tobytes()
    assert got["meta"].mnId == 42 and got["meta"].agent == 3 and got["meta"].mnScaleLevels == 8
    for key in ("kun", "uright", "depth", "mp_flags", "mp_pos", "bow_word", "bow_value", "fv_node", "fv_off",
                "fv_feat"):
        assert np.array_equal(got[key], ref[key]), key
    if full:
        assert np.array_equal(got["kun"], extra["kun"]) and np.array_equal(got["uright"], extra["uright"])
        assert np.array_equal(got["mp_flags"], extra["mp_flags"]) and np.array_equal(got["mp_pos"], extra["mp_pos"])
        assert np.array_equal(got["bow_word"], extra["bow"][0]) and np.array_equal(got["bow_value"], extra["bow"][1])
        if n:
            assert np.array_equal(got["fv_node"], extra["fv"][0]) and np.array_equal(got["fv_feat"], extra["fv"][2])
    else:
        # mono keyframe, no MapPoints: mvKeysUn = mvKeys, mvuRight = mvDepth = -1
        assert np.array_equal(got["kun"][:, 0], k["x"]) and np.all(got["uright"] == -1)
        assert got["flags"] == 0


def test_capacity_error():
    meta, k, d, extra = _keyframe(50, full=False)
    with pytest.raises(RuntimeError, match="ECAPACITY"):
        exchange.pack_host(meta, k, d, 49)


def _corrupt(buf, fn):
    b = buf.copy()
    fn(b)
    return b


def test_parse_rejects_malformed_slots():
    meta, k, d, extra = _keyframe(300, seed=5)
    cap = 400
    buf = exchange.pack_host(meta, k, d, cap, **extra)
    exchange.parse(buf)
    off, total = exchange.layout(cap)
    sec = {name: off[i] for i, name in enumerate(exchange.SLOT_SECTIONS)}
    u32 = lambda b: b[:128].view(np.uint32)  # noqa: E731
    bad = {
        "magic": lambda b: u32(b).__setitem__(0, 0),
        "version": lambda b: u32(b).__setitem__(1, 1),
        "n > cap": lambda b: u32(b).__setitem__(2, cap + 1),
        "cap vs bytes": lambda b: u32(b).__setitem__(3, cap + 64),
        "nbow > cap": lambda b: u32(b).__setitem__(4, cap + 1),
        "offset": lambda b: u32(b).__setitem__(8 + 3, off[3] + 256),
        "levels": lambda b: b[128:128 + 704].view(np.int32).__setitem__(38 + 1, 99),
        "octave": lambda b: b[sec["KPS"] + 20:sec["KPS"] + 24].view(np.int32).__setitem__(0, 8),
        "fv off": lambda b: b[sec["FVOFF"] + 4:sec["FVOFF"] + 8].view(np.int32).__setitem__(0, 10 ** 6),
        "fv feat": lambda b: b[sec["FVFEAT"]:sec["FVFEAT"] + 4].view(np.int32).__setitem__(0, 300),
        "fv node order": lambda b: b[sec["FVNODE"] + 4:sec["FVNODE"] + 8].view(np.uint32).__setitem__(0, 0),
        "bow order": lambda b: b[sec["BOWWORD"] + 4:sec["BOWWORD"] + 8].view(np.uint32).__setitem__(0, 0),
    }
    for name, fn in bad.items():
        with pytest.raises(RuntimeError, match="EARG"):
            exchange.parse(_corrupt(buf, fn))
            pytest.fail(name)
    with pytest.raises(RuntimeError, match="EARG"):
        exchange.parse(buf[:total - 256])  # truncated
    # a larger receive buffer than the slot is fine
    exchange.parse(np.concatenate([buf, np.zeros(512, np.uint8)]))
