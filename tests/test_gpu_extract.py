"""GPU parity: ORBextractor::operator() on the HIP path vs the CPU oracle, bit-exact.

Every field of every keypoint (x, y, size, angle, response, octave) and every descriptor
byte must match, in the reference's order (ORBextractor.cc:1075-1104)."""
import numpy as np
import pytest

import oracle_py
import orbamd

pytestmark = pytest.mark.gpu

CONFIGS = [
    # (W, H, nfeatures) -- BASELINE configs C2, C3 (per image), C4 (per image), mono-init 2x
    (640, 480, 1000),
    (752, 480, 1200),
    (1241, 376, 2000),
    (640, 480, 2000),
]


def _compare(kg, dg, ko, do):
    assert len(kg) == len(ko), "keypoint count %d vs oracle %d" % (len(kg), len(ko))
    for f in ("octave", "x", "y", "response", "size", "angle"):
        a, b = kg[f], ko[f]
        bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
        assert bad.size == 0, "field %s differs at %s: gpu %s oracle %s" % (f, bad[:5], a[bad[:5]], b[bad[:5]])
    bad = np.nonzero((dg != do).any(axis=1))[0]
    assert bad.size == 0, "descriptors differ at %d rows, first %s" % (bad.size, bad[:5])


@pytest.mark.parametrize("W,H,nf", CONFIGS)
def test_extract_bit_exact(W, H, nf):
    frames = orbamd.synth_frames(0, 0, 2, W, H)
    ext = orbamd.ORBextractor(nf, 1.2, 8, 20, 7, max_width=W, max_height=H)
    orc = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    for f in range(frames.shape[0]):
        kg, dg = ext(frames[f])
        ko, do = orc(frames[f])
        _compare(kg, dg, ko, do)
        # stage isolation: pyramid levels (public mvImagePyramid)
        for l in range(8):
            np.testing.assert_array_equal(ext.pyramid_level(l), orc.pyramid(l), err_msg="pyramid level %d" % l)


def test_extract_other_agents_and_frames():
    W, H = 640, 480
    ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    for agent, t in ((1, 5), (3, 97), (7, 301)):
        img = orbamd.synth_frames(agent, t, 1, W, H)[0]
        kg, dg = ext(img)
        ko, do = orc(img)
        _compare(kg, dg, ko, do)


def test_extract_noise_and_flat_edge_cases():
    rng = np.random.default_rng(7)
    ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    noise = rng.integers(0, 256, (480, 640), dtype=np.uint8)  # dense corners: octree stress
    kg, dg = ext(noise)
    ko, do = orc(noise)
    _compare(kg, dg, ko, do)
    flat = np.full((480, 640), 128, np.uint8)  # no corners at all
    kg, dg = ext(flat)
    ko, do = orc(flat)
    assert len(kg) == len(ko) == 0 and dg is None
    # low contrast: only the minThFAST fallback fires (ORBextractor.cc:812-816)
    low = (128 + (rng.integers(0, 2, (480, 640)) * 12)).astype(np.uint8)
    kg, dg = ext(low)
    ko, do = orc(low)
    _compare(kg, dg, ko, do)
    # duplicated corners in the 6-px cell overlaps + saturated regions
    img = np.zeros((480, 640), np.uint8)
    img[::7, :] = 255
    img[:, ::11] = 255
    kg, dg = ext(img)
    ko, do = orc(img)
    _compare(kg, dg, ko, do)


@pytest.mark.parametrize("B", [6, 4, 2])
def test_batch_device_matches_host_path(B):
    """small batches (< 64 frames: run_extract_levels' two queue lists) at several sizes, three steps on one
    pipeline (the graph replays), every frame against the oracle and the device error word clean"""
    torch = pytest.importorskip("torch")
    W, H = 640, 480
    frames = orbamd.synth_frames(2, 10, B, W, H)
    pipe = orbamd.device.BatchPipeline(torch, W, H, B)
    fr = torch.from_numpy(frames).cuda()
    for _ in range(3):
        pipe.step(fr)
    torch.cuda.synchronize()
    pipe.check_error()
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    for b in range(B):
        kg, dg, _ = pipe.host_results(b)
        ko, do = orc(frames[b])
        _compare(kg, dg, ko, do)
    pipe.close()


@pytest.mark.parametrize("W,H,nf", CONFIGS[:3])
def test_large_batch_whole_frame_pyramid(W, H, nf):
    """Batches >= kPyrFramesMinBatch (64) build the pyramid with one workgroup per frame
    (k_pyramid_frames); pyramid levels and keypoints must still match the oracle bit for bit."""
    torch = pytest.importorskip("torch")
    B = 64
    frames = orbamd.synth_frames(5, 3, B, W, H)
    pipe = orbamd.device.BatchPipeline(torch, W, H, B, nfeatures=nf)
    fr = torch.from_numpy(frames).cuda()
    pipe.extract(fr)
    pipe.check_error()
    torch.cuda.synchronize()
    orc = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    for b in (0, 37, B - 1):
        kg, dg, _ = pipe.host_results(b)
        ko, do = orc(frames[b])
        _compare(kg, dg, ko, do)
        for l in range(8):
            np.testing.assert_array_equal(pipe.ext.pyramid_level(l, frame=b), orc.pyramid(l),
                                          err_msg="frame %d pyramid level %d" % (b, l))
    pipe.close()


@pytest.mark.parametrize("W,offset", [(641, 0), (640, 1)])
def test_large_batch_unaligned_rows_separate_blur(W, offset):
    """A >= 64-frame batch whose level-0 rows are not 4-byte aligned (a 641-byte row pitch, or frames starting one
    byte into the buffer) cannot take the fused describe (k_describe_blur's LDS-DMA moves dwords): the pyramid falls
    back to the per-level kernels, the blur runs in k_blur_strips on the handle's lazily created side stream (its
    buffer allocated at this first unaligned call) and k_describe joins it. Keypoints, descriptors and every pyramid
    level against the oracle, over two steps on one pipeline (the second reuses the side stream and blur buffer)."""
    torch = pytest.importorskip("torch")
    lib = orbamd.load()
    H, B = 480, 64
    frames = orbamd.synth_frames(6, 4, B, W, H)
    buf = torch.zeros(B * H * W + offset, dtype=torch.uint8, device="cuda")
    fr = buf[offset:].view(B, H, W)
    fr.copy_(torch.from_numpy(frames).cuda())
    assert lib.orbx_describe_blur_fused(fr.data_ptr(), fr.stride(0), fr.stride(1)) == 0
    pipe = orbamd.device.BatchPipeline(torch, W, H, B)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    for step in range(2):
        pipe.extract(fr)
        pipe.check_error()
        torch.cuda.synchronize()
        for b in (0, 29, B - 1):
            kg, dg, _ = pipe.host_results(b)
            ko, do = orc(frames[b])
            _compare(kg, dg, ko, do)
            for l in range(8):
                np.testing.assert_array_equal(pipe.ext.pyramid_level(l, frame=b), orc.pyramid(l),
                                              err_msg="step %d frame %d pyramid level %d" % (step, b, l))
    pipe.close()


PARAMS = [
    # (W, H, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST): other my.yaml settings / odd sizes
    (641, 479, 1000, 1.2, 8, 20, 7),
    (320, 240, 500, 1.2, 5, 20, 7),
    (800, 600, 1500, 1.3, 6, 12, 5),
    (512, 384, 800, 1.15, 10, 25, 9),
    (1024, 768, 3000, 1.2, 8, 20, 7),
]


@pytest.mark.parametrize("W,H,nf,sf,nl,ini,mini", PARAMS)
def test_extract_other_parameters(W, H, nf, sf, nl, ini, mini):
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) beyond the default config:
    odd frame sizes, other scale factors / level counts / thresholds (ORBextractor.cc:410-470)."""
    frames = orbamd.synth_frames(1, 2, 2, W, H)
    ext = orbamd.ORBextractor(nf, sf, nl, ini, mini, max_width=W, max_height=H)
    orc = oracle_py.OracleExtractor(nf, sf, nl, ini, mini)
    for f in range(frames.shape[0]):
        kg, dg = ext(frames[f])
        ko, do = orc(frames[f])
        _compare(kg, dg, ko, do)


def test_host_path_graph_replay_and_size_changes():
    """orbx_extract captures its per-frame work as a hipGraph (eager first call per geometry, captured
    second, replayed after): many frames and alternating frame sizes on one handle, every call
    bit-exact vs the oracle, and the eager path (stage profiling on) gives the same."""
    ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7, max_width=752, max_height=480)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    a = orbamd.synth_frames(0, 3, 4, 640, 480)
    b = orbamd.synth_frames(1, 5, 3, 752, 480)
    seq = [a[0], a[1], a[2], b[0], b[1], a[3], b[2]]
    sums = []
    for img in seq:
        kg, dg = ext(img)
        ko, do = orc(img)
        _compare(kg, dg, ko, do)
        sums.append(int(dg.astype(np.int64).sum()))
    ext.close()
    # the eager path (every call launched stage by stage: stage profiling on disables the graph)
    e2 = orbamd.ORBextractor(1000, 1.2, 8, 20, 7, max_width=752, max_height=480)
    assert orbamd.load().orbx_profile_enable(e2._h, 0x1F) == 0
    assert [int(e2(i)[1].astype(np.int64).sum()) for i in seq] == sums
    e2.close()


def test_host_path_keeps_the_sticky_batch_error():
    """an error raised by a device batch stays set across host-path extractions (orbx_extract has its own
    per-call word) until orbx_check_error reports it, once (the host path used to zero it)"""
    W, H = 640, 480
    frames = orbamd.synth_frames(0, 0, 2, W, H)
    ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7, max_width=W, max_height=H)
    lib = orbamd.load()
    ext(frames[0])
    assert lib.orbx_check_error(ext._h, None) == 0
    assert lib.orbx_debug_raise_error(ext._h, 4, None) == 0
    kg, _ = ext(frames[1])  # a host-path call between the failing batch and the check
    assert len(kg) > 900
    assert lib.orbx_check_error(ext._h, None) == -2  # ORBX_EDEVICE
    assert lib.orbx_check_error(ext._h, None) == 0   # cleared by the read


def test_host_pyramid_delivery():
    """orbx_set_host_pyramid (the eager mvImagePyramid of the host path, ORBextractor.cc:1107-1132): the levels the
    octree launch's extra workgroups copy into pinned host memory equal the oracle's pyramid on consecutive distinct
    frames (captured-graph replays included) and the device copy (orbx_pyramid_level); ORBX_EARG when off, before the
    first call and for a stage-profiled call; the keypoints stay bit-exact with the copy on."""
    import ctypes as C
    W, H = 752, 480
    frames = orbamd.synth_frames(3, 7, 4, W, H)
    ext = orbamd.ORBextractor(1200, 1.2, 8, 20, 7, max_width=W, max_height=H)
    orc = oracle_py.OracleExtractor(1200, 1.2, 8, 20, 7)
    lib = orbamd.load()
    p, pitch, w, h = C.c_void_p(), C.c_size_t(), C.c_int(), C.c_int()

    def level(lv):
        rc = lib.orbx_host_pyramid_level(ext._h, lv, C.byref(p), C.byref(pitch), C.byref(w), C.byref(h))
        if rc:
            return rc
        buf = (C.c_uint8 * (pitch.value * h.value)).from_address(p.value)
        return np.frombuffer(buf, np.uint8).reshape(h.value, pitch.value)[:, :w.value].copy()

    assert lib.orbx_set_host_pyramid(ext._h, 1) == 0
    assert level(0) == -1  # nothing delivered yet
    for f in range(frames.shape[0]):
        kg, dg = ext(frames[f])
        ko, do = orc(frames[f])
        _compare(kg, dg, ko, do)
        for lv in range(8):
            got = level(lv)
            assert isinstance(got, np.ndarray), (f, lv, got)
            np.testing.assert_array_equal(got, orc.pyramid(lv), err_msg="frame %d level %d" % (f, lv))
            np.testing.assert_array_equal(got, ext.pyramid_level(lv))
    assert lib.orbx_set_host_pyramid(ext._h, 0) == 0
    ext(frames[0])
    assert level(1) == -1  # off: no host copy
    assert lib.orbx_set_host_pyramid(ext._h, 1) == 0
    assert lib.orbx_profile_enable(ext._h, 0x1F) == 0
    ext(frames[1])
    assert level(1) == -1  # a stage-profiled call delivers none
    ext.close()


@pytest.mark.gpu
def test_host_pyramid_caller_targets():
    """orbx_set_host_pyramid_target (the storage of the drop-in's refcounted mvImagePyramid, so a level a caller keeps
    is not overwritten by the next call, as with the reference's per-call Mats, ORBextractor.cc:1114-1115): each call
    fills the registered target set before it, level 0 at offset 0 and levels 1..L-1 after it, bit-exact against the
    oracle, captured-graph replays included; a target filled earlier keeps its frame; a target smaller than
    orbx_host_pyramid_bytes is rejected; NULL returns to the handle's own memory."""
    import ctypes as C
    W, H = 640, 480
    frames = orbamd.synth_frames(4, 3, 5, W, H)
    ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7, max_width=W, max_height=H)
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    lib = orbamd.load()
    assert lib.orbx_set_host_pyramid(ext._h, 1) == 0
    nb = C.c_size_t()
    assert lib.orbx_host_pyramid_bytes(ext._h, W, H, C.byref(nb)) == 0
    page = 4096
    need = (nb.value + page - 1) // page * page
    raw = [np.zeros(need + page, np.uint8) for _ in range(2)]
    tgt = [r[(-r.ctypes.data) % page:][:need] for r in raw]  # page-aligned views
    for t in tgt:
        assert lib.orbx_host_register(t.ctypes.data, need) == 0
    p, pitch, w, h = C.c_void_p(), C.c_size_t(), C.c_int(), C.c_int()

    def level(lv):
        assert lib.orbx_host_pyramid_level(ext._h, lv, C.byref(p), C.byref(pitch), C.byref(w), C.byref(h)) == 0
        buf = (C.c_uint8 * (pitch.value * h.value)).from_address(p.value)
        return p.value, np.frombuffer(buf, np.uint8).reshape(h.value, pitch.value)[:, :w.value].copy()

    try:
        want = []
        for f in range(frames.shape[0]):
            k = f % 2
            assert lib.orbx_set_host_pyramid_target(ext._h, tgt[k].ctypes.data, need) == 0
            kg, dg = ext(frames[f])
            ko, do = orc(frames[f])
            _compare(kg, dg, ko, do)
            lv_f = [orc.pyramid(lv).copy() for lv in range(8)]
            for lv in range(8):
                addr, got = level(lv)
                assert tgt[k].ctypes.data <= addr < tgt[k].ctypes.data + need, (f, lv)
                np.testing.assert_array_equal(got, lv_f[lv], err_msg="frame %d level %d" % (f, lv))
            if f:
                # the other target still holds the previous frame (level 0 at offset 0, w x h contiguous)
                prev = tgt[1 - k][:W * H].reshape(H, W)
                np.testing.assert_array_equal(prev, want[-1][0])
            want.append(lv_f)
        assert lib.orbx_set_host_pyramid_target(ext._h, tgt[0].ctypes.data, need - page) == 0
        img = np.ascontiguousarray(frames[0])
        cap = ext.max_keypoints(W, H)
        kbuf, dbuf, n = np.empty(cap * 24, np.uint8), np.empty(cap * 32, np.uint8), C.c_int()
        rc = lib.orbx_extract(ext._h, img.ctypes.data, W, H, W, kbuf.ctypes.data, dbuf.ctypes.data, cap, C.byref(n))
        assert rc == -1  # ORBX_EARG: the target cannot hold the frame's levels
        assert lib.orbx_set_host_pyramid_target(ext._h, None, 0) == 0
        ext(frames[2])
        addr, got = level(3)
        assert not (tgt[0].ctypes.data <= addr < tgt[0].ctypes.data + need)
        np.testing.assert_array_equal(got, want[2][3])
    finally:
        ext.close()
        for t in tgt:
            assert lib.orbx_host_unregister(t.ctypes.data) == 0
