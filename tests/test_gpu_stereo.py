"""GPU parity: Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641) on the HIP path
(k_stereo over the device-resident pyramids) vs the CPU oracle, bit-exact on mvuRight and
mvDepth (raw float bits) and the kept count."""
import numpy as np
import pytest

import oracle_py
import orbamd

pytestmark = pytest.mark.gpu

MBF, MB = 47.90639384423901, 0.11  # EuRoC-like rig: fx 435.2, baseline 0.11 m


def _pair(agent, t, W, H, dx):
    return orbamd.synth_frames(agent, t, 1, W, H)[0], orbamd.synth_frames(agent, t, 1, W, H, dx=dx)[0]


def _check(ur, dp, n, uo, do, no):
    assert n == no, "kept %d vs oracle %d" % (n, no)
    bad = np.nonzero(ur.view(np.uint32) != uo.view(np.uint32))[0]
    assert bad.size == 0, "mvuRight differs at %s: %s vs %s" % (bad[:5], ur[bad[:5]], uo[bad[:5]])
    bad = np.nonzero(dp.view(np.uint32) != do.view(np.uint32))[0]
    assert bad.size == 0, "mvDepth differs at %s: %s vs %s" % (bad[:5], dp[bad[:5]], do[bad[:5]])


@pytest.mark.parametrize("W,H,nf,dx,agent,t", [(752, 480, 1200, 8, 0, 0), (752, 480, 1200, 17, 3, 9),
                                               (1241, 376, 2000, 12, 1, 2), (640, 480, 1000, 1, 2, 33),
                                               (640, 480, 1000, 26, 5, 7)])
def test_stereo_host_path_bit_exact(W, H, nf, dx, agent, t):
    L, R = _pair(agent, t, W, H, dx)
    el = orbamd.ORBextractor(nf, 1.2, 8, 20, 7, max_width=W, max_height=H)
    er = orbamd.ORBextractor(nf, 1.2, 8, 20, 7, max_width=W, max_height=H)
    ol = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    orr = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    kl, dl = el(L)
    kr, dr = er(R)
    ko, do_ = ol(L)
    kro, dro = orr(R)
    assert kl.tobytes() == ko.tobytes() and kr.tobytes() == kro.tobytes()
    ur, dp, n = orbamd.compute_stereo_matches(el, er, kl, dl, kr, dr, MBF, MB)
    uo, dpo, no = oracle_py.compute_stereo_matches(ol, orr, ko, do_, kro, dro, MBF, MB)
    assert n > 0
    _check(ur, dp, n, uo, dpo, no)


def test_stereo_empty_and_mismatched():
    W, H = 640, 480
    L, R = _pair(0, 0, W, H, 8)
    el = orbamd.ORBextractor(1000, 1.2, 8, 20, 7)
    er = orbamd.ORBextractor(1000, 1.2, 8, 20, 7)
    kl, dl = el(L)
    kr, dr = er(np.full((H, W), 77, np.uint8))
    assert len(kr) == 0
    ur, dp, n = orbamd.compute_stereo_matches(el, er, kl, dl, kr, dr, MBF, MB)
    assert n == 0 and (ur == -1).all() and (dp == -1).all()
    # same handle on both sides is rejected (its single-frame pyramid holds one image)
    with pytest.raises(RuntimeError):
        orbamd.compute_stereo_matches(el, el, kl, dl, kl, dl, MBF, MB)


def test_stereo_batch_device_matches_oracle():
    torch = pytest.importorskip("torch")
    W, H, nf, B = 752, 480, 1200, 6
    dev = torch.device("cuda", 0)
    left = orbamd.synth_frames(4, 10, B, W, H)
    right = orbamd.synth_frames(4, 10, B, W, H, dx=9)
    # one handle holding left and right images in one batch (frames 0..B-1 left, B..2B-1 right)
    ext = orbamd.ORBextractor(nf, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=2 * B)
    stride = ext.max_keypoints(W, H)
    frames = torch.from_numpy(np.concatenate([left, right])).to(dev)
    kps = torch.empty((2 * B, stride, 6), dtype=torch.float32, device=dev)
    desc = torch.empty((2 * B, stride, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    ext.extract_batch_device(frames, kps, desc, cnt, st)
    fl = torch.arange(B, dtype=torch.int32, device=dev)
    fr = fl + B
    ur = torch.empty((B, stride), dtype=torch.float32, device=dev)
    dp = torch.empty((B, stride), dtype=torch.float32, device=dev)
    ns = torch.zeros(B, dtype=torch.int32, device=dev)
    orbamd.frame.stereo_matches_batch_device(ext, ext, fl, fr, kps, desc, cnt, kps, desc, cnt, MBF, MB, ur, dp, ns,
                                             st)
    torch.cuda.synchronize()
    assert orbamd.load().orbx_check_error(ext._h, st) == 0
    ol = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    orr = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    for p in range(B):
        ko, do_ = ol(left[p])
        kro, dro = orr(right[p])
        n = int(cnt[p].item())
        assert n == len(ko)
        uo, dpo, no = oracle_py.compute_stereo_matches(ol, orr, ko, do_, kro, dro, MBF, MB)
        _check(ur[p, :n].cpu().numpy(), dp[p, :n].cpu().numpy(), int(ns[p].item()), uo, dpo, no)
