"""CPU: the oracle's Frame-level restatements (oracle/orb_oracle_frame.c) against independent
numpy/pure-Python restatements written from the reference text.

Frame::ComputeStereoMatches (ORB_SLAM2.1/src/Frame.cc:470-641) is restated below line by line
with float32 scalars; parity with the reference itself is unpinned (OpenCV absent).
"""
import numpy as np
import pytest

import oracle_py
import orbamd

f32 = np.float32


def roundf(v):
    """C roundf (half away from zero) for v >= 0; v - floor(v) is exact for floats."""
    fl = np.floor(v)
    return f32(fl + (1 if v - fl >= 0.5 else 0))


def stereo_py(ol, orr, kl, dl, kr, dr, mbf, mb):
    """Pure-Python restatement of Frame::ComputeStereoMatches (Frame.cc:470-641)."""
    tabs = ol.tables()
    scale, inv = tabs["scale"], tabs["inv_scale"]
    N = len(kl)
    ur = np.full(N, -1, np.float32)
    dp = np.full(N, -1, np.float32)
    nRows = ol.level_size(0)[1]
    rows = [[] for _ in range(nRows)]
    for iR in range(len(kr)):
        y = f32(kr["y"][iR])
        r = f32(2.0) * scale[kr["octave"][iR]]
        maxr = int(np.ceil(f32(y + r)))
        minr = int(np.floor(f32(y - r)))
        for yi in range(minr, maxr + 1):
            rows[yi].append(iR)
    maxD = f32(mbf) / f32(mb)
    pyrL = [ol.pyramid(l) for l in range(8)]
    pyrR = [orr.pyramid(l) for l in range(8)]
    hd = np.unpackbits(dl, axis=1)
    hr = np.unpackbits(dr, axis=1)
    vdi = []
    for iL in range(N):
        lev = int(kl["octave"][iL])
        vL, uL = f32(kl["y"][iL]), f32(kl["x"][iL])
        cand = rows[int(vL)]
        if not cand:
            continue
        minU, maxU = f32(uL - maxD), uL
        best, bestR = 100, 0
        for iR in cand:
            o = int(kr["octave"][iR])
            if o < lev - 1 or o > lev + 1:
                continue
            uR = f32(kr["x"][iR])
            if minU <= uR <= maxU:
                d = int(np.count_nonzero(hd[iL] != hr[iR]))
                if d < best:
                    best, bestR = d, iR
        if best >= 75:
            continue
        sf = inv[lev]
        suL = roundf(f32(uL * sf))
        svL = roundf(f32(vL * sf))
        suR0 = roundf(f32(f32(kr["x"][bestR]) * sf))
        PL, PR = pyrL[lev], pyrR[lev]
        r0, c0 = int(svL) - 5, int(suL) - 5
        IL = PL[r0:r0 + 11, c0:c0 + 11].astype(np.int64)
        IL = IL - IL[5, 5]
        if suR0 < 0 or suR0 + 11 >= PR.shape[1]:
            continue
        vd = []
        for inc in range(-5, 6):
            cc = int(suR0) + inc - 5
            IR = PR[r0:r0 + 11, cc:cc + 11].astype(np.int64)
            IR = IR - IR[5, 5]
            vd.append(int(np.abs(IL - IR).sum()))
        bi = int(np.argmin(vd))  # first minimum, like `dist < bestDist`
        if bi in (0, 10):
            continue
        d1, d2, d3 = f32(vd[bi - 1]), f32(vd[bi]), f32(vd[bi + 1])
        deltaR = f32(f32(d1 - d3) / f32(f32(2) * f32(f32(d1 + d3) - f32(2) * d2)))
        if deltaR < -1 or deltaR > 1:
            continue
        bestuR = f32(scale[lev] * f32(f32(suR0 + f32(bi - 5)) + deltaR))
        disp = f32(uL - bestuR)
        if disp >= 0 and disp < maxD:
            if disp <= 0:
                disp = f32(0.01)
                bestuR = f32(float(uL) - 0.01)
            dp[iL] = f32(f32(mbf) / disp)
            ur[iL] = bestuR
            vdi.append((vd[bi], iL))
    vdi.sort()
    kept = len(vdi)
    if vdi:
        med = f32(vdi[len(vdi) // 2][0])
        th = f32(f32(f32(1.5) * f32(1.4)) * med)
        for d, i in reversed(vdi):
            if f32(d) < th:
                break
            ur[i] = dp[i] = -1
            kept -= 1
    return ur, dp, kept


@pytest.mark.parametrize("W,H,nf,dx,agent", [(752, 480, 1200, 8, 0), (640, 480, 1000, 3, 2),
                                             (1241, 376, 2000, 20, 1)])
def test_stereo_oracle_matches_restatement(W, H, nf, dx, agent):
    L = orbamd.synth_frames(agent, 4, 1, W, H)[0]
    R = orbamd.synth_frames(agent, 4, 1, W, H, dx=dx)[0]
    ol = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    orr = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    kl, dl = ol(L)
    kr, dr = orr(R)
    mbf, mb = 47.90639384423901, 0.11
    ur, dp, n = oracle_py.compute_stereo_matches(ol, orr, kl, dl, kr, dr, mbf, mb)
    ur2, dp2, n2 = stereo_py(ol, orr, kl, dl, kr, dr, mbf, mb)
    assert n == n2 and n > len(kl) // 4
    np.testing.assert_array_equal(ur.view(np.uint32), ur2.view(np.uint32))
    np.testing.assert_array_equal(dp.view(np.uint32), dp2.view(np.uint32))
    # a fronto-parallel scene at disparity dx: the kept matches sit within a pixel of it
    v = ur >= 0
    assert np.abs((kl["x"][v] - ur[v]) - dx).max() < 2.5


def test_stereo_oracle_no_right_keypoints():
    W, H = 640, 480
    L = orbamd.synth_frames(0, 0, 1, W, H)[0]
    ol = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    orr = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    kl, dl = ol(L)
    orr(np.full((H, W), 128, np.uint8))  # flat right image: no keypoints
    ur, dp, n = oracle_py.compute_stereo_matches(ol, orr, kl, dl, kl[:0], dl[:0], 40.0, 0.1)
    assert n == 0 and (ur == -1).all() and (dp == -1).all()
