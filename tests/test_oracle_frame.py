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


# ------------------------------------------------------------------ SearchByProjection
import proj_scenes as ps  # noqa: E402


def grid_py(F):
    g = {}
    for i in range(F.n):
        px = int(roundf_signed(f32(f32(F.x[i] - F.min_x) * F.grid_w_inv)))
        py = int(roundf_signed(f32(f32(F.y[i] - F.min_y) * F.grid_h_inv)))
        if 0 <= px < 64 and 0 <= py < 48:
            g.setdefault((px, py), []).append(i)
    return g


def roundf_signed(v):
    return roundf(v) if v >= 0 else -roundf(-v)


def area_py(F, g, x, y, r, minL=-1, maxL=-1):
    """Frame::GetFeaturesInArea (Frame.cc:332-389)."""
    x, y, r = f32(x), f32(y), f32(r)
    x0 = max(0, int(np.floor(f32(f32(f32(x - F.min_x) - r) * F.grid_w_inv))))
    if x0 >= 64:
        return []
    x1 = min(63, int(np.ceil(f32(f32(f32(x - F.min_x) + r) * F.grid_w_inv))))
    if x1 < 0:
        return []
    y0 = max(0, int(np.floor(f32(f32(f32(y - F.min_y) - r) * F.grid_h_inv))))
    if y0 >= 48:
        return []
    y1 = min(47, int(np.ceil(f32(f32(f32(y - F.min_y) + r) * F.grid_h_inv))))
    if y1 < 0:
        return []
    check = minL > 0 or maxL >= 0
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for k in g.get((ix, iy), []):
                if check:
                    if F.octave[k] < minL:
                        continue
                    if maxL >= 0 and F.octave[k] > maxL:
                        continue
                if abs(f32(F.x[k] - x)) < r and abs(f32(F.y[k] - y)) < r:
                    out.append(k)
    return out


def local_py(F, mp, th, nnratio):
    """ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) (ORBmatcher.cc:45-129)."""
    g = grid_py(F)
    bits = np.unpackbits(F.desc, axis=1)
    occ = F.occupied.astype(bool).copy()
    match = np.full(F.n, -1, np.int32)
    nm = 0
    for i in range(mp.n):
        if not mp.track_in_view[i] or mp.bad[i]:
            continue
        lvl = int(mp.track_level[i])
        r = f32(2.5) if float(mp.track_view_cos[i]) > 0.998 else f32(4.0)
        if th != 1.0:
            r = f32(r * f32(th))
        rad = f32(r * F.scale_factors[lvl])
        qb = np.unpackbits(mp.desc[i])
        best, bl, best2, bl2, bi = 256, -1, 256, -1, -1
        for idx in area_py(F, g, mp.track_proj_x[i], mp.track_proj_y[i], rad, lvl - 1, lvl):
            if occ[idx]:
                continue
            if F.uright is not None and F.uright[idx] > 0:
                if abs(f32(mp.track_proj_xr[i] - F.uright[idx])) > rad:
                    continue
            dist = int(np.count_nonzero(bits[idx] != qb))
            if dist < best:
                best2, best, bl2, bl, bi = best, dist, bl, int(F.octave[idx]), idx
            elif dist < best2:
                bl2, best2 = int(F.octave[idx]), dist
        if best <= 100:
            if bl == bl2 and f32(best) > f32(f32(nnratio) * f32(best2)):
                continue
            match[bi] = i
            occ[bi] = bool(mp.has_obs[i])
            nm += 1
    return nm, match


@pytest.mark.parametrize("seed,stereo,th", [(1, True, 3.0), (2, False, 1.0), (3, True, 5.0)])
def test_projection_local_oracle_matches_restatement(seed, stereo, th):
    F, mps = ps.local_scene(seed, stereo)
    n, m = oracle_py.search_by_projection_local(F, mps, th, 0.8)
    n2, m2 = local_py(F, mps, th, 0.8)
    assert n == n2 and n > F.n // 4
    np.testing.assert_array_equal(m, m2)


def test_projection_variants_oracle_sanity():
    F, Tcw, mps, Tl = ps.last_frame_scene(4)
    n, m = oracle_py.search_by_projection_last_frame(F, Tcw, mps, Tl, 7.0, False, True)
    assert n > F.n // 4 and n >= (m >= 0).sum()  # has_obs == 0 claimers can be overwritten (last wins)
    F, Tcw, mps = ps.keyframe_scene(5)
    n, m = oracle_py.search_by_projection_keyframe(F, Tcw, mps, 10.0, 100, True)
    assert n > F.n // 4 and n == (m >= 0).sum()  # every claim occupies
    F, Scw, mps = ps.sim3_scene(6)
    n, m = oracle_py.search_by_projection_sim3(F, Scw, mps, 10)
    assert n > F.n // 8 and n == (m >= 0).sum()


# ------------------------------------------------------------------ Fuse x2 (ORBmatcher.cc:825-1100)
import ctypes as _C  # noqa: E402

_libm = _C.CDLL("libm.so.6")
_libm.logf.restype = _C.c_float
_libm.logf.argtypes = [_C.c_float]


def _gemm33_fast(A, x, c):
    """cv::Mat A*x + c, 3x3 by 3x1 (OpenCV's small-matrix gemm: float products and sums, + c in double)."""
    out = []
    for i in range(3):
        t0 = f32(f32(f32(A[i][0] * x[0]) + f32(A[i][1] * x[1])) + f32(A[i][2] * x[2]))
        out.append(f32(float(t0) + float(c[i])))
    return out


def _norm3(v):
    return f32(np.sqrt(sum(float(a) * float(a) for a in v)))


def _dot3(a, b):
    return sum(float(x) * float(y) for x, y in zip(a, b))


def _predict_scale(max_dist, d, F):
    """MapPoint::PredictScale (MapPoint.cc:385-417), logf of the float ratio."""
    ratio = f32(f32(max_dist) / f32(d))
    n = int(np.ceil(f32(f32(_libm.logf(float(ratio))) / f32(F.log_scale_factor))))
    return min(max(n, 0), len(F.scale_factors) - 1)


def fuse_py(F, mp, th, R, t, Ow, inv=None, sim3=False):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th) (ORBmatcher.cc:825-975) or, with sim3, Fuse(pKF, Scw,
    vpPoints, th, vpReplacePoint) (:977-1100): per MapPoint the bestIdx that the reference fuses."""
    g = grid_py(F)
    bits = np.unpackbits(F.desc, axis=1)
    best = np.full(mp.n, -1, np.int32)
    for i in range(mp.n):
        if mp.skip[i] or mp.bad[i]:
            continue
        p = [f32(v) for v in mp.pos[i]]
        pc = _gemm33_fast(R, p, t)
        if pc[2] < f32(0):
            continue
        invz = f32(1.0 / float(pc[2])) if sim3 else f32(f32(1) / pc[2])
        u = f32(f32(f32(F.fx) * f32(pc[0] * invz)) + f32(F.cx))
        v = f32(f32(f32(F.fy) * f32(pc[1] * invz)) + f32(F.cy))
        if not (u >= F.min_x and u < F.max_x and v >= F.min_y and v < F.max_y):
            continue
        ur = f32(u - f32(f32(F.bf) * invz))
        PO = [f32(p[k] - f32(Ow[k])) for k in range(3)]
        d3 = _norm3(PO)
        if d3 < f32(f32(0.8) * f32(mp.min_dist[i])) or d3 > f32(f32(1.2) * f32(mp.max_dist[i])):
            continue
        if _dot3(PO, mp.normal[i]) < 0.5 * float(d3):
            continue
        lvl = _predict_scale(mp.max_dist[i], d3, F)
        rad = f32(f32(th) * f32(F.scale_factors[lvl]))
        qb = np.unpackbits(mp.desc[i])
        bd, bi = 1 << 30, -1
        for idx in area_py(F, g, u, v, rad):
            kl = int(F.octave[idx])
            if kl < lvl - 1 or kl > lvl:
                continue
            if not sim3:
                ex, ey = f32(u - F.x[idx]), f32(v - F.y[idx])
                if F.uright is not None and F.uright[idx] >= 0:
                    er = f32(ur - F.uright[idx])
                    e2 = f32(f32(f32(ex * ex) + f32(ey * ey)) + f32(er * er))
                    if float(f32(e2 * inv[kl])) > 7.8:
                        continue
                else:
                    e2 = f32(f32(ex * ex) + f32(ey * ey))
                    if float(f32(e2 * inv[kl])) > 5.99:
                        continue
            dist = int(np.count_nonzero(bits[idx] != qb))
            if dist < bd:
                bd, bi = dist, idx
        if bd <= 50:
            best[i] = bi
    return int((best >= 0).sum()), best


@pytest.mark.parametrize("seed,stereo,th", [(3, True, 3.0), (4, False, 3.0), (5, True, 5.0)])
def test_fuse_oracle_matches_restatement(seed, stereo, th):
    F, Tcw, Ow, mps, inv = ps.fuse_scene(seed, stereo)
    n, b = oracle_py.fuse(F, Tcw, Ow, mps, th, inv)
    R = [[f32(Tcw[r][c]) for c in range(3)] for r in range(3)]
    t = [f32(Tcw[r][3]) for r in range(3)]
    n2, b2 = fuse_py(F, mps, th, R, t, Ow, inv)
    assert n == n2 and n > mps.n // 4
    np.testing.assert_array_equal(b, b2)


def test_fuse_sim3_oracle_matches_restatement():
    F, Scw, mps = ps.fuse_sim3_scene(6)
    n, b = oracle_py.fuse_sim3(F, Scw, mps, 4.0)
    scw = f32(np.sqrt(sum(float(Scw[0][c]) * float(Scw[0][c]) for c in range(3))))
    inv = f32(1.0 / float(scw))
    R = [[f32(Scw[r][c] * inv) for c in range(3)] for r in range(3)]
    t = [f32(Scw[r][3] * inv) for r in range(3)]
    Ow = [f32(-sum(float(R[k][i]) * float(t[k]) for k in range(3))) for i in range(3)]
    n2, b2 = fuse_py(F, mps, 4.0, R, t, Ow, sim3=True)
    assert n == n2 and n > mps.n // 4
    np.testing.assert_array_equal(b, b2)


# ------------------------------------------------------------------ ComputeDistinctiveDescriptors
def distinctive_scene(seed, big=False):
    rng = np.random.default_rng(seed)
    sizes = list(rng.integers(0, 70, 300)) + [1, 2, 3, 0]
    if big:
        sizes += [1100, 1500]
    rows = []
    for n in sizes:
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        obs = np.repeat(base[None], n, 0)
        if n:
            obs = ps.flip_bits(rng, obs, 30)
            dup = rng.random(n) < 0.1  # exact duplicates -> median ties
            obs[dup] = obs[0]
        rows.append(obs)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    return off, np.concatenate(rows).astype(np.uint8)


def distinctive_py(off, desc):
    out = []
    for p in range(len(off) - 1):
        d = desc[off[p]:off[p + 1]]
        n = len(d)
        if n == 0:
            out.append(-1)
            continue
        bits = np.unpackbits(d, axis=1).astype(np.int32)
        D = (bits[:, None, :] != bits[None, :, :]).sum(-1)
        med = np.sort(D, axis=1)[:, int(0.5 * (n - 1))]
        out.append(int(np.argmin(med)))  # first minimum
    return np.array(out, np.int32)


def test_distinctive_oracle_matches_restatement():
    off, desc = distinctive_scene(1)
    np.testing.assert_array_equal(oracle_py.compute_distinctive_descriptors(off, desc), distinctive_py(off, desc))


# ------------------------------------------------------------------ SearchForInitialization (ORBmatcher.cc:405-520)
def init_py(F1, F2, prev, window, nnratio, check_ori):
    """literal restatement: in-order queries, vMatchedDistance / vnMatches21 with stealing, rotation bins
    that keep stolen entries, ComputeThreeMaxima, vbPrevMatched update"""
    g = grid_py(F2)
    b2 = np.unpackbits(F2.desc, axis=1)
    m12 = np.full(F1.n, -1, np.int32)
    md = np.full(F2.n, 2 ** 31 - 1, np.int64)
    m21 = np.full(F2.n, -1, np.int64)
    hist = [[] for _ in range(30)]
    nm = 0
    for i1 in range(F1.n):
        l1 = int(F1.octave[i1])
        if l1 > 0:
            continue
        cand = area_py(F2, g, prev[i1, 0], prev[i1, 1], float(window), l1, l1)
        if not cand:
            continue
        qb = np.unpackbits(F1.desc[i1])
        best, best2, bi = 2 ** 31 - 1, 2 ** 31 - 1, -1
        for i2 in cand:
            dist = int(np.count_nonzero(b2[i2] != qb))
            if md[i2] <= dist:
                continue
            if dist < best:
                best2, best, bi = best, dist, i2
            elif dist < best2:
                best2 = dist
        if best <= 50 and f32(best) < f32(f32(best2) * f32(nnratio)):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                nm -= 1
            m12[i1], m21[bi], md[bi] = bi, i1, best
            nm += 1
            if check_ori:
                rot = f32(F1.angle[i1] - F2.angle[bi])
                if rot < 0:
                    rot = f32(rot + f32(360))
                b = int(roundf(float(f32(rot * f32(1.0 / 30)))))
                hist[0 if b == 30 else b].append(i1)
    if check_ori:
        sizes = [len(h) for h in hist]
        i1s = [-1, -1, -1]
        m = [0, 0, 0]
        for i, sz in enumerate(sizes):
            if sz > m[0]:
                m, i1s = [sz, m[0], m[1]], [i, i1s[0], i1s[1]]
            elif sz > m[1]:
                m, i1s = [m[0], sz, m[1]], [i1s[0], i, i1s[1]]
            elif sz > m[2]:
                m[2], i1s[2] = sz, i
        if m[1] < f32(f32(0.1) * f32(m[0])):
            i1s[1] = i1s[2] = -1
        elif m[2] < f32(f32(0.1) * f32(m[0])):
            i1s[2] = -1
        for i in range(30):
            if i in i1s:
                continue
            for idx1 in hist[i]:
                if m12[idx1] >= 0:
                    m12[idx1] = -1
                    nm -= 1
    prev = prev.copy()
    for i1 in np.nonzero(m12 >= 0)[0]:
        prev[i1] = (F2.x[m12[i1]], F2.y[m12[i1]])
    return nm, m12, prev


@pytest.mark.parametrize("seed,noise,check_ori,ratio", [(1, 0.0, True, 0.9), (2, 3.0, True, 0.9), (3, 0.0, False, 0.7)])
def test_search_for_initialization_oracle_matches_restatement(seed, noise, check_ori, ratio):
    F1, F2, prev = ps.init_scene(seed, prev_noise=noise)
    n, m, p = oracle_py.search_for_initialization(F1, F2, prev, 100, ratio, check_ori)
    n2, m2, p2 = init_py(F1, F2, prev, 100, ratio, check_ori)
    assert n == n2 and n > 100
    np.testing.assert_array_equal(m, m2)
    np.testing.assert_array_equal(p, p2)


# ------------------------------------------------------------------ SearchBySim3 (ORBmatcher.cc:1102-1326)
def sim3_py(KF1, T1w, mp1, KF2, T2w, mp2, s12, R12, t12, th):
    inv_s = f32(1.0 / float(s12))
    sR12 = [[f32(R12[r][c] * s12) for c in range(3)] for r in range(3)]
    sR21 = [[f32(R12[c][r] * inv_s) for c in range(3)] for r in range(3)]
    t21 = [f32(-float(f32(f32(f32(sR21[r][0] * t12[0]) + f32(sR21[r][1] * t12[1])) + f32(sR21[r][2] * t12[2]))))
           for r in range(3)]
    fx, fy, cx, cy = KF1.fx, KF1.fy, KF1.cx, KF1.cy

    def direction(KF, T, mp, sR, t):
        g = grid_py(KF)
        bits = np.unpackbits(KF.desc, axis=1)
        R = [[f32(T[r][c]) for c in range(3)] for r in range(3)]
        tw = [f32(T[r][3]) for r in range(3)]
        out = np.full(mp.n, -1, np.int32)
        for i in range(mp.n):
            if mp.skip[i] or mp.bad[i]:
                continue
            pc = _gemm33_fast(sR, _gemm33_fast(R, [f32(v) for v in mp.pos[i]], tw), t)
            if pc[2] < 0:
                continue
            invz = f32(1.0 / float(pc[2]))
            u = f32(f32(fx * f32(pc[0] * invz)) + cx)
            v = f32(f32(fy * f32(pc[1] * invz)) + cy)
            if not (u >= KF.min_x and u < KF.max_x and v >= KF.min_y and v < KF.max_y):
                continue
            d3 = _norm3(pc)
            if d3 < f32(f32(0.8) * mp.min_dist[i]) or d3 > f32(f32(1.2) * mp.max_dist[i]):
                continue
            lvl = _predict_scale(mp.max_dist[i], d3, KF)
            rad = f32(f32(th) * KF.scale_factors[lvl])
            qb = np.unpackbits(mp.desc[i])
            bd, bi = 2 ** 31 - 1, -1
            for idx in area_py(KF, g, u, v, rad):
                if KF.octave[idx] < lvl - 1 or KF.octave[idx] > lvl:
                    continue
                dist = int(np.count_nonzero(bits[idx] != qb))
                if dist < bd:
                    bd, bi = dist, idx
            if bd <= 100:
                out[i] = bi
        return out

    v1 = direction(KF2, T1w, mp1, sR21, t21)
    v2 = direction(KF1, T2w, mp2, sR12, [f32(x) for x in t12])
    m12 = np.full(mp1.n, -1, np.int32)
    for i1 in range(mp1.n):
        if v1[i1] >= 0 and v2[v1[i1]] == i1:
            m12[i1] = v1[i1]
    return int((m12 >= 0).sum()), m12


@pytest.mark.parametrize("seed", [2, 5])
def test_search_by_sim3_oracle_matches_restatement(seed):
    sc = ps.sim3_pair_scene(seed)
    n, m = oracle_py.search_by_sim3(*sc)
    n2, m2 = sim3_py(*sc)
    assert n == n2 and n > 100
    np.testing.assert_array_equal(m, m2)
