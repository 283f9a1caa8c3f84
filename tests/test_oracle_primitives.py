"""Independent numpy restatements of the OpenCV 3.x primitives vs the oracle (no GPU).

These check the oracle's literal C translation against definitions written from the
published algorithm in a different form (vectorised numpy, pure-Python loops for the
quadtree), so an error has to be made twice to slip through."""
import math

import numpy as np
import pytest

import oracle_py
import orbamd

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1),
        (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast_numpy(img, t):
    """cv::FAST(img, kps, t, nonmax=true) from the definition: 9 contiguous of 16 ring pixels
    all > p+t or all < p-t; score = cornerScore<16>; 3x3 strict NMS; row-major order."""
    img = img.astype(np.int32)
    h, w = img.shape
    sc = np.zeros((h, w), np.int32)
    ys, xs = np.mgrid[3:h - 3, 3:w - 3]
    p = img[3:h - 3, 3:w - 3]
    d = np.stack([p - img[ys + dy, xs + dx] for dx, dy in RING], -1)  # v - ring
    best_dark = np.full(p.shape, -10**9)
    best_bright = np.full(p.shape, -10**9)
    for k in range(16):
        idx = [(k + j) % 16 for j in range(9)]
        best_dark = np.maximum(best_dark, d[..., idx].min(-1))
        best_bright = np.maximum(best_bright, (-d[..., idx]).min(-1))
    corner = (best_dark > t) | (best_bright > t)
    score = np.maximum(np.maximum(best_dark, best_bright), t) - 1
    sc[3:h - 3, 3:w - 3] = np.where(corner, score, 0)
    out = []
    for i in range(3, h - 3):
        for j in range(3, w - 3):
            s = sc[i, j]
            if s > 0 and all(s > sc[i + a, j + b] for a in (-1, 0, 1) for b in (-1, 0, 1) if (a or b)):
                out.append((j, i, s))
    return np.array(out, np.float32).reshape(-1, 3)


@pytest.mark.parametrize("seed,t", [(0, 20), (1, 7), (2, 40), (3, 0)])
def test_fast_matches_definition(seed, t):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (40, 43), dtype=np.uint8)
    img[10:20, 5:30] = 200  # flat region + edges
    got = oracle_py.fast(img, t)
    exp = fast_numpy(img, t)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("t", [0, 7, 20, 60, 255])
def test_fast_vector_form_equals_scalar(t):
    """the oracle's AVX2 FAST step (32 pixels, OpenCV FAST_t's vector form) equals its scalar form: noise,
    flat areas, saturated pixels (v + t > 255, v - t < 0) and every row-tail width; and the whole extractor"""
    rng = np.random.default_rng(100 + t)
    imgs = [rng.integers(0, 256, (48, w), dtype=np.uint8) for w in (7, 35, 36, 37, 67, 68, 100)]
    sat = rng.integers(0, 256, (40, 90), dtype=np.uint8)
    sat[5:30, 10:80] = np.where(rng.random((25, 70)) < 0.5, 0, 255).astype(np.uint8)
    imgs.append(sat)
    try:
        for img in imgs:
            oracle_py.set_fast_simd(True)
            a = oracle_py.fast(img, t)
            oracle_py.set_fast_simd(False)
            b = oracle_py.fast(img, t)
            assert np.array_equal(a, b), img.shape
        if t == 20:
            orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
            for img in orbamd.synth_frames(1, 0, 2, 640, 480):
                oracle_py.set_fast_simd(True)
                ka, da = orc(img)
                oracle_py.set_fast_simd(False)
                kb, db = orc(img)
                assert np.array_equal(ka.view(np.uint8), kb.view(np.uint8)) and np.array_equal(da, db)
    finally:
        oracle_py.set_fast_simd(True)


def test_fast_pretest_lerp_exact():
    """k_fast_cells2's byte-SWAR pretest compares with v_lerp_u8 (per byte (a + b + r) >> 1):
    bright = bit 7 of lerp(lerp(c, 255 - v, r_b), 255 - M_b, 1) must equal c > v + t, and
    notdark = bit 7 of lerp(lerp(c, 255 - v, r_d), 255 - M_d, 1) must equal NOT c < v - t, for every
    (c, v, t) in [0, 255]^3 (t = 255: the bright bound is clamped, so only c > v + t => bright)."""
    c = np.arange(256, dtype=np.int32)[:, None]
    v = np.arange(256, dtype=np.int32)[None, :]

    def lerp(a, b, r):
        return (a + b + r) >> 1

    for t in range(256):
        rb, rd = t & 1, 1 - (t & 1)
        mb_c = min((t + 256 + rb) >> 1, 255)
        md_c = (256 - t - (t & 1)) >> 1
        bright = (lerp(lerp(c, 255 - v, rb), 255 - mb_c, 1) & 0x80) != 0
        notdark = (lerp(lerp(c, 255 - v, rd), 255 - md_c, 1) & 0x80) != 0
        assert lerp(lerp(c, 255 - v, rb), 255 - mb_c, 1).max() <= 255
        if t < 255:
            assert np.array_equal(bright, c > v + t), t
        else:
            assert not (c > v + t).any() or bright[c > v + t].all()
        assert np.array_equal(notdark, ~(c < v - t)), t


def test_fast_on_synthetic_cell_roi():
    frame = orbamd.synth_frames(0, 0, 1, 640, 480)[0]
    roi = frame[100:138, 200:237]
    for t in (20, 7):
        assert np.array_equal(oracle_py.fast(roi, t), fast_numpy(roi, t))


def resize_numpy(src, dw, dh):
    """INTER_LINEAR 8U fixed point (OpenCV 3.x resizeGeneric_, SSE2 vertical span)."""
    sh, sw = src.shape
    scale_x = 1.0 / (dw / sw)
    scale_y = 1.0 / (dh / sh)
    S = src.astype(np.int64)

    def coef(n, scale, limit, clamp_frac):
        f = np.array([np.float32((i + 0.5) * scale - 0.5) for i in range(n)], np.float32)
        si = np.floor(f).astype(np.int64)
        fr = (f - si.astype(np.float32)).astype(np.float32)
        if clamp_frac:
            neg = si < 0
            fr[neg] = 0
            si[neg] = 0
            hi = si >= limit - 1
            fr[hi] = 0
            si[hi] = limit - 1
        a0 = np.rint((np.float32(1) - fr) * np.float32(2048)).astype(np.int64)
        a1 = np.rint(fr * np.float32(2048)).astype(np.int64)
        return si, a0, a1

    sx, a0, a1 = coef(dw, scale_x, sw, True)
    sy, b0, b1 = coef(dh, scale_y, sh, False)
    r0 = np.clip(sy, 0, sh - 1)
    r1 = np.clip(sy + 1, 0, sh - 1)
    sx1 = np.minimum(sx + 1, sw - 1)
    h0 = S[r0][:, sx] * a0 + S[r0][:, sx1] * a1
    h1 = S[r1][:, sx] * a0 + S[r1][:, sx1] * a1
    simd_end = 0
    while simd_end <= dw - 16:
        simd_end += 16
    while simd_end < dw - 4:
        simd_end += 4
    B0, B1 = b0[:, None], b1[:, None]
    v_simd = (((h0 >> 4) * B0) >> 16) + (((h1 >> 4) * B1) >> 16) + 2 >> 2
    v_scal = (h0 * B0 + h1 * B1 + (1 << 21)) >> 22
    v = np.where(np.arange(dw)[None, :] < simd_end, v_simd, v_scal)
    return np.clip(v, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("sw,sh,dw,dh", [(640, 480, 533, 400), (533, 400, 444, 333), (257, 193, 214, 161),
                                         (1241, 376, 1034, 313), (214, 161, 179, 134)])
def test_resize_matches_definition(sw, sh, dw, dh):
    rng = np.random.default_rng(sw)
    src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    assert np.array_equal(oracle_py.resize_linear(src, dw, dh), resize_numpy(src, dw, dh))


def gauss_numpy(src):
    k = np.array([18, 34, 49, 55, 49, 34, 18], np.int64)
    h, w = src.shape
    pad = np.pad(src.astype(np.int64), 3, mode="reflect")  # numpy "reflect" == REFLECT_101
    rows = sum(k[i] * pad[:, i:i + w] for i in range(7))
    s = sum(k[i] * rows[i:i + h, :] for i in range(7))
    rhe = (s + 0x7FFF + ((s >> 16) & 1)) >> 16
    half_up = (s + (1 << 15)) >> 16
    v = np.where(np.arange(w)[None, :] < (w & ~3), rhe, half_up)
    return np.clip(v, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("w,h", [(640, 480), (179, 134), (309, 231), (67, 70)])
def test_gauss_matches_definition(w, h):
    rng = np.random.default_rng(w * h)
    src = rng.integers(0, 256, (h, w), dtype=np.uint8)
    src[:20, :20] = 255  # saturation path
    assert np.array_equal(oracle_py.gauss7(src), gauss_numpy(src))


def test_fast_atan2_close_to_atan2():
    rng = np.random.default_rng(5)
    for y, x in rng.integers(-20000, 20000, (500, 2)):
        a = oracle_py.fast_atan2(float(y), float(x))
        e = math.degrees(math.atan2(y, x)) % 360
        assert abs((a - e + 180) % 360 - 180) < 0.3
    assert oracle_py.fast_atan2(0.0, 0.0) == 0.0


def test_descriptor_distance():
    rng = np.random.default_rng(9)
    for _ in range(200):
        a = rng.integers(0, 256, 32, dtype=np.uint8)
        b = rng.integers(0, 256, 32, dtype=np.uint8)
        assert oracle_py.descriptor_distance(a, b) == int(np.unpackbits(a ^ b).sum())


# ---------------------------------------------------------------- DistributeOctTree ---
def distribute_octtree_py(keys, minX, maxX, minY, maxY, N):
    """Pure-Python literal restatement of ORBextractor.cc:539-763 (std::list semantics,
    pointer tie-break pinned to creation order)."""
    seq = [0]

    class Node:
        def __init__(self, ul, ur, bl, br, ks):
            self.UL, self.UR, self.BL, self.BR, self.k = ul, ur, bl, br, ks
            self.nomore = False
            self.seq = None

    def divide(n):
        hx = math.ceil((n.UR[0] - n.UL[0]) / 2)
        hy = math.ceil((n.BR[1] - n.UL[1]) / 2)
        n1 = Node(n.UL, (n.UL[0] + hx, n.UL[1]), (n.UL[0], n.UL[1] + hy), (n.UL[0] + hx, n.UL[1] + hy), [])
        n2 = Node(n1.UR, n.UR, n1.BR, (n.UR[0], n.UL[1] + hy), [])
        n3 = Node(n1.BL, n1.BR, n.BL, (n1.BR[0], n.BL[1]), [])
        n4 = Node(n3.UR, n2.BR, n3.BR, n.BR, [])
        for kp in n.k:
            if kp[0] < n1.UR[0]:
                (n1 if kp[1] < n1.BR[1] else n3).k.append(kp)
            elif kp[1] < n1.BR[1]:
                n2.k.append(kp)
            else:
                n4.k.append(kp)
        for c in (n1, n2, n3, n4):
            c.nomore = len(c.k) == 1
        return n1, n2, n3, n4

    def create(n):
        n.seq = seq[0]
        seq[0] += 1
        return n

    nIni = int(np.round(np.float32(maxX - minX) / np.float32(maxY - minY)))  # floats: ties irrelevant here
    hX = np.float32(maxX - minX) / np.float32(nIni)
    lst = []
    for i in range(nIni):
        ulx = int(np.float32(hX * np.float32(i)))
        urx = int(np.float32(hX * np.float32(i + 1)))
        lst.append(create(Node((ulx, 0), (urx, 0), (ulx, maxY - minY), (urx, maxY - minY), [])))
    roots = list(lst)
    for kp in keys:
        roots[int(np.float32(kp[0]) / hX)].k.append(kp)
    lst = [n for n in lst if len(n.k) > 0]
    for n in lst:
        n.nomore = len(n.k) == 1
    finish = False
    vsz = []
    while not finish:
        prev = len(lst)
        vsz = []
        nexp = 0
        i = 0
        while i < len(lst):
            n = lst[i]
            if n.nomore:
                i += 1
                continue
            front = []
            for c in divide(n):
                if c.k:
                    create(c)
                    front.insert(0, c)
                    if len(c.k) > 1:
                        nexp += 1
                        vsz.append(c)
            del lst[i]
            lst[:0] = front
            i += len(front)
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + nexp * 3 > N:
            while not finish:
                prev = len(lst)
                vprev = sorted(vsz, key=lambda n: (len(n.k), n.seq))
                vsz = []
                for n in reversed(vprev):
                    front = []
                    for c in divide(n):
                        if c.k:
                            create(c)
                            front.insert(0, c)
                            if len(c.k) > 1:
                                vsz.append(c)
                    lst.remove(n)
                    lst[:0] = front
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    out = []
    for n in lst:
        best = n.k[0]
        for kp in n.k[1:]:
            if kp[2] > best[2]:
                best = kp
        out.append(best)
    return out


@pytest.mark.parametrize("agent,t", [(0, 0), (3, 11)])
def test_octree_matches_python_restatement(agent, t):
    frame = orbamd.synth_frames(agent, t, 1, 640, 480)[0]
    orc = oracle_py.OracleExtractor()
    orc(frame)
    nfeat = orc.tables()["nfeat"]
    for l in (0, 3, 7):
        w, h = orc.level_size(l)
        cand = [tuple(r) for r in orc.candidates(l)]
        exp = distribute_octtree_py(cand, 16, w - 16, 16, h - 16, int(nfeat[l]))
        got = orc.octree(l)
        exp = np.array([(x + 16, y + 16, r) for x, y, r in exp], np.float32)
        assert np.array_equal(got, exp), "level %d" % l
