"""Oracle vs committed regression vectors (tests/golden, made by make_golden.py). No GPU."""
import glob
import hashlib
import os

import numpy as np
import pytest

import oracle_py
import orbamd

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(path):
    g = np.load(path)
    W, H, nf = int(g["W"]), int(g["H"]), int(g["nfeatures"])
    frames = orbamd.synth_frames(int(g["agent"]), int(g["t0"]), 2, W, H)
    orc = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    res = []
    for i in range(2):
        assert hashlib.sha256(frames[i].tobytes()).digest() == g["frame_sha%d" % i].tobytes(), "generator drift"
        k, d = orc(frames[i])
        assert np.array_equal(k.view(np.uint8).reshape(-1, 24), g["kps%d" % i])
        assert np.array_equal(d, g["desc%d" % i])
        res.append((k, d))
    t = orc.tables()
    v1 = orbamd.KeyFrameView(res[1][0], res[1][1], t["scale"], t["sigma2"])
    v0 = orbamd.KeyFrameView(res[0][0], res[0][1], t["scale"], t["sigma2"])
    n, m = oracle_py.search_for_triangulation(v1, v0, g["F12"], float(g["ex"]), float(g["ey"]), False, False)
    assert n == int(g["tri_n"]) and np.array_equal(m, g["tri_match"])
