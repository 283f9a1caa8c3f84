#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz -- regression vectors produced by the CPU oracle.

The reference ships no tests or fixtures and cannot be compiled here without OpenCV/DBoW2
stand-ins (DESIGN.md "Oracle"), so these vectors pin the oracle against drift (and give the
GPU parity tests a second, stored target); they do not pin it to a reference binary.
Inputs are the deterministic synthetic frames (orbx_synth_frames), stored by seed.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "cooperative-orb-slam_amd"), os.path.join(ROOT, "oracle")]
import oracle_py  # noqa: E402
import orbamd  # noqa: E402

CASES = [
    # name, W, H, nfeatures, agent, t0, nframes
    ("c2_640x480_1000", 640, 480, 1000, 0, 0, 2),
    ("c3_752x480_1200", 752, 480, 1200, 1, 3, 2),
    ("c4_1241x376_2000", 1241, 376, 2000, 2, 7, 2),
]


def main():
    F12, ex, ey = orbamd.device.default_geometry()
    for name, W, H, nf, agent, t0, n in CASES:
        orc = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
        tabs = orc.tables()
        frames = orbamd.synth_frames(agent, t0, n, W, H)
        out = {"W": W, "H": H, "nfeatures": nf, "agent": agent, "t0": t0, "F12": F12, "ex": ex, "ey": ey}
        res = []
        for i in range(n):
            k, d = orc(frames[i])
            out["kps%d" % i] = k.view(np.uint8).reshape(-1, 24)
            out["desc%d" % i] = d
            out["frame_sha%d" % i] = np.frombuffer(__import__("hashlib").sha256(frames[i].tobytes()).digest(),
                                                   np.uint8)
            res.append((k, d))
        v1 = orbamd.KeyFrameView(res[1][0], res[1][1], tabs["scale"], tabs["sigma2"])
        v0 = orbamd.KeyFrameView(res[0][0], res[0][1], tabs["scale"], tabs["sigma2"])
        nm, m = oracle_py.search_for_triangulation(v1, v0, F12, ex, ey, False, False)
        out["tri_match"] = m
        out["tri_n"] = nm
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, [len(r[0]) for r in res], "matches", nm)


if __name__ == "__main__":
    main()
