#!/usr/bin/env python3
"""Pass rate of k_fast_cells2's cardinal pretest on the synthetic C2 frames, per threshold
(level 0 only): the share of band pixels whose FAST strength the kernel has to compute."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cooperative-orb-slam_amd"))
import orbamd  # noqa: E402


def main():
    frames = orbamd.synth_frames(0, 0, 2, 640, 480)
    for f in frames:
        im = f.astype(np.int32)
        v = im[3:-3, 3:-3]
        ring = (im[6:, 3:-3], im[3:-3, 6:], im[:-6, 3:-3], im[3:-3, :-6])
        for t in (7, 20):
            b = [c > v + t for c in ring]
            d = [c < v - t for c in ring]
            cand = np.zeros_like(v, dtype=bool)
            for k in range(4):
                cand |= (b[k] & b[(k + 1) % 4]) | (d[k] & d[(k + 1) % 4])
            print("t=%d pass rate %.4f" % (t, cand.mean()))


if __name__ == "__main__":
    main()
