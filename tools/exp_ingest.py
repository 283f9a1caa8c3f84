#!/usr/bin/env python3
"""Ingest-leg experiment: the bench schedule with every step's frames uploaded from pinned host
memory (bench.run_ingest), over copy-stream counts and chunk shapes, beside the box's raw pinned H2D bandwidth (one
stream and 4 streams of large copies, nothing else on the GPU). Prints one line per setting.

usage: python3 tools/exp_ingest.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cooperative-orb-slam_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import orbamd  # noqa: E402
from orbamd.agent import AgentSchedule  # noqa: E402


def raw_h2d(nstreams, mb=1536, reps=4):
    dev = torch.device("cuda", 0)
    per = mb * (1 << 20) // nstreams
    src = [torch.empty(per, dtype=torch.uint8).pin_memory() for _ in range(nstreams)]
    dst = [torch.empty(per, dtype=torch.uint8, device=dev) for _ in range(nstreams)]
    st = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for s, a, b in zip(st, src, dst):
            with torch.cuda.stream(s):
                b.copy_(a, non_blocking=True)
    torch.cuda.synchronize()
    return reps * nstreams * per / (time.perf_counter() - t0) / 1e9


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    W, H, B, P, pool = 640, 480, 3072, 3, 2
    for n in (1, 2, 4, 8):
        print("raw pinned H2D, %d stream(s): %.1f GB/s" % (n, raw_h2d(n)), flush=True)
    frames = orbamd.synth_frames(0, 0, pool * B, W, H, scene=0)
    sched = AgentSchedule(torch, frames, W, H, P, device=0, pool=pool)
    for i in range(5):
        sched.step(first=i == 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        sched.step(first=i == 0)
    torch.cuda.synchronize()
    print("resident: %.1f frames/s" % (steps * B / (time.perf_counter() - t0)), flush=True)
    for nst, ch in ((3, 1), (4, 2), (4, 4), (4, 8), (8, 4), (8, 8), (12, 4), (16, 8), (3, 1), (4, 4)):
        r = bench.run_ingest(torch, sched, frames, pool, steps, B, W, H, 1, False, None, lambda v, dtype=None: v, nst, ch)
        print("ingest %2d copy streams, %d chunks/graph: %.1f frames/s, %.2f GB/s" % (
            nst, r["chunks_per_graph"], r["frames_per_s"], r["h2d_GBs_per_gpu"]), flush=True)
    sched.close()


if __name__ == "__main__":
    main()
