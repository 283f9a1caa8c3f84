#!/usr/bin/env python3
"""A/B experiment: one extraction+match graph over B frames vs P concurrent graphs over B/P frames
each (separate handles and HIP streams), to fill the GPU during the latency-bound tail stages
(octree, describe, match). Prints frames/s per configuration."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cooperative-orb-slam_amd"))


def run(torch, orbamd, frames_np, P, steps=20, warm=3, offset=False):
    B = frames_np.shape[0]
    dev = torch.device("cuda", 0)
    sub = B // P
    pipes = [orbamd.device.BatchPipeline(torch, 640, 480, sub) for _ in range(P)]
    streams = [torch.cuda.Stream(dev, priority=0) for _ in range(P)]
    fr = [torch.from_numpy(frames_np[p * sub:(p + 1) * sub]).to(dev) for p in range(P)]
    torch.cuda.synchronize()

    evs = [torch.cuda.Event() for _ in range(P)]

    def step():
        for p in range(P):
            if offset and p > 0:
                # graph p starts its step once graph p-1's extraction of this step is done: its FAST then
                # overlaps graph p-1's matcher / next pyramid instead of running in lockstep with it
                streams[p].wait_event(evs[p - 1])
            pipes[p].extract(fr[p], streams[p].cuda_stream)
            evs[p].record(streams[p])
            pipes[p].match_pairs(streams[p].cuda_stream)

    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    for p in pipes:
        p.close()
    return B * steps / el


def main():
    import torch
    import orbamd
    cfgs = [(1024, 4, True), (2048, 4, True), (1024, 3, True), (1536, 3, True)]
    for B, P, off in cfgs:
        frames = orbamd.synth_frames(0, 0, B, 640, 480)
        if True:
            if True:
                print("B=%d P=%d offset=%d frames/s=%.0f" % (B, P, off, run(torch, orbamd, frames, P, offset=off)),
                      flush=True)


if __name__ == "__main__":
    main()
