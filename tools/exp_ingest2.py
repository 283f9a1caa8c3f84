#!/usr/bin/env python3
"""Ingest-leg coupling experiment (round 6): with 2 resident batches, the upload of step i waits (a stream wait on
the copy stream) for step i-2 to finish on every graph. The copy streams share the process's 4 hardware queues with
the graph streams, so that wait can hold a graph's queue while a later graph of step i-2 is still running; which
graph it holds depends on the queue the copy stream landed on, i.e. on how many streams were created before it.
Interleaved rounds of: pool 2 / 3 batches x stream wait / host wait, fresh copy streams per run, and pool 3 with
one set of copy streams reused.

usage: python3 tools/exp_ingest2.py [steps] [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cooperative-orb-slam_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import orbamd  # noqa: E402
from orbamd.agent import AgentSchedule  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    W, H, B, P, pool = 640, 480, 3072, 3, 3
    frames = orbamd.synth_frames(0, 0, pool * B, W, H, scene=0)
    sched = AgentSchedule(torch, frames, W, H, P, device=0, pool=pool)
    for i in range(5):
        sched.step(first=i == 0)
    torch.cuda.synchronize()
    fixed = [torch.cuda.Stream(0) for _ in range(4)]
    ident = lambda v, dtype=None: v  # noqa: E731
    variants = [("pool2 stream-wait", 2, False, None), ("pool3 stream-wait", 3, False, None),
                ("pool2 host-wait", 2, True, None), ("pool3 host-wait", 3, True, None),
                ("pool3 stream-wait fixed", 3, False, fixed)]
    for r in range(rounds):
        for name, up, hw, cs in variants:
            res = bench.run_ingest(torch, sched, frames, up, steps, B, W, H, 1, False, None, ident, 4, 8,
                                   copy_streams=cs, host_wait=hw)
            print("r%d %-24s %.1f frames/s %.2f GB/s" % (r, name, res["frames_per_s"], res["h2d_GBs_per_gpu"]),
                  flush=True)
    sched.close()


if __name__ == "__main__":
    main()
