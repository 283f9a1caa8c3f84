#!/usr/bin/env python3
"""Experiment: the cost of the per-step exchange as the agent count grows, on ONE GPU.

The bench step at N agents does, per rank, the same extraction + intra-agent matching as at N=1 plus a
cross-agent SearchForTriangulation of its keyframe against N slots. This runs the bench schedule
(orbamd.agent.AgentSchedule) with world=K slots filled by a device-side replicate of this agent's slot
instead of the RCCL all-gather (so the all-gather's xGMI latency is NOT included) and reports the step
rate with the exchange on and off and the exchange stage time. Results are timing only (no check)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cooperative-orb-slam_amd"))


def main():
    import torch
    import orbamd
    from orbamd.agent import AgentSchedule
    W, H, B, P = 640, 480, 1024, 4
    frames = orbamd.synth_frames(0, 0, B, W, H)
    steps = int(os.environ.get("XS_STEPS", "200"))

    def replicate(out, inp):
        out.view(-1, inp.numel()).copy_(inp.view(1, -1).expand(out.numel() // inp.numel(), -1))

    for K in [int(k) for k in os.environ.get("XS_K", "1 2 4 8").split()]:
        sched = AgentSchedule(torch, frames, W, H, P, device=0, rank=0, world=K,
                              allgather=replicate if K > 1 else None)
        res = {}
        for xchg in (True, False):
            for _ in range(20):
                sched.step(xchg=xchg)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(steps):
                sched.step(xchg=xchg, first=i == 0)
            torch.cuda.synchronize()
            res[xchg] = B * steps / (time.perf_counter() - t)
        # exchange alone (pack + replicate + slot match), back to back on graph 0's stream
        st = sched.streams[0]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(st)
        for _ in range(50):
            sched.exchange()
        e1.record(st)
        torch.cuda.synchronize()
        print("K=%d frames/s with exchange %.0f without %.0f (%.1f%%); exchange alone %.1f us" %
              (K, res[True], res[False], 100.0 * (res[True] / res[False] - 1.0), e0.elapsed_time(e1) / 50 * 1e3),
              flush=True)
        sched.close()


if __name__ == "__main__":
    main()
