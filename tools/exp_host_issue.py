#!/usr/bin/env python3
"""Experiment: is the bench step bound by the host's issue of it? Runs the bench schedule (orbamd.agent.AgentSchedule,
C2, 1024 frames over 4 graphs, 2-batch pool) with and without the per-step exchange and reports, per step, the host
time spent inside sched.step() (the Python + HIP API issue of every launch) against the GPU's step time (wall clock
over many steps, synchronised at both ends). Timing only (no check)."""
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
    frames = orbamd.synth_frames(0, 0, 2 * B, W, H)
    steps = 400
    def run(sched, xchg, tag):
        for i in range(20):
            sched.step(xchg=xchg, first=i == 0)
        torch.cuda.synchronize()
        issue = 0.0
        t = time.perf_counter()
        for i in range(steps):
            a = time.perf_counter()
            sched.step(xchg=xchg, first=i == 0)
            issue += time.perf_counter() - a
        torch.cuda.synchronize()
        wall = time.perf_counter() - t
        print("%-34s frames/s %.0f  step %.3f ms  host issue per step %.3f ms (%.0f %% of the step)"
              % (tag, B * steps / wall, wall / steps * 1e3, issue / steps * 1e3, 100 * issue / wall), flush=True)

    # one configuration per process (HIP stream / HW queue assignment starts fresh): A = the bench's exchange object
    # with the exchange issued, A0 = the same object with it skipped, B = an object built without the exchange
    # (bench.py --no-exchange), C = B plus the exchange's vocabulary created afterwards, D = B plus one more matcher
    # context (one more HIP stream) created afterwards
    cfg = os.environ.get("XCFG", "A")
    sched = AgentSchedule(torch, frames, W, H, P, device=0, pool=2, exchange=cfg in ("A", "A0"))
    extra = None
    if cfg == "C":
        from orbamd.agent import SYNTH_VOC_SEED
        from orbamd.vocabulary import L1_NORM, TF_IDF, ORBVocabulary, synth_vocabulary_full
        k, L, par, leaf, vdesc, w = synth_vocabulary_full(seed=SYNTH_VOC_SEED)
        extra = ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, par, leaf, vdesc, w, device=0)
    elif cfg == "D":
        import ctypes as C
        extra = C.c_void_p()
        assert orbamd.load().orbm_create(0, C.byref(extra)) == 0
    for rnd in (1, 2):
        run(sched, cfg == "A", "%s r%d" % (cfg, rnd))
    sched.close()

if __name__ == "__main__":
    main()
