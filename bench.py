#!/usr/bin/env python3
"""bench.py -- frames/s of ORB extract + match (BASELINE.json metric) on 1..N MI355X.

One step = one pass of the hot path over one batch of B synthetic 640x480 frames already
resident in HBM:  ORBextractor::operator() on every frame (nfeatures 1000, 1.2, 8 levels,
FAST 20/7) + SearchForTriangulation of frame b against frame b-1 (one BoW node holding all
features = the BASELINE "BF" configuration) + the cooperative exchange: each agent packs its
latest keyframe (keypoints + descriptors) and RCCL-all-gathers it, then matches it against
every agent's slot. One process per GPU = one agent; frames are
agent-private, so per-GPU work is fixed as N grows ("weak" scaling). The B frames of a step are
split over P concurrent extraction+match graphs (own handle and HIP stream each; frame b of a
graph is matched against frame b-1 of the same graph), staggered so that one graph's FAST
overlaps another graph's latency-bound tail (octree, describe, match) -- default 1024 frames as
4 graphs of 256.

Launch (N>1): python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
              --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cooperative-orb-slam_amd"))

VALU_PEAK_GINST = 1228.8  # 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU op (G wave-instr/s)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def level_sizes(W, H, nlevels=8, scale=1.2):
    """Level sizes exactly as ComputePyramid (ORBextractor.cc:1111-1112) with float math."""
    import numpy as np
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(scale))))
    out = []
    for sc in s:
        inv = np.float32(1.0) / sc
        out.append((int(np.rint(np.float32(W) * inv)), int(np.rint(np.float32(H) * inv))))
    return out


def algorithmic_bytes(W, H, nkp):
    """Per-frame algorithmic HBM bytes (DESIGN.md "Roofline"): the SURVEY 8(d) figure
    B_extract = sum_l W_l*H_l (read each level once) + sum_{l>=1} W_l*H_l (write levels 1..7)
    + 64*N, and the per-stage split used for the dominant-kernel roofline."""
    ls = level_sizes(W, H)
    px = [w * h for w, h in ls]
    total = sum(px) + sum(px[1:]) + 64 * nkp
    per_stage = {
        "pyramid": sum(px[:-1]) + sum(px[1:]),   # read level l-1, write level l
        "fast_cells": sum(px),                   # read every level once
        "octree": 0,                             # candidate keys only (reported, not priced)
        "blur": 2 * sum(px),                     # read + write every level
        "describe": nkp * (31 * 31 + 37 * 37 + 56),  # IC patch + BRIEF patch + 24B kp + 32B desc
    }
    return total, per_stage


def cpu_baseline(frames, seconds, threads):
    """Oracle ("port") timed on host cores: extract + BF SearchForTriangulation vs the previous
    frame, one independent frame stream per thread (ctypes releases the GIL). Returns frames/s,
    frames, seconds, and the per-stage seconds per frame summed over the threads' extractors
    (oracle stage timers + the matcher timed around its call)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    import orbamd
    F12, ex, ey = orbamd.device.default_geometry()
    count = [0] * threads
    stage = [None] * threads
    match_s = [0.0] * threads
    stop = time.perf_counter() + seconds

    def work(tid):
        orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
        tabs = orc.tables()
        prev = None
        i = tid
        while time.perf_counter() < stop:
            img = frames[i % len(frames)]
            k, d = orc(img)
            cur = orbamd.KeyFrameView(k, d, tabs["scale"], tabs["sigma2"])
            if prev is not None:
                tm = time.perf_counter()
                oracle_py.search_for_triangulation(cur, prev, F12, ex, ey, False, False)
                match_s[tid] += time.perf_counter() - tm
            prev = cur
            count[tid] += 1
            i += threads
        stage[tid] = orc.stage_times()[0]

    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    n = max(sum(count), 1)
    per = {k: sum(st[k] for st in stage) / n for k in stage[0]}
    per["match"] = sum(match_s) / max(n - threads, 1)
    return sum(count) / el, sum(count), el, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="frames per step per GPU")
    ap.add_argument("--pipes", type=int, default=4,
                    help="concurrent extraction+match graphs per GPU (each over batch/pipes frames, own handle "
                         "and HIP stream), staggered: graph p starts a step when graph p-1 finished extracting it")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--prio", choices=("none", "lead", "lead1"), default="none",
                    help="HIP stream priorities of the graphs: lead = the first half of the staggered graphs (the ones "
                         "in their latency-bound tail stages) high, lead1 = graph 0 only")
    ap.add_argument("--no-exchange", action="store_true")
    ap.add_argument("--stagger", choices=("each", "once", "none"), default="each",
                    help="graph p starts extracting after graph p-1's extraction: every step / only in the "
                         "first step of a run (the phase offset then persists) / never")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    import orbamd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal hooks (defaults = the product setting): ORBAMD_DIST_BACKEND=gloo and
    # ORBAMD_BENCH_DEVICE=0 run a multi-rank bench on a one-GPU box (tools/rehearse_ranks.sh)
    backend = os.environ.get("ORBAMD_DIST_BACKEND", "nccl")
    local = int(os.environ.get("ORBAMD_BENCH_DEVICE", local))
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    W, H, B, P = args.width, args.height, args.batch, args.pipes
    assert B % P == 0, "--batch must be a multiple of --pipes"
    sub = B // P
    frames_np = orbamd.synth_frames(rank, 0, B, W, H)  # agent = rank
    frames = [torch.from_numpy(frames_np[p * sub:(p + 1) * sub]).to(dev) for p in range(P)]
    pipes = [orbamd.device.BatchPipeline(torch, W, H, sub, device=local) for _ in range(P)]
    lo_prio, hi_prio = torch.cuda.Stream.priority_range()
    n_hi = {"none": 0, "lead": P // 2, "lead1": 1}[args.prio]
    streams = [torch.cuda.Stream(dev, priority=hi_prio if p < n_hi else lo_prio) for p in range(P)]
    pipe = pipes[0]
    slot_bytes = pipe.slot_bytes()
    my_slot = torch.zeros(slot_bytes, dtype=torch.uint8, device=dev)
    all_slots = torch.zeros(world * slot_bytes, dtype=torch.uint8, device=dev)
    xmatch = torch.empty((world, pipe.stride), dtype=torch.int32, device=dev)
    xn = torch.zeros(world, dtype=torch.int32, device=dev)

    ag_events = []  # (start, end) around the all-gather alone, timed steps only

    def exchange(ag=None):
        # this agent's latest keyframe -> RCCL all-gather -> match against every agent's slot
        with torch.cuda.stream(streams[0]):
            pipe.pack(0, my_slot, streams[0].cuda_stream)
            if ag is not None:
                ag[0].record(streams[0])
            if world > 1:
                dist.all_gather_into_tensor(all_slots, my_slot)
            else:
                all_slots.copy_(my_slot)
            if ag is not None:
                ag[1].record(streams[0])
            pipe.match_packed(0, all_slots, world, xmatch, xn, streams[0].cuda_stream)

    done = [torch.cuda.Event() for _ in range(P)]

    def step(ev=None, xev=None, extract=True, match=True, xchg=True, first=True):
        for p in range(P):
            st = streams[p].cuda_stream
            if extract:
                if p > 0 and (args.stagger == "each" or (args.stagger == "once" and first)):
                    # staggered graphs: graph p's extraction (FAST-heavy) overlaps graph p-1's matcher and the
                    # latency-bound tail stages instead of running in lockstep with them
                    streams[p].wait_event(done[p - 1])
                pipes[p].extract(frames[p], st)
                done[p].record(streams[p])
            if match:
                if ev is not None:
                    ev[p][0].record(streams[p])
                pipes[p].match_pairs(st)
                if ev is not None:
                    ev[p][1].record(streams[p])
        if xchg and not args.no_exchange:
            if xev is not None:
                xev[0].record(streams[0])
            ag = None
            if xev is not None:
                ag = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ag_events.append(ag)
            exchange(ag)
            if xev is not None:
                xev[1].record(streams[0])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    lib = orbamd.load()
    import ctypes as C
    stages = ["pyramid", "fast_cells", "octree", "blur", "describe"]

    def run_profiled(mask, nsteps, timed):
        """nsteps steps with HIP event pairs around the stages in `mask` (each on the stream its
        kernel runs on; the overlapped schedule is unchanged) and torch events around the matcher."""
        for pp in pipes:
            lib.orbx_profile_enable(pp.ext._h, mask)
        evs = [[[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(P)]
               for _ in range(nsteps)]
        xevs = [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(nsteps)]
        if timed and world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for i in range(nsteps):
            step(evs[i], xevs[i], first=i == 0)
        torch.cuda.synchronize()
        if timed and world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        acc = [0.0] * 5
        ncalls = 0
        for pp in pipes:
            ms = (C.c_double * 5)()
            nc = C.c_int()
            lib.orbx_profile_read(pp.ext._h, ms, C.byref(nc))
            lib.orbx_profile_enable(pp.ext._h, 0)
            for i in range(5):
                acc[i] += ms[i]
            ncalls += nc.value
        st = {k: acc[i] / max(ncalls, 1) for i, k in enumerate(stages) if (mask >> i) & 1}
        st["match"] = sum(e[p][0].elapsed_time(e[p][1]) for e in evs for p in range(P)) / (nsteps * P)
        if not args.no_exchange:
            st["exchange"] = sum(x[0].elapsed_time(x[1]) for x in xevs) / nsteps
            st["allgather"] = sum(a.elapsed_time(b) for a, b in ag_events) / max(len(ag_events), 1)
            ag_events.clear()
        return elapsed, st

    def run_part(nsteps, **kw):
        """untimed breakdown pass: wall time of nsteps steps doing only part of the work"""
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nsteps):
            step(first=i == 0, **kw)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    # 1) stage split (untimed): every stage bracketed, same schedule
    _, stage_ms = run_profiled(0x1F, args.steps, False)
    dom = max(stages, key=lambda k: stage_ms[k])
    # 2) timed region: only the dominant kernel bracketed (its live launch duration for the roofline)
    el, dom_live = run_profiled(1 << stages.index(dom), args.steps, True)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # 3) extract-only and match-only rates, untimed breakdown passes; and the box's
    # measured device-to-device copy bandwidth (read + write bytes of a 1 GiB copy) beside the nominal peak
    copy_gbs = None
    if rank == 0:
        a = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        b2 = torch.empty_like(a)
        b2.copy_(a)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        for _ in range(5):
            b2.copy_(a)
        c1.record()
        torch.cuda.synchronize()
        copy_gbs = 2.0 * 5 * (1 << 30) / (c0.elapsed_time(c1) * 1e-3) / 1e9
        del a, b2
    extract_fps = B * args.steps / run_part(args.steps, match=False, xchg=False)
    match_pps = B * args.steps / run_part(args.steps, extract=False, xchg=False)
    nkp = float(sum(pp.counts.float().mean().item() for pp in pipes) / P)
    nmatch = float(sum(pp.nmatch.float().mean().item() for pp in pipes) / P)

    total_frames = world * B * args.steps
    value = total_frames / el
    result = None
    if rank == 0:
        b_frame, per_stage = algorithmic_bytes(W, H, nkp)
        dom_ms = dom_live[dom]
        # one launch of the dominant kernel processes one graph's sub-batch (B / P frames)
        achieved = per_stage[dom] * sub / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 and per_stage[dom] > 0 else 0.0
        traffic = valu_insts = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            try:
                rec = json.load(open(pmc_path)).get(dom, {})
                traffic = rec.get("hbm_bytes_per_launch")
                valu_insts = rec.get("valu_insts_per_launch")
            except Exception:
                traffic = valu_insts = None
        result = {
            "metric": "frames/sec ORB extract+match, 640x480 mono, 1000 feat/frame",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic textured pan, SURVEY.md 8(d)); resident in HBM",
            "config": {"workload": "C2: synthetic %dx%d uint8, nfeatures 1000, scale 1.2, 8 levels, FAST 20/7; "
                                   "extract + BF SearchForTriangulation vs previous frame + per-step keyframe "
                                   "all-gather & cross-agent match" % (W, H),
                       "frames_per_step_per_gpu": B, "graphs_per_gpu": P,
                       "parallelism": "agent-per-gpu x%d" % world},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "algorithmic_bytes_per_launch": per_stage[dom] * sub,
                         "launch_ms": round(dom_ms, 4),
                         "measured_copy_GBs": round(copy_gbs, 1) if copy_gbs else None,
                         "frac_vs_copy": round(achieved / copy_gbs, 5) if copy_gbs else None},
            # what actually bounds these byte/integer kernels: vector-instruction issue
            # (wave64 VALU op = 2 cycles on a SIMD-32; 1024 SIMDs at 2.4 GHz)
            "valu_issue": None if not valu_insts else {
                "insts_per_launch": valu_insts, "achieved_Ginst_s": round(valu_insts / (dom_ms * 1e-3) / 1e9, 1),
                "peak_Ginst_s": VALU_PEAK_GINST, "frac": round(valu_insts / (dom_ms * 1e-3) / 1e9 / VALU_PEAK_GINST, 4)},
            "pipeline_hbm": {"bytes_per_frame": b_frame, "achieved_GBs": round(b_frame * value / world / 1e9, 2),
                             "frac": round(b_frame * value / world / 1e9 / HBM_PEAK_GBS, 5)},
            "stage_ms_per_step": {k: round(v, 4) for k, v in stage_ms.items()},
            "per_gpu_frames_per_s": round(value / world, 2),
            "extract_only_frames_per_s_per_gpu": round(extract_fps, 1),
            "match_only_pairs_per_s_per_gpu": round(match_pps, 1),
            "kp_per_frame": round(nkp, 1),
            "matches_per_pair": round(nmatch, 1),
        }
    # the CPU baseline is measured at N=1 only (rank 0); multi-GPU lines report null
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        # median of 5 short runs on all host cores, then the reference's own
        # architecture: one Tracking thread ((i), median of 3), with the oracle's stage split
        runs = [cpu_baseline(frames_np, args.cpu_seconds / 5, threads) for _ in range(5)]
        fps = sorted(r[0] for r in runs)[2]
        nfr, sec = sum(r[1] for r in runs), sum(r[2] for r in runs)
        runs1 = [cpu_baseline(frames_np, max(args.cpu_seconds / 6, 1.0), 1) for _ in range(3)]
        fps1, nfr1, sec1, per1 = sorted(runs1, key=lambda r: r[0])[1]
        result["cpu_baseline"] = {"value": round(fps, 2), "unit": "frames/s", "cores": threads, "kind": "port",
                                  "sample": "median of 5 runs, %d synthetic 640x480 frames in %.1f s in total (extract + "
                                            "BF triangulation vs previous) on %d threads, oracle/orb_oracle.c -O3 "
                                            "-ffp-contract=off; 1-thread leg: median of 3 runs (%d frames in %.1f s)"
                                            % (nfr, sec, threads, nfr1, sec1),
                                  "value_1thread": round(fps1, 2),
                                  "stage_ms_per_frame_1thread": {k: round(v * 1e3, 3) for k, v in per1.items()}}
        result["speedup_vs_cpu"] = round(value / fps, 1)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    for pp in pipes:
        pp.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
