#!/usr/bin/env python3
"""bench.py -- frames/s of ORB extract + match (BASELINE.json metric) on 1..N MI355X.

One step = one pass of the hot path over one batch of B synthetic frames already resident in HBM
(orbamd.agent.AgentSchedule): ORBextractor::operator() on every frame (C2: nfeatures 1000, 1.2,
8 levels, FAST 20/7) + SearchForTriangulation of frame b against frame b-1 (one BoW node holding
all features = the BASELINE "BF" configuration) + the cooperative exchange: each agent packs its
latest keyframe into a keyframe slot, RCCL-all-gathers it, then matches it against every agent's
slot. One process per GPU = one agent; frames are agent-private, so
per-GPU work is fixed as N grows ("weak" scaling). The B frames are split over P concurrent,
staggered extraction+match graphs (default 3840 frames as 3 graphs of 1280).

After the timed region the run checks itself: every graph's device error flags, then sampled
frames (first / middle / last of every graph) with their match rows and the cross-agent matches,
bit-compared against the CPU oracle (oracle/check_schedule.py, the checker); "bit_exact" in the
JSON line, exit status 3 on a mismatch. The frames form a pool of --pool resident batches and
consecutive steps process consecutive batches, so the last step's correct outputs differ from the
step before: a stage that stopped launching fails the check ("stale_guard").

Beside `value` (frames already in HBM) the "ingest" leg reports the rate with every step's frames
uploaded from pinned host memory on a copy stream, overlapped with the previous step's compute
(ORBextractor::operator() takes a host image, ORBextractor.cc:1043-1050).

--config c2 (default, the BASELINE metric) | c3 (752x480, 1200 features) | c4 (1241x376, 2000
features): the BASELINE configs 3 (EuRoC MH01 stereo) and 4 (KITTI 00 stereo) as the stereo frames they name:
each frame is a rectified left/right pair (synthetic: the right image is the left crop shifted by a fixed
disparity), both images extracted, Frame::ComputeStereoMatches on the device, and SearchForTriangulation's stereo
branch against the previous frame (ORB_SLAM2.1/src/Frame.cc:80-92, 471-645; ORBmatcher.cc:703-749); `value` is
stereo frames (pairs) per second. --mono runs their left images alone (the rounds 1-5 lines).

Launch (N>1): python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
              --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
(--dist at N=1 under torch.distributed.run: the same RCCL process group and out-of-place all-gather
as N>1, with one rank.)
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cooperative-orb-slam_amd"))

VALU_PEAK_GINST = 1228.8  # 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU op (G wave-instr/s)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
ALONE_LAUNCHES = 7  # roofline.alone: launches of the priced kernel with nothing else on the GPU (median)
FP4_MFMA_PEAK_TOPS = 10000.0  # dense fp4 (MX-scaled f8f6f4) MFMA, 4x the 2.5 PF dense bf16 rate (MI355X_MICROARCH.md "Matrix cores")

CONFIGS = {
    "c2": dict(W=640, H=480, nfeatures=1000, name="C2: synthetic 640x480 uint8, nfeatures 1000"),
    # stereo: the rig (orbamd.device.STEREO_RIGS: Camera.bf and mb = bf / fx of EuRoC.yaml / KITTI00-02.yaml) and the
    # synthetic right image's disparity in pixels (orbx_synth_scene_frames dx)
    "c3": dict(W=752, H=480, nfeatures=1200, stereo="euroc", dx=11,
               name="C3: synthetic 752x480 uint8 (EuRoC geometry), nfeatures 1200"),
    "c4": dict(W=1241, H=376, nfeatures=2000, stereo="kitti", dx=19,
               name="C4: synthetic 1241x376 uint8 (KITTI geometry), nfeatures 2000"),
}


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
        # the unblurred levels (IC_Angle patches) and the blurred levels (rBRIEF patches) read once each, 24 B
        # keypoint + 32 B descriptor written per keypoint (overlapping patches re-read from L2 are not HBM bytes)
        "describe": 2 * sum(px) + 56 * nkp,
    }
    return total, per_stage


def describe_touched_bytes(sched, W, H, fused):
    """describe's algorithmic HBM bytes per frame, from this run's keypoints (first / middle / last frame of every
    graph in the last step): the union, per level, of the level pixels its patches read, each read once (patches of
    neighbouring keypoints overlap; the overlap is an L2 hit, not HBM traffic), plus 56 B written per keypoint
    (24 B keypoint + 32 B descriptor). Fused (k_describe_blur): the unblurred 43x43 window around each keypoint
    (the blur's source rows and columns +-21, which contain IC_Angle's 31x31 window); separate blur: the unblurred
    31x31 IC_Angle window plus the blurred 37x37 rBRIEF window."""
    import numpy as np
    ls = level_sizes(W, H)
    scale = [np.float32(1.0)]
    for _ in range(1, len(ls)):
        scale.append(np.float32(np.float64(scale[-1]) * np.float64(np.float32(1.2))))
    tot, nfr = 0.0, 0
    for p in range(sched.P):
        for b in sorted({0, sched.sub // 2, sched.sub - 1}):
            k = sched.frame_results(p, b)[0]
            nb = 56 * len(k)
            for lv, (w, h) in enumerate(ls):
                sel = k[k["octave"] == lv]
                if not len(sel):
                    continue
                xs = np.rint(sel["x"] / scale[lv]).astype(np.int64)
                ys = np.rint(sel["y"] / scale[lv]).astype(np.int64)
                for r in ((21,) if fused else (15, 18)):
                    m = np.zeros((h, w), bool)
                    for x, y in zip(xs, ys):
                        m[max(y - r, 0):y + r + 1, max(x - r, 0):x + r + 1] = True
                    nb += int(m.sum())
            tot += nb
            nfr += 1
    return tot / max(nfr, 1)


def host_cpu_info():
    """nproc / affinity / cgroup quota / CPU model of the host this process runs on."""
    info = {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "model": None}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
    except Exception:
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return info


def cpu_baseline(frames, threads, seconds=None, nframes=None, nfeatures=1000, stereo=None):
    """Oracle ("port") timed on host cores: extract + BF SearchForTriangulation vs the previous
    frame, one independent frame stream per thread (ctypes releases the GIL). Stops after `seconds`
    or once `nframes` frames are done in total. Returns frames/s, frames, seconds, per-stage seconds
    per frame (oracle stage timers + the matcher timed around its call). stereo=(mbf, mb): frames are
    [N, 2, H, W] pairs and a frame is the stereo Frame's work: both images extracted (the reference runs the
    two extractions on two threads, Frame.cc:80-81; here each thread's frame stream runs them in turn, and
    every core runs its own stream), ComputeStereoMatches, and the stereo SearchForTriangulation."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    import orbamd
    F12, ex, ey = orbamd.device.default_geometry()
    count = [0] * threads
    stage = [None] * threads
    match_s = [0.0] * threads
    stop = time.perf_counter() + (seconds if seconds else 1e9)
    total = [0]
    lock = threading.Lock()

    stereo_s = [0.0] * threads

    def work(tid):
        orc = oracle_py.OracleExtractor(nfeatures, 1.2, 8, 20, 7)
        orr = oracle_py.OracleExtractor(nfeatures, 1.2, 8, 20, 7) if stereo else None
        tabs = orc.tables()
        prev = None
        i = tid
        while time.perf_counter() < stop:
            if nframes is not None:
                with lock:
                    if total[0] >= nframes:
                        break
                    total[0] += 1
            img = frames[i % len(frames)]
            ur = None
            if stereo:
                k, d = orc(img[0])
                kr, dr = orr(img[1])
                ts = time.perf_counter()
                ur = oracle_py.compute_stereo_matches(orc, orr, k, d, kr, dr, stereo[0], stereo[1])[0]
                stereo_s[tid] += time.perf_counter() - ts
            else:
                k, d = orc(img)
            cur = orbamd.KeyFrameView(k, d, tabs["scale"], tabs["sigma2"], uright=ur)
            if prev is not None:
                tm = time.perf_counter()
                oracle_py.search_for_triangulation(cur, prev, F12, ex, ey, False, False)
                match_s[tid] += time.perf_counter() - tm
            prev = cur
            count[tid] += 1
            i += threads
        stage[tid] = orc.stage_times()[0]
        if stereo:  # both extractors' stage timers
            for k2, v in orr.stage_times()[0].items():
                stage[tid][k2] = stage[tid].get(k2, 0.0) + v

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
    if stereo:
        per["stereo"] = sum(stereo_s) / n
    return sum(count) / el, sum(count), el, per


def run_ingest(torch, sched, frames_np, pool, nsteps, B, W, H, world, use_dist, dist, reduce_max, nstreams=4,
               chunks=0, copy_streams=None, host_wait=False):
    """The schedule with every step's B frames uploaded from pinned host memory (the frame pool, batch
    i mod pool at step i) into the device batch the step processes, on `nstreams` copy streams whatever the
    graph count (several DMA engines in flight: round 3's fourth copy stream was +36 %, and tying the streams to
    the graphs lost it when the step went to 3 graphs): each graph's frames are cut into ceil(nstreams / P)
    contiguous chunks dealt round-robin over the streams in graph order, and graph p starts extracting as soon
    as its own chunks have arrived. Upload i waits for step i-pool (the previous user of that device batch), so
    an upload overlaps the previous step's compute. Returns frames/s over nsteps after `pool` warm-up steps and
    the H2D rate achieved (bytes per frame uploaded, max over ranks). chunks: chunks per graph (0: ceil(nstreams / P)).
    pool may be below the schedule's batch count (the first `pool` batches are cycled); copy_streams: reuse these
    streams instead of creating nstreams; host_wait: the host waits for the batch's previous user (step i - pool) to
    finish before enqueueing its upload, instead of a stream wait on the copy streams."""
    P, sub, dev = sched.P, sched.sub, sched.dev
    per = sched.images_per_frame  # 2 for stereo pairs (left + right image per frame)
    host = [torch.from_numpy(sched.host_batch(frames_np, r)).pin_memory() for r in range(pool)]
    copy_st = list(copy_streams) if copy_streams else [torch.cuda.Stream(dev) for _ in range(max(1, nstreams))]
    nst = len(copy_st)
    k = chunks or -(-nst // P)  # chunks per graph (default: enough to give every copy stream one)
    imgs = per * sub
    cuts = [(j * imgs // k, (j + 1) * imgs // k) for j in range(k)]
    up = [[[torch.cuda.Event() for _ in range(k)] for _ in range(P)] for _ in range(pool)]
    done = [[torch.cuda.Event() for _ in range(P)] for _ in range(pool)]
    used = [False] * pool

    def one(i):
        r = i % pool
        if host_wait and used[r]:
            for e in done[r]:
                e.synchronize()
        for p in range(P):
            dst = sched.device_images(r, p)
            for j, (a, b) in enumerate(cuts):
                cs = copy_st[(p * k + j) % nst]
                with torch.cuda.stream(cs):
                    if used[r] and not host_wait:
                        for e in done[r]:
                            cs.wait_event(e)
                    dst[a:b].copy_(host[r][p * imgs + a:p * imgs + b], non_blocking=True)
                    up[r][p][j].record(cs)
        sched.step(batch=r, wait=up[r], first=i == 0)
        for p in range(P):
            done[r][p].record(sched.streams[p])
        used[r] = True

    for i in range(pool):
        one(i)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(nsteps):
        one(pool + i)
    torch.cuda.synchronize()
    el = reduce_max(time.perf_counter() - t0)
    fps = world * B * nsteps / el
    return {"frames_per_s": round(fps, 1), "per_gpu_frames_per_s": round(fps / world, 1),
            "h2d_GBs_per_gpu": round(per * B * W * H * nsteps / el / 1e9, 2), "steps": nsteps, "seconds": round(el, 3),
            "copy_streams": nst, "chunks_per_graph": k, "upload_waits": "host" if host_wait else "stream",
            "source": "pinned host memory, %d batches of %d frames uploaded round-robin (one batch per step) on %d "
                      "copy streams (%d chunks per graph), overlapped with the previous step's compute; each graph "
                      "starts on its own frames' arrival; an upload waits for the batch's previous step (%s)"
                      % (pool, B, nst, k, "on the host" if host_wait else "stream wait on the copy streams")}


def launch_ranks(n, argv):
    """`bench.py --gpus N` called directly (no WORLD_SIZE in the environment) with N > 1: start N ranks
    under torch.distributed.run as a child process and exit with its status (rank 0 prints the JSON line
    to the inherited stdout). Runs before anything in this process touches the GPU. With the product
    backend (nccl = RCCL) every rank needs its own visible device."""
    import socket
    import subprocess
    backend = os.environ.get("ORBAMD_DIST_BACKEND", "nccl")
    if backend == "nccl" and "ORBAMD_BENCH_DEVICE" not in os.environ:
        import torch  # device_count() does not initialise the GPU on this image
        ndev = torch.cuda.device_count()
        if n > ndev:
            print("bench.py: --gpus %d needs %d visible GPUs (one agent per GPU over RCCL); %d visible"
                  % (n, n, ndev), file=sys.stderr, flush=True)
            return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


def default_batch(per):
    """frames per step per GPU: 3 graphs of 1280 frames (C2; 3 x 1024 measured 2.5 % slower on the round-6 kernels,
    3 x 1536 equal, 3 x 1792 / 2048 and 2 x 2048 slower: profiles/r06zk_shape*.log), or 1536 stereo pairs (3 x 512 pairs =
    1024 images per graph at C3 / C4, where 3 x 640 pairs is equal)"""
    return 3840 if per == 1 else 1536


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per step per GPU (0: 3840 = 3 graphs of 1280, or 1536 stereo pairs = 3072 images at "
                         "c3 / c4)")
    ap.add_argument("--mono", action="store_true",
                    help="c3 / c4: their left images alone (monocular frames) instead of the stereo pairs the configs name")
    ap.add_argument("--pipes", type=int, default=3,
                    help="concurrent extraction+match graphs per GPU (each over batch/pipes frames, own handle "
                         "and HIP stream), staggered: graph p starts a step when graph p-1 finished extracting it")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="all-cores CPU leg: total seconds (5 runs)")
    ap.add_argument("--cpu-frames-1t", type=int, default=0,
                    help="1-thread CPU leg: frames (0 = 2000 at c2, 1000 at c3/c4)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this process may use (affinity set capped by the cgroup quota)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the post-run bit-exact check")
    ap.add_argument("--prio", choices=("none", "lead", "lead1"), default="none",
                    help="HIP stream priorities of the graphs: lead = the first half of the staggered graphs (the ones "
                         "in their latency-bound tail stages) high, lead1 = graph 0 only")
    ap.add_argument("--no-exchange", action="store_true")
    ap.add_argument("--alias-frames", action="store_true",
                    help="measurement hook (orbx_debug_alias_frames): every frame of a graph's batch is its frame 0 and "
                         "shares one pyramid / blur buffer, so every stage reads L2-resident data (the L2-residency "
                         "bound, DESIGN.md 6.0); outputs are frame 0's, the self-check is skipped")
    ap.add_argument("--serial-stages", action="store_true",
                    help="measurement hook (orbx_debug_serial): every extraction stage in order on its graph's stream, so "
                         "a kernel trace times each kernel alone (with --pipes 1)")
    ap.add_argument("--exchange-stream", choices=("auto", "own", "graph0"), default="auto",
                    help="where the keyframe exchange runs: its own stream, off graph 0's critical path (only the pack + "
                         "keyframe copy holds graph 0's next extraction), or in order on graph 0's stream; auto = own when "
                         "a collective runs (N > 1, --dist), graph 0's at N = 1 (profiles/r03_exp_exchange_stream.log)")
    ap.add_argument("--roof-kernel", choices=("auto", "pyramid", "fast_cells", "octree", "blur", "describe"),
                    default="auto", help="extraction kernel priced in `roofline` (timed live in the timed region); auto = "
                                         "the largest stage of this run's own stage split")
    ap.add_argument("--sustain", type=float, default=6.0,
                    help="seconds of the untimed sustained pass after the timed region (0: skip)")
    ap.add_argument("--pool", type=int, default=3,
                    help="resident batches of distinct frames; step k processes batch k mod pool (stale-output guard; "
                         "the ingest leg re-uploads batch k mod pool, so its upload for step k waits for step k - pool)")
    ap.add_argument("--dist", action="store_true",
                    help="use torch.distributed and the out-of-place RCCL all-gather even at world 1")
    ap.add_argument("--collective", choices=("rccl", "torch"), default="rccl",
                    help="the keyframe all-gather across ranks: rccl = liborbamd's RCCL communicator (orbx_comm_allgather: "
                         "ncclAllGather on the exchange's own HIP stream, no collective-owned stream; torch.distributed runs "
                         "the gloo control plane: unique-id broadcast, barriers, max-over-ranks timing), torch = "
                         "torch.distributed's ProcessGroupNCCL all_gather_into_tensor (its internal RCCL stream)")
    ap.add_argument("--ingest-streams", type=int, default=4, help="copy streams of the ingest leg")
    ap.add_argument("--ingest-chunks", type=int, default=8,
                    help="upload chunks per graph in the ingest leg, dealt round-robin over the copy streams (4 streams x 8 "
                         "chunks: 53.7 GB/s of the box's 54 GB/s pinned H2D, profiles/r06c_exp_ingest.log)")
    ap.add_argument("--ingest-wait", choices=("host", "stream"), default="host",
                    help="how an upload waits for the batch's previous user (step k - pool): host = the enqueueing thread "
                         "waits on its events before issuing the copies, stream = a stream wait on the copy streams, "
                         "which holds whichever graph's hardware queue the copy stream shares (pool 3: 175-179k vs "
                         "145k frames/s, profiles/r06i_exp_ingest2.log)")
    ap.add_argument("--ingest-steps", type=int, default=100,
                    help="steps of the ingest leg (frames uploaded from pinned host memory each step; 0: skip)")
    ap.add_argument("--scene", choices=("shared", "private"), default="shared",
                    help="shared: every agent (rank) views one synthetic environment from its own crop offset "
                         "(orbx_synth_scene_frames, 12 px per agent along the pan), so the cross-agent matchers find the "
                         "other agents' features as A1 does on A2's keyframes; private: a texture per agent. Rank 0's "
                         "frames are the same in both modes")
    ap.add_argument("--stagger", choices=("each", "once", "none", "every4", "every8", "every16", "pyr_each", "pyr_every8",
                                          "fast_each", "fast_every8", "fast_once"),
                    default="every8",
                    help="graph p starts extracting after graph p-1's extraction: every step / only in the "
                         "first step of a run (the phase offset then persists) / never / in the first step and every "
                         "K-th step after it; pyr_ / fast_: after graph p-1's pyramid / FAST instead (a third of the step "
                         "apart at 3 graphs)")
    ap.add_argument("--launch-frames", action="store_true",
                    help="print the images one stage launch processes (--batch / --pipes frames, x2 for stereo pairs) and "
                         "the graph count, and exit (no GPU use)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    if args.launch_frames:  # images one stage launch processes (stereo: a graph's left + right images)
        per = 1 if args.mono or "stereo" not in cfg else 2
        print(per * ((args.batch or default_batch(per)) // args.pipes), args.pipes)
        return
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import numpy as np
    import torch
    import torch.distributed as dist
    import orbamd
    from orbamd._lib import check as lib_check
    from orbamd.agent import AgentSchedule

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal hooks (defaults = the product setting): ORBAMD_DIST_BACKEND=gloo and
    # ORBAMD_BENCH_DEVICE=0 run a multi-rank bench on a one-GPU box (tools/rehearse_ranks.sh)
    backend = os.environ.get("ORBAMD_DIST_BACKEND", "nccl")
    local = int(os.environ.get("ORBAMD_BENCH_DEVICE", local))
    use_dist = world > 1 or args.dist
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr, flush=True)
        sys.exit(2)
    # the data-path collective: liborbamd's RCCL communicator (default), torch's ProcessGroupNCCL, or (one-GPU
    # rehearsals, ORBAMD_DIST_BACKEND=gloo) gloo through host memory
    coll = args.collective if backend == "nccl" else "gloo"
    if use_dist:
        torch.cuda.set_device(local)
        if coll == "torch":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # control plane only: barriers, max-over-ranks timing, the RCCL unique id
            dist.init_process_group("gloo")
        assert dist.get_world_size() == world
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ctl_dev = dev if coll == "torch" else torch.device("cpu")

    def reduce_max(v, dtype=None):
        """max over ranks of a host number (the whole job's time is its slowest rank's)"""
        if not use_dist:
            return v
        t = torch.tensor([v], dtype=dtype or torch.float64, device=ctl_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item()
    comm = None
    if use_dist and coll == "rccl":
        import ctypes as C
        lib0 = orbamd.load()
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            lib_check(lib0.orbx_comm_unique_id(uid), "orbx_comm_unique_id")
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0)
        uid = (C.c_uint8 * 128).from_buffer_copy(box[0])
        h = C.c_void_p()
        lib_check(lib0.orbx_comm_create(uid, world, rank, local, C.byref(h)), "orbx_comm_create")
        comm = h

    W, H, P = cfg["W"], cfg["H"], args.pipes
    rig = None if args.mono or "stereo" not in cfg else orbamd.device.STEREO_RIGS[cfg["stereo"]]
    per = 2 if rig else 1  # images per frame
    B = args.batch or default_batch(per)
    assert B % P == 0, "--batch must be a multiple of --pipes"
    assert args.pool >= 1
    sub = B // P
    imgs = per * sub  # images one extraction launch processes
    scene = 0 if args.scene == "shared" else None

    def agent_frames(r, t0, n):
        """agent r's frames t0 .. t0+n-1: uint8 [n, H, W], or [n, 2, H, W] stereo pairs (the right image: the crop
        shifted by the config's disparity)"""
        left = orbamd.synth_frames(r, t0, n, W, H, scene=scene)
        if not rig:
            return left
        return np.stack([left, orbamd.synth_frames(r, t0, n, W, H, dx=cfg["dx"], scene=scene)], axis=1)
    frames_np = agent_frames(rank, 0, args.pool * B)  # agent = rank; pool batches back to back
    def allgather(out, inp):
        # RCCL over xGMI on the current (exchange) stream; gloo (the one-GPU rehearsal): through host memory
        if coll == "rccl":
            lib_check(orbamd.load().orbx_comm_allgather(comm, inp.data_ptr(), out.data_ptr(), inp.numel(),
                                                        torch.cuda.current_stream(dev).cuda_stream), "orbx_comm_allgather")
        elif coll == "torch":
            dist.all_gather_into_tensor(out, inp)
        else:
            o = torch.empty(out.numel(), dtype=torch.uint8)
            dist.all_gather_into_tensor(o, inp.cpu().clone())
            out.copy_(o.to(out.device))

    lo_prio, hi_prio = torch.cuda.Stream.priority_range()
    n_hi = {"none": 0, "lead": P // 2, "lead1": 1}[args.prio]
    # auto: torch's collective on the exchange's own stream (off graph 0's chain while it waits on its internal stream);
    # liborbamd's RCCL in order on graph 0's stream, as the N = 1 exchange (no stream beyond the graphs')
    async_x = args.exchange_stream == "own" or (args.exchange_stream == "auto" and use_dist and coll == "torch")
    sched = AgentSchedule(torch, frames_np, W, H, P, device=local, rank=rank, world=world,
                          allgather=allgather if use_dist else None,
                          stagger=args.stagger, exchange=not args.no_exchange,
                          priorities=[hi_prio if p < n_hi else lo_prio for p in range(P)], nfeatures=cfg["nfeatures"],
                          pool=args.pool, async_exchange=async_x, stereo=rig)
    pipes = sched.pipes
    if args.serial_stages:
        for pp in pipes:
            assert orbamd.load().orbx_debug_serial(pp.ext._h, 1) == 0
    if args.alias_frames:
        args.no_check = True
        for pp in pipes:
            assert orbamd.load().orbx_debug_alias_frames(pp.ext._h, 1) == 0

    for _ in range(args.warmup):
        sched.step()
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
        sevs = ([[[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(P)]
                 for _ in range(nsteps)] if rig else None)
        if timed and use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for i in range(nsteps):
            # the timed pass records only the dominant kernel's event pairs (inside the graphs); the matcher /
            # exchange split comes from the untimed stage pass
            if timed:
                sched.step(first=i == 0)
            else:
                sched.step(evs[i], xevs[i], first=i == 0, sev=sevs[i] if rig else None)
        torch.cuda.synchronize()
        if timed and use_dist:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        acc = [0.0] * 5
        ncalls = 0
        for pp in pipes:
            ms = (C.c_double * 5)()
            nc = C.c_int()
            # a failing read (an unrecorded stage event pair) must stop the run, not leave a HIP error behind
            lib_check(lib.orbx_profile_read(pp.ext._h, ms, C.byref(nc)), "orbx_profile_read")
            lib.orbx_profile_enable(pp.ext._h, 0)
            for i in range(5):
                acc[i] += ms[i]
            ncalls += nc.value
        st = {k: acc[i] / max(ncalls, 1) for i, k in enumerate(stages) if (mask >> i) & 1}
        if timed:
            return elapsed, st
        st["match"] = sum(e[p][0].elapsed_time(e[p][1]) for e in evs for p in range(P)) / (nsteps * P)
        if rig:
            st["stereo"] = sum(e[p][0].elapsed_time(e[p][1]) for e in sevs for p in range(P)) / (nsteps * P)
        if not args.no_exchange:
            st["exchange"] = sum(x[0].elapsed_time(x[1]) for x in xevs) / nsteps
            st["allgather"] = sum(a.elapsed_time(b) for a, b in sched.ag_events) / max(len(sched.ag_events), 1)
            sched.ag_events.clear()
        return elapsed, st

    def run_part(nsteps, **kw):
        """untimed breakdown pass: wall time of nsteps steps doing only part of the work"""
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nsteps):
            sched.step(first=i == 0, **kw)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    # 1) stage split (untimed): every stage bracketed, same schedule
    _, stage_ms = run_profiled(0x1F, args.steps, False)
    # the roofline kernel: the extraction stage with the largest live time in this run's own stage split (every
    # stage bracketed by HIP events on the stream it runs on, same overlapped schedule); --roof-kernel overrides
    ranked = sorted(stages, key=lambda k: -stage_ms[k])
    dom = ranked[0] if args.roof_kernel == "auto" else args.roof_kernel
    # a second stage within 5 % of the largest is priced beside it (`roofline.co_dominant`): the split's event pairs
    # cannot rank two stages that close (round-4 review)
    co = (ranked[1] if args.roof_kernel == "auto" and stage_ms[ranked[1]] >= 0.95 * stage_ms[dom] else None)
    # 2) timed region: only the priced kernels bracketed (their live launch durations for the roofline)
    el, dom_live = run_profiled((1 << stages.index(dom)) | ((1 << stages.index(co)) if co else 0), args.steps, True)
    last_batch, prev_batch = sched.last_batch, (sched.last_batch - 1) % args.pool
    el = reduce_max(el)
    # 3) self-check of the last timed step (error flags on every rank; oracle bit-compare of sampled frames,
    # their match rows and the cross-agent matches)
    err_msg = None
    try:
        sched.check_errors()
    except RuntimeError as e:
        err_msg = str(e)
    check = None
    agent_kf = lambda r, t: agent_frames(r, t, 1)[0]  # noqa: E731 (agent r's keyframe image / stereo pair)
    if not args.no_check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from check_schedule import check_schedule
        check = check_schedule(sched, frames_np, nfeatures=cfg["nfeatures"], agent_frames=agent_kf)
    ok_local = err_msg is None and (check is None or check["bit_exact"])
    ok_all = ok_local
    if use_dist:
        ok_all = int(reduce_max(0 if ok_local else 1, torch.int32)) == 0
    # 3b) the priced kernels alone (untimed, after the check): graph 0 re-extracts the last batch in stage order with
    # every other graph idle, one step at a time, the priced stages bracketed by HIP events; the live launch above is
    # the kernel's share of a chip running the other graphs, this is its own speed (roofline.alone)
    alone_ms = {}
    pp0 = pipes[0]
    lib.orbx_debug_serial(pp0.ext._h, 1)
    for kern in [dom] + ([co] if co else []):
        vals = []
        for _ in range(ALONE_LAUNCHES):
            lib.orbx_profile_enable(pp0.ext._h, 1 << stages.index(kern))
            pp0.extract(sched.frames[last_batch][0], sched.streams[0].cuda_stream, stereo=False)
            torch.cuda.synchronize()
            ms = (C.c_double * 5)()
            nc = C.c_int()
            lib_check(lib.orbx_profile_read(pp0.ext._h, ms, C.byref(nc)), "orbx_profile_read")
            vals.append(ms[stages.index(kern)] / max(nc.value, 1))
        alone_ms[kern] = sorted(vals)[len(vals) // 2]
    lib.orbx_profile_enable(pp0.ext._h, 0)
    lib.orbx_debug_serial(pp0.ext._h, 0)
    # 4) extract-only and match-only rates, untimed breakdown passes; and the box's
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
    # 4b) ingest leg (untimed for `value`): every step's frames are uploaded from pinned host memory on a
    # copy stream into the device batch that step processes, overlapped with the previous step's compute;
    # checked against the oracle like the timed region
    ingest = None
    if args.ingest_steps > 0:
        if use_dist:
            dist.barrier()
        ingest = run_ingest(torch, sched, frames_np, args.pool, args.ingest_steps, B, W, H, world, use_dist, dist,
                            reduce_max, args.ingest_streams, args.ingest_chunks,
                            host_wait=args.ingest_wait == "host")
        if not args.no_check:
            chk = check_schedule(sched, frames_np, nfeatures=cfg["nfeatures"], agent_frames=agent_kf)
            ingest["bit_exact"] = bool(chk["bit_exact"])
            ok_all = ok_all and chk["bit_exact"]
    # 5) sustained pass (untimed for `value`): the full schedule for ~--sustain seconds, which reports the
    # steady-state rate over thousands of steps and keeps the GPU busy long enough for a utilisation sampler
    # to see it. The step count comes from the max-over-ranks timing, so every rank runs the same number of
    # exchange all-gathers.
    sustained = None
    if args.sustain > 0:
        n_sus = max(1, int(math.ceil(args.sustain / (el / args.steps))))
        if use_dist:
            dist.barrier()
        sus_s = reduce_max(run_part(n_sus))
        sustained = {"seconds": round(sus_s, 3), "steps": n_sus, "frames_per_s": round(world * B * n_sus / sus_s, 1)}
    nkp = float(sum(pp.counts.float().mean().item() for pp in pipes) / P)
    nmatch = float(sum(pp.nmatch.float().mean().item() for pp in pipes) / P)

    total_frames = world * B * args.steps
    value = total_frames / el
    result = None
    if rank == 0:
        b_frame, per_stage = algorithmic_bytes(W, H, nkp)
        # describe's bytes from this run's keypoints: the union of the pixels its patches read (the blur folded into
        # describe when no separate blur stage ran)
        f0 = sched.frames[0][0]
        fused = bool(lib.orbx_describe_blur_fused(f0.data_ptr(), f0.stride(0), f0.stride(1)))
        per_stage["describe"] = describe_touched_bytes(sched, W, H, fused)
        if fused:
            per_stage["blur"] = 0
        # counter passes of this configuration (tools/prof_round.sh for c2, tools/pmc_config.sh for c3 / c4), taken
        # at 256 frames per launch
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json" if args.config == "c2" else
                                "pmc_traffic_%s.json" % args.config)
        pmc = {}
        if os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))
            except Exception:
                pmc = {}
            if pmc.get("frames_per_launch", 256) != imgs:  # counters of another launch size do not price this one
                pmc = {}
        sel = ("largest stage of this run's stage split (%s)" % ", ".join("%s %.3f ms" % (k, stage_ms[k]) for k in stages)
               if args.roof_kernel == "auto" else "--roof-kernel")

        def price(kern):
            """the kernel's roofline at its live launch duration in the timed region (one launch = one graph's
            sub-batch of B / P frames, `imgs` images): VALU issue from the counter pass, algorithmic bytes against
            HBM; `alone`: the same launch with nothing else on the GPU (its own efficiency, measured after the timed
            region: graph 0's extraction in stage order, one launch at a time)"""
            k_ms = dom_live[kern]
            hbm_gbs = per_stage[kern] * imgs / (k_ms * 1e-3) / 1e9 if k_ms > 0 and per_stage[kern] > 0 else 0.0
            rec = pmc.get(kern, {})
            traffic, valu_insts = rec.get("hbm_bytes_per_launch"), rec.get("valu_insts_per_launch")
            valu_gs = valu_insts / (k_ms * 1e-3) / 1e9 if valu_insts and k_ms > 0 else None
            a_ms = alone_ms.get(kern)
            alone = None
            if a_ms:
                alone = {"launch_ms": round(a_ms, 4), "share_of_live": round(a_ms / k_ms, 4) if k_ms > 0 else None,
                         "alg_hbm_frac": round(per_stage[kern] * imgs / (a_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                         "valu_frac": (round(valu_insts / (a_ms * 1e-3) / 1e9 / VALU_PEAK_GINST, 4) if valu_insts
                                       else None),
                         "counter_hbm_frac": (round(traffic / (a_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic
                                              else None),
                         "how": "graph 0 alone on the GPU (orbx_debug_serial), HIP events around the stage, median of "
                                "%d launches" % ALONE_LAUNCHES}
            hbm = {"achieved": round(hbm_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(hbm_gbs / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_launch": round(per_stage[kern] * imgs),
                   "measured_copy_GBs": round(copy_gbs, 1) if copy_gbs else None,
                   "frac_vs_copy": round(hbm_gbs / copy_gbs, 5) if copy_gbs else None}
            if valu_gs is not None and valu_gs / VALU_PEAK_GINST > hbm_gbs / HBM_PEAK_GBS:
                # the byte/integer kernels are bound by vector-instruction issue, not HBM
                return {"bound": "valu", "kernel": kern, "achieved": round(valu_gs, 1), "peak": VALU_PEAK_GINST,
                        "unit": "G wave64 VALU instr/s", "frac": round(valu_gs / VALU_PEAK_GINST, 4),
                        "traffic": traffic, "valu_insts_per_launch": valu_insts, "launch_ms": round(k_ms, 4),
                        "hbm": hbm, "alone": alone}
            return {"bound": "hbm", "kernel": kern, "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm["frac"], "traffic": traffic, "launch_ms": round(k_ms, 4), "hbm": hbm, "alone": alone}

        roof = price(dom)
        roof["selected_by"] = sel
        roof["describe_form"] = "k_describe_blur (blur fused)" if fused else "k_blur_strips + k_describe"
        if co:
            roof["co_dominant"] = price(co)
        # the matcher on the matrix cores (fp4 +-1 operands, v_mfma_scale_f32_32x32x64_f8f6f4): algorithmic ops =
        # n1*n2 distances x 256 bits x 2 per pair
        m_ms = stage_ms.get("match", 0.0)
        m_tops = nkp * nkp * 512 * sub / (m_ms * 1e-3) / 1e12 if m_ms > 0 else 0.0
        # the live launch shares the chip with the other graphs' extraction; the match-only pass (every graph's
        # matcher, nothing else on the GPU, wall clock incl. the rotation filter) gives the matcher's own rate
        mo_tops = nkp * nkp * 512 * match_pps / 1e12
        # every stage's roofline at its live launch time in the stage pass (one launch = one graph's sub-batch):
        # VALU issue and HBM fractions from the counter passes of this configuration, algorithmic bytes beside
        # them; plus the whole step's VALU issue rate (every stage's VALU wave-instructions x P launches per step
        # / ms_per_step)
        stage_roof, step_valu = {}, 0.0
        for k in stages + ["match"] + (["stereo"] if rig else []):
            if k == "blur" and fused:
                continue  # no separate blur stage ran (the event pair around nothing reads a few microseconds)
            ms = stage_ms.get(k, 0.0)
            rec = pmc.get(k, {})
            vi, hb = rec.get("valu_insts_per_launch"), rec.get("hbm_bytes_per_launch")
            alg = round(per_stage.get(k, 0) * imgs) if k in per_stage else None
            row = {"launch_ms": round(ms, 4), "valu_insts_per_launch": vi, "hbm_bytes_per_launch": hb}
            if ms > 0:
                if vi:
                    row["valu_frac"] = round(vi / (ms * 1e-3) / 1e9 / VALU_PEAK_GINST, 4)
                if hb:
                    row["hbm_frac"] = round(hb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                if alg:
                    row["alg_bytes_per_launch"] = alg
                    row["alg_hbm_frac"] = round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            if vi:
                step_valu += vi * P
            stage_roof[k] = row
        step_s = el / args.steps
        step_valu_roof = ({"valu_insts_per_step": step_valu, "achieved": round(step_valu / step_s / 1e9, 1),
                           "peak": VALU_PEAK_GINST, "unit": "G wave64 VALU instr/s",
                           "frac": round(step_valu / step_s / 1e9 / VALU_PEAK_GINST, 4)} if step_valu else None)
        result = {
            "metric": ("frames/sec ORB extract+match, 640x480 mono, 1000 feat/frame" if args.config == "c2" else
                       "stereo frames/sec ORB extract(L+R)+stereo match+match, %dx%d, %d feat/image" % (W, H, cfg["nfeatures"])
                       if rig else "frames/sec ORB extract+match, %dx%d left images, %d feat/frame"
                       % (W, H, cfg["nfeatures"])),
            "value": round(value, 2),
            "unit": "stereo frames/s" if rig else "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic textured pan, SURVEY.md 8(d)); resident in HBM",
            "config": {"workload": cfg["name"] + ", scale 1.2, 8 levels, FAST 20/7; " +
                                   ("stereo pairs (right image at disparity %d px; mbf %.4f, mb %.5f): extract left + right "
                                    "+ ComputeStereoMatches + BF SearchForTriangulation (stereo branch)" % (cfg["dx"], rig[0], rig[1])
                                    if rig else "extract + BF SearchForTriangulation") +
                                   " vs previous frame + per-step keyframe BoW + slot all-gather & cross-agent "
                                   "SearchForTriangulation and SearchByBoW(KF,KF)",
                       "config": args.config, "stereo": bool(rig), "frames_per_step_per_gpu": B,
                       "images_per_step_per_gpu": per * B, "graphs_per_gpu": P,
                       "graph_stagger": args.stagger, "scene": args.scene,
                       "exchange_stream": "own" if async_x else "graph 0's",
                       "parallelism": "agent-per-gpu x%d" % world},
            "bit_exact": bool(ok_all) if check is not None else None,
            "checked_frames": check["checked_frames"] if check else 0,
            "checked_pairs": check["checked_pairs"] if check else 0,
            "checked_slots": check["checked_slots"] if check else 0,
            "slot_bow_matches": check.get("slot_bow_matches") if check else None,
            "device_errors": err_msg,
            "roofline": roof,
            "match_roofline": {"bound": "mfma", "kernel": "k_tri_mfma", "achieved": round(m_tops, 2),
                               "peak": FP4_MFMA_PEAK_TOPS, "unit": "fp4 TOPS", "frac": round(m_tops / FP4_MFMA_PEAK_TOPS, 4),
                               "launch_ms": round(m_ms, 4),
                               "match_only": {"achieved": round(mo_tops, 2), "frac": round(mo_tops / FP4_MFMA_PEAK_TOPS, 4),
                                              "what": "whole-GPU rate of the match-only pass (wall clock)"}},
            "stage_rooflines": stage_roof,
            "step_valu_issue": step_valu_roof,
            "pipeline_hbm": {"bytes_per_image": b_frame, "achieved_GBs": round(b_frame * per * value / world / 1e9, 2),
                             "frac": round(b_frame * per * value / world / 1e9 / HBM_PEAK_GBS, 5)},
            "stage_ms_per_step": {k: round(v, 4) for k, v in stage_ms.items()},
            "per_gpu_frames_per_s": round(value / world, 2),
            "extract_only_frames_per_s_per_gpu": round(extract_fps, 1),
            "match_only_pairs_per_s_per_gpu": round(match_pps, 1),
            "kp_per_image": round(nkp, 1),
            "matches_per_pair": round(nmatch, 1),
            "sustained": sustained,
            "ingest": ingest,
            "stale_guard": {"frame_pool_batches": args.pool, "checked_step_batch": last_batch,
                            "previous_step_batch": prev_batch,
                            "note": "consecutive steps process different resident batches, so a stage that did not "
                                    "launch in the checked (last timed) step leaves the previous batch's outputs and "
                                    "fails the oracle check" if args.pool > 1 else
                                    "pool of 1: repeated frames, a skipped launch would not be detected"},
            "collective": ("rccl ncclAllGather by liborbamd (orbx_comm_allgather) on %s stream, out-of-place slot "
                           "buffer; gloo control plane" % ("the exchange's own" if async_x else "graph 0's")
                           if use_dist and coll == "rccl" else
                           "rccl all_gather_into_tensor (torch ProcessGroupNCCL, out-of-place slot buffer)"
                           if use_dist and coll == "torch"
                           else "gloo all_gather through host memory (rehearsal)" if use_dist
                           else "none (N=1: the keyframe slot is packed in place)"),
        }
        if check is not None and check["mismatches"]:
            result["mismatches"] = check["mismatches"]
    # the CPU baseline is measured at N=1 only (rank 0); multi-GPU lines report null
    if rank == 0 and world == 1 and not args.no_cpu:
        info = host_cpu_info()
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from check_schedule import host_threads
        threads = args.cpu_threads or host_threads()
        nf1 = args.cpu_frames_1t or (2000 if args.config == "c2" else 1000)
        # median of 5 short runs on every usable host core (the headline ratio), then the
        # reference's own architecture: one Tracking thread ((i), >= 2000 frames at C2) with the oracle's stage split
        if rig:
            nf1 = args.cpu_frames_1t or 500
        runs = [cpu_baseline(frames_np, threads, seconds=args.cpu_seconds / 5, nfeatures=cfg["nfeatures"], stereo=rig)
                for _ in range(5)]
        fps = sorted(r[0] for r in runs)[2]
        nfr, sec = sum(r[1] for r in runs), sum(r[2] for r in runs)
        fps1, nfr1, sec1, per1 = cpu_baseline(frames_np, 1, nframes=nf1, nfeatures=cfg["nfeatures"], stereo=rig)
        result["cpu_baseline"] = {
            "value": round(fps, 2), "unit": "stereo frames/s" if rig else "frames/s", "cores": threads, "kind": "port",
            "sample": "median of 5 runs, %d synthetic %dx%d %s in %.1f s in total (%s vs "
                      "previous) on %d threads (every CPU of the affinity set, capped by the cgroup quota), "
                      "oracle/orb_oracle.c -O3 -march=x86-64-v3 -ffp-contract=off (a restatement; cv::FAST in OpenCV's SSE2 "
                      "vector form (detection + cornerScore), the other stages compiler-vectorised, no IPP); "
                      "1-thread leg: %d frames in %.1f s" % (nfr, W, H, "stereo pairs" if rig else "frames", sec,
                                                             "extract L + R + ComputeStereoMatches + stereo BF "
                                                             "triangulation" if rig else "extract + BF triangulation",
                                                             threads, nfr1, sec1),
            "host": info,
            "value_1thread": round(fps1, 2),
            "frames_1thread": nfr1,
            "stage_ms_per_frame_1thread": {k: round(v * 1e3, 3) for k, v in per1.items()}}
        result["speedup_vs_cpu"] = round(value / fps, 1)
        result["speedup_vs_cpu_1thread"] = round(value / fps1, 1)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    sched.close()
    if use_dist:
        dist.barrier()
        if comm is not None:
            orbamd.load().orbx_comm_destroy(comm)
        dist.destroy_process_group()
    if not ok_all:
        sys.exit(3)


if __name__ == "__main__":
    main()
