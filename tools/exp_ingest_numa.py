#!/usr/bin/env python3
"""Ingest-leg variance (round 6): the same ingest setting read 124k-175k frames/s across passes and runs. Host-side
suspects: the NUMA node the pinned frame pool lives on against the GPU's PCIe root, and the CPUs the enqueueing thread
runs on. Prints the box topology (the GPU's NUMA node, this process's allowed CPUs per node) and, in interleaved
rounds, the ingest rate with the pinned pool first-touched (a) wherever the process runs and (b) after binding the
process to the GPU's NUMA node's CPUs, plus the raw pinned H2D rate of each pool.

usage: python3 tools/exp_ingest_numa.py [steps] [rounds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cooperative-orb-slam_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import orbamd  # noqa: E402
from orbamd.agent import AgentSchedule  # noqa: E402


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def gpu_numa_node(dev=0):
    p = torch.cuda.get_device_properties(dev)
    bdf = "%04x:%02x:%02x.0" % (getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
    try:
        return int(open("/sys/bus/pci/devices/%s/numa_node" % bdf).read()), bdf
    except OSError:
        return -1, bdf


def raw_h2d(src, dst):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return 3 * src.numel() / (time.perf_counter() - t0) / 1e9


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    node, bdf = gpu_numa_node()
    allowed = sorted(os.sched_getaffinity(0))
    nodes = {}
    for d in sorted(os.listdir("/sys/devices/system/node")):
        if d.startswith("node"):
            nodes[int(d[4:])] = [c for c in cpulist(open("/sys/devices/system/node/%s/cpulist" % d).read())
                                 if c in allowed]
    print("GPU %s on NUMA node %d; allowed CPUs per node: %s" % (bdf, node, {k: len(v) for k, v in nodes.items()}),
          flush=True)
    W, H, B, P, pool = 640, 480, 3072, 3, 2
    frames = orbamd.synth_frames(0, 0, pool * B, W, H, scene=0)
    sched = AgentSchedule(torch, frames, W, H, P, device=0, pool=pool)
    for i in range(5):
        sched.step(first=i == 0)
    torch.cuda.synchronize()
    dst = torch.empty(B * W * H, dtype=torch.uint8, device="cuda")
    for r in range(rounds):
        for mode in ("default", "gpu_node"):
            if mode == "gpu_node" and node >= 0 and nodes.get(node):
                os.sched_setaffinity(0, nodes[node])
            else:
                os.sched_setaffinity(0, allowed)
            src = torch.from_numpy(frames[:B].reshape(-1)).pin_memory()  # first touched on the current CPUs
            h2d = raw_h2d(src, dst)
            del src
            res = bench.run_ingest(torch, sched, frames, pool, steps, B, W, H, 1, False, None,
                                   lambda v, dtype=None: v, 4, 8)
            print("r%d %-8s raw H2D %.1f GB/s | ingest %.1f frames/s %.2f GB/s" % (
                r, mode, h2d, res["frames_per_s"], res["h2d_GBs_per_gpu"]), flush=True)
    os.sched_setaffinity(0, allowed)
    sched.close()


if __name__ == "__main__":
    main()
