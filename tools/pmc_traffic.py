#!/usr/bin/env python3
"""HBM traffic per launch of each pipeline stage from separate FETCH_SIZE / WRITE_SIZE
rocprofv3 --pmc passes. Both counters are in KiB (x1024 bytes). FETCH_SIZE reports exactly half the bytes
read on gfx950 for every load width these kernels use (1, 4, 8, 16 B per lane and 4-B LDS-DMA, measured by
tools/fetch_calib.hip over a 1 GiB buffer: profiles/r05_fetch_size_calibration.txt; MI355X_MICROARCH.md
documents the half for 16-B lanes), so it is doubled here; WRITE_SIZE reads the bytes exactly.
For a stage launched with different grids (FAST: level-0 and other-level launches in the
overlapped schedule, one whole-grid launch in the stage-serial profiling pass) the whole-grid
launch is reported, which is the launch bench.py's roofline times.
Optionally a counter pass with SQ_INSTS_VALU adds the VALU instructions per launch.
usage: pmc_traffic.py fetch.csv write.csv out.json [valu_pass.csv [frames_per_launch]]
(frames_per_launch, default 256: the bench's B / P, recorded so bench.py prices launches of that size only)"""
import collections
import csv
import json
import sys

STAGES = {"pyramid": ("k_pyramid_frames", "k_resize_tiled", "k_resize_level"), "fast_cells": ("k_fast_cells2",),
          "octree": ("k_octree",), "blur": ("k_blur_strips",), "describe": ("k_describe",),
          "match": ("k_tri_mfma",), "stereo": ("k_stereo",)}  # k_stereo_median's smaller grid is not the one priced


def load(path, counter):
    per = collections.defaultdict(list)  # (stage, grid) -> values
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for st, ks in STAGES.items():
            if any(k in name for k in ks):
                per[(st, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return per


fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
valu = load(sys.argv[4], "SQ_INSTS_VALU") if len(sys.argv) > 4 else {}
out = {}
for st in STAGES:
    grids = sorted(g for (s, g) in fetch if s == st)
    if not grids:
        continue
    g = grids[-1]
    f = 2.0 * sum(fetch[(st, g)]) / len(fetch[(st, g)])  # calibrated: FETCH_SIZE tallies half the bytes
    w = sum(write.get((st, g), [0.0])) / max(len(write.get((st, g), [0.0])), 1)
    out[st] = {"grid": g, "dispatches": len(fetch[(st, g)]), "FETCH_SIZE_KiB_raw_avg_per_dispatch": f / 2.0,
               "fetch_KiB_avg_per_dispatch_corrected": f,
               "WRITE_SIZE_KiB_avg_per_dispatch": w, "hbm_bytes_per_launch": (f + w) * 1024.0}
    if (st, g) in valu:
        out[st]["valu_insts_per_launch"] = sum(valu[(st, g)]) / len(valu[(st, g)])
out["frames_per_launch"] = int(sys.argv[5]) if len(sys.argv) > 5 else 256
json.dump(out, open(sys.argv[3], "w"), indent=1)
for k, v in out.items():
    if not isinstance(v, dict):
        continue
    print("%-10s grid %9d  fetch %10.0f KiB  write %9.0f KiB  -> %.1f MB/launch" % (
        k, v["grid"], v["fetch_KiB_avg_per_dispatch_corrected"], v["WRITE_SIZE_KiB_avg_per_dispatch"],
        v["hbm_bytes_per_launch"] / 1e6))
