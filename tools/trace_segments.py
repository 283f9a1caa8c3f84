#!/usr/bin/env python3
"""Average duration of each pipeline kernel per segment of a `bench.py` run, from a rocprofv3 kernel trace.

bench.py launches every stage kernel once per graph and step in this order: warm-up steps, the untimed
stage-split pass, the timed region, the `roofline.alone` launches (graph 0's extraction alone on the GPU, ALONE
launches of every extraction stage: 7 per priced kernel), the extract-only pass, (match-only: no extraction kernels),
then the ingest leg. rocprofv3 --stats averages over all of them; the ingest leg's launches overlap differently
(PCIe-bound steps), so the timed region's own average is what bench.py's event-timed `launch_ms` is
compared with.
usage: trace_segments.py run_kernel_trace.csv STEPS WARMUP [PIPES] [ALONE]"""
import csv
import sys

KERNELS = (("fast_cells", "k_fast_cells2"), ("pyramid", "k_pyramid_frames"), ("describe", "k_describe"),
           ("blur", "k_blur_strips"), ("octree", "k_octree"), ("match", "k_tri_mfma"), ("stereo", "k_stereo"))


def kernel(row):
    """the kernel's own name: orbamd::k_describe_blur(...) -> k_describe_blur"""
    return row["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].replace("void ", "").strip()


def main():
    path, steps, warm = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    pipes = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    alone = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    rows = list(csv.DictReader(open(path)))
    w, s = warm * pipes, steps * pipes
    for stage, name in KERNELS:
        ks = sorted((r for r in rows if kernel(r).startswith(name) and not kernel(r).endswith("_median")),
                    key=lambda r: int(r["Start_Timestamp"]))
        if not ks:
            continue
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ks]
        segs = [("warmup", 0, w), ("stage_split", w, w + s), ("timed", w + s, w + 2 * s)]
        if stage in ("match", "stereo"):  # not in the alone launches; the matcher runs in the match-only pass
            segs += [("match_only" if stage == "match" else "extract_only", w + 2 * s, w + 3 * s),
                     ("ingest", w + 3 * s, len(d))]
        else:
            a = w + 2 * s + alone
            segs += [("alone", w + 2 * s, a), ("extract_only", a, a + s), ("ingest", a + s, len(d))]
        out = ["%s=%d x %.4f ms" % (n, b - a, sum(d[a:b]) / (b - a)) for n, a, b in segs if b > a]
        print("%-10s launches %4d, all %.4f ms | %s" % (stage, len(d), sum(d) / max(len(d), 1), " | ".join(out)))


if __name__ == "__main__":
    main()
