#!/usr/bin/env python3
"""Print the kernel timeline of one step from a rocprofv3 --kernel-trace CSV.
usage: timeline.py run_kernel_trace.csv [anchor_kernel] [occurrence] [count]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_resize_tiled"
occ = int(sys.argv[3]) if len(sys.argv) > 3 else 42
cnt = int(sys.argv[4]) if len(sys.argv) > 4 else 20
ks = [(r["Kernel_Name"].split("(")[0].replace("orbamd::", "").replace("void ", ""), int(r["Start_Timestamp"]),
       int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows]
idx = [i for i, k in enumerate(ks) if k[0].startswith(anchor)]
i0 = max(idx[min(occ, len(idx) - 1)] - 3, 0)
t0 = ks[i0][1]
for k in ks[i0:i0 + cnt]:
    print("%-24s q%-3s %8.1f %8.1f  dur %7.1f us" % (k[0][:24], k[3], (k[1] - t0) / 1e3, (k[2] - t0) / 1e3, (k[2] - k[1]) / 1e3))
