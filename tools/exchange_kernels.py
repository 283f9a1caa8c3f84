"""Per-kernel launch statistics of the exchange step's kernels from a rocprofv3 kernel trace.

usage: python3 tools/exchange_kernels.py <kernel_trace.csv>
"""
import collections
import csv
import sys

KEYS = ("k_voc", "k_pack_slot", "k_tri_slots", "k_bow_slots", "k_rot_slots")


def main(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0]
        if any(k in n for k in KEYS):
            d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in sorted(d.items()):
        v.sort()
        print("%-60s %5d launches, mean %.1f us, median %.1f us, max %.1f us"
              % (n, len(v), sum(v) / len(v), v[len(v) // 2], max(v)))


if __name__ == "__main__":
    main(sys.argv[1])
