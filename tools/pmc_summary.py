#!/usr/bin/env python3
"""Per-kernel per-wave summary of a rocprofv3 --pmc counter_collection.csv."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("orbamd::", "").replace("void ", "")
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "at::" in k or "rocclr" in k or "pack" in k:
        continue
    d = {c: sum(x) / len(x) for c, x in v.items()}
    w = d.get("SQ_WAVES", 0)
    if not w:
        continue
    print("%-22s waves %7d cyc/wave %8.0f valu/wave %6.0f vmem/wave %5.1f lds/wave %6.1f wait %.2f waitinst %.2f"
          % (k[:22], w, 4 * d["SQ_WAVE_CYCLES"] / w, d["SQ_INSTS_VALU"] / w, d["SQ_INSTS_VMEM_RD"] / w,
             d["SQ_INSTS_LDS"] / w, d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]))
