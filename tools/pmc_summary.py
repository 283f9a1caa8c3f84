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
    g = lambda c: d.get(c, float("nan"))
    # SQ_WAVE_CYCLES / SQ_BUSY_CYCLES count in quad-cycles on gfx950 (x4)
    print("%-22s waves %7d cyc/wave %8.0f valu/wave %6.0f valu_total(M) %7.1f vmem/wave %5.1f lds/wave %6.1f wait %.2f waitinst %.2f"
          % (k[:22], w, 4 * g("SQ_WAVE_CYCLES") / w, g("SQ_INSTS_VALU") / w, g("SQ_INSTS_VALU") / 1e6,
             g("SQ_INSTS_VMEM_RD") / w, g("SQ_INSTS_LDS") / w, g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
             g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES")))
