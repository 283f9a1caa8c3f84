#!/usr/bin/env python3
"""Per-kernel per-wave summary of rocprofv3 --pmc counter_collection.csv files (several passes
are merged by kernel name; values are averaged over the dispatches of a kernel).
usage: pmc_summary.py pass_a.csv [pass_b.csv ...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
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
    print("%-22s waves %7d cyc/wave %7.0f valu/wave %6.0f valu(M) %6.1f vmem/wave %5.1f lds/wave %5.1f "
          "salu/wave %5.0f wait %.2f waitinst %.2f ldsconf %.2f"
          % (k[:22], w, 4 * g("SQ_WAVE_CYCLES") / w, g("SQ_INSTS_VALU") / w, g("SQ_INSTS_VALU") / 1e6,
             g("SQ_INSTS_VMEM_RD") / w, g("SQ_INSTS_LDS") / w, g("SQ_INSTS_SALU") / w,
             g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"),
             g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_INSTS_LDS"), 1)))
