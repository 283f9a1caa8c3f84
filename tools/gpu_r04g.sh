#!/bin/bash
# round 4 evidence: the one-frame call (fork after resize 1), then the bench's kernel trace + stats and the PMC
# passes (tools/prof_round.sh), the timed region's per-kernel averages, the reduction to profiles-sized files
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04g
tools/gpu_run.sh \
  "300 ${T}_latency tests/cpp/build/bench_latency 2000" \
  "300 ${T}_latency_kt rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_latency_kt -o run -- tests/cpp/build/bench_latency 200" || exit $?
tools/prof_round.sh $T || exit $?
kt=$(find gpurun_out/${T}_kt -name '*kernel_trace.csv' | head -n 1)
python3 tools/trace_segments.py "$kt" 10 2 > gpurun_out/${T}_timed_region_kernels.txt || exit $?
python3 - "$kt" > gpurun_out/${T}_exchange_kernels.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    if any(k in n for k in ("k_voc", "k_pack_slot", "k_tri_slots", "k_bow_slots", "k_rot_slots")):
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items()):
    print("%-60s %5d launches, mean %.1f us, max %.1f us" % (n, len(v), sum(v) / len(v), max(v)))
PY
tools/prof_reduce.sh $T
