#!/bin/bash
# Every pipeline kernel alone on the GPU (VERDICT r05 item 6 / DESIGN.md 6.0): one graph of 1024 images per launch
# (C2: 1024 frames; C3 / C4: 512 stereo pairs), every stage in order on its stream (--serial-stages), under a
# kernel trace; the per-kernel averages are the kernels' own speed at the bench's launch size.
# usage: tools/alone_trace.sh <tag> [config]
T=$1; C=${2:-c2}
B=1024; [ "$C" != c2 ] && B=512
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_alone_$C -o run -- \
  python3 bench.py --config $C --pipes 1 --batch $B --serial-stages --steps 10 --warmup 2 --no-cpu --sustain 0 \
  --ingest-steps 0 --no-check > gpurun_out/${T}_alone_$C.log 2>&1 || exit $?
st=$(find gpurun_out/${T}_alone_$C -name '*kernel_stats.csv' | head -n 1)
python3 - "$st" <<'PY' | tee gpurun_out/${T}_alone_${C}_summary.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("%-28s %8s %10s %10s" % ("kernel", "calls", "avg_ms", "total_ms"))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].split("(")[0].replace("void ", "")[:28]
    print("%-28s %8s %10.4f %10.2f" % (name, r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
