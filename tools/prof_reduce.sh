#!/bin/bash
# Reduce a tools/prof_session.sh run on the GPU box to the files kept under profiles/ (the raw kernel
# traces exceed what gpurun copies back): one-step timeline, kernel stats, PMC traffic JSON + summary.
# usage: tools/prof_reduce.sh <tag> [frames_per_launch]
T=${1:-r02}
O=gpurun_out
one() { find "$1" -name "$2" 2>/dev/null | head -n 1; }
kt=$(one $O/${T}_kt '*kernel_trace.csv')
[ -n "$kt" ] && python3 tools/timeline.py "$kt" k_pyramid_frames 30 40 > $O/${T}_timeline_step.txt
for d in kt iso rows; do
  s=$(one $O/${T}_$d '*kernel_stats.csv'); [ -n "$s" ] && cp "$s" $O/${T}_${d}_kernel_stats.csv
done
fe=$(one $O/${T}_fetch '*counter_collection.csv'); wr=$(one $O/${T}_write '*counter_collection.csv')
pa=$(one $O/${T}_pmc_a '*counter_collection.csv'); pb=$(one $O/${T}_pmc_b '*counter_collection.csv')
python3 tools/pmc_traffic.py "$fe" "$wr" $O/${T}_pmc_traffic.json "$pa" ${2:-256}
python3 tools/pmc_summary.py "$pa" "$pb" > $O/${T}_pmc_summary.txt
for f in fetch write pmc_a pmc_b; do
  c=$(one $O/${T}_$f '*counter_collection.csv'); [ -n "$c" ] && gzip -c "$c" > $O/${T}_${f}.csv.gz
done
rm -rf $O/${T}_kt $O/${T}_iso $O/${T}_rows $O/${T}_fetch $O/${T}_write $O/${T}_pmc_a $O/${T}_pmc_b
du -sh $O
