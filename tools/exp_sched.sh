#!/bin/bash
# Extraction schedule experiment: ORBX_SCHED = default (blur on a side stream) / serial (one stream per
# graph) / split (level-0 FAST beside the pyramid), 4 staggered graphs of 256 frames.
for s in default serial split; do
  v=$(ORBX_SCHED=$s timeout -k 10 120 python bench.py --sustain 0 --no-cpu --steps 20 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")
  echo "sched=$s frames/s,ms = $v"
done
