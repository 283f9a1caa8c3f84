#!/bin/bash
# stagger modes at the driver's bench arguments (--steps 20 --warmup 5) with the sustained pass (~2000 steps) and the
# ingest leg on: the timed value and the steady-state rate of each mode, interleaved rounds.
# usage: tools/exp_stagger_sustain.sh [rounds] [modes...]
R=${1:-3}; shift
modes=${*:-each once}
summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"], "sustained", d["sustained"]["frames_per_s"], "ingest", d["ingest"]["frames_per_s"], d["bit_exact"])'
for r in $(seq 1 "$R"); do for m in $modes; do
  v=$(timeout -k 10 180 python bench.py --no-cpu --steps 20 --warmup 5 --stagger $m | python -c "$summ") || exit $?
  echo "r$r stagger=$m (driver args, sustain 6 s, ingest leg): $v"
done; done
