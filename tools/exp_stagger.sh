#!/bin/bash
# graph stagger modes of bench.py (see --stagger), interleaved rounds, at the driver's short timed region
# (--steps 20 --warmup 5) and at bench.py's default 200 timed steps.
# usage: tools/exp_stagger.sh [rounds]
R=${1:-4}
summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"], d["bit_exact"])'
for r in $(seq 1 "$R"); do
  for m in each once none; do
    for st in "20 5" "200 20"; do
      set -- $st
      v=$(timeout -k 10 120 python bench.py --sustain 0 --no-cpu --ingest-steps 0 --steps $1 --warmup $2 --stagger $m \
          | python -c "$summ") || exit $?
      echo "r$r stagger=$m steps=$1 warmup=$2: $v"
    done
  done
done
