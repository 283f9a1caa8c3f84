#!/bin/bash
# frames per step x graphs under the every-8th-step stagger, at the driver's bench arguments (--steps 20 --warmup 5)
# with the sustained pass on; interleaved rounds. usage: tools/exp_batches3.sh [rounds] "B P" ...
R=${1:-2}; shift
cfgs=("$@")
summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"], "sustained", d["sustained"]["frames_per_s"], d["bit_exact"])'
for r in $(seq 1 "$R"); do for cfg in "${cfgs[@]}"; do
  read -r b p <<< "$cfg"
  v=$(timeout -k 10 180 python bench.py --no-cpu --ingest-steps 0 --steps 20 --warmup 5 --batch $b --pipes $p | python -c "$summ") || exit $?
  echo "r$r batch=$b pipes=$p: $v"
done; done
