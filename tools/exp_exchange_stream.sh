#!/bin/bash
# keyframe exchange on its own stream (default) vs in order on graph 0's stream (--exchange-stream own / graph0), at the driver's
# bench arguments with the sustained pass; interleaved rounds. usage: tools/exp_exchange_stream.sh [rounds]
R=${1:-3}
summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"], "sustained", d["sustained"]["frames_per_s"], "exchange_ms", d["stage_ms_per_step"]["exchange"], d["bit_exact"])'
for r in $(seq 1 "$R"); do for f in "--exchange-stream own" "--exchange-stream graph0"; do
  v=$(timeout -k 10 180 python bench.py --no-cpu --ingest-steps 0 --steps 20 --warmup 5 $f | python -c "$summ") || exit $?
  echo "r$r $f: $v"
done; done
