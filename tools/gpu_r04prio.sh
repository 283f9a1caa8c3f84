#!/bin/bash
# round 4: the exchange below the graphs -- every graph's stream at high priority with the exchange on its own
# (default-priority) stream, against the default (exchange on graph 0's stream, no priorities); two rounds
export TMPDIR=/tmp
T=r04prio
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "exchange=%.3f" % s["exchange"])'
for r in 1 2; do
  for a in "" "--prio all --exchange-stream own" "--prio all"; do
    out=$(timeout -k 10 180 python bench.py --sustain 0 --no-cpu $a | python -c "$summ") || exit $?
    echo "r$r [${a:-default}] $out" | tee -a gpurun_out/${T}_ab.log
  done
done
