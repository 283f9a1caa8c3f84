#!/bin/bash
# round 4: the exchange on its own stream vs on graph 0's stream (the default at N = 1) with the round-4 exchange
# (BoW transform + both slot matchers), three interleaved rounds of the default C2 bench
export TMPDIR=/tmp
T=r04v
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match","exchange")))'
for r in 1 2 3; do
  for x in graph0 own; do
    out=$(timeout -k 10 180 python bench.py --sustain 0 --no-cpu --exchange-stream $x | python -c "$summ") || exit $?
    echo "r$r exchange-stream=$x $out" | tee -a gpurun_out/${T}_xstream_ab.log
  done
done
