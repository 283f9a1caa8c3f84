#!/bin/bash
# round 4: what the per-step exchange (keyframe BoW + pack + slot SearchForTriangulation + slot SearchByBoW) costs
# the step: the default C2 / C4 bench against --no-exchange, two interleaved rounds, plus the exchange's kernel trace
export TMPDIR=/tmp
T=r04w
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], " ".join("%s=%.3f" % (k, s.get(k, 0)) for k in ("pyramid","fast_cells","octree","blur","describe","match","exchange")))'
for r in 1 2; do
  for c in c2 c4; do
    for x in "" "--no-exchange"; do
      out=$(timeout -k 10 180 python bench.py --sustain 0 --no-cpu --config $c $x | python -c "$summ") || exit $?
      echo "r$r $c ${x:-exchange} $out" | tee -a gpurun_out/${T}_exchange_cost.log
    done
  done
done
