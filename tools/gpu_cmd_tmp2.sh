#!/bin/bash
# scratch: C4 / C3 interleaved rounds of two variants
summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d["stage_ms_per_step"]; m=d["match_roofline"]; print("%.0f" % d["value"], "match_only_pps=%.0f" % d["match_only_pairs_per_s_per_gpu"], "mo_frac=%.4f live_frac=%.4f" % (m["match_only"]["frac"], m["frac"]), " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","describe","match")))'
for r in 1 2 3; do
  for c in c4 c3; do
    for v in $VARS; do
      out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 120 python bench.py --config $c --sustain 0 --no-cpu --steps 20 | python -c "$summ") || exit $?
      echo "r$r $c $v: $out"
    done
  done
done
