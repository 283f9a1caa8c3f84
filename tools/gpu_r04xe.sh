#!/bin/bash
# round 4 diagnostic: what the per-step exchange costs the step. full = the shipped exchange; empty = the same
# launches (same grids, LDS, streams, memsets) with every exchange kernel returning at once (variant xempty; its
# slot check fails by construction); none = --no-exchange. Three interleaved C2 rounds.
export TMPDIR=/tmp
T=r04xe
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s["exchange"], "sustained=%.0f" % d["sustained"]["frames_per_s"])'
for r in 1 2 3; do
  for v in full empty none; do
    unset ORBAMD_LIB_VARIANT; a=""
    [ $v = empty ] && export ORBAMD_LIB_VARIANT=xempty
    [ $v = none ] && a="--no-exchange"
    out=$(timeout -k 10 180 python bench.py --no-cpu $a | python -c "$summ")
    echo "r$r $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
