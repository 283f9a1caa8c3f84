#!/bin/bash
# round 4: C2 bench with the vocabulary stream created lazily (new) against HEAD's library (vold, the stream created
# at orbv_create), interleaved on one box: default arguments (three rounds) and the driver's arguments (two)
export TMPDIR=/tmp
T=r04vs2
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s.get("exchange", 0.0), "sustained=%.0f" % (d.get("sustained") or {}).get("frames_per_s", 0))'
for r in 1 2 3; do
  for v in new vold; do
    if [ $v = new ]; then unset ORBAMD_LIB_VARIANT; else export ORBAMD_LIB_VARIANT=$v; fi
    out=$(timeout -k 10 180 python bench.py --no-cpu 2>/dev/null | python -c "$summ") || exit $?
    echo "r$r default $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
for r in 1 2; do
  for v in new vold; do
    if [ $v = new ]; then unset ORBAMD_LIB_VARIANT; else export ORBAMD_LIB_VARIANT=$v; fi
    out=$(timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu 2>/dev/null | python -c "$summ") || exit $?
    echo "r$r driver-args $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
