#!/bin/bash
# round 4: the bench's graph streams created before the pipelines' library handles (first) or after them (the
# current order, last), interleaved C2 lines at the default and the driver's arguments
export TMPDIR=/tmp
T=r04sf
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s.get("exchange", 0.0), "sustained=%.0f" % (d.get("sustained") or {}).get("frames_per_s", 0))'
for r in 1 2 3; do
  for v in first last; do
    if [ $v = first ]; then export ORBAMD_STREAMS_FIRST=1; else unset ORBAMD_STREAMS_FIRST; fi
    out=$(timeout -k 10 180 python bench.py --no-cpu 2>/dev/null | python -c "$summ") || exit $?
    echo "r$r default $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
for v in first last; do
  if [ $v = first ]; then export ORBAMD_STREAMS_FIRST=1; else unset ORBAMD_STREAMS_FIRST; fi
  out=$(timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu 2>/dev/null | python -c "$summ") || exit $?
  echo "driver-args $v $out" | tee -a gpurun_out/${T}_bench.log
done
