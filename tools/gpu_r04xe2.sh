#!/bin/bash
# round 4 diagnostic, second half of tools/gpu_r04xe.sh: full vs --no-exchange in the same session
export TMPDIR=/tmp
T=r04xe2
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s.get("exchange", 0.0), "sustained=%.0f" % (d.get("sustained") or {}).get("frames_per_s", 0))'
for r in 1 2 3; do
  for v in full none; do
    a=""; [ $v = none ] && a="--no-exchange"
    out=$(timeout -k 10 180 python bench.py --no-cpu $a 2>gpurun_out/${T}_err_$v.log | python -c "$summ")
    echo "r$r $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
