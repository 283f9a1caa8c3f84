#!/bin/bash
# round 4: k_voc_bow in 256-thread workgroups (new) against HEAD's 1024-thread kernel (mid): C2 bench lines without
# the profiler, three interleaved rounds
export TMPDIR=/tmp
T=r04bt2
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s["exchange"])'
for r in 1 2 3; do
  for v in new mid; do
    if [ $v = new ]; then unset ORBAMD_LIB_VARIANT; else export ORBAMD_LIB_VARIANT=$v; fi
    out=$(timeout -k 10 180 python bench.py --sustain 0 --no-cpu | python -c "$summ") || exit $?
    echo "r$r $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
