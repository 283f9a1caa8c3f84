#!/bin/bash
# round 4: the per-step keyframe exchange rotating over the graphs (frame 0 of graph k mod P in step k, in order on
# that graph's stream) against graph 0's every step: schedule / exchange parity, then interleaved C2 bench lines
# and one C4 pair
export TMPDIR=/tmp
T=r04rot
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_schedule.py tests/test_gpu_exchange.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], d["checked_slots"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s["exchange"], "sustained=%.0f" % d["sustained"]["frames_per_s"])'
for r in 1 2 3; do
  for v in rotate graph0; do
    out=$(timeout -k 10 180 python bench.py --no-cpu --exchange-stream $v | python -c "$summ") || exit $?
    echo "r$r c2 $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
for v in rotate graph0; do
  out=$(timeout -k 10 180 python bench.py --no-cpu --config c4 --exchange-stream $v | python -c "$summ") || exit $?
  echo "c4 $v $out" | tee -a gpurun_out/${T}_bench.log
done
