#!/bin/bash
# extraction schedule x HW queue count, overlapped default bench (timing only). usage: tools/exp_sched2.sh
for r in 1 2; do
for cfg in "default 4" "serial 4" "serial_blur_first 4" "default 8" "serial_blur_first 8"; do
  set -- $cfg
  if [ $1 = default ]; then unset ORBX_SCHED; else export ORBX_SCHED=$1; fi
  out=$(GPU_MAX_HW_QUEUES=$2 timeout -k 10 120 python bench.py --sustain 0 --no-cpu --no-check --steps 20 | python -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"])') || exit 1
  echo "r$r sched $1 queues $2: $out"
done; done
