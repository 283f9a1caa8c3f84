#!/bin/bash
# frames/s of the default schedule under different HW-queue counts and the per-graph serial schedule
# (each graph's stages on its own stream only): 4 graphs x 256 frames, no CPU leg, no check
run() { timeout -k 10 180 env "$@" python bench.py --sustain 0 --no-cpu --no-check --steps 30 | \
  python -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"])'; }
for r in 1 2; do
  echo "r$r default:            $(run X=1)"
  echo "r$r ORBX_SCHED=serial:  $(run ORBX_SCHED=serial)"
  echo "r$r GPU_MAX_HW_QUEUES=8: $(run GPU_MAX_HW_QUEUES=8)"
  echo "r$r GPU_MAX_HW_QUEUES=8 serial: $(run GPU_MAX_HW_QUEUES=8 ORBX_SCHED=serial)"
done
