#!/bin/bash
# round 4 final head: the C3 and C4 bench lines (driver arguments)
export TMPDIR=/tmp
T=r04fin3
tools/gpu_run.sh \
  "300 ${T}_bench_c3 python3 bench.py --config c3 --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_bench_c4 python3 bench.py --config c4 --gpus 1 --steps 20 --warmup 5" || exit $?
