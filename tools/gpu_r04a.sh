#!/bin/bash
# round 4: GPU suite + driver-args bench + default bench on the current head
export TMPDIR=/tmp
tools/gpu_run.sh \
  "600 r04a_tests python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread" \
  "300 r04a_bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "300 r04a_bench python3 bench.py"
