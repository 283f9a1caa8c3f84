#!/bin/bash
# round 4: exchange / schedule GPU tests after the cross-agent SearchByBoW, then the driver-args bench
export TMPDIR=/tmp
tools/gpu_run.sh \
  "600 r04b_tests python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_schedule.py tests/test_gpu_cache.py tests/test_cpp_dropin.py -m gpu -x -v --timeout 240 --timeout-method thread" \
  "300 r04b_bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5"
