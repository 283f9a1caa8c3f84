#!/bin/bash
# HW-queue experiment: bench.py throughput vs GPU_MAX_HW_QUEUES (HIP's per-process hardware queues,
# default 4) and the number of concurrent graphs. One process per setting (the variable is read at
# HIP init). Prints one line per configuration.
for q in 4 8 16; do
  for p in 4 6 8; do
    v=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --sustain 0 --no-cpu --pipes $p --batch $((256 * p)) --steps 20 \
        | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")
    echo "queues=$q pipes=$p frames/s,ms = $v"
  done
done
