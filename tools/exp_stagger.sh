#!/bin/bash
# graph stagger modes of bench.py (see --stagger)
for m in each once none; do
  v=$(timeout -k 10 120 python bench.py --sustain 0 --no-cpu --steps 20 --stagger $m \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['stage_ms_per_step']['fast_cells'])")
  echo "stagger=$m frames/s, FAST ms = $v"
done
