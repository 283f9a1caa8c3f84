#!/bin/bash
# frames per step (B) x graphs (P): smaller per-graph batches shrink the working set (frames +
# pyramid + blurred pyramid) that the concurrent graphs keep in L2 / MALL
for cfg in "512 4" "768 4" "1024 4" "512 2" "2048 8"; do
  set -- $cfg
  v=$(timeout -k 10 120 python bench.py --sustain 0 --no-cpu --steps 20 --batch $1 --pipes $2 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'])")
  echo "B=$1 P=$2 frames/s = $v"
done
