#!/bin/bash
# frames per step x graphs x stagger sweep of the default bench (timing only). usage: tools/exp_batches2.sh
for r in 1 2; do
for cfg in "1024 4 each" "1024 4 once" "1024 4 none" "1024 2 each" "2048 4 each" "1536 3 each" "2048 8 each" "768 3 each"; do
  set -- $cfg
  out=$(timeout -k 10 120 python bench.py --sustain 0 --no-cpu --no-check --steps 20 --batch $1 --pipes $2 --stagger $3 | python -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"])') || exit 1
  echo "r$r batch $1 pipes $2 stagger $3: $out"
done; done
