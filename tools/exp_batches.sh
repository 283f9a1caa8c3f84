#!/bin/bash
# frames/s of the current head at several (frames per step, graphs) splits (no CPU leg, no check)
for cfg in "1024 4" "1024 2" "2048 4" "2048 8" "1536 6" "1024 8"; do
  set -- $cfg
  out=$(timeout -k 10 180 python bench.py --sustain 0 --no-cpu --no-check --steps 20 --batch $1 --pipes $2 | \
    python -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f" % d["value"])') || exit $?
  echo "batch $1 pipes $2: $out frames/s"
done
