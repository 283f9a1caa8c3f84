#!/bin/bash
# k_pyramid_frames workgroups per frame (row bands with halo): bench throughput for 1, 2 and 4 parts
for p in 1 2 4; do
  v=$(ORBX_PYR_PARTS=$p timeout -k 10 120 python bench.py --no-cpu --steps 20 \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['stage_ms_per_step']['pyramid'])")
  echo "pyr_parts=$p frames/s, pyramid ms = $v"
done
