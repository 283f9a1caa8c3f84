#!/bin/bash
# Marginal cost of each stage in the overlapped bench schedule: variants built with
# -DORBX_SKIP_WARM=<bit> (capi.cpp skip_warm) skip one stage after warm-up; the frames/s gained is that
# stage's share of the step. usage: tools/exp_marginal.sh v1 v2 ... (run on the GPU box)
for r in 1 2; do for v in "$@"; do
  out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 120 python bench.py --sustain 0 --no-cpu --no-check --steps 30 --warmup 20 | python -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f %.3f" % (d["value"], d["ms_per_step"]))') || exit 1
  echo "r$r $v $out"; done; done
