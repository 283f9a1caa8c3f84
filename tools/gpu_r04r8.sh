#!/bin/bash
# round 4: 8-rank rehearsal of bench.py on one GPU over gloo with the round-4 exchange (keyframe BoW, slot
# SearchForTriangulation and SearchByBoW against all 8 slots), and bench.py --gpus 2 launching its own ranks
export TMPDIR=/tmp
tools/gpu_run.sh \
  "400 r04_rehearse_8ranks_gloo tools/rehearse_ranks.sh 8" \
  "300 r04_bench_gpus2_gloo env ORBAMD_DIST_BACKEND=gloo ORBAMD_BENCH_DEVICE=0 python3 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu --batch 512 --pipes 2 --sustain 0" || exit $?
grep '^{' gpurun_out/r04_rehearse_8ranks_gloo.log | head -c 1500
