#!/bin/bash
# Multi-rank rehearsal of bench.py on a one-GPU box: N ranks (default 2) share cuda:0 and exchange over
# gloo (the product run uses one GPU per rank and RCCL). Checks the barrier / max-over-ranks timing,
# the all-gather exchange and the single JSON line of rank 0.
N=${1:-2}
export ORBAMD_DIST_BACKEND=gloo ORBAMD_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus "$N" --steps 5 --warmup 1 --no-cpu --batch 512 --pipes 2
