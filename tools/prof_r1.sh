#!/bin/bash
# Round-1 profiling session on the GPU box (see tools/gpu_run.sh for the stop-on-fault rule).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh \
  "600 gputests python -m pytest tests -m gpu -q" \
  "300 bench256 python bench.py --steps 20 --warmup 3 --batch 256 --cpu-seconds 10" \
  "300 prof_kt rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o run -- python3 bench.py --steps 10 --warmup 2 --batch 256 --no-cpu" \
  "300 prof_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --batch 256 --no-cpu" \
  "300 prof_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 bench.py --steps 3 --warmup 1 --batch 256 --no-cpu"
