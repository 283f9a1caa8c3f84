#!/bin/bash
# Profiling session on the GPU box: kernel trace + stats, then PMC passes (one counter group per
# pass, no tracing domains combined with --pmc). Outputs under gpurun_out/<tag>_*.
# usage: tools/prof_round.sh <tag>
export TMPDIR=/tmp
T=${1:-r01}
R=$GRAFT_REPO_ROOT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --sustain 0"
tools/gpu_run.sh \
  "300 ${T}_kt rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --sustain 0" \
  "300 ${T}_pmc_a rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/${T}_pmc_a -o run -- $B" \
  "300 ${T}_pmc_b rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM --output-format csv -d $R/gpurun_out/${T}_pmc_b -o run -- $B" \
  "300 ${T}_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${T}_fetch -o run -- $B" \
  "300 ${T}_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${T}_write -o run -- $B"
